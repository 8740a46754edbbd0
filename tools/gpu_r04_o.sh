#!/bin/bash
# Round 4: the crc variant with the next input's loads ahead of the copy stores (frame_crc_prefetch).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/crc_pf_ab.py > gpurun_out/r04_crc_pf_ab.log 2>&1 || { echo "AB rc=$?"; tail -20 gpurun_out/r04_crc_pf_ab.log; exit 1; }
cat gpurun_out/r04_crc_pf_ab.log
echo R04_O_OK
