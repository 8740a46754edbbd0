#!/bin/bash
# Round 4: one-wave bitsliced kernel with the next input's loads issued before each network
# (bs_prefetch 2 / 4) against none, C3 encode / decodes (bytes checked against the LDS tables).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/bs_wave_ab.py c3pf > gpurun_out/r04_bs_prefetch_ab.log 2>&1 || { echo "AB rc=$?"; tail -20 gpurun_out/r04_bs_prefetch_ab.log; exit 1; }
grep summary gpurun_out/r04_bs_prefetch_ab.log
echo R04_L_OK
