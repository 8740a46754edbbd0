#!/bin/bash
# Round 4: copy-through one-wave bitsliced kernel with the next input's loads issued before the
# current input's copy stores (bs_prefetch 2 / 4) -- framed encode / decode-join A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/frame_wave_ab.py > gpurun_out/r04_frame_wave_pf_ab2.log 2>&1 || { echo "AB rc=$?"; tail -20 gpurun_out/r04_frame_wave_pf_ab2.log; exit 1; }
cat gpurun_out/r04_frame_wave_pf_ab2.log
echo R04_M_OK
