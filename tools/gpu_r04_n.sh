#!/bin/bash
# Round 4: copy-through on the one-wave bitsliced kernel by default with the next input's loads ahead
# of the copy stores (bs_wave_copy 1, bs_prefetch 2): the framing tests, then the framed A/Bs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/r04_frame_tests_n.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_frame_tests_n.log; exit 1; }
tail -1 gpurun_out/r04_frame_tests_n.log
timeout -k 10 300 python tools/cover_ab.py > gpurun_out/r04_cover_ab5.log 2>&1 || { echo "COVER rc=$?"; tail -20 gpurun_out/r04_cover_ab5.log; exit 1; }
cat gpurun_out/r04_cover_ab5.log
timeout -k 10 300 python tools/frame_bench.py --reps 4 --no-crc-sweep > gpurun_out/r04_frame_bench.log 2>&1 || { echo "FB rc=$?"; tail -20 gpurun_out/r04_frame_bench.log; exit 1; }
grep -v amdgpu gpurun_out/r04_frame_bench.log | head -40
echo R04_N_OK
