#!/bin/bash
# Round 4: framed flat-XOR decode-join (frame_xor_copy) and the late copy (bs_late_copy): the framing
# tests, then the two A/Bs.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/r04_frame_tests_r.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_frame_tests_r.log; exit 1; }
tail -1 gpurun_out/r04_frame_tests_r.log
timeout -k 10 300 python tools/xor_decode_ab.py > gpurun_out/r04_xor_decode_ab.log 2>&1 || { echo "AB rc=$?"; tail -20 gpurun_out/r04_xor_decode_ab.log; exit 1; }
cat gpurun_out/r04_xor_decode_ab.log
timeout -k 10 400 python tools/late_copy_ab.py > gpurun_out/r04_late_copy_ab.log 2>&1 || { echo "LC rc=$?"; tail -20 gpurun_out/r04_late_copy_ab.log; exit 1; }
cat gpurun_out/r04_late_copy_ab.log
echo R04_R_OK
