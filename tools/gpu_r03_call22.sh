#!/bin/bash
# Round-3: realigned copy-through loads (gf16_realign_kernel): framed tests, A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py tests/test_gpu_frontend.py > gpurun_out/r03_frame_tests7.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_frame_tests7.log; exit 1; }
tail -1 gpurun_out/r03_frame_tests7.log
timeout -k 10 400 python3 tools/realign_ab.py > gpurun_out/r03_realign_ab.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03_realign_ab.log; exit 1; }
cat gpurun_out/r03_realign_ab.log
echo CALL22_OK
