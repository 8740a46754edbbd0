#!/bin/bash
# Round-3: the bitsliced crc variant for 5-8 outputs (fold-each), framed copy grid default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/r03_frame_tests4.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_frame_tests4.log; exit 1; }
tail -1 gpurun_out/r03_frame_tests4.log
timeout -k 10 400 python3 tools/frame_c5_bench.py > gpurun_out/r03_frame_c5_crc2.log 2>&1 || { echo C5F_FAILED; tail -20 gpurun_out/r03_frame_c5_crc2.log; exit 1; }
cat gpurun_out/r03_frame_c5_crc2.log
echo CALL18_OK
