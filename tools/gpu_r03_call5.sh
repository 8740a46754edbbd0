#!/bin/bash
# Round-3 GPU call: bitsliced copy-through framed paths (tests + C5 framed bench), the bitsliced
# golden / JIT tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_frame.py -k "bitsliced or copy_through or join" tests/test_gpu_bitslice.py tests/test_gpu_bitslice_golden.py > gpurun_out/r03_bs_frame_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03_bs_frame_tests.log; exit 1; }
tail -1 gpurun_out/r03_bs_frame_tests.log
timeout -k 10 300 python3 tools/frame_c5_bench.py > gpurun_out/r03_frame_c5.log 2>&1 || { echo C5_FRAME_FAILED; tail -20 gpurun_out/r03_frame_c5.log; exit 1; }
cat gpurun_out/r03_frame_c5.log | grep op
echo CALL5_OK
