#!/bin/bash
# Round-3: flat-XOR tile width A/B (tools/xor_threads_ab.py), then the XOR GPU tests with 64-thread tiles.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 tools/xor_threads_ab.py > gpurun_out/r03_xor_threads_ab2.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03_xor_threads_ab2.log; exit 1; }
cat gpurun_out/r03_xor_threads_ab2.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_xor.py tests/test_gpu_xor_batch.py tests/test_gpu_frontend.py > gpurun_out/r03_xor_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_xor_tests.log; exit 1; }
tail -1 gpurun_out/r03_xor_tests.log
