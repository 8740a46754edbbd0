#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/c3_tile_ab.py c2 chunk > gpurun_out/r03_c2_chunk_ab2.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03_c2_chunk_ab2.log; exit 1; }
cat gpurun_out/r03_c2_chunk_ab2.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_device.py > gpurun_out/r03_c2_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_c2_tests.log; exit 1; }
tail -1 gpurun_out/r03_c2_tests.log
