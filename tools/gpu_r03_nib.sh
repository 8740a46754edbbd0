#!/bin/bash
# Round-3: nibble piece tables in the bitsliced crc variant -- fused-CRC frame tests, then the A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py -k "fused_crc_matches_split" > gpurun_out/r03_nib_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_nib_tests.log; exit 1; }
tail -1 gpurun_out/r03_nib_tests.log
timeout -k 10 500 python3 tools/crc_nib_ab.py > gpurun_out/r03_crc_nib_ab.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03_crc_nib_ab.log; exit 1; }
cat gpurun_out/r03_crc_nib_ab.log
