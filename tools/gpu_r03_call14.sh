#!/bin/bash
# Round-3: flat-XOR one-workgroup-per-tile default (XOR tests) and the launch-shape ceiling of the
# codec access patterns (mix_grid_probe).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -k "xor or flat" tests/ -m gpu > gpurun_out/r03_xor_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_xor_tests.log; exit 1; }
tail -1 gpurun_out/r03_xor_tests.log
timeout -k 10 400 python3 tools/mix_grid_probe.py > gpurun_out/r03_mix_grid_probe.log 2>&1 || { echo PROBE_FAILED; tail -20 gpurun_out/r03_mix_grid_probe.log; exit 1; }
cat gpurun_out/r03_mix_grid_probe.log
timeout -k 10 400 python3 tools/stream_chunk_ab.py > gpurun_out/r03_stream_chunk_ab.log 2>&1 || { echo CHUNK_FAILED; tail -20 gpurun_out/r03_stream_chunk_ab.log; exit 1; }
cat gpurun_out/r03_stream_chunk_ab.log
echo CALL14_OK
