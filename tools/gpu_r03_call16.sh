#!/bin/bash
# Round-3: fused-CRC test without skips, split CRC launch-shape sweep, framed benches on the
# one-workgroup-per-tile bitsliced kernel.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_frame.py -k fused_crc_matches_split -rs > gpurun_out/r03_fused_crc_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_fused_crc_tests.log; exit 1; }
tail -1 gpurun_out/r03_fused_crc_tests.log
timeout -k 10 300 python3 tools/crc_grid_sweep.py > gpurun_out/r03_crc_grid_sweep.log 2>&1 || { echo CRC_FAILED; tail -20 gpurun_out/r03_crc_grid_sweep.log; exit 1; }
cat gpurun_out/r03_crc_grid_sweep.log
timeout -k 10 300 python3 tools/frame_c5_bench.py > gpurun_out/r03_frame_c5_grid.log 2>&1 || { echo C5F_FAILED; tail -20 gpurun_out/r03_frame_c5_grid.log; exit 1; }
cat gpurun_out/r03_frame_c5_grid.log
timeout -k 10 400 python3 tools/frame_bench.py --no-crc-sweep > gpurun_out/r03_frame_bench6.log 2>&1 || { echo FB_FAILED; tail -20 gpurun_out/r03_frame_bench6.log; exit 1; }
cat gpurun_out/r03_frame_bench6.log
echo CALL16_OK
