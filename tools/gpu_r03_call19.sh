#!/bin/bash
# Round-3: lane-shift fold in the bitsliced crc variant (C3 A/B), framed tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/r03_frame_tests5.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_frame_tests5.log; exit 1; }
tail -1 gpurun_out/r03_frame_tests5.log
timeout -k 10 500 python3 tools/frame_bench.py --no-crc-sweep --fused-sweep > gpurun_out/r03_fused_sweep_lane.log 2>&1 || { echo FB_FAILED; tail -20 gpurun_out/r03_fused_sweep_lane.log; exit 1; }
grep -E 'fused_crc|"checksum": 2' gpurun_out/r03_fused_sweep_lane.log
echo CALL19_OK
