#!/bin/bash
# Round-3: lane-shift fold default (1 position set) for the C3 crc variant: framed tests, sweep,
# C5 CRC bench, the framed-CRC profile.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py tests/test_gpu_bitslice_golden.py > gpurun_out/r03_frame_tests6.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_frame_tests6.log; exit 1; }
tail -1 gpurun_out/r03_frame_tests6.log
timeout -k 10 500 python3 tools/frame_bench.py --no-crc-sweep --fused-sweep > gpurun_out/r03_fused_sweep_lane2.log 2>&1 || { echo FB_FAILED; tail -20 gpurun_out/r03_fused_sweep_lane2.log; exit 1; }
grep -E 'fused_crc|"checksum": 2' gpurun_out/r03_fused_sweep_lane2.log
timeout -k 10 400 python3 tools/frame_c5_bench.py > gpurun_out/r03_frame_c5_crc3.log 2>&1 || { echo C5F_FAILED; tail -20 gpurun_out/r03_frame_c5_crc3.log; exit 1; }
grep crc32 gpurun_out/r03_frame_c5_crc3.log
bash tools/gpu_prof_frame_crc.sh || exit 1
echo CALL20_OK
