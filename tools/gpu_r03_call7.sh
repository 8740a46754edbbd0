#!/bin/bash
# Round-3: fused CRC framed encode with the codec on nibble tables -- parity tests, then the
# interleaved fused sweep (tools/frame_bench.py --fused-sweep).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_frame.py -k "fused" > gpurun_out/r03_fused_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/r03_fused_tests.log; exit 1; }
tail -1 gpurun_out/r03_fused_tests.log
timeout -k 10 400 python3 tools/frame_bench.py --no-crc-sweep --fused-sweep --reps 5 > gpurun_out/r03_fused_sweep.log 2>&1 || { echo SWEEP_FAILED; tail -20 gpurun_out/r03_fused_sweep.log; exit 1; }
grep fused_crc gpurun_out/r03_fused_sweep.log
echo CALL7_OK
