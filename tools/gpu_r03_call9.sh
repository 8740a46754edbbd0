#!/bin/bash
# Round-3: whole GPU suite with the bitsliced crc variant as the default, its rocprofv3 evidence,
# the framed bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_gpu_tests2.log 2>&1 || { echo GPU_TESTS_FAILED; tail -40 gpurun_out/r03_gpu_tests2.log; exit 1; }
tail -1 gpurun_out/r03_gpu_tests2.log
bash tools/gpu_prof_frame_crc.sh || exit 1
timeout -k 10 300 python3 tools/frame_bench.py --no-crc-sweep --reps 5 > gpurun_out/r03_frame_bench4.log 2>&1 || { echo FRAME_BENCH_FAILED; tail -20 gpurun_out/r03_frame_bench4.log; exit 1; }
grep '"op": "frame_encode"' gpurun_out/r03_frame_bench4.log
echo CALL9_OK
