#!/bin/bash
# Round-3 GPU check: the whole -m gpu suite, then the framed-path bench (systematic decode) and
# the flat-XOR geometry sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03_gpu_tests.log 2>&1 || { echo GPU_TESTS_FAILED; tail -40 gpurun_out/r03_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r03_gpu_tests.log
timeout -k 10 240 python3 tools/frame_bench.py --no-crc-sweep --reps 5 > gpurun_out/r03_frame_bench.log 2>&1 || { echo FRAME_BENCH_FAILED; tail -20 gpurun_out/r03_frame_bench.log; exit 1; }
grep systematic gpurun_out/r03_frame_bench.log
timeout -k 10 300 python3 tools/xor_geom_sweep.py --rounds 5 > gpurun_out/r03_xor_geom.log 2>&1 || { echo XOR_GEOM_FAILED; tail -20 gpurun_out/r03_xor_geom.log; exit 1; }
echo CALL2_OK
