#!/bin/bash
# Round-3 GPU call: streaming join re-check, framed bench, flat-XOR geometry sweep, per-call
# latency beside the reference codec, the default bench line and a 2-rank gloo rehearsal.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_frame.py -k "stream or systematic or split or join or decode" > gpurun_out/r03_frame_tests.log 2>&1 || { echo FRAME_TESTS_FAILED; tail -30 gpurun_out/r03_frame_tests.log; exit 1; }
tail -1 gpurun_out/r03_frame_tests.log
timeout -k 10 240 python3 tools/frame_bench.py --no-crc-sweep --reps 5 > gpurun_out/r03_frame_bench2.log 2>&1 || { echo FRAME_BENCH_FAILED; tail -20 gpurun_out/r03_frame_bench2.log; exit 1; }
grep systematic gpurun_out/r03_frame_bench2.log | grep '"lost": \[\]'
timeout -k 10 300 python3 tools/xor_geom_sweep.py --rounds 5 > gpurun_out/r03_xor_geom.log 2>&1 || { echo XOR_GEOM_FAILED; tail -20 gpurun_out/r03_xor_geom.log; exit 1; }
timeout -k 10 300 python3 tools/latency_bench.py --reps 25 > gpurun_out/r03_latency_bench.log 2>&1 || { echo LATENCY_FAILED; tail -20 gpurun_out/r03_latency_bench.log; exit 1; }
tail -1 gpurun_out/r03_latency_bench.log
timeout -k 10 300 python3 bench.py > gpurun_out/r03_bench_default.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r03_bench_default.log; exit 1; }
ECAMD_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 10 --warmup 2 --no-c5 > gpurun_out/r03_rehearsal_2ranks.log 2>&1 || { echo REHEARSAL_FAILED; tail -20 gpurun_out/r03_rehearsal_2ranks.log; exit 1; }
echo CALL3_OK
