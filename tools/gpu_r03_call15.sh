#!/bin/bash
# Round-3: full GPU suite on the round's defaults (bitsliced / XOR one workgroup per tile, C2 stream
# chunks), the C2 bench line and the C2 chunk A/B (default rule vs grid-stride).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/ -m gpu > gpurun_out/r03_gpu_tests_full2.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_gpu_tests_full2.log; exit 1; }
tail -1 gpurun_out/r03_gpu_tests_full2.log
timeout -k 10 300 python3 bench.py --config c2 --steps 20 --warmup 5 > gpurun_out/r03_bench_c2.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r03_bench_c2.log; exit 1; }
tail -1 gpurun_out/r03_bench_c2.log
CHUNKS=-1,0,2 SLOTS=0 timeout -k 10 300 python3 tools/stream_chunk_ab.py > gpurun_out/r03_stream_chunk_ab2.log 2>&1 || { echo CHUNK_FAILED; tail -20 gpurun_out/r03_stream_chunk_ab2.log; exit 1; }
cat gpurun_out/r03_stream_chunk_ab2.log
echo CALL15_OK
