#!/bin/bash
# Round-3: framed bench with the bitsliced-launch counter, the flat-XOR profile on another box.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/frame_bench.py --no-crc-sweep --reps 5 > gpurun_out/r03_frame_bench5.log 2>&1 || { echo FRAME_BENCH_FAILED; tail -20 gpurun_out/r03_frame_bench5.log; exit 1; }
grep '"op": "frame_encode"' gpurun_out/r03_frame_bench5.log
timeout -k 10 200 python3 tools/frame_crc_prof.py > gpurun_out/r03_frame_crc_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r03_frame_crc_prof.log; exit 1; }
cat gpurun_out/r03_frame_crc_prof.log | grep path
echo CALL10_OK
