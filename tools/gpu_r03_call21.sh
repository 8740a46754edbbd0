#!/bin/bash
# Round-3: rocprofv3 of the flat-XOR kernel on its one-workgroup-per-tile default, and of the
# systematic framed decode (streaming join), each with FETCH / WRITE passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_prof_xor.sh || exit 1
grep '^{' gpurun_out/prof_trace_xor.log
bash tools/gpu_prof_join.sh || exit 1
timeout -k 10 500 python3 tools/frame_bench.py --no-crc-sweep > gpurun_out/r03_frame_bench8.log 2>&1 || { echo FB_FAILED; tail -20 gpurun_out/r03_frame_bench8.log; exit 1; }
grep -E "swift|minus" gpurun_out/r03_frame_bench8.log
echo CALL21_OK
