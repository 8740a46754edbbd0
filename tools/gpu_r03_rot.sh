#!/bin/bash
# Round-3: launch shape of the stream kernel for the C3 mixed decode (tools/mixed_shape_ab.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python3 tools/mixed_shape_ab.py > gpurun_out/r03_mixed_shape_ab.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03_mixed_shape_ab.log; exit 1; }
cat gpurun_out/r03_mixed_shape_ab.log
