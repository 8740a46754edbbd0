#!/bin/bash
# Round-3: C5 bitsliced launch-grid A/B at 32 and 128 stripes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/c5_grid_ab.py > gpurun_out/r03_c5_grid_ab.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03_c5_grid_ab.log; exit 1; }
grep '"op"' gpurun_out/r03_c5_grid_ab.log
C5_S=128 timeout -k 10 300 python3 tools/c5_grid_ab.py > gpurun_out/r03_c5_grid_ab128.log 2>&1 || { echo AB128_FAILED; tail -20 gpurun_out/r03_c5_grid_ab128.log; exit 1; }
grep '"op"' gpurun_out/r03_c5_grid_ab128.log
echo CALL11_OK
