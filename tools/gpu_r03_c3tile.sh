#!/bin/bash
# Round-3: C3 stream kernel in one-wave-tile shapes (tools/c3_tile_ab.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/c3_tile_ab.py > gpurun_out/r03_c3_tile_ab.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03_c3_tile_ab.log; exit 1; }
cat gpurun_out/r03_c3_tile_ab.log
