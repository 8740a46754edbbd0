#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 tools/c3_tile_ab.py c2 chunk > gpurun_out/r03_c2_chunk_ab.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03_c2_chunk_ab.log; exit 1; }
cat gpurun_out/r03_c2_chunk_ab.log
