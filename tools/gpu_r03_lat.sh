#!/bin/bash
# Round-3: per-call latency A/B of the copy helpers' batch threshold (tools/latency_ab.py).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 800 python3 tools/latency_ab.py > gpurun_out/r03_latency_ab5.log 2>&1 || { echo LATAB_FAILED; tail -20 gpurun_out/r03_latency_ab5.log; exit 1; }
echo LAT_OK
