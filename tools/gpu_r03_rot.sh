#!/bin/bash
# Round-3: tile-width probe of the C5 rebuild patterns (tools/rot_probe.py geom5).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/rot_probe.py geom5 > gpurun_out/r03_geom5_probe.log 2>&1 || { echo PROBE_FAILED; tail -20 gpurun_out/r03_geom5_probe.log; exit 1; }
cat gpurun_out/r03_geom5_probe.log
