#!/bin/bash
# Round-3: tile-width probe of the C3 contiguous and mixed write patterns (tools/rot_probe.py geom).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/rot_probe.py geom > gpurun_out/r03_geom_probe3.log 2>&1 || { echo PROBE_FAILED; tail -20 gpurun_out/r03_geom_probe3.log; exit 1; }
cat gpurun_out/r03_geom_probe3.log
