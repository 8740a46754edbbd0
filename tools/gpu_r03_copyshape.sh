#!/bin/bash
# Round-3: split / join tile shape -- frame tests with the shapes, then the A/B (tools/copy_shape_ab.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 tools/copy_shape_ab.py sizes > gpurun_out/r03_copy_shape_ab2.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03_copy_shape_ab2.log; exit 1; }
cat gpurun_out/r03_copy_shape_ab2.log
