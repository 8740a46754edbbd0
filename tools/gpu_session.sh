#!/bin/bash
# Development GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
export SKP_LAUNCH=1
for v in 0 1; do
  if [ $v = 1 ]; then export SKP_H2D=1; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_skh$v" -o run --output-format csv -- python3 tools/small_kernel_probe.py 416 300 > gpurun_out/r05_skh$v.log 2>&1 || { echo FAILED; tail -20 gpurun_out/r05_skh$v.log; exit 1; }
  grep case gpurun_out/r05_skh$v.log
done
echo ALL_OK
