#!/bin/bash
# Development GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 1024 4096 16384; do
  echo "== small_chunks $c"
  ECAMD_TUNE=small_chunks=$c timeout -k 10 300 python3 tools/latency_bench.py --codec own > gpurun_out/r05_lat_sc$c.log 2>&1 || exit 1
done
echo ALL_OK
