#!/bin/bash
# Development GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r05_gpu_tests_skipbs.log 2>&1; rc=$?
tail -25 gpurun_out/r05_gpu_tests_skipbs.log | cut -c1-250
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python3 tools/latency_bench.py --codec own > gpurun_out/r05_lat_skipbs.log 2>&1 || exit 1
echo ALL_OK
