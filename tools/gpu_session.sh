#!/bin/bash
# Development GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -2 "gpurun_out/r05_$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; tail -30 "gpurun_out/r05_$name.log"; exit 1; }; }
step small_tests 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests
step percall_new_trace 150 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_percall_new" -o run --output-format csv -- python3 tools/percall_trace.py 4096 300
ECAMD_TUNE=small_lane=2 step percall_l2_trace 150 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_percall_l2" -o run --output-format csv -- python3 tools/percall_trace.py 4096 300
step lat_l4 600 python3 tools/latency_bench.py --codec own
ECAMD_TUNE=small_lane=2 step lat_l2 600 python3 tools/latency_bench.py --codec own
ECAMD_PERCALL_BAR_KIB=64 step lat_bar 600 python3 tools/latency_bench.py --codec own
echo ALL_OK
