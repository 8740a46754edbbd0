#!/bin/bash
# Development GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -2 "gpurun_out/r05_$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; tail -30 "gpurun_out/r05_$name.log"; exit 1; }; }
ECAMD_PERCALL_ZEROCOPY_MODE=3 ECAMD_TUNE=small_lane=4 step lat_m3l4a 400 python3 tools/latency_bench.py --codec own
step lat_m2c 400 python3 tools/latency_bench.py --codec own
ECAMD_PERCALL_ZEROCOPY_MODE=3 ECAMD_TUNE=small_lane=4 step lat_m3l4b 400 python3 tools/latency_bench.py --codec own
ECAMD_PERCALL_ZEROCOPY_MODE=3 ECAMD_TUNE=small_lane=16 step lat_m3l16 400 python3 tools/latency_bench.py --codec own
echo ALL_OK
