#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -1 "gpurun_out/r05_$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; exit 1; }; }
ECAMD_PERCALL_BAR_KIB=1024 step tests_bar 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frontend.py tests/test_gpu_threaded.py tests/test_gpu_reference_api.py tests/test_ref_api_slap.py tests/test_gpu_errors.py tests/test_foreign_codec.py tests/test_percall_devices.py
for rep in a b; do
step lat3_def$rep 300 python -u tools/latency_bench.py --codec own --reps 25
ECAMD_PERCALL_BAR_KIB=1024 step lat3_bar$rep 300 python -u tools/latency_bench.py --codec own --reps 25
done
echo ALL_OK
