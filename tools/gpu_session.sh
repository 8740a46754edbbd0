#!/bin/bash
# Development GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -1 "gpurun_out/r05_$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; tail -30 "gpurun_out/r05_$name.log"; exit 1; }; }
step frame_tests_lds 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py tests/test_gpu_frontend.py
B="python3 $R/tools/frame_crc_prof.py wave_crc"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_crcwave3" -o run --output-format csv -- $B > gpurun_out/r05_crcwave3_prof.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/r05_crcwave3_prof.log; exit 1; }
grep '^{' gpurun_out/r05_crcwave3_prof.log
echo ALL_OK
