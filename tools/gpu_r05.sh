#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -1 "gpurun_out/r05_$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; tail -30 "gpurun_out/r05_$name.log"; exit 1; }; }
step smoke_mid 400 python -c "import __graft_entry__ as g; g.smoke()"
step bench_mid 600 python bench.py
tail -1 gpurun_out/r05_bench_mid.log
echo ALL_OK
