#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -2 "gpurun_out/r05_$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; exit 1; }; }
step tests_bs 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bitslice_wave.py tests/test_gpu_jit_shipped.py tests/test_gpu_bitslice_golden.py tests/test_gpu_bitslice.py
step ab_ncap 900 python -u tools/bs_wave_ab.py c3ncap c5ncap2
grep summary gpurun_out/r05_ab_ncap.log
step ab_xorcap 900 python -u tools/xor_threads_ab.py xor_per_cu 0,6,7,8,12
cat gpurun_out/r05_ab_xorcap.log | grep -v amdgpu
echo ALL_OK
