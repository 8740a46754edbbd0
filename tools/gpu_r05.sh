#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -2 "gpurun_out/r05_$name.log" | cut -c1-400; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; exit 1; }; }
step tests_percall 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frontend.py tests/test_gpu_threaded.py tests/test_gpu_reference_api.py tests/test_ref_api_slap.py tests/test_gpu_errors.py tests/test_foreign_codec.py
ECAMD_PERCALL_ZEROCOPY_KIB=0 step lat_zc0 300 python -u tools/latency_bench.py --codec own --reps 25
ECAMD_PERCALL_ZEROCOPY_KIB=256 step lat_zc256 300 python -u tools/latency_bench.py --codec own --reps 25
ECAMD_PERCALL_ZEROCOPY_KIB=4096 step lat_zc4096 300 python -u tools/latency_bench.py --codec own --reps 25
LD_LIBRARY_PATH=$R/oracle/_ref step lat_ref 300 python -u tools/latency_bench.py --codec ref --reps 25
step ab_crccap 600 python -u tools/frame_knob_ab.py frame_crc_per_cu 0,1,2 --ct crc --ops encode
grep -v amdgpu gpurun_out/r05_ab_crccap.log
step ab_c5tile 400 python -u tools/bs_wave_ab.py c5tile
grep summary gpurun_out/r05_ab_c5tile.log
echo ALL_OK
