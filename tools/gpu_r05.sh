#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -2 "gpurun_out/r05_$name.log" | cut -c1-400; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; exit 1; }; }
step ab_crccap 600 python -u tools/frame_knob_ab.py frame_crc_per_cu 0,1,2 --ct crc --ops encode
grep -v amdgpu gpurun_out/r05_ab_crccap.log
step ab_c5tile 400 python -u tools/bs_wave_ab.py c5tile
grep summary gpurun_out/r05_ab_c5tile.log
echo ALL_OK
