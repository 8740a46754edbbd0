#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -2 "gpurun_out/r05_$name.log" | cut -c1-400; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; exit 1; }; }
step prof 900 bash tools/gpu_prof.sh r05 c3
B="python3 bench.py --gpus 1 --steps 20 --warmup 5 --config c3 --no-c5 --no-scatter --no-cpu-baseline"
step pmc_sq 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/r05_pmc_sq" -o run --output-format csv -- $B
step ab_copycap2 600 python -u tools/frame_wave_ab.py cap2
cat gpurun_out/r05_ab_copycap2.log | grep -v amdgpu
echo ALL_OK
