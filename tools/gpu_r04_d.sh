#!/bin/bash
# Round 4: rocprofv3 evidence of the driver's bench command with the one-wave bitsliced C3 default
# (kernel trace + FETCH / WRITE / LDS passes, tools/gpu_prof.sh) and one SQ pass of the same
# command (VALU issue, wait shares) summarised by tools/summarize_pmc.py; then the second form of the
# DPP realign (the last lane's load in the same burst) for the split / join and the copy-through
# stream kernel, and the bitsliced framed-CRC work-unit sweep.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_prof.sh r04 c3 || exit 1
B="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --config c3 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/pmc_sq_c3" -o run --output-format csv -- $B > gpurun_out/pmc_sq_c3.log 2>&1 || { echo "SQ FAILED rc=$?"; tail -20 gpurun_out/pmc_sq_c3.log; exit 1; }
python3 tools/summarize_pmc.py gpurun_out/r04_c3_pmc_sq.json gpurun_out/pmc_sq_c3 --command "$B" || exit 1
timeout -k 10 300 python tools/copy_shape_ab.py dpp > gpurun_out/r04_copy_dpp_ab2.log 2>&1 || { echo "DPP rc=$?"; exit 1; }
timeout -k 10 300 python tools/realign_ab.py > gpurun_out/r04_realign_ab2.log 2>&1 || { echo "REALIGN rc=$?"; exit 1; }
timeout -k 10 300 python tools/frame_bench.py --fused-sweep --no-crc-sweep --reps 4 > gpurun_out/r04_fused_sweep.log 2>&1 || { echo "FUSED rc=$?"; exit 1; }
echo R04_D_OK
