#!/bin/bash
# One PMC pass (SQ issue / wait / LDS counters) over tools/frame_bench.py: what bounds
# the fused CRC framed encode kernel, beside the plain framed encode in the same run.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/tools/frame_bench.py --no-crc-sweep --reps 4"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d "$R/gpurun_out/prof_sq_fused" -o run --output-format csv -- $B > gpurun_out/prof_sq_fused.log 2>&1 || { echo "SQ FAILED rc=$?"; tail -20 gpurun_out/prof_sq_fused.log; exit 1; }
echo PROF_FUSED_OK
