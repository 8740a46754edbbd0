#!/bin/bash
# C5 lookup-engine variants (tools/c5_variants.py): HIP-event times, then rocprofv3 kernel trace
# and SQ / LDS counter passes, each its own run.  Usage: tools/gpu_prof_c5.sh [variant specs...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/tools/c5_variants.py $*"
timeout -k 10 200 $B > gpurun_out/c5_variants.log 2>&1 || { echo "C5 VARIANTS FAILED rc=$?"; tail -20 gpurun_out/c5_variants.log; exit 1; }
cat gpurun_out/c5_variants.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace_c5v" -o run --output-format csv -- $B > gpurun_out/prof_trace_c5v.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/prof_trace_c5v.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --kernel-trace -d "$R/gpurun_out/prof_sqa_c5v" -o run --output-format csv -- $B > gpurun_out/prof_sqa_c5v.log 2>&1 || { echo "SQA FAILED rc=$?"; tail -20 gpurun_out/prof_sqa_c5v.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR --kernel-trace -d "$R/gpurun_out/prof_sqb_c5v" -o run --output-format csv -- $B > gpurun_out/prof_sqb_c5v.log 2>&1 || { echo "SQB FAILED rc=$?"; tail -20 gpurun_out/prof_sqb_c5v.log; exit 1; }
echo PROF_C5_OK
