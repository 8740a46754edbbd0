#!/bin/bash
# PMC passes over tools/frame_bench.py for the CRC kernels (LDS / VALU balance).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/tools/frame_bench.py --reps 1"
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d "$R/gpurun_out/cprof_a" -o run --output-format csv -- $B > gpurun_out/cprof_a.log 2>&1 || { echo "A FAILED rc=$?"; tail -20 gpurun_out/cprof_a.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --kernel-trace -d "$R/gpurun_out/cprof_b" -o run --output-format csv -- $B > gpurun_out/cprof_b.log 2>&1 || { echo "B FAILED rc=$?"; tail -20 gpurun_out/cprof_b.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE SQ_INSTS_VMEM_RD --kernel-trace -d "$R/gpurun_out/cprof_c" -o run --output-format csv -- $B > gpurun_out/cprof_c.log 2>&1 || { echo "C FAILED rc=$?"; tail -20 gpurun_out/cprof_c.log; exit 1; }
echo PROF_OK
