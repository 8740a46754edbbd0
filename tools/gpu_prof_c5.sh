#!/bin/bash
# rocprofv3 kernel trace + separate PMC passes of tools/c5_prof.py (C5 steady state, bitsliced and
# LDS-table kernels), summarised into profiles/<round>_c5_summary.json.  Usage: gpu_prof_c5.sh
# then, where gpurun_out/ was merged back (windows = the steady launches, tools/c5_prof.py docstring):
#   tools/summarize_prof.py c5 r02 --command "python3 tools/c5_prof.py" --algo-bytes 3758096384 \
#     --window bs_encode:ecamd_bs_kernel:38:20 --window bs_rebuild8_data:ecamd_bs_kernel:68:20 \
#     --window bs_rebuild8_mixed:ecamd_bs_kernel:98:20 --window lds_encode:gf16_hybrid_kernel:36:20 \
#     --window lds_rebuild8_data:gf16_hybrid_kernel:66:20 --window lds_rebuild8_mixed:gf16_hybrid_kernel:96:20
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/tools/c5_prof.py"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace_c5" -o run --output-format csv -- $B > gpurun_out/prof_trace_c5.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/prof_trace_c5.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/prof_fetch_c5" -o run --output-format csv -- $B > gpurun_out/prof_fetch_c5.log 2>&1 || { echo "FETCH FAILED rc=$?"; tail -20 gpurun_out/prof_fetch_c5.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/prof_write_c5" -o run --output-format csv -- $B > gpurun_out/prof_write_c5.log 2>&1 || { echo "WRITE FAILED rc=$?"; tail -20 gpurun_out/prof_write_c5.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d "$R/gpurun_out/prof_lds_c5" -o run --output-format csv -- $B > gpurun_out/prof_lds_c5.log 2>&1 || { echo "LDS FAILED rc=$?"; tail -20 gpurun_out/prof_lds_c5.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_IFETCH SQ_INSTS_VMEM SQ_INSTS_SALU --kernel-trace -d "$R/gpurun_out/prof_stall_c5" -o run --output-format csv -- $B > gpurun_out/prof_stall_c5.log 2>&1 || { echo "STALL FAILED rc=$?"; tail -20 gpurun_out/prof_stall_c5.log; exit 1; }
grep '^{' gpurun_out/prof_trace_c5.log
echo PROF_C5_OK
