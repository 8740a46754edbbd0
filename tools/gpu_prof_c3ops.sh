#!/bin/bash
# rocprofv3 kernel trace + FETCH / WRITE passes of tools/c5_prof.py at C3 (PROF_CFG=c3): encode,
# decode {0,1,2,3} and the mixed {0,5,10,13}, 30 launches each, on the one-wave bitsliced kernel
# then on the LDS-table stream kernel.  Summarise where gpurun_out/ was merged back:
#   PROF_CFG=c3 tools/summarize_prof.py c3ops r04 --command "PROF_CFG=c3 python3 tools/c5_prof.py" \
#     --algo-bytes 3758096384 --window bs_encode:ecamd_bs_kernel:38:20 \
#     --window bs_decode_0123:ecamd_bs_kernel:68:20 --window bs_decode_mixed:ecamd_bs_kernel:98:20 \
#     (the LDS-table passes run as 2 launches each: their HIP-event rates are in the log)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp PROF_CFG=c3
B="python3 $R/tools/c5_prof.py"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace_c3ops" -o run --output-format csv -- $B > gpurun_out/prof_trace_c3ops.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/prof_trace_c3ops.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/prof_fetch_c3ops" -o run --output-format csv -- $B > gpurun_out/prof_fetch_c3ops.log 2>&1 || { echo "FETCH FAILED rc=$?"; tail -20 gpurun_out/prof_fetch_c3ops.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/prof_write_c3ops" -o run --output-format csv -- $B > gpurun_out/prof_write_c3ops.log 2>&1 || { echo "WRITE FAILED rc=$?"; tail -20 gpurun_out/prof_write_c3ops.log; exit 1; }
grep '^{' gpurun_out/prof_trace_c3ops.log
echo PROF_C3OPS_OK
