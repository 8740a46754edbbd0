#!/bin/bash
# rocprofv3 kernel trace + HBM PMC passes of tools/join_prof.py (streaming join:
# systematic framed decode, C3 and Swift segments).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/tools/join_prof.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace_join" -o run --output-format csv -- $B > gpurun_out/prof_trace_join.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/prof_trace_join.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/prof_fetch_join" -o run --output-format csv -- $B > gpurun_out/prof_fetch_join.log 2>&1 || { echo "FETCH FAILED rc=$?"; tail -20 gpurun_out/prof_fetch_join.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/prof_write_join" -o run --output-format csv -- $B > gpurun_out/prof_write_join.log 2>&1 || { echo "WRITE FAILED rc=$?"; tail -20 gpurun_out/prof_write_join.log; exit 1; }
grep '^{' gpurun_out/prof_trace_join.log
echo PROF_JOIN_OK
