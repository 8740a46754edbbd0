#!/bin/bash
# rocprofv3 kernel trace + PMC passes (separate runs) of tools/xor_prof.py: flat_xor_hd batch
# encode / decode at (3,3,3) 4 KiB and (10,6,4) 1 MiB.  Usage: tools/gpu_prof_xor.sh
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/tools/xor_prof.py"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace_xor" -o run --output-format csv -- $B > gpurun_out/prof_trace_xor.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/prof_trace_xor.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/prof_fetch_xor" -o run --output-format csv -- $B > gpurun_out/prof_fetch_xor.log 2>&1 || { echo "FETCH FAILED rc=$?"; tail -20 gpurun_out/prof_fetch_xor.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/prof_write_xor" -o run --output-format csv -- $B > gpurun_out/prof_write_xor.log 2>&1 || { echo "WRITE FAILED rc=$?"; tail -20 gpurun_out/prof_write_xor.log; exit 1; }
echo PROF_XOR_OK
