#!/bin/bash
# rocprofv3 kernel trace + HBM PMC passes of tools/frame_bench.py (framing / CRC kernels).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/tools/frame_bench.py --reps 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/fprof_trace" -o run --output-format csv -- $B > gpurun_out/fprof_trace.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/fprof_trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/fprof_fetch" -o run --output-format csv -- $B > gpurun_out/fprof_fetch.log 2>&1 || { echo "FETCH FAILED rc=$?"; tail -20 gpurun_out/fprof_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/fprof_write" -o run --output-format csv -- $B > gpurun_out/fprof_write.log 2>&1 || { echo "WRITE FAILED rc=$?"; tail -20 gpurun_out/fprof_write.log; exit 1; }
find gpurun_out/fprof_* -name '*.csv' | head -20
echo PROF_OK
