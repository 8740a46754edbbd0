#!/bin/bash
# Round 6: HIP API + kernel trace of one-thread 4 KiB per-call encodes (tools/percall_trace.py), to see
# where the ~20 us of a small call go (launch call, synchronisation, kernel).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace --stats -d "$R/gpurun_out/r06_api_4096" -o run --output-format csv -- python3 tools/percall_trace.py 4096 400 1 > gpurun_out/r06_api_4096.log 2>&1 || { echo "TRACE FAILED"; tail -20 gpurun_out/r06_api_4096.log; exit 1; }
grep median gpurun_out/r06_api_4096.log
echo API_OK
