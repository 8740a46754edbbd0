#!/bin/bash
# rocprofv3 kernel trace + HBM PMC passes of tools/frame_crc_prof.py (framed CRC32 encode at C3:
# the bitsliced crc variant, then the LDS-table fused kernel).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/tools/frame_crc_prof.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace_framecrc" -o run --output-format csv -- $B > gpurun_out/prof_trace_framecrc.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/prof_trace_framecrc.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/prof_fetch_framecrc" -o run --output-format csv -- $B > gpurun_out/prof_fetch_framecrc.log 2>&1 || { echo "FETCH FAILED rc=$?"; tail -20 gpurun_out/prof_fetch_framecrc.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/prof_write_framecrc" -o run --output-format csv -- $B > gpurun_out/prof_write_framecrc.log 2>&1 || { echo "WRITE FAILED rc=$?"; tail -20 gpurun_out/prof_write_framecrc.log; exit 1; }
grep '^{' gpurun_out/prof_trace_framecrc.log
echo PROF_FRAMECRC_OK
