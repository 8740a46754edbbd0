#!/bin/bash
# Sweep + rocprofv3 kernel trace / PMC passes of bench.py (development tool).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
CFG="${1:-c3}"
timeout -k 10 300 python bench.py --config "$CFG" > gpurun_out/bench_full_$CFG.log 2>&1 || { echo "BENCH FAILED rc=$?"; tail -20 gpurun_out/bench_full_$CFG.log; exit 1; }
tail -1 gpurun_out/bench_full_$CFG.log
B="python3 $R/bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace_$CFG" -o run --output-format csv -- $B > gpurun_out/prof_trace_$CFG.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/prof_trace_$CFG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/prof_fetch_$CFG" -o run --output-format csv -- $B > gpurun_out/prof_fetch_$CFG.log 2>&1 || { echo "FETCH FAILED rc=$?"; tail -20 gpurun_out/prof_fetch_$CFG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/prof_write_$CFG" -o run --output-format csv -- $B > gpurun_out/prof_write_$CFG.log 2>&1 || { echo "WRITE FAILED rc=$?"; tail -20 gpurun_out/prof_write_$CFG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-trace -d "$R/gpurun_out/prof_lds_$CFG" -o run --output-format csv -- $B > gpurun_out/prof_lds_$CFG.log 2>&1 || { echo "LDS FAILED rc=$?"; tail -20 gpurun_out/prof_lds_$CFG.log; exit 1; }
find gpurun_out/prof_* -name '*.csv' | head -20
echo PROF_OK
