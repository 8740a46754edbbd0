#!/bin/bash
# rocprofv3 evidence for the bench line: kernel trace + separate PMC passes of EXACTLY the driver's
# command (python3 bench.py --gpus 1 --steps 20 --warmup 5), then tools/summarize_prof.py picks
# the timed launches of the dominant kernel.  Usage: tools/gpu_prof.sh [round] [cfg]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
RND="${1:-r02}"
CFG="${2:-c3}"
B="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --config $CFG"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_trace_$CFG" -o run --output-format csv -- $B > gpurun_out/prof_trace_$CFG.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/prof_trace_$CFG.log; exit 1; }
grep '^{' gpurun_out/prof_trace_$CFG.log | tail -1 > gpurun_out/bench_prof_$CFG.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/prof_fetch_$CFG" -o run --output-format csv -- $B --no-cpu-baseline > gpurun_out/prof_fetch_$CFG.log 2>&1 || { echo "FETCH FAILED rc=$?"; tail -20 gpurun_out/prof_fetch_$CFG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/prof_write_$CFG" -o run --output-format csv -- $B --no-cpu-baseline > gpurun_out/prof_write_$CFG.log 2>&1 || { echo "WRITE FAILED rc=$?"; tail -20 gpurun_out/prof_write_$CFG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES --kernel-trace -d "$R/gpurun_out/prof_lds_$CFG" -o run --output-format csv -- $B --no-cpu-baseline > gpurun_out/prof_lds_$CFG.log 2>&1 || { echo "LDS FAILED rc=$?"; tail -20 gpurun_out/prof_lds_$CFG.log; exit 1; }
find gpurun_out/prof_*_$CFG -name '*.csv' | head -20
echo PROF_OK
