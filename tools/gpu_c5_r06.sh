#!/bin/bash
# Round 6, VERDICT r05 #1: isolated counters of C5's 16 KiB-tile dispatches at today's defaults (SQ pass,
# FETCH / WRITE passes, kernel trace of `bench.py --config c5 --no-scatter --no-cpu-baseline`), then the
# 20-read / 8-write probe in the codec's launch shapes under per-CU caps (tools/c5_ceiling.py).
# Outputs under gpurun_out/r06_c5_*; summaries go to profiles/ (tools/summarize_pmc.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --config c5 --no-scatter --no-cpu-baseline"
echo "command: $B"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r06_c5_trace" -o run --output-format csv -- $B > gpurun_out/r06_c5_trace.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/r06_c5_trace.log; exit 1; }
grep '^{' gpurun_out/r06_c5_trace.log | tail -1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/r06_c5_pmc_sq" -o run --output-format csv -- $B > gpurun_out/r06_c5_pmc_sq.log 2>&1 || { echo "SQ FAILED rc=$?"; tail -20 gpurun_out/r06_c5_pmc_sq.log; exit 1; }
echo SQ_OK
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/r06_c5_pmc_fetch" -o run --output-format csv -- $B > gpurun_out/r06_c5_pmc_fetch.log 2>&1 || { echo "FETCH FAILED rc=$?"; tail -20 gpurun_out/r06_c5_pmc_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/r06_c5_pmc_write" -o run --output-format csv -- $B > gpurun_out/r06_c5_pmc_write.log 2>&1 || { echo "WRITE FAILED rc=$?"; tail -20 gpurun_out/r06_c5_pmc_write.log; exit 1; }
echo PMC_OK
timeout -k 10 300 python3 -u tools/c5_ceiling.py 3 > gpurun_out/r06_c5_ceiling.log 2>&1 || { echo "CEILING FAILED rc=$?"; tail -20 gpurun_out/r06_c5_ceiling.log; exit 1; }
echo C5_R06_OK
