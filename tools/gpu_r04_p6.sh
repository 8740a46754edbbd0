#!/bin/bash
# Round 4, final validation: the whole GPU suite, smoke(), the driver's bench command, the 2-rank gloo
# rehearsal (cpu_baseline and per-rank fields at N > 1).  First failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_tests_final6.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_gpu_tests_final6.log; exit 1; }
tail -1 gpurun_out/r04_gpu_tests_final6.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke_final6.log 2>&1 || { echo "SMOKE rc=$?"; tail -20 gpurun_out/r04_smoke_final6.log; exit 1; }
tail -1 gpurun_out/r04_smoke_final6.log
timeout -k 10 300 python bench.py > gpurun_out/r04_bench_final6.log 2>&1 || { echo "BENCH rc=$?"; tail -20 gpurun_out/r04_bench_final6.log; exit 1; }
tail -1 gpurun_out/r04_bench_final6.log | cut -c1-400
ECAMD_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 > gpurun_out/r04_rehearsal_2ranks_final6.log 2>&1 || { echo "REHEARSAL rc=$?"; tail -20 gpurun_out/r04_rehearsal_2ranks_final6.log; exit 1; }
tail -1 gpurun_out/r04_rehearsal_2ranks_final6.log | cut -c1-300
echo R04_P6_OK
