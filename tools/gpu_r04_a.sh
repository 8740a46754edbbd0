#!/bin/bash
# Round 4, first GPU session: the GPU tests, the driver's bench command, the 2-rank gloo rehearsal
# (cpu_baseline and per-rank fields at N>1) and the one-wave bitsliced A/B.  Every GPU step has its
# own time limit; the first failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_tests1.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_gpu_tests1.log; exit 1; }
timeout -k 10 240 python bench.py > gpurun_out/r04_bench1.log 2>&1 || { echo "BENCH rc=$?"; exit 1; }
ECAMD_DIST_BACKEND=gloo timeout -k 10 240 python bench.py --gpus 2 > gpurun_out/r04_rehearsal1.log 2>&1 || { echo "REHEARSAL rc=$?"; exit 1; }
timeout -k 10 240 python tools/bs_wave_ab.py > gpurun_out/r04_bs_wave_ab1.log 2>&1 || { echo "AB rc=$?"; exit 1; }
echo R04_A_OK
