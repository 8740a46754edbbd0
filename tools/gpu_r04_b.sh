#!/bin/bash
# Round 4, second GPU session: the GPU tests with the one-wave bitsliced default, the driver's bench
# command, the bs_wave A/B (C3, C2, C5).  First failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_tests2.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_gpu_tests2.log; exit 1; }
timeout -k 10 240 python bench.py > gpurun_out/r04_bench2.log 2>&1 || { echo "BENCH rc=$?"; tail -20 gpurun_out/r04_bench2.log; exit 1; }
timeout -k 10 300 python tools/bs_wave_ab.py > gpurun_out/r04_bs_wave_ab2.log 2>&1 || { echo "AB rc=$?"; tail -20 gpurun_out/r04_bs_wave_ab2.log; exit 1; }
echo R04_B_OK
