#!/bin/bash
# Round 4: the whole GPU suite, smoke() and the driver's default bench command after the framing
# changes (realigned loads, encode tails, join tiles).  First failure ends the script.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_gpu_tests3.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_gpu_tests3.log; exit 1; }
tail -2 gpurun_out/r04_gpu_tests3.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke3.log 2>&1 || { echo "SMOKE rc=$?"; tail -20 gpurun_out/r04_smoke3.log; exit 1; }
tail -1 gpurun_out/r04_smoke3.log
timeout -k 10 300 python bench.py > gpurun_out/r04_bench3.log 2>&1 || { echo "BENCH rc=$?"; tail -20 gpurun_out/r04_bench3.log; exit 1; }
tail -1 gpurun_out/r04_bench3.log | cut -c1-600
echo R04_K_OK
