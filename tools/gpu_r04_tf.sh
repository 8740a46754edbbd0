#!/bin/bash
# frame_tail_fork: the framed GPU tests (default on), then the A/B (padded framed encode, tails on a side stream)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_frame.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_tf_tests.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_tf_tests.log; exit 1; }
tail -1 gpurun_out/r04_tf_tests.log
timeout -k 10 400 python tools/tail_fork_ab.py > gpurun_out/r04_tail_fork_ab4.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r04_tail_fork_ab4.log; exit 1; }
cat gpurun_out/r04_tail_fork_ab4.log
