#!/bin/bash
# dpp_reduce default: the framed and bitslice GPU tests
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_bitslice_golden.py tests/test_gpu_bitslice.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_dv_tests.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_dv_tests.log; exit 1; }
tail -1 gpurun_out/r04_dv_tests.log
