#!/bin/bash
# Round-3: frontend / per-call GPU tests only.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frontend.py tests/test_foreign_codec.py tests/test_gpu_threaded.py tests/test_gpu_errors.py > gpurun_out/r03_fe_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_fe_tests.log; exit 1; }
tail -1 gpurun_out/r03_fe_tests.log
