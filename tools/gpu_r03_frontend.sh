#!/bin/bash
# Round-3: per-call host path (frontend zeroing skipped in front of this repo's codec, copies shared
# with helper threads) -- frontend / per-call tests, the A/B (tools/percall_ab.py), per-call latency.
# Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frontend.py tests/test_foreign_codec.py tests/test_gpu_threaded.py tests/test_gpu_device.py tests/test_gpu_errors.py > gpurun_out/r03_frontend_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_frontend_tests.log; exit 1; }
tail -1 gpurun_out/r03_frontend_tests.log
timeout -k 10 500 python3 tools/percall_ab.py > gpurun_out/r03_percall_ab4.log 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/r03_percall_ab4.log; exit 1; }
cat gpurun_out/r03_percall_ab4.log
timeout -k 10 600 python3 tools/latency_ab.py > gpurun_out/r03_latency_ab4.log 2>&1 || { echo LATAB_FAILED; tail -20 gpurun_out/r03_latency_ab4.log; exit 1; }
