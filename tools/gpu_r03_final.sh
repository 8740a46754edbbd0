#!/bin/bash
# Round-3 final check: smoke, the driver's bench command, the flat-XOR profile (1 KiB tiles), then the
# whole GPU suite. Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_final2.log 2>&1 || { echo "SMOKE FAILED"; tail -20 gpurun_out/r03_smoke_final2.log; exit 1; }
tail -1 gpurun_out/r03_smoke_final2.log
timeout -k 10 300 python bench.py > gpurun_out/r03_bench_final2.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/r03_bench_final2.log; exit 1; }
tail -1 gpurun_out/r03_bench_final2.log

timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests_final2.log 2>&1
rc=$?
echo "PYTEST_RC=$rc"; tail -3 gpurun_out/r03_gpu_tests_final2.log
exit $rc
