#!/bin/bash
# One GPU call of the development loop: new tests first, the driver's bench command, the rocprof
# evidence for it, the flat-XOR profile, then the whole GPU suite.  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
RND="${1:-r02}"
FIRST="${2:-}"
if [ -n "$FIRST" ]; then
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread $FIRST > gpurun_out/pytest_first.log 2>&1 || { echo "FIRST TESTS FAILED rc=$?"; tail -40 gpurun_out/pytest_first.log; exit 1; }
  tail -3 gpurun_out/pytest_first.log
fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || { echo "BENCH FAILED rc=$?"; tail -20 gpurun_out/bench_driver.log; exit 1; }
tail -1 gpurun_out/bench_driver.log
bash tools/gpu_prof.sh "$RND" c3 || exit 1
bash tools/gpu_prof_xor.sh || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "PYTEST_RC=$rc"; tail -15 gpurun_out/pytest_gpu.log
exit $rc
