#!/bin/bash
# Round 6, VERDICT r05 #2 / #6: the shipped-kernel and stress tests on the GPU, then tools/rebuild_prof.py
# (cold process, empty JIT cache: every (10,4) single-destination reconstruct and a 4-pattern
# decode_multi at C3) under a rocprofv3 kernel trace.  Outputs under gpurun_out/r06_rebuild_*.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_jit_shipped.py tests/test_gpu_bitslice_wave.py tests/test_ref_api_stress.py > gpurun_out/r06_rebuild_tests.log 2>&1 || { echo "TESTS FAILED rc=$?"; tail -40 gpurun_out/r06_rebuild_tests.log; exit 1; }
tail -3 gpurun_out/r06_rebuild_tests.log
C=$(mktemp -d); chmod 700 "$C"
ECAMD_JIT_CACHE="$C" timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r06_rebuild_trace" -o run --output-format csv -- python3 tools/rebuild_prof.py 20 > gpurun_out/r06_rebuild_prof.log 2>&1 || { echo "PROF FAILED rc=$?"; tail -20 gpurun_out/r06_rebuild_prof.log; exit 1; }
grep '^{' gpurun_out/r06_rebuild_prof.log
echo REBUILD_OK
