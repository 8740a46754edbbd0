#!/bin/bash
# CRC pass fold by DPP + readlane: framed GPU tests (checksums vs the oracle), then the frame bench
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_frontend.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_cd_tests.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_cd_tests.log; exit 1; }
tail -1 gpurun_out/r04_cd_tests.log
timeout -k 10 400 python tools/frame_bench.py > gpurun_out/r04_frame_bench2.log 2>&1 || { echo "bench rc=$?"; tail -20 gpurun_out/r04_frame_bench2.log; exit 1; }
head -12 gpurun_out/r04_frame_bench2.log
