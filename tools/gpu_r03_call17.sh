#!/bin/bash
# Round-3: single-owner straddle chunks in the streaming join, its grid A/B (frame_bench systematic
# decode), CRC grid default.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/r03_frame_tests2.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_frame_tests2.log; exit 1; }
tail -1 gpurun_out/r03_frame_tests2.log
timeout -k 10 400 python3 tools/frame_bench.py --no-crc-sweep > gpurun_out/r03_frame_bench7.log 2>&1 || { echo FB_FAILED; tail -20 gpurun_out/r03_frame_bench7.log; exit 1; }
grep -v '"op": "frame_encode' gpurun_out/r03_frame_bench7.log
echo CALL17_OK
