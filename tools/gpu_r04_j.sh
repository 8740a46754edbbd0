#!/bin/bash
# Round 4: join tiles aligned to the object (frame_join_align A/B), crc variant back on unaligned loads;
# framing tests, join A/B, cover A/B.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/r04_frame_tests_j.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_frame_tests_j.log; exit 1; }
tail -1 gpurun_out/r04_frame_tests_j.log
timeout -k 10 300 python tools/copy_shape_ab.py align > gpurun_out/r04_join_align_ab.log 2>&1 || { echo "ALIGN rc=$?"; tail -20 gpurun_out/r04_join_align_ab.log; exit 1; }
cat gpurun_out/r04_join_align_ab.log
timeout -k 10 300 python tools/cover_ab.py > gpurun_out/r04_cover_ab4.log 2>&1 || { echo "COVER rc=$?"; tail -20 gpurun_out/r04_cover_ab4.log; exit 1; }
cat gpurun_out/r04_cover_ab4.log
echo R04_J_OK
