#!/bin/bash
# Round 4: realigned object-chunk loads in the bitsliced copy-through / crc kernels (knob bs_realign):
# the framing tests, then the cover A/B (crc variant, realigned vs unaligned loads) and the one-wave
# copy-through A/B (bs_wave_copy, now with realigned loads on Swift's segments).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/r04_frame_tests_g.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_frame_tests_g.log; exit 1; }
tail -2 gpurun_out/r04_frame_tests_g.log
timeout -k 10 300 python tools/cover_ab.py > gpurun_out/r04_cover_ab2.log 2>&1 || { echo "COVER rc=$?"; tail -20 gpurun_out/r04_cover_ab2.log; exit 1; }
cat gpurun_out/r04_cover_ab2.log
timeout -k 10 300 python tools/frame_wave_ab.py > gpurun_out/r04_frame_wave_ab2.log 2>&1 || { echo "WAVE rc=$?"; tail -20 gpurun_out/r04_frame_wave_ab2.log; exit 1; }
cat gpurun_out/r04_frame_wave_ab2.log
echo R04_G_OK
