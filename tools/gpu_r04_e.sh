#!/bin/bash
# Round 4: the partly fused framed CRC32 encode (knob frame_crc_cover) -- its parity tests and the
# framing tests around it, then its A/B against the codec + separate CRC pass.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/r04_frame_tests_e.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_frame_tests_e.log; exit 1; }
tail -3 gpurun_out/r04_frame_tests_e.log
timeout -k 10 300 python tools/cover_ab.py > gpurun_out/r04_cover_ab.log 2>&1 || { echo "COVER rc=$?"; tail -20 gpurun_out/r04_cover_ab.log; exit 1; }
cat gpurun_out/r04_cover_ab.log
echo R04_E_OK
