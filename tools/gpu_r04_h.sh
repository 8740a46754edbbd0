#!/bin/bash
# Round 4: join with the straddling chunk in the load burst, split with the payload's last chunk
# masked (no byte loop), one-wave bitsliced copy-through for unaligned object chunks (bs_wave_copy 2):
# the framing tests, the join / split shape A/B, the copy-through A/B, the Swift encode traces.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/r04_frame_tests_h.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_frame_tests_h.log; exit 1; }
tail -2 gpurun_out/r04_frame_tests_h.log
timeout -k 10 300 python tools/copy_shape_ab.py dpp > gpurun_out/r04_copy_dpp_ab3.log 2>&1 || { echo "DPP rc=$?"; tail -20 gpurun_out/r04_copy_dpp_ab3.log; exit 1; }
cat gpurun_out/r04_copy_dpp_ab3.log
timeout -k 10 300 python tools/frame_wave_ab.py > gpurun_out/r04_frame_wave_ab3.log 2>&1 || { echo "WAVE rc=$?"; tail -20 gpurun_out/r04_frame_wave_ab3.log; exit 1; }
cat gpurun_out/r04_frame_wave_ab3.log
bash tools/gpu_prof_swift.sh || exit 1
echo R04_H_OK
