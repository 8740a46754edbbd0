#!/bin/bash
# Round 4: the payloads' rest by split + plain encode of their last tiles (frame_tail_bs), work units
# of one tile for odd tile counts: framing tests, cover A/B, Swift encode traces.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frame.py > gpurun_out/r04_frame_tests_i.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_frame_tests_i.log; exit 1; }
tail -2 gpurun_out/r04_frame_tests_i.log
timeout -k 10 300 python tools/cover_ab.py > gpurun_out/r04_cover_ab3.log 2>&1 || { echo "COVER rc=$?"; tail -20 gpurun_out/r04_cover_ab3.log; exit 1; }
cat gpurun_out/r04_cover_ab3.log
bash tools/gpu_prof_swift.sh || exit 1
timeout -k 10 300 python tools/copy_shape_ab.py obj > gpurun_out/r04_join_obj_ab.log 2>&1 || { echo "OBJ rc=$?"; tail -20 gpurun_out/r04_join_obj_ab.log; exit 1; }
cat gpurun_out/r04_join_obj_ab.log
echo R04_I_OK
