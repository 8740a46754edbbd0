#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -1 "gpurun_out/r05_$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; tail -30 "gpurun_out/r05_$name.log"; exit 1; }; }
step crcwave_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_frame.py -k crc_wave
step ab_crcwave_dma 600 python -u tools/frame_knob_ab.py frame_crc_wave_dma 0,1 --ct crc --ops encode
step ab_crcwave_dma2 600 python -u tools/frame_knob_ab.py frame_crc_wave_dma 0,1 --ct crc --ops encode
grep frac gpurun_out/r05_ab_crcwave_dma.log gpurun_out/r05_ab_crcwave_dma2.log
echo ALL_OK
