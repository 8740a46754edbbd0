#!/bin/bash
# CRC32 pass span A/B on the Swift segment CRC32 encode (its tail checksum)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py -x -q --timeout 300 --timeout-method thread -k "cover_crc or padded" > gpurun_out/r04_tc_tests.log 2>&1 || { echo "TESTS rc=$?"; tail -30 gpurun_out/r04_tc_tests.log; exit 1; }
tail -1 gpurun_out/r04_tc_tests.log
timeout -k 10 300 python tools/tail_crc_ab.py > gpurun_out/r04_tail_crc_ab2.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r04_tail_crc_ab2.log; exit 1; }
cat gpurun_out/r04_tail_crc_ab2.log
