#!/bin/bash
# Round-3: fused CRC framed encode sweep (LDS-table kernel vs the bitsliced crc variant).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python3 tools/frame_bench.py --no-crc-sweep --fused-sweep --reps 5 > gpurun_out/r03_fused_sweep3.log 2>&1 || { echo SWEEP_FAILED; tail -20 gpurun_out/r03_fused_sweep3.log; exit 1; }
grep fused_crc gpurun_out/r03_fused_sweep3.log
echo CALL8_OK
