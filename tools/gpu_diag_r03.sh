#!/bin/bash
# Round-3 diagnostics (development): what bounds the flat-XOR (10,6) encode and the fused-CRC
# framed encode.  XOR kernel variants + the codec-shaped streaming probe of the (10 read, 6 write)
# pattern, then one SQ PMC pass each over tools/xor_prof.py and tools/frame_bench.py.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 python3 tools/xor_sweep.py > gpurun_out/r03_xor_sweep.log 2>&1 || { echo "XOR SWEEP FAILED"; tail -20 gpurun_out/r03_xor_sweep.log; exit 1; }
timeout -k 10 200 python3 tools/mix_sweep.py --k 10 --m 6 --policies 2/2,0/2,2/0 --geoms 256x2,256x3,256x4 --rounds 3 --out gpurun_out/r03_mix_10_6.jsonl > gpurun_out/r03_mix_10_6.log 2>&1 || { echo "MIX FAILED"; tail -20 gpurun_out/r03_mix_10_6.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES --kernel-trace -d "$R/gpurun_out/r03_pmc_xor" -o run --output-format csv -- python3 tools/xor_prof.py > gpurun_out/r03_pmc_xor.log 2>&1 || { echo "PMC XOR FAILED"; tail -20 gpurun_out/r03_pmc_xor.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_ANY --kernel-trace -d "$R/gpurun_out/r03_pmc_fused" -o run --output-format csv -- python3 tools/frame_bench.py --no-crc-sweep --reps 4 > gpurun_out/r03_pmc_fused.log 2>&1 || { echo "PMC FUSED FAILED"; tail -20 gpurun_out/r03_pmc_fused.log; exit 1; }
echo DIAG_OK
