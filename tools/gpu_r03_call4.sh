#!/bin/bash
# Round-3 GPU call: realigned streaming copies (tests + framed bench), flat-XOR defaults (tests +
# rocprofv3 trace / FETCH / WRITE of tools/xor_prof.py), an LDS-utilisation PMC pass of the fused
# CRC framed encode.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_frame.py tests/test_gpu_xor_batch.py tests/test_gpu_xor.py > gpurun_out/r03_frame_xor_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_frame_xor_tests.log; exit 1; }
tail -1 gpurun_out/r03_frame_xor_tests.log
timeout -k 10 240 python3 tools/frame_bench.py --no-crc-sweep --reps 5 > gpurun_out/r03_frame_bench3.log 2>&1 || { echo FRAME_BENCH_FAILED; tail -20 gpurun_out/r03_frame_bench3.log; exit 1; }
grep systematic gpurun_out/r03_frame_bench3.log | grep '"lost": \[\]'
bash tools/gpu_prof_xor.sh || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d "$PWD/gpurun_out/r03_pmc_fused_lds" -o run --output-format csv -- python3 tools/frame_bench.py --no-crc-sweep --reps 4 > gpurun_out/r03_pmc_fused_lds.log 2>&1 || { echo PMC_FUSED_FAILED; tail -20 gpurun_out/r03_pmc_fused_lds.log; exit 1; }
echo CALL4_OK
