#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/tools/frame_crc_prof.py bitsliced_crc wave_crc"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_crcwave" -o run --output-format csv -- $B > gpurun_out/r05_crcwave_prof.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/r05_crcwave_prof.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/pmc_crcwave_a" -o run --output-format csv -- $B > gpurun_out/pmc_crcwave_a.log 2>&1 || { echo "PMC A FAILED rc=$?"; tail -20 gpurun_out/pmc_crcwave_a.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/pmc_crcwave_b" -o run --output-format csv -- $B > gpurun_out/pmc_crcwave_b.log 2>&1 || { echo "PMC B FAILED rc=$?"; tail -20 gpurun_out/pmc_crcwave_b.log; exit 1; }
python3 tools/summarize_pmc.py gpurun_out/r05_crcwave_pmc.json gpurun_out/pmc_crcwave_a gpurun_out/pmc_crcwave_b --kernel ecamd_bs_kernel --command "$B" || exit 1
grep '^{' gpurun_out/r05_crcwave_prof.log
echo ALL_OK
