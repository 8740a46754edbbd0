#!/bin/bash
# Round 4: what bounds the framed CRC32 encode on the kernel that runs (the bitsliced crc variant,
# ecamd_bs_kernel): two SQ PMC passes over tools/frame_crc_prof.py (which also runs the LDS-table
# fused kernel after it), each in its own rocprofv3 run, summarised by tools/summarize_pmc.py into
# gpurun_out/r04_framecrc_pmc.json.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 $R/tools/frame_crc_prof.py"
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/pmc_framecrc_a" -o run --output-format csv -- $B > gpurun_out/pmc_framecrc_a.log 2>&1 || { echo "PMC A FAILED rc=$?"; tail -20 gpurun_out/pmc_framecrc_a.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/pmc_framecrc_b" -o run --output-format csv -- $B > gpurun_out/pmc_framecrc_b.log 2>&1 || { echo "PMC B FAILED rc=$?"; tail -20 gpurun_out/pmc_framecrc_b.log; exit 1; }
python3 tools/summarize_pmc.py gpurun_out/r04_framecrc_pmc.json gpurun_out/pmc_framecrc_a gpurun_out/pmc_framecrc_b --command "$B" || exit 1
grep '^{' gpurun_out/pmc_framecrc_a.log
echo PMC_FRAMECRC_OK
