#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -1 "gpurun_out/r05_$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; tail -30 "gpurun_out/r05_$name.log"; exit 1; }; }
step ab_crcwave_wpe 600 python -u tools/frame_knob_ab.py frame_crc_wave_wpe 0,2 --ct crc --ops encode
grep frac gpurun_out/r05_ab_crcwave_wpe.log
B="python3 $R/tools/frame_crc_prof.py wave_crc"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_crcwave2" -o run --output-format csv -- $B > gpurun_out/r05_crcwave2_prof.log 2>&1 || { echo "TRACE FAILED rc=$?"; tail -20 gpurun_out/r05_crcwave2_prof.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/pmc_crcwave2_a" -o run --output-format csv -- $B > gpurun_out/pmc_crcwave2_a.log 2>&1 || { echo "PMC A FAILED rc=$?"; tail -20 gpurun_out/pmc_crcwave2_a.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/pmc_crcwave2_b" -o run --output-format csv -- $B > gpurun_out/pmc_crcwave2_b.log 2>&1 || { echo "PMC B FAILED rc=$?"; tail -20 gpurun_out/pmc_crcwave2_b.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_crcwave2_c" -o run --output-format csv -- $B > gpurun_out/pmc_crcwave2_c.log 2>&1 || { echo "PMC C FAILED rc=$?"; tail -20 gpurun_out/pmc_crcwave2_c.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_crcwave2_d" -o run --output-format csv -- $B > gpurun_out/pmc_crcwave2_d.log 2>&1 || { echo "PMC D FAILED rc=$?"; tail -20 gpurun_out/pmc_crcwave2_d.log; exit 1; }
python3 tools/summarize_pmc.py gpurun_out/r05_crcwave2_pmc.json gpurun_out/pmc_crcwave2_a gpurun_out/pmc_crcwave2_b gpurun_out/pmc_crcwave2_c gpurun_out/pmc_crcwave2_d --kernel ecamd_bs_kernel --command "$B" || exit 1
grep '^{' gpurun_out/r05_crcwave2_prof.log
echo ALL_OK
