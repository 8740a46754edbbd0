#!/bin/bash
# rocprofv3 counter passes (each its own run) of tools/bs_probe.py: SQ issue / wait cycles and
# instruction-cache behaviour of the bitsliced probe kernel; the counter list of this GPU too.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_IFETCH SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/bsp1 -o run --output-format csv -- python3 tools/bs_probe.py > gpurun_out/bsp1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/bsp2 -o run --output-format csv -- python3 tools/bs_probe.py > gpurun_out/bsp2.log 2>&1
echo rc=$?
