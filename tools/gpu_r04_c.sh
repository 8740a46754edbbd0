#!/bin/bash
# Round 4, third GPU session: DPP realign A/B of the copy-through stream kernel (stream_realign 2),
# the framed CRC32 PMC passes, the per-call A/B (direct-into-object decode, staging-pack tees).
# First failure ends the script.  (Its first version also ran tools/bs_wave_ab.py c2 c5,
# tools/copy_shape_ab.py dpp and tools/frame_wave_ab.py: profiles/r04_bs_wave_ab3.log,
# r04_copy_dpp_ab.log, r04_frame_wave_ab.log.)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python tools/realign_ab.py > gpurun_out/r04_realign_ab.log 2>&1 || { echo "REALIGN rc=$?"; tail -20 gpurun_out/r04_realign_ab.log; exit 1; }
bash tools/gpu_pmc_framecrc.sh || exit 1
timeout -k 10 600 python tools/percall_ab.py 2 > gpurun_out/r04_percall_ab.log 2>&1 || { echo "PERCALL rc=$?"; tail -20 gpurun_out/r04_percall_ab.log; exit 1; }
echo R04_C_OK
