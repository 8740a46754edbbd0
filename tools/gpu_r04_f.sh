#!/bin/bash
# Round 4: per-operation C3 trace (encode, decode {0,1,2,3}, mixed {0,5,10,13}) on the one-wave
# bitsliced kernel and the LDS-table kernel (tools/gpu_prof_c3ops.sh), then the unaligned-copy probe.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_prof_c3ops.sh || exit 1
timeout -k 10 300 python tools/unaligned_probe.py > gpurun_out/r04_unaligned_probe.log 2>&1 || { echo "PROBE rc=$?"; tail -20 gpurun_out/r04_unaligned_probe.log; exit 1; }
cat gpurun_out/r04_unaligned_probe.log
echo R04_F_OK
