#!/bin/bash
# realign_lane A/B on Swift segments: base / rlane / base / rlane, separate JIT caches
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04_rlane_ab.log; : > $L
for i in 1 2; do
  ECAMD_JIT_CACHE=/tmp/jit_base timeout -k 10 180 python tools/rlane_ab.py >> $L 2>&1 || { echo "base rc=$?"; tail -20 $L; exit 1; }
  ECAMD_BS_RLANE=1 ECAMD_JIT_CACHE=/tmp/jit_rl timeout -k 10 180 python tools/rlane_ab.py >> $L 2>&1 || { echo "rlane rc=$?"; tail -20 $L; exit 1; }
done
cat $L
