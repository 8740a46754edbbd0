#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do for RL in 0 1; do
  rm -rf /tmp/jc_$RL; mkdir -p /tmp/jc_$RL
  ECAMD_JIT_CACHE=/tmp/jc_$RL ECAMD_BS_RLANE=$RL timeout -k 10 300 python -u tools/frame_shape_ab.py 1048572,4194300 > gpurun_out/r05_rlane_${RL}_$i.log 2>&1 || { echo "RUN FAILED"; tail -20 gpurun_out/r05_rlane_${RL}_$i.log; exit 1; }
  sed "s/^/rl$RL /" gpurun_out/r05_rlane_${RL}_$i.log | grep frac
done; done
echo ALL_OK
