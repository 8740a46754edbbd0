#!/bin/bash
# dpp_reduce A/B on the framed CRC32 encode (C5 fold-each, C3): bpermute / dpp / bpermute / dpp
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
L=gpurun_out/r04_dppred_ab.log; : > $L
for i in 1 2; do
  ECAMD_BS_DPPRED=0 ECAMD_JIT_CACHE=/tmp/jit_base timeout -k 10 240 python tools/dppred_ab.py >> $L 2>&1 || { echo "base rc=$?"; tail -20 $L; exit 1; }
  ECAMD_BS_DPPRED=1 ECAMD_JIT_CACHE=/tmp/jit_dpp timeout -k 10 240 python tools/dppred_ab.py >> $L 2>&1 || { echo "dpp rc=$?"; tail -20 $L; exit 1; }
done
grep '^{' $L
