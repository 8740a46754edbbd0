#!/bin/bash
# bs_realign A/B (one-wave copy-through encode, unaligned object chunks)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/bs_realign_ab.py > gpurun_out/r04_bs_realign_ab.log 2>&1 || { echo "rc=$?"; tail -20 gpurun_out/r04_bs_realign_ab.log; exit 1; }
cat gpurun_out/r04_bs_realign_ab.log
