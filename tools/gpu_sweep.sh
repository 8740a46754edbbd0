#!/bin/bash
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python tools/kernel_sweep.py "$@" > gpurun_out/sweep.log 2>&1; rc=$?
cat gpurun_out/sweep.log | grep -v amdgpu.ids
exit $rc
