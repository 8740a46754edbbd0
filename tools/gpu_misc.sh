#!/bin/bash
# e2e host<->GPU rates + 2-rank bench rehearsal on one GPU (gloo coordination).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python tools/e2e_bench.py > gpurun_out/e2e.log 2>&1 || { echo "E2E FAILED rc=$?"; tail -30 gpurun_out/e2e.log; exit 1; }
tail -1 gpurun_out/e2e.log
ECAMD_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 --stripes 64 > gpurun_out/bench_2rank.log 2>&1 || { echo "2RANK FAILED rc=$?"; tail -30 gpurun_out/bench_2rank.log; exit 1; }
grep '"metric"' gpurun_out/bench_2rank.log
