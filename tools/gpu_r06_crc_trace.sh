#!/bin/bash
# Round 6: kernel traces of one-thread CHKSUM_CRC32 per-call encodes (tools/percall_trace.py) with the
# checksums fused into the small-launch kernel (default) and without (ECAMD_PERCALL_FUSE_CRC=0).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for size in 4096 16384 65536; do
  for fuse in 1 0; do
    ECAMD_PERCALL_FUSE_CRC=$fuse timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r06_crctr_${size}_$fuse" -o run --output-format csv -- python3 tools/percall_trace.py $size 300 2 > gpurun_out/r06_crctr_${size}_$fuse.log 2>&1 || { echo "TRACE FAILED $size $fuse"; tail -20 gpurun_out/r06_crctr_${size}_$fuse.log; exit 1; }
    grep median gpurun_out/r06_crctr_${size}_$fuse.log
  done
done
echo CRCTR_OK
