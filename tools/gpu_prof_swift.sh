#!/bin/bash
# rocprofv3 kernel traces of tools/swift_prof.py: the Swift-segment framed encode with CRC32 (cover
# path) and without; per-kernel stats land in gpurun_out/prof_swift_{crc,none}/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 2 1; do
  tag=$([ $c = 2 ] && echo crc || echo none)
  SWIFT_CHKSUM=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_swift_$tag" -o run --output-format csv -- python3 "$R/tools/swift_prof.py" > gpurun_out/prof_swift_$tag.log 2>&1 || { echo "TRACE $tag FAILED rc=$?"; tail -20 gpurun_out/prof_swift_$tag.log; exit 1; }
  grep '^{' gpurun_out/prof_swift_$tag.log
done
echo PROF_SWIFT_OK
