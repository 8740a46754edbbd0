#!/bin/bash
# Same-box A/B of bitsliced-kernel generator variants (tools/c5_prof.py per variant, each in its own
# process and JIT cache dir; the LDS-table kernel in every run as the control), two interleaved
# rounds.  Variants: name:ECAMD_BS_LAZY:ECAMD_BS_BARRIER:ECAMD_JIT_CAP_MAX.  Usage: c5_ab.sh [variant...]
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
VARIANTS=("$@")
[ ${#VARIANTS[@]} -eq 0 ] && VARIANTS=(lazy_bar_64:1:1:64 lazy_nobar_64:1:0:64 eager_bar_48:0:1:48 eager_nobar_48:0:0:48 lazy_nobar_48:1:0:48)
for rnd in 1 2; do
  for v in "${VARIANTS[@]}"; do
    IFS=: read -r name lazy bar cap <<< "$v"
    out=$(ECAMD_BS_LAZY=$lazy ECAMD_BS_BARRIER=$bar ECAMD_JIT_CAP_MAX=$cap ECAMD_JIT_CACHE=/tmp/ecamd-ab-$name \
          C5_MODES="2:2,0:0" timeout -k 10 240 python3 -u tools/c5_prof.py) || { echo "FAILED $name"; exit 1; }
    echo "$out" | sed "s/^{/{\"variant\": \"$name\", \"round\": $rnd, /"
  done
done
