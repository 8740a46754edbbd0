#!/bin/bash
# Round 6 A/B: the markers between back-to-back C3 launches (bench's per-pass timing events, the
# bitsliced launch's completion event) -- bench value and per-launch time, 3 interleaved rounds.
# (Ran at cc4ca13 with two development toggles since removed: BENCH_PASS_EVENTS in bench.py and the
# bs_launch_event tune knob; summary and decision in profiles/r06_gap_ab.json.)
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
for rnd in 1 2 3; do
  for v in "1 1" "0 1" "1 0" "0 0"; do
    set -- $v
    BENCH_PASS_EVENTS=$1 ECAMD_TUNE=bs_launch_event=$2 timeout -k 10 150 python3 bench.py --no-c5 --no-scatter --no-cpu-baseline > gpurun_out/r06_gap_tmp.log 2>&1 || { echo "BENCH FAILED"; tail -5 gpurun_out/r06_gap_tmp.log; exit 1; }
    python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/r06_gap_tmp.log') if l.startswith('{')][-1])
print(json.dumps({'round':$rnd,'pass_events':$1,'launch_event':$2,'value':d['value'],'ms_per_step':d['ms_per_step'],'launch_ms':d['roofline']['launch_ms']}))
" | tee -a gpurun_out/r06_gap_ab.log
  done
done
echo GAP_OK
