#!/bin/bash
# Final check of a round (usage: tools/gpu_final_check.sh [round]): the whole GPU suite, smoke, the default
# bench, the 2-rank rehearsal, and the rocprofv3 evidence of the driver's bench command (summarise it
# afterwards with tools/summarize_prof.py c3 <round> --kernel ecamd_bs_kernel --pre 4 --per-pass 1 ...).
# Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
RND="${1:-r05}"
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/${RND}_$name.log" 2>&1; local rc=$?; tail -1 "gpurun_out/${RND}_$name.log" | cut -c1-300; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; tail -30 "gpurun_out/${RND}_$name.log"; exit 1; }; }
step gpu_tests_final 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests
step smoke_final 400 python -c "import __graft_entry__ as g; g.smoke()"
step bench_final 600 python bench.py
bash tools/gpu_rehearsal_2ranks.sh "$RND" || exit 1
bash tools/gpu_prof.sh "$RND" c3 > gpurun_out/${RND}_prof_final.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/${RND}_prof_final.log; exit 1; }
grep -c . gpurun_out/bench_prof_c3.json
echo ALL_OK
