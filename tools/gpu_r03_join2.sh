#!/bin/bash
# Round-3: one-wave 1 KiB split / join tiles -- frame tests, the join profile (trace + PMC), a bench line
# with both copy probes. Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_frame.py tests/test_gpu_xor.py tests/test_gpu_xor_batch.py > gpurun_out/r03_frame_tests_join2.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_frame_tests_join2.log; exit 1; }
tail -1 gpurun_out/r03_frame_tests_join2.log
bash tools/gpu_prof_join.sh || exit 1
python3 tools/summarize_prof.py join r03b --command "python3 tools/join_prof.py" --algo-bytes 5368709120 \
    --window systematic_c3:frame_join_stream_kernel:5:20 --window systematic_swift:frame_join_stream_kernel:30:20 \
    > gpurun_out/r03b_join_summarize.log 2>&1 || { echo SUMMARIZE_FAILED; tail -5 gpurun_out/r03b_join_summarize.log; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03_bench_copyprobes.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r03_bench_copyprobes.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r03_bench_copyprobes.log').read().strip().splitlines()[-1])
r=d['roofline'];print(d['value'],r['frac'],r['copy_peak_measured'],r['copy_probes'],r['frac_of_measured_copy'])"
