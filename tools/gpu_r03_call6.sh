#!/bin/bash
# Round-3: the driver's bench command twice, then its rocprofv3 evidence (tools/gpu_prof.sh r03 c3).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench_driver_$i.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/r03_bench_driver_$i.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], r['frac'], r['frac_of_measured_copy'], r['encode_pass_ms'], r['decode_pass_ms'])" gpurun_out/r03_bench_driver_$i.log
done
bash tools/gpu_prof.sh r03 c3 || exit 1
echo CALL6_OK
