#!/bin/bash
# Round-3: the driver's bench command twice (C5 fields with the longer warm-up). Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r03_bench_c5warm_$i.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/r03_bench_c5warm_$i.log; exit 1; }
  python -c "
import json;d=json.loads(open('gpurun_out/r03_bench_c5warm_$i.log').read().strip().splitlines()[-1])
c=d['c5'];print(d['value'],d['roofline']['frac'],c['encode_frac'],c['rebuild8_data_frac'],c['rebuild8_mixed_frac'],c['lds_rebuild8_data_frac'])"
done
