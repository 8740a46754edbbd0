#!/bin/bash
# Round-3: bitsliced one-workgroup-per-tile default -- bitslice tests, the C5 profile, the bench line;
# flat-XOR grid A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bitslice.py tests/test_gpu_bitslice_golden.py > gpurun_out/r03_bs_tests3.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r03_bs_tests3.log; exit 1; }
tail -1 gpurun_out/r03_bs_tests3.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench_driver_3.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r03_bench_driver_3.log; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], json.dumps(d['c5']))" gpurun_out/r03_bench_driver_3.log
timeout -k 10 400 python3 tools/xor_geom_sweep.py --rounds 3 --wgs 2,3 --slots 32 --grid 0,1 > gpurun_out/r03_xor_grid.log 2>&1 || { echo XOR_FAILED; tail -20 gpurun_out/r03_xor_grid.log; exit 1; }
grep encode gpurun_out/r03_xor_grid.log
timeout -k 10 300 python3 tools/c3_bitslice_ab.py > gpurun_out/r03_c3_bitslice_ab.log 2>&1 || { echo C3AB_FAILED; tail -20 gpurun_out/r03_c3_bitslice_ab.log; exit 1; }
cat gpurun_out/r03_c3_bitslice_ab.log
bash tools/gpu_prof_c5.sh || exit 1
echo CALL13_OK
