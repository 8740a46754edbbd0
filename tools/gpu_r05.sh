#!/bin/bash
# Round-5 GPU session (rewritten per call; history keeps earlier versions).  Stops at the first failure.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r05_$name.log" 2>&1; local rc=$?; tail -4 "gpurun_out/r05_$name.log"; [ $rc -eq 0 ] || { echo "STEP $name FAILED rc=$rc"; exit 1; }; }
step tests_new 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_bitslice_wave.py tests/test_gpu_jit_shipped.py "tests/test_gpu_frame.py::test_stream_contexts_bounded"
step ab_narrow 500 python -u tools/bs_wave_ab.py c3n c5n c2n
step ab_ring 300 python -u tools/bs_wave_ab.py c3ring
step pmc_c3 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace -d "$R/gpurun_out/r05_pmc_c3" -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --config c3 --no-c5 --no-scatter --no-cpu-baseline
python3 tools/summarize_pmc.py gpurun_out/r05_c3_pmc_sq.json gpurun_out/r05_pmc_c3 --kernel ecamd_bs_kernel --command "bench.py --gpus 1 --steps 20 --warmup 5 --config c3 --no-c5 --no-scatter --no-cpu-baseline"
echo ALL_OK
