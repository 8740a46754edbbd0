#!/bin/bash
# Round-3 (final): 2-rank gloo rehearsal of the multi-GPU bench on the box's one GPU.
set -o pipefail
mkdir -p gpurun_out
ECAMD_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline > gpurun_out/r03_rehearsal_2ranks_final.log 2>&1 || { echo REHEARSAL_FAILED; tail -20 gpurun_out/r03_rehearsal_2ranks_final.log; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r03_rehearsal_2ranks_final.log').read().strip().splitlines()[-1])
print(d['n_gpus'],d['ranks_seen'],d['value'],d['coord_backend'],d['shared_devices'],d.get('peer_scatter',{}).get('bytes_exact'),d['roofline']['trace'])"
