#!/bin/bash
# 2-rank gloo rehearsal of the multi-GPU bench on the box's one GPU (usage: gpu_rehearsal_2ranks.sh [round]).
set -o pipefail
mkdir -p gpurun_out
RND="${1:-r05}"
LOG=gpurun_out/${RND}_rehearsal_2ranks.log
ECAMD_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu-baseline > $LOG 2>&1 || { echo REHEARSAL_FAILED; tail -20 $LOG; exit 1; }
python -c "
import json;d=json.loads(open('$LOG').read().strip().splitlines()[-1])
print(d['n_gpus'],d['ranks_seen'],d['value'],d['coord_backend'],d['shared_devices'],d.get('peer_scatter',{}).get('bytes_exact'),d['roofline'].get('trace'))"
