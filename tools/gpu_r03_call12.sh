#!/bin/bash
# Round-3: framed bench with the launch counter, framed-CRC HIP-event check, C5 grid A/B.
set -o pipefail
bash tools/gpu_r03_call10.sh || exit 1
bash tools/gpu_r03_call11.sh || exit 1
echo CALL12_OK
