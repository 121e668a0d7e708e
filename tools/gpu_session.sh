#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zj: which weight gradients gain from the side stream: option side_mask 3 (default: decoder and
# encoder wgrads beside the dgrad chains), 2 (decoder's in order on the main stream), 1 (encoder's
# in order), 0 (both), alternating, C2 / C3 / C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5zj_$1|120|python bench.py --config $2 $BQ $3 > gpurun_out/r5zj_$1.json"; }
rot() { for m in 3 2 1 0; do echo "$(r ${1}_m${m}$2 $1 "--opt side_mask=$m")"; done; }
mapfile -t S < <(rot C2 1; rot C3 1; rot C5 1; rot C2 2; rot C3 2)
bash tools/gpu_steps.sh "${S[@]}"
