#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zzb: option side_mask at C5 (r5zj measured C2 / C3 only): 3 (default) vs 2 (decoder weight
# gradients in order on the caller's stream) vs 1, alternating, final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5zzb_$1|120|python bench.py --config $2 $BQ $3 > gpurun_out/r5zzb_$1.json"; }
bash tools/gpu_steps.sh \
  "$(r c5_m3a C5)" "$(r c5_m2a C5 "--opt side_mask=2")" "$(r c5_m1a C5 "--opt side_mask=1")" \
  "$(r c5_m3b C5)" "$(r c5_m2b C5 "--opt side_mask=2")" "$(r c5_m1b C5 "--opt side_mask=1")"
