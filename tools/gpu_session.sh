#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r6l: the early Adam's layer-0 chunks (option early_chunks 2, the default, vs 1) with the bits
# path and pinned chunk plans -- C2 / C3 / C5 alternating twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 100"
r() { echo "r6l_$1|150|python bench.py $B --config $2 $3 > gpurun_out/r6l_$1.json"; }
bash tools/gpu_steps.sh \
  "$(r c2_2a C2)" "$(r c2_1a C2 "--opt early_chunks=1")" "$(r c3_2a C3)" "$(r c3_1a C3 "--opt early_chunks=1")" \
  "$(r c5_2a C5)" "$(r c5_1a C5 "--opt early_chunks=1")" \
  "$(r c2_2b C2)" "$(r c2_1b C2 "--opt early_chunks=1")" "$(r c3_2b C3)" "$(r c3_1b C3 "--opt early_chunks=1")" \
  "$(r c5_2b C5)" "$(r c5_1b C5 "--opt early_chunks=1")"
