#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5i: the planner's ring-fill rule (single-product GEMMs whose 192-row ring tiles fill one round
# stay on the ring kernel) against the rebuilt eight-phase kernel: default vs libmvae_norf.so (the
# rule off: the layer-0 and hidden forwards on the eight-phase kernel), alternating, C3 / C5 / C2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
NR=MVAE_LIB=magic_amd/libmvae_norf.so
r() { echo "r5i_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5i_$1.json"; }
bash tools/gpu_steps.sh \
  "$(r c3_d1 C3)" "$(r c3_n1 C3 $NR)" "$(r c3_d2 C3)" "$(r c3_n2 C3 $NR)" \
  "$(r c5_d1 C5)" "$(r c5_n1 C5 $NR)" "$(r c5_d2 C5)" "$(r c5_n2 C5 $NR)" \
  "$(r c2_d1 C2)" "$(r c2_n1 C2 $NR)" "$(r c2_d2 C2)" "$(r c2_n2 C2 $NR)"
