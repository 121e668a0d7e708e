#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5w (r5v repeated, HEAD's library first in each pair, 100 steps): the eight-phase kernel's image-reusing walk for f32x plane pairs (k-tiles in twos, pairs
# between; an operand image its buffer already holds is not copied again): tests, then whole
# steps against HEAD's library (libmvae_head.so), alternating, C2 (f32x) / C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5w_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5w_$1.json"; }
H="MVAE_LIB=magic_amd/libmvae_head.so"
bash tools/gpu_steps.sh \
  "$(r c2_h1 C2 "$H")" "$(r c2_n1 C2)" "$(r c2_h2 C2 "$H")" "$(r c2_n2 C2)" "$(r c2_h3 C2 "$H")" "$(r c2_n3 C2)" \
  "$(r c2_h4 C2 "$H")" "$(r c2_n4 C2)" "$(r c3_h1 C3 "$H")" "$(r c3_n1 C3)" "$(r c3_h2 C3 "$H")" "$(r c3_n2 C3)"
