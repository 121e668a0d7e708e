#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zr: the planner's split-K fixed cost 4 -> 8 us (C2's f32x hidden forward unsplit at 192x128):
# plans of both libraries at C2 / C3 / C5, then the steps against the parent, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5zr_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5zr_$1.json"; }
H="MVAE_LIB=magic_amd/libmvae_head.so"
p() { echo "r5zr_plan_$1_$2|120|$3 python bench.py --config $1 $BQ --steps 2 --create-opt plan_log=1 > gpurun_out/r5zr_plan_$1_$2.json"; }
bash tools/gpu_steps.sh \
  "$(p C2 h "$H")" "$(p C2 n)" "$(p C3 h "$H")" "$(p C3 n)" "$(p C5 h "$H")" "$(p C5 n)" \
  "$(r c2_h1 C2 "$H")" "$(r c2_n1 C2)" "$(r c2_h2 C2 "$H")" "$(r c2_n2 C2)" "$(r c2_h3 C2 "$H")" "$(r c2_n3 C2)" \
  "$(r c3_h1 C3 "$H")" "$(r c3_n1 C3)" "$(r c3_h2 C3 "$H")" "$(r c3_n2 C3)" \
  "$(r c5_h1 C5 "$H")" "$(r c5_n1 C5)" "$(r c5_h2 C5 "$H")" "$(r c5_n2 C5)"
