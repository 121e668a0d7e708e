#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zza: the planner's split-K fixed cost 8 us only for plane-pair products (4 us again for single
# products: C5's decoder layer 1 back to 256x128 split 2): plans of both libraries, C5 / C3 A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5zza_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5zza_$1.json"; }
H="MVAE_LIB=magic_amd/libmvae_head.so"
p() { echo "r5zza_plan_$1_$2|120|$3 python bench.py --config $1 $BQ --steps 2 --create-opt plan_log=1 > gpurun_out/r5zza_plan_$1_$2.json"; }
bash tools/gpu_steps.sh \
  "$(p C2 h "$H")" "$(p C2 n)" "$(p C3 h "$H")" "$(p C3 n)" "$(p C5 h "$H")" "$(p C5 n)" \
  "$(r c5_h1 C5 "$H")" "$(r c5_n1 C5)" "$(r c5_h2 C5 "$H")" "$(r c5_n2 C5)" "$(r c5_h3 C5 "$H")" "$(r c5_n3 C5)"
