#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5m: (1) what staging the next batch's de-interleave beside the step would cost the step: a
# shadow pass of the step's input into a scratch image on a low-priority stream (create options
# diag_shadow_deint = grid (-1 the normal launch, > 0 persistent workgroups), diag_shadow_at =
# 0 after the forward's pass, 1 at the backward, 2 at the encoder backward); (2) the early Adam
# on a capped float4 grid (option adam_side_grid) vs its one-thread-per-element launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
r() { echo "r5m_$1|120|python bench.py --config $2 $BQ $3 > gpurun_out/r5m_$1.json"; }
sh() { echo "--create-opt diag_shadow_deint=$1 --create-opt diag_shadow_at=$2"; }
E="--opt early_adam=1"
bash tools/gpu_steps.sh \
  "r5m_t|300|python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_r2.py -k early_adam" \
  "$(r c3_d1 C3)" "$(r c3_sf0 C3 "$(sh -1 0)")" "$(r c3_s64a1 C3 "$(sh 64 1)")" "$(r c3_s128a1 C3 "$(sh 128 1)")" \
  "$(r c3_s256a1 C3 "$(sh 256 1)")" "$(r c3_s128a0 C3 "$(sh 128 0)")" "$(r c3_s128a2 C3 "$(sh 128 2)")" "$(r c3_d2 C3)" \
  "$(r c3_e0 C3 "$E")" "$(r c3_e128 C3 "$E --opt adam_side_grid=128")" "$(r c3_e512 C3 "$E --opt adam_side_grid=512")" "$(r c3_d3 C3)" \
  "$(r c2_d1 C2)" "$(r c2_g128 C2 "--opt adam_side_grid=128")" "$(r c2_s128a1 C2 "$(sh 128 1)")" "$(r c2_sf0 C2 "$(sh -1 0)")" \
  "$(r c2_g512 C2 "--opt adam_side_grid=512")" "$(r c2_d2 C2)"
