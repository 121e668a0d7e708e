#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zm: the decoder's two hidden layers in one enc_chain launch (create option dec_chain): the
# A/B (r5zl ran the plan and the tests: 472 passed): C3 / C5 against the parent commit's library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5zm_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5zm_$1.json"; }
H="MVAE_LIB=magic_amd/libmvae_head.so"
bash tools/gpu_steps.sh \
  "$(r c3_h1 C3 "$H")" "$(r c3_n1 C3)" "$(r c3_h2 C3 "$H")" "$(r c3_n2 C3)" "$(r c3_h3 C3 "$H")" "$(r c3_n3 C3)" \
  "$(r c5_h1 C5 "$H")" "$(r c5_n1 C5)" "$(r c5_h2 C5 "$H")" "$(r c5_n2 C5)"
