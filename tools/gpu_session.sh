#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zn: the latent head as the encoder chain's last, linear layer (fp32 rows of ms; create option
# head_chain): the plan at C3, chain tests + parity / golden / r2, then C3 / C5 against the parent.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5zn_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5zn_$1.json"; }
H="MVAE_LIB=magic_amd/libmvae_head.so"
bash tools/gpu_steps.sh \
  "r5zn_plan|120|python bench.py --config C3 $BQ --steps 3 --create-opt plan_log=1 > gpurun_out/r5zn_plan.json" \
  "r5zn_t|600|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_r5.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_r2.py" \
  "$(r c3_h1 C3 "$H")" "$(r c3_n1 C3)" "$(r c3_h2 C3 "$H")" "$(r c3_n2 C3)" "$(r c3_h3 C3 "$H")" "$(r c3_n3 C3)" \
  "$(r c5_h1 C5 "$H")" "$(r c5_n1 C5)" "$(r c5_h2 C5 "$H")" "$(r c5_n2 C5)"
