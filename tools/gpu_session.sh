#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5y: (1) early Adam: one side-stream join per step (in mvae_adam) instead of two; (2) the
# de-interleave's plane stores non-temporal (libmvae_nts.so, on top of (1)); against HEAD's
# library (libmvae_head.so), alternating, C3 / C2. Tests of the step paths first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5y_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5y_$1.json"; }
H="MVAE_LIB=magic_amd/libmvae_head.so"; T="MVAE_LIB=magic_amd/libmvae_nts.so"
bash tools/gpu_steps.sh \
  "r5y_t|600|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_r2.py tests/test_gpu_dp.py tests/test_gpu_parity.py" \
  "$(r c3_h1 C3 "$H")" "$(r c3_n1 C3)" "$(r c3_t1 C3 "$T")" "$(r c3_h2 C3 "$H")" "$(r c3_n2 C3)" "$(r c3_t2 C3 "$T")" \
  "$(r c2_h1 C2 "$H")" "$(r c2_n1 C2)" "$(r c2_t1 C2 "$T")" "$(r c2_h2 C2 "$H")" "$(r c2_n2 C2)" "$(r c2_t2 C2 "$T")"
