#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5ze: the eight-phase image-reusing walk on the f32x BCE head too (bce_split's remainder then
# agrees to fp32 rounding instead of bitwise): tests, then C2 against HEAD's library, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5ze_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5ze_$1.json"; }
H="MVAE_LIB=magic_amd/libmvae_head.so"
bash tools/gpu_steps.sh \
  "r5ze_t|600|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_r2.py tests/test_gpu_parity.py tests/test_gpu_golden.py" \
  "$(r c2_h1 C2 "$H")" "$(r c2_n1 C2)" "$(r c2_h2 C2 "$H")" "$(r c2_n2 C2)" "$(r c2_h3 C2 "$H")" "$(r c2_n3 C2)"
