#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zx: option early_chunks (default 2): under the early Adam the single-call backward runs the
# layer-0 weight gradient in 2 row chunks, chunk 0's Adam beside chunk 1's GEMM. Tests, then
# C2 / C3 / C5 against the parent commit's library, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5zx_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5zx_$1.json"; }
H="MVAE_LIB=magic_amd/libmvae_head.so"
bash tools/gpu_steps.sh \
  "r5zx_t|600|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_r2.py tests/test_gpu_dp.py tests/test_gpu_r3.py tests/test_gpu_parity.py tests/test_gpu_golden.py" \
  "$(r c2_h1 C2 "$H")" "$(r c2_n1 C2)" "$(r c2_h2 C2 "$H")" "$(r c2_n2 C2)" "$(r c2_h3 C2 "$H")" "$(r c2_n3 C2)" \
  "$(r c3_h1 C3 "$H")" "$(r c3_n1 C3)" "$(r c3_h2 C3 "$H")" "$(r c3_n2 C3)" \
  "$(r c5_h1 C5 "$H")" "$(r c5_n1 C5)" "$(r c5_h2 C5 "$H")" "$(r c5_n2 C5)"
