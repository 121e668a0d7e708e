#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5k: the column statistics and the metric + loss sums each in one launch (last-arriver fixed-
# order reductions): parity / determinism / DP tests, then whole steps vs HEAD's two-launch forms
# (libmvae_head.so, tools/build_rev.sh), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
HD=MVAE_LIB=magic_amd/libmvae_head.so
r() { echo "r5k_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5k_$1.json"; }
bash tools/gpu_steps.sh \
  "r5k_tests|600|$T tests/test_gpu_parity.py tests/test_gpu_r2.py tests/test_gpu_golden.py tests/test_gpu_dp.py" \
  "$(r c3_n1 C3)" "$(r c3_h1 C3 $HD)" "$(r c3_n2 C3)" "$(r c3_h2 C3 $HD)" \
  "$(r c2_n1 C2)" "$(r c2_h1 C2 $HD)" "$(r c2_n2 C2)" "$(r c2_h2 C2 $HD)"
