#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r6g: after removing the LDS-image bits form: the bits tests, then same-box step A/B of the bits
# path (bf16: C3 / C5) -- bits=1 (default) vs bits=0, alternating, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
B="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 100"
r() { echo "r6g_$1|150|python bench.py $B --config $2 $3 > gpurun_out/r6g_$1.json"; }
bash tools/gpu_steps.sh \
  "r6g_t|300|$T -x tests/test_gpu_r6.py tests/test_gpu_r2.py" \
  "$(r c3_1a C3)" "$(r c3_0a C3 "--create-opt bits=0")" "$(r c3_1b C3)" "$(r c3_0b C3 "--create-opt bits=0")" \
  "$(r c5_1a C5)" "$(r c5_0a C5 "--create-opt bits=0")" "$(r c5_1b C5)" "$(r c5_0b C5 "--create-opt bits=0")"
