#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r6i: bits on in f32x too (default): the whole suite; then the default bench line (C2 + configs)
# bits=1 vs bits=0, alternating twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
B="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --steps 50"
r() { echo "r6i_$1|300|python bench.py $B $2 > gpurun_out/r6i_$1.json"; }
bash tools/gpu_steps.sh \
  "r6i_all|800|$T -m gpu tests" \
  "$(r 1a)" "$(r 0a "--create-opt bits=0")" "$(r 1b)" "$(r 0b "--create-opt bits=0")"
