#!/bin/bash
# r7d: x3 with the planner's x3 cost (tile N 128 plans for the f32x weight gradients); tests; C2 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r7d_tx|600|$T -m gpu tests/test_gpu_x3.py" \
  "r7d_c2_plan|200|python bench.py --config C2 $A --create-opt x3=1,plan_log=1" \
  "r7d_c2_x0|200|python bench.py --config C2 $A --create-opt x3=0" \
  "r7d_c2_x1|200|python bench.py --config C2 $A --create-opt x3=1" \
  "r7d_c2_x0b|200|python bench.py --config C2 $A --create-opt x3=0" \
  "r7d_c2_x1b|200|python bench.py --config C2 $A --create-opt x3=1"
