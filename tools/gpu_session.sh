#!/bin/bash
# r6zp: the 256x256 plane-stacked form (x3=2: C2's hidden weight gradients) -- tests, C2 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r6zp_tx|600|$T -m gpu tests/test_gpu_x3.py" \
  "r6zp_c2_1|200|python bench.py --config C2 $A --create-opt x3=1" \
  "r6zp_c2_2|200|python bench.py --config C2 $A --create-opt x3=2" \
  "r6zp_c2_1b|200|python bench.py --config C2 $A --create-opt x3=1" \
  "r6zp_c2_2b|200|python bench.py --config C2 $A --create-opt x3=2" \
  "r6zp_c2_1c|200|python bench.py --config C2 $A --create-opt x3=1" \
  "r6zp_c2_2c|200|python bench.py --config C2 $A --create-opt x3=2"
