#!/bin/bash
# r7c: the plane-stacked f32x ring kernel (x3): kernel + step tests, C2 A/B; cs_one A/B at C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r7c_tx|600|$T -m gpu tests/test_gpu_x3.py" \
  "r7c_c2_x1|200|python bench.py --config C2 $A --create-opt x3=1" \
  "r7c_c2_x0|200|python bench.py --config C2 $A --create-opt x3=0" \
  "r7c_c2_x1b|200|python bench.py --config C2 $A --create-opt x3=1" \
  "r7c_c2_x0b|200|python bench.py --config C2 $A --create-opt x3=0" \
  "r7c_c3_1|200|python bench.py --config C3 $A" \
  "r7c_c3_0|200|python bench.py --config C3 $A --create-opt cs_one=0" \
  "r7c_c3_1b|200|python bench.py --config C3 $A" \
  "r7c_c3_0b|200|python bench.py --config C3 $A --create-opt cs_one=0"
