#!/bin/bash
# r7b: cs_one with LDS-staged last-chunk sums; full GPU suite; same-box A/B at C3 / C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r7b_c3_1|200|python bench.py --config C3 $A" \
  "r7b_c3_0|200|python bench.py --config C3 $A --create-opt cs_one=0" \
  "r7b_c3_1b|200|python bench.py --config C3 $A" \
  "r7b_c3_0b|200|python bench.py --config C3 $A --create-opt cs_one=0" \
  "r7b_c2_1|200|python bench.py --config C2 $A" \
  "r7b_c2_0|200|python bench.py --config C2 $A --create-opt cs_one=0" \
  "r7b_t|900|$T -m gpu tests"
