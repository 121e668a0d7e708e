#!/bin/bash
# r7a: one-launch column statistics (cs_one) tests and same-box A/B at C2 / C3 (cosine)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r7a_t|400|$T -m gpu tests/test_gpu_r6.py -k 'cs_one or xbw'" \
  "r7a_c2_1|200|python bench.py --config C2 $A" \
  "r7a_c2_0|200|python bench.py --config C2 $A --create-opt cs_one=0" \
  "r7a_c2_1b|200|python bench.py --config C2 $A" \
  "r7a_c2_0b|200|python bench.py --config C2 $A --create-opt cs_one=0" \
  "r7a_c3_1|200|python bench.py --config C3 $A" \
  "r7a_c3_0|200|python bench.py --config C3 $A --create-opt cs_one=0"
