#!/bin/bash
# r6zg: xbw_split auto (on where the layer-0 forward leaves CUs: C3 / C5; off at C2) against off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r6zg_t|400|$T -m gpu tests/test_gpu_r6.py" \
  "r6zg_c3_a|200|python bench.py --config C3 $A" \
  "r6zg_c3_0|200|python bench.py --config C3 $A --create-opt xbw_split=0" \
  "r6zg_c3_b|200|python bench.py --config C3 $A" \
  "r6zg_c3_1|200|python bench.py --config C3 $A --create-opt xbw_split=0" \
  "r6zg_c2_a|200|python bench.py --config C2 $A" \
  "r6zg_c2_0|200|python bench.py --config C2 $A --create-opt xbw_split=0" \
  "r6zg_c5_a|200|python bench.py --config C5 $A" \
  "r6zg_c5_0|200|python bench.py --config C5 $A --create-opt xbw_split=0"
