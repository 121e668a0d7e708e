#!/bin/bash
# r6zm: coalesced de-interleave loads (deint_variant 8 / 9): bitwise tests, isolated A/B with the
# input cached or not (variant + 1000: four X images in turn), step A/B at C3 / C2; x3 tests (live skip)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q -x --timeout 300 --timeout-method thread -p no:cacheprovider"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r6zm_t|600|$T -m gpu tests/test_gpu_r6.py -k 'coalesced or cs_one' tests/test_gpu_x3.py" \
  "r6zm_db|300|python tools/deint_bench.py --config C3 --variants 0,8,1000,1008,7,9,1007,1009 --rounds 3 && python tools/deint_bench.py --config C2 --variants 0,8,1000,1008 --rounds 3" \
  "r6zm_c3_d|200|python bench.py --config C3 $A" \
  "r6zm_c3_8|200|python bench.py --config C3 $A --create-opt deint_variant=8" \
  "r6zm_c3_db|200|python bench.py --config C3 $A" \
  "r6zm_c3_8b|200|python bench.py --config C3 $A --create-opt deint_variant=8" \
  "r6zm_c2_d|200|python bench.py --config C2 $A" \
  "r6zm_c2_8|200|python bench.py --config C2 $A --create-opt deint_variant=8" \
  "r6zm_c2_db|200|python bench.py --config C2 $A" \
  "r6zm_c2_8b|200|python bench.py --config C2 $A --create-opt deint_variant=8"
