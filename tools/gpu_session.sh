#!/bin/bash
# r6zb: the de-interleave with non-temporal loads of X (deint variant 6) -- isolated and in-step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r6zb_deint|200|python tools/deint_bench.py --config C3 --variants 0,6,0,6 --rounds 3 && python tools/deint_bench.py --config C2 --variants 0,6 --rounds 3" \
  "r6zb_c3_v0a|200|python bench.py --config C3 $A --create-opt deint_variant=0" \
  "r6zb_c3_v6a|200|python bench.py --config C3 $A --create-opt deint_variant=6" \
  "r6zb_c3_v0b|200|python bench.py --config C3 $A --create-opt deint_variant=0" \
  "r6zb_c3_v6b|200|python bench.py --config C3 $A --create-opt deint_variant=6" \
  "r6zb_c2_v0a|200|python bench.py --config C2 $A --create-opt deint_variant=0" \
  "r6zb_c2_v6a|200|python bench.py --config C2 $A --create-opt deint_variant=6"
