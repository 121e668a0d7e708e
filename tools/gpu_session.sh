#!/bin/bash
# r6ze: the de-interleave without its weight-gradient words (deint variant 7, diagnostics)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "r6ze_deint|200|python tools/deint_bench.py --config C3 --variants 0,7,0,7 --rounds 3 && python tools/deint_bench.py --config C2 --variants 0,7 --rounds 3"
