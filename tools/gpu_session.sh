#!/bin/bash
# r6zo: the de-interleave right after a 1 ms bf16 GEMM on random operands (+2000) or a 1 GB memset
# (+4000), each launch timed alone, against back-to-back launches -- why the in-step pass is slower
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "r6zo_db|400|python tools/deint_bench.py --config C3 --variants 7,2007,4007,1007,3007,5007 --rounds 3 --iters 10 && python tools/deint_bench.py --config C2 --variants 0,2000,4000 --rounds 3 --iters 10"
