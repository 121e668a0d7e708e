#!/bin/bash
# Round-4 session i: stamped eight-phase build with linear DMA source addresses (diag 2) vs the
# swizzled images, single workgroup (L2 warm) and 4096^3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 3"
bash tools/gpu_steps.sh \
  "r4i_probe|200|MVAE_BENCH_SPLIT=1 $S --config C3 --variants 22 --diag 0,2,1 --shapes l2_one,square4096"
