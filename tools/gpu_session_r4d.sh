#!/bin/bash
# Round-4 session d: stamped eight-phase 32x32 build under diag switches: 0 base, 1 no DMA in the
# loop, 64 no fragment reads, 128 no stagger, 65 neither DMA nor reads
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "r4d_stamps|300|MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 3 --config C3 --variants 22 --diag 0,1,64,128,65 --shapes square4096,enc_fwd_0,enc_bwd_w_0"
