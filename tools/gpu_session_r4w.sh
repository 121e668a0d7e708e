#!/bin/bash
# Round-4 session w: eight-phase kernel DMA / fragment-read placement experiments (stamped build,
# diag 4 = lgkmcnt(0) before each phase's DMA, diag 8 = DMA issued before the phase's reads)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 3"
bash tools/gpu_steps.sh \
  "r4w_st0|90|$S --config C3 --variants 22 --shapes square4096,enc_fwd_0,enc_bwd_w_0" \
  "r4w_st4|90|$S --config C3 --variants 22 --diag 4 --shapes square4096,enc_fwd_0,enc_bwd_w_0" \
  "r4w_st8|90|$S --config C3 --variants 22 --diag 8 --shapes square4096,enc_fwd_0,enc_bwd_w_0" \
  "r4w_st0b|90|$S --config C3 --variants 22 --shapes square4096,enc_fwd_0,enc_bwd_w_0"
