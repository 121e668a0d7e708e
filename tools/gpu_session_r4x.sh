#!/bin/bash
# Round-4 session x: split-K choice on the layer-0 pair (eight-phase kernel) under the power limit
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
G="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3 --iters 10"
bash tools/gpu_steps.sh \
  "r4x_c3_s0|60|$G --config C3 --shapes enc_bwd_w_0,enc_fwd_0,dec_bwd_w_out,dec_bwd_d_out --variants 29" \
  "r4x_c3_s1|60|MVAE_BENCH_SPLIT=1 $G --config C3 --shapes enc_bwd_w_0,enc_fwd_0,dec_bwd_w_out,dec_bwd_d_out --variants 29" \
  "r4x_c3_s2|60|MVAE_BENCH_SPLIT=2 $G --config C3 --shapes enc_bwd_w_0,enc_fwd_0,dec_bwd_w_out,dec_bwd_d_out --variants 29" \
  "r4x_c3_s4|60|MVAE_BENCH_SPLIT=4 $G --config C3 --shapes enc_bwd_w_0,enc_fwd_0,dec_bwd_w_out,dec_bwd_d_out --variants 29" \
  "r4x_c2_s0|60|$G --config C2 --shapes enc_bwd_w_0,enc_fwd_0,dec_bwd_w_out,dec_bwd_d_out --variants 45" \
  "r4x_c2_s1|60|MVAE_BENCH_SPLIT=1 $G --config C2 --shapes enc_bwd_w_0,enc_fwd_0,dec_bwd_w_out,dec_bwd_d_out --variants 45" \
  "r4x_c2_s2|60|MVAE_BENCH_SPLIT=2 $G --config C2 --shapes enc_bwd_w_0,enc_fwd_0,dec_bwd_w_out,dec_bwd_d_out --variants 45"
