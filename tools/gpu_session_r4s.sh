#!/bin/bash
# Round-4 session s: split-K slabs vs narrower ring tiles on the short-K GEMMs (C2 f32x, C3 bf16)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
G="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3 --iters 10"
SH=enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,dec_fwd_2,dec_bwd_d_2,dec_bwd_w_2,enc_fwd_0,dec_bwd_d_out,dec_bwd_w_out
bash tools/gpu_steps.sh \
  "r4s_c2|240|$G --config C2 --shapes $SH --variants 32,47,43,44" \
  "r4s_c3|240|$G --config C3 --shapes $SH --variants 16,31,27,28"
