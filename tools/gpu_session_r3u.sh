#!/bin/bash
# Round-3 session u: s_setprio 1 around each k16-step of the ring kernel (diag 32 A/B switch)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues"
SH=enc_fwd_0,enc_bwd_w_0,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out,enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,square4096
bash tools/gpu_steps.sh \
  "r3u_c3|300|$S --shapes $SH --config C3 --variants 28 --rounds 3 --diag 0,32" \
  "r3u_c2|300|$S --shapes $SH --config C2 --variants 44 --rounds 3 --diag 0,32"
