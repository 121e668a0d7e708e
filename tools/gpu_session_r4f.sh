#!/bin/bash
# Round-4 session f: eight-phase epilogue always 16-B where aligned; stamps on L2-resident probes
# (latency vs per-CU DMA bandwidth) and on the step shapes; A/B vs the ring kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3"
SH=enc_fwd_0,enc_bwd_w_0,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out,enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,square4096
bash tools/gpu_steps.sh \
  "r4f_stamps|300|MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 5 --config C3 --variants 22 --diag 0,1 --shapes l2_one,l2_64,square4096,dec_bwd_d_out,enc_fwd_0" \
  "r4f_ab_c3|300|$S --shapes $SH --config C3 --variants 31,22" \
  "r4f_ab_c2|300|$S --shapes $SH --config C2 --variants 47,38"
TH=head_fwd,head_bwd_d,head_bwd_w,dec_fwd_1,dec_bwd_w_1,dec_bwd_d_z,dec_fwd_2,dec_bwd_d_2,dec_bwd_w_2
bash tools/gpu_steps.sh \
  "r4f_thin_c3|300|$S --shapes $TH --config C3 --variants 16,29,19" \
  "r4f_thin_c2|300|$S --shapes $TH --config C2 --variants 0,9,45"
