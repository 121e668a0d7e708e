#!/bin/bash
# Round-4 session g: stamped eight-phase build (prologue / k-loop / epilogue per workgroup) on
# the step's shapes and on L2-resident probes without split-K
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 3 --variants 22"
bash tools/gpu_steps.sh \
  "r4g_probe|200|MVAE_BENCH_SPLIT=1 $S --config C3 --diag 0,1 --shapes l2_one,l2_64" \
  "r4g_c3|300|$S --config C3 --diag 0 --shapes square4096,enc_fwd_0,dec_bwd_d_out,enc_fwd_h,dec_fwd_2,dec_bwd_w_2,enc_bwd_w_h"
S2="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3"
SH=enc_fwd_0,enc_bwd_w_0,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out,enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,head_fwd,head_bwd_d,head_bwd_w,dec_fwd_1,dec_bwd_w_1,dec_bwd_d_z,dec_fwd_2,dec_bwd_d_2,dec_bwd_w_2
bash tools/gpu_steps.sh \
  "r4g_plan_c3|300|$S2 --shapes $SH --config C3 --variants 16,31,29" \
  "r4g_plan_c2|300|$S2 --shapes $SH --config C2 --variants 32,47,45,35,43,0"
