#!/bin/bash
# Round-4 session q: epilogue ablation on the step's epilogue shapes (ring kernel diag bits:
# 2 no global stores, 4 no LDS transpose, 8 no transcendental math), C3 and C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
G="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3 --iters 10"
SH=dec_fwd_out,enc_fwd_h,enc_bwd_d_h,dec_fwd_2
bash tools/gpu_steps.sh \
  "r4q_epi_c3|200|$G --config C3 --shapes $SH --variants 31,29 --diag 0,2,4,8,14" \
  "r4q_epi_c2|200|$G --config C2 --shapes $SH --variants 47,45 --diag 0,2,4,8,14"
