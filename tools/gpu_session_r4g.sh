#!/bin/bash
# Round-4 session g: stamped eight-phase build (prologue / k-loop / epilogue per workgroup) on
# the step's shapes and on L2-resident probes without split-K
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 3 --variants 22"
bash tools/gpu_steps.sh \
  "r4g_probe|200|MVAE_BENCH_SPLIT=1 $S --config C3 --diag 0,1 --shapes l2_one,l2_64" \
  "r4g_c3|300|$S --config C3 --diag 0 --shapes square4096,enc_fwd_0,dec_bwd_d_out,enc_fwd_h,dec_fwd_2,dec_bwd_w_2,enc_bwd_w_h"
