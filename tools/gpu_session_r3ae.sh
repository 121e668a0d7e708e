#!/bin/bash
# Round-3 session ae: how much of the ring kernel's k-loop is spent at iteration boundaries
# (counted vmcnt for the next images + the raw barrier), stamped builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="MVAE_BENCH_PLANES_ONLY=1 MVAE_STAMPS=1 python tools/gemm_bench.py --epilogues --rounds 1"
bash tools/gpu_steps.sh \
  "r3ae_c3|200|$S --config C3 --shapes enc_fwd_0,enc_fwd_h,dec_bwd_d_out --variants 16,28" \
  "r3ae_c2|200|$S --config C2 --shapes enc_fwd_0,dec_bwd_d_out --variants 32"
