#!/bin/bash
# Round-3 session w: ring-kernel fragment-read placement (MVAE_QGAP=1: the next k16-step's reads
# in the first 7 of 8 MFMA gaps) vs default, two library builds, alternating processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SH=enc_fwd_0,enc_bwd_w_0,dec_fwd_out,dec_bwd_d_out,enc_fwd_h,enc_bwd_d_h,square4096
S="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --shapes $SH --rounds 2"
bash tools/gpu_steps.sh \
  "r3w_a1|200|$S --config C3 --variants 28" \
  "r3w_b1|200|MVAE_LIB=magic_amd/libmvae_alt1.so $S --config C3 --variants 28" \
  "r3w_a2|200|$S --config C3 --variants 28" \
  "r3w_b2|200|MVAE_LIB=magic_amd/libmvae_alt1.so $S --config C3 --variants 28" \
  "r3w_a3|200|$S --config C2 --variants 44" \
  "r3w_b3|200|MVAE_LIB=magic_amd/libmvae_alt1.so $S --config C2 --variants 44"
