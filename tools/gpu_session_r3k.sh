#!/bin/bash
# Round-3 session k: does the row-stride alignment of the GEMM outputs set the epilogue's store
# time? A/B of the step's GEMM shapes with 16-B (default), 128-B and 256-B padded row strides.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SH=enc_fwd_h,enc_bwd_d_h,dec_fwd_out,dec_bwd_d_out,head_bwd_d
GB="python tools/gemm_bench.py --shapes $SH --epilogues --rounds 3"
bash tools/gpu_steps.sh \
  "r3k_pad8|200|MVAE_BENCH_PLANES_ONLY=1 $GB --config C3 --variants 16" \
  "r3k_pad64|200|MVAE_BENCH_LDPAD=64 MVAE_BENCH_PLANES_ONLY=1 $GB --config C3 --variants 16" \
  "r3k_pad128|200|MVAE_BENCH_LDPAD=128 MVAE_BENCH_PLANES_ONLY=1 $GB --config C3 --variants 16" \
  "r3k_stamps|200|MVAE_BENCH_PLANES_ONLY=1 MVAE_STAMPS=1 python tools/gemm_bench.py --config C3 --shapes enc_fwd_h --variants 28 --epilogues --rounds 1 && MVAE_BENCH_LDPAD=64 MVAE_BENCH_PLANES_ONLY=1 MVAE_STAMPS=1 python tools/gemm_bench.py --config C3 --shapes enc_fwd_h --variants 28 --epilogues --rounds 1" \
  "r3k_pad8_c2|200|MVAE_BENCH_PLANES_ONLY=1 $GB --config C2 --variants 32" \
  "r3k_pad64_c2|200|MVAE_BENCH_LDPAD=64 MVAE_BENCH_PLANES_ONLY=1 $GB --config C2 --variants 32"
