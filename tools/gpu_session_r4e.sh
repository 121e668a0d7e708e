#!/bin/bash
# Round-4 session e: eight-phase kernel with 4/4/8/8 fragment reads per phase (A-sub 0 prefetched
# in q4) and contiguous half images (full-line DMA of row-contiguous operands): tests, stamps,
# A/B vs the ring kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
S="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3"
SH=enc_fwd_0,enc_bwd_w_0,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out,enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,square4096
bash tools/gpu_steps.sh \
  "r4e_tests|400|$PT tests/test_gpu_r3.py -k 'e8_kernel or e8_epilogues'" \
  "r4e_stamps|300|MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 3 --config C3 --variants 22,21 --diag 0,1,64 --shapes square4096,enc_fwd_0,enc_bwd_w_0" \
  "r4e_ab_c3|300|$S --shapes $SH --config C3 --variants 31,22,21" \
  "r4e_ab_c2|300|$S --shapes $SH --config C2 --variants 47,38"
