#!/bin/bash
# Round-4 session h: eight-phase kernel with the DMA issued between the MFMAs (variants 7 / 8):
# tests, stamps, A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
S="MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 3"
S2="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3"
SH=enc_fwd_0,enc_bwd_w_0,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out,enc_bwd_d_h,head_bwd_d,square4096
bash tools/gpu_steps.sh \
  "r4h_tests|400|$PT tests/test_gpu_r3.py -k 'e8_kernel or e8_epilogues'" \
  "r4h_probe|200|MVAE_BENCH_SPLIT=1 $S --config C3 --variants 22,23,24 --shapes l2_one" \
  "r4h_stamps|300|$S --config C3 --variants 22,23 --shapes square4096,enc_fwd_0" \
  "r4h_ab_c3|300|$S2 --shapes $SH --config C3 --variants 31,22,23,24" \
  "r4h_ab_c2|300|$S2 --shapes $SH --config C2 --variants 47,38,39"
