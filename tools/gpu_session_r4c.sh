#!/bin/bash
# Round-4 session c: batch-producer contraction fix; eight-phase 16x16x32 variant (5) tests;
# stamped eight-phase builds (per-slot cycles) for 32x32 (6) and 16x16 (5); A/B 15 / 6 / 5
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
S="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3"
SH=enc_fwd_0,enc_bwd_w_0,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out,enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,square4096
bash tools/gpu_steps.sh \
  "r4c_tests|400|$PT tests/test_input_pipeline.py tests/test_gpu_r3.py -k 'e8_kernel or e8_epilogues or batch_producer'" \
  "r4c_stamps|300|MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 3 --config C3 --variants 22,21 --shapes square4096,enc_fwd_0,enc_bwd_w_0,dec_bwd_d_out" \
  "r4c_ab_c3|300|$S --shapes $SH --config C3 --variants 31,22,21" \
  "r4c_ab_c2|300|$S --shapes $SH --config C2 --variants 47,38,37"
