#!/bin/bash
# Round-4 session b (buffer-resource DMA): eight-phase kernel (gemm_bf16e.hip) correctness, then ring (15) vs
# eight-phase (13) A/B on the step's shapes in one process per config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
S="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3"
SH=enc_fwd_0,enc_bwd_w_0,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out,enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,square4096
bash tools/gpu_steps.sh \
  "r4b_e8_tests|400|$PT tests/test_gpu_r3.py tests/test_input_pipeline.py -k 'e8_kernel or e8_epilogues or batch_producer'" \
  "r4b_ab_c3|300|$S --shapes $SH --config C3 --variants 31,29" \
  "r4b_ab_c2|300|$S --shapes $SH --config C2 --variants 47,45"
