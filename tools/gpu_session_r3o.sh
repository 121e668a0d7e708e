#!/bin/bash
# Round-3 session o: after the padded-epilogue fix, which kernel/tile serves the 500-wide GEMMs
# best? A/B of the ring kernel at tile N 256 (v12) / 128 (v11), the twin 128x128 kernel (v13) and
# the planner's default (v0), C2 (f32x) and C3 (bf16); and the plans the step uses.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SH=enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,head_fwd,head_bwd_d,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out,enc_fwd_0,enc_bwd_w_0
GB="python tools/gemm_bench.py --shapes $SH --epilogues --rounds 3"
bash tools/gpu_steps.sh \
  "r3o_c3|300|MVAE_BENCH_PLANES_ONLY=1 $GB --config C3 --variants 16,27,28,29" \
  "r3o_c2|300|MVAE_BENCH_PLANES_ONLY=1 $GB --config C2 --variants 32,43,44,45" \
  "r3o_plans|300|MVAE_PLAN_LOG=1 python bench.py --no-cpu-baseline --pmc off --steps 2 --warmup 1 > gpurun_out/r3o_plans.json 2> gpurun_out/r3o_plans.err"
