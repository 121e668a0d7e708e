#!/bin/bash
# Round-4 session m: eight-phase kernel reusing unchanged plane images (f32x pairs) + snake pair
# order: full GPU suite, stamps, A/B vs the ring kernels, default bench line, de-interleave NT A/B,
# persistent / staggered eight-phase A/B (C3 step regions)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
S="MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 3"
S2="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3"
SH=enc_fwd_0,enc_bwd_w_0,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out,enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,dec_fwd_2,square4096
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline"
bash tools/gpu_steps.sh \
  "r4m_tests|200|$PT tests -m gpu" \
  "r4m_stamps|90|$S --config C2 --variants 38 --shapes enc_fwd_0,dec_fwd_out" \
  "r4m_ab_c2|200|$S2 --shapes $SH --config C2 --variants 47,45,32" \
  "r4m_bench|240|python bench.py --no-cpu-baseline --pmc off > gpurun_out/r4m_bench.json 2> gpurun_out/r4m_bench.err" \
  "r4m_deint_nt1|80|python bench.py --config C3 $BQ > gpurun_out/r4m_deint_nt1.json 2> gpurun_out/r4m_deint_nt1.err" \
  "r4m_deint_nt0|80|MVAE_DEINT_NT=0 python bench.py --config C3 $BQ > gpurun_out/r4m_deint_nt0.json 2> gpurun_out/r4m_deint_nt0.err" \
  "r4m_persist0|80|MVAE_E8_PERSIST=1 python bench.py --config C3 $BQ > gpurun_out/r4m_persist0.json 2> gpurun_out/r4m_persist0.err" \
  "r4m_persist8|80|MVAE_E8_PERSIST=1 MVAE_E8_STAGGER=8 python bench.py --config C3 $BQ > gpurun_out/r4m_persist8.json 2> gpurun_out/r4m_persist8.err"
