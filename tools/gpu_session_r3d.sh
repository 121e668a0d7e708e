#!/bin/bash
# Round-3 session d: full GPU suite after fast tanh + bf16-plane DACT aux + long-row latent
# forward; row-alignment A/B of the GEMM epilogue stores; C5 / C3 / C2 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SH=enc_fwd_h,enc_bwd_d_h,dec_fwd_out,dec_bwd_d_out
bash tools/gpu_steps.sh \
  "r3d_tests|900|$PT tests -m gpu" \
  "r3d_ab_pad8|200|python tools/gemm_bench.py --config C3 --shapes $SH --variants 31,29 --epilogues --rounds 3" \
  "r3d_ab_pad64|200|MVAE_BENCH_LDPAD=64 python tools/gemm_bench.py --config C3 --shapes $SH --variants 31,29 --epilogues --rounds 3" \
  "r3d_bench_c5|200|python bench.py --config C5 --no-cpu-baseline --pmc off" \
  "r3d_bench_c3|200|python bench.py --config C3 --no-cpu-baseline --pmc off" \
  "r3d_bench_c3_f32aux|200|MVAE_DACT_F32AUX=1 python bench.py --config C3 --no-cpu-baseline --pmc off" \
  "r3d_bench_c2|200|python bench.py --no-cpu-baseline --pmc off"
