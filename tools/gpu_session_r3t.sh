#!/bin/bash
# Round-3 session t: rational tanh (one rcp), hardware-log BCE fast path: full GPU suite, BCE/ACT
# GEMM A/B with stamps, bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
S="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues"
bash tools/gpu_steps.sh \
  "r3t_tests|900|$PT tests -m gpu" \
  "r3t_ab|300|$S --shapes dec_fwd_out,enc_fwd_h,enc_bwd_d_h --config C3 --variants 28 --rounds 3 --diag 0,8 && $S --shapes dec_fwd_out,enc_fwd_h,enc_bwd_d_h --config C2 --variants 44 --rounds 3" \
  "r3t_bench|300|python bench.py --no-cpu-baseline --pmc off > gpurun_out/r3t_bench.json 2> gpurun_out/r3t_bench.err"
