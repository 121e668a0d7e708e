#!/bin/bash
# Round-3 session y: 192-row ring tiles (MI = 3) in the planner. Full GPU suite, GEMM A/B against
# MVAE_TM192=0 on the 500-wide shapes, plans, bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SH=enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,head_fwd,head_bwd_d,enc_fwd_0,dec_bwd_d_out
S="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --shapes $SH --rounds 2 --variants"
bash tools/gpu_steps.sh \
  "r3y_tests|900|$PT tests -m gpu" \
  "r3y_ab|300|$S 16 --config C3 && MVAE_TM192=0 $S 16 --config C3 && $S 32 --config C2 && MVAE_TM192=0 $S 32 --config C2" \
  "r3y_bench|300|MVAE_PLAN_LOG=1 python bench.py --no-cpu-baseline --pmc off > gpurun_out/r3y_bench.json 2> gpurun_out/r3y_bench.err" \
  "r3y_bench0|300|MVAE_TM192=0 python bench.py --no-cpu-baseline --pmc off > gpurun_out/r3y_bench0.json 2> gpurun_out/r3y_bench0.err"
