#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zt: C2's f32x hidden shapes on the eight-phase kernel (forced: variants 13 / 14, prec 2 -> 45 / 46)
# against the planner's ring-kernel plans, split-K 1 and 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
GB="python tools/gemm_bench.py --config C2 --epilogues --variants 32,45,46 --rounds 5 --shapes enc_fwd_h,enc_bwd_d_h,dec_fwd_2,dec_bwd_d_2,dec_bwd_w_2,enc_bwd_w_h"
bash tools/gpu_steps.sh "r5zt_plan|300|$GB" "r5zt_s1|300|MVAE_BENCH_SPLIT=1 $GB" "r5zt_s2|300|MVAE_BENCH_SPLIT=2 $GB"
