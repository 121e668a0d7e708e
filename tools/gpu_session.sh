#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zg: C2's f32x hidden / decoder GEMMs (with their step epilogues, outputs as planes) on the
# planner's kernel (32) vs the eight-phase kernel forced (45: with the image-reusing walk) and its
# planner split -- the planner's e8 rule predates the walk.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,dec_fwd_2,dec_bwd_d_2,dec_bwd_w_2,enc_fwd_0,enc_bwd_w_0,dec_fwd_out,dec_bwd_d_out,dec_bwd_w_out"
bash tools/gpu_steps.sh \
  "r5zg|300|MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --config C2 --variants 32,45 --rounds 5 --epilogues --shapes $S"
