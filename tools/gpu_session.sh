#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zu: C2's thin GEMMs (latent head, decoder layer 1) in the fp32-accurate forms: the f32x ring
# kernel on any shape (v35 = prec 2 + variant 3, the step's thin_ring plan), native fp32 MFMA (v0),
# the fp32 VALU kernel (v9), with their epilogues.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
GB="python tools/gemm_bench.py --config C2 --epilogues --variants 35,0,9 --rounds 5 --shapes head_fwd,head_bwd_d,head_bwd_w,dec_fwd_1,dec_bwd_w_1,dec_bwd_d_z"
bash tools/gpu_steps.sh "r5zu|300|$GB"
