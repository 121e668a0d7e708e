#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5p: is the layer-0 forward's k-loop bound by streaming X from HBM? Cost per k-tile (K
# differences 5001 -> 10001, split 1) of the eight-phase (29) and ring (31) kernels on the
# 24576 x 500 shape (X 491 MB, past the 256 MB last-level cache) vs 6144 x 500 (X 123 MB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
X="--extra f10:24576:500:10001:0:0:1 --extra f5:24576:500:5001:0:0:1 --extra q10:6144:500:10001:0:0:1 --extra q5:6144:500:5001:0:0:1 --extra s10:24576:512:10000:0:0:1 --extra s5:24576:512:5000:0:0:1"
bash tools/gpu_steps.sh \
  "r5p_l0|240|MVAE_BENCH_SPLIT=1 python tools/gemm_bench.py --variants 29,31 --rounds 5 --shapes none $X"
