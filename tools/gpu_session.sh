#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zz2: the default bench line again after the per-step PMC traffic fix (r5zz: tests, smoke,
# rocprof summaries of the same tree).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_steps.sh \
  "r5zz2_bench|500|python bench.py > gpurun_out/r5zz2_bench.json 2> gpurun_out/r5zz2_bench.err"
