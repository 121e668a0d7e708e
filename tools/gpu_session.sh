#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5t: what bounds the fused encoder chain: its region time with parts removed (create option
# diag_chain: 1 no weight DMA after the first steps, 2 no MFMAs, 4 no block copy-out), C3 / C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 10"
r() { echo "r5t_$1|120|python bench.py --config $2 $BQ $3 > gpurun_out/r5t_$1.json"; }
d() { echo "--create-opt diag_chain=$1"; }
bash tools/gpu_steps.sh \
  "r5t_t|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_r5.py" \
  "$(r c3_d0 C3)" "$(r c3_d1 C3 "$(d 1)")" "$(r c3_d2 C3 "$(d 2)")" "$(r c3_d4 C3 "$(d 4)")" "$(r c3_d3 C3 "$(d 3)")" \
  "$(r c3_d7 C3 "$(d 7)")" "$(r c5_d0 C5)" "$(r c5_d1 C5 "$(d 1)")" "$(r c5_d2 C5 "$(d 2)")"
