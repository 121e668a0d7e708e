#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zy: early_chunks 2 (even halves) vs 3 (3/4 + 1/4 of the layer-0 rows: a shorter exposed tail),
# C2 / C3 / C5, alternating in one library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5zy_$1|120|python bench.py --config $2 $BQ $3 > gpurun_out/r5zy_$1.json"; }
T="--opt early_chunks=3"
bash tools/gpu_steps.sh \
  "r5zy_t|300|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_r2.py -k early" \
  "$(r c2_e2a C2)" "$(r c2_e3a C2 "$T")" "$(r c2_e2b C2)" "$(r c2_e3b C2 "$T")" "$(r c2_e2c C2)" "$(r c2_e3c C2 "$T")" \
  "$(r c3_e2a C3)" "$(r c3_e3a C3 "$T")" "$(r c3_e2b C3)" "$(r c3_e3b C3 "$T")" \
  "$(r c5_e2a C5)" "$(r c5_e3a C5 "$T")" "$(r c5_e2b C5)" "$(r c5_e3b C5 "$T")"
