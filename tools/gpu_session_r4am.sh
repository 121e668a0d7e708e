#!/bin/bash
# Round-4 session am: the inexact-pixel flag in two alternating slots (no per-step memset launch)
# -- full GPU suite with its alternating-batch test; in-step A/B against the memset restored
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
M=MVAE_AB_DYN_MEMSET=1
bash tools/gpu_steps.sh \
  "r4am_tests|200|$PT tests -m gpu" \
  "$(run r4am_c2_new1 '' C2)" "$(run r4am_c2_old1 $M C2)" "$(run r4am_c2_old2 $M C2)" "$(run r4am_c2_new2 '' C2)" \
  "$(run r4am_c3_new1 '' C3)" "$(run r4am_c3_old1 $M C3)" "$(run r4am_c3_old2 $M C3)" "$(run r4am_c3_new2 '' C3)"
