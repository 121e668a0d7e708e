#!/bin/bash
# Round-4 session ag: input staging (mvae_stage_input) -- full suite, then in-step A/B against
# in-line de-interleave (--no-stage), alternating, C2 and C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
run() { echo "$1|90|python bench.py --config $3 $BQ $2 > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "r4ag_tests|200|$PT tests -m gpu" \
  "$(run r4ag_c2_on1 '' C2)" "$(run r4ag_c2_off1 --no-stage C2)" "$(run r4ag_c2_off2 --no-stage C2)" "$(run r4ag_c2_on2 '' C2)" \
  "$(run r4ag_c3_on1 '' C3)" "$(run r4ag_c3_off1 --no-stage C3)" "$(run r4ag_c3_off2 --no-stage C3)" "$(run r4ag_c3_on2 '' C3)" \
  "$(run r4ag_c5_on1 '' C5)" "$(run r4ag_c5_off1 --no-stage C5)"
