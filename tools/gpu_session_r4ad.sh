#!/bin/bash
# Round-4 session ad: early Adam (the blocks after layer 0 on the side stream beside the layer-0
# weight gradient) -- bitwise test, full suite, in-step A/B (MVAE_EARLY_ADAM is the bench's own
# switch via the DataParallelStep default; the A/B uses the engine option through an env hook)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "r4ad_tests|200|$PT tests -m gpu" \
  "$(run r4ad_c2_on '' C2)" "$(run r4ad_c2_off MVAE_NO_EARLY_ADAM=1 C2)" "$(run r4ad_c2_on2 '' C2)" "$(run r4ad_c2_off2 MVAE_NO_EARLY_ADAM=1 C2)" \
  "$(run r4ad_c3_on '' C3)" "$(run r4ad_c3_off MVAE_NO_EARLY_ADAM=1 C3)"
