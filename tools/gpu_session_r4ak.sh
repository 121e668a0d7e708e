#!/bin/bash
# Round-4 session ak: planner -- the 192-row ring rule only for real one-round fills (C3/C5
# decoder-output dgrad back on the eight-phase kernel); in-step check C3 / C5 and the GEMM suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "r4ak_tests|200|$PT tests -m gpu" \
  "$(run r4ak_c3 '' C3)" "$(run r4ak_c5 '' C5)" "$(run r4ak_c3b '' C3)"
