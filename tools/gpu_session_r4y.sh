#!/bin/bash
# Round-4 session y: de-interleave with 8 pixels per thread (MVAE_DEINT=8) -- parity tests under it
# and the in-step A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "r4y_tests|200|MVAE_DEINT=8 $PT tests/test_gpu_parity.py tests/test_gpu_r2.py tests/test_gpu_r3.py" \
  "$(run r4y_c3_d4 '' C3)" "$(run r4y_c3_d8 MVAE_DEINT=8 C3)" "$(run r4y_c3_d4b '' C3)" "$(run r4y_c3_d8b MVAE_DEINT=8 C3)" \
  "$(run r4y_c2_d4 '' C2)" "$(run r4y_c2_d8 MVAE_DEINT=8 C2)"
