#!/bin/bash
# Round-4 session an: LDS-staged de-interleave (lane-contiguous loads; MVAE_DEINT=1) -- full GPU
# suite with it forced, in-step A/B against the default 8-pixel kernel at C2 / C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
L=MVAE_DEINT=1
bash tools/gpu_steps.sh \
  "r4an_tests_lds|200|$L $PT tests -m gpu" \
  "$(run r4an_c3_lds1 $L C3)" "$(run r4an_c3_def1 '' C3)" "$(run r4an_c3_def2 '' C3)" "$(run r4an_c3_lds2 $L C3)" \
  "$(run r4an_c2_lds1 $L C2)" "$(run r4an_c2_def1 '' C2)" "$(run r4an_c2_def2 '' C2)" "$(run r4an_c2_lds2 $L C2)"
