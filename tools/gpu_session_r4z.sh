#!/bin/bash
# Round-4 session z: de-interleave at 8 pixels per thread by default -- full GPU suite, the 16-pixel
# form's parity, in-step A/B of 4 / 8 / 16 pixels per thread
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "r4z_tests|200|$PT tests -m gpu" \
  "r4z_tests16|200|MVAE_DEINT=16 $PT tests/test_gpu_parity.py tests/test_gpu_r2.py -k 'step or deint or grey or wide'" \
  "$(run r4z_c3_d8 '' C3)" "$(run r4z_c3_d16 MVAE_DEINT=16 C3)" "$(run r4z_c3_d4 MVAE_DEINT=4 C3)" \
  "$(run r4z_c3_d8b '' C3)" "$(run r4z_c3_d16b MVAE_DEINT=16 C3)"
