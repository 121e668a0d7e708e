#!/bin/bash
# Round-4 session u: grouped tile order (MVAE_TILE_GROUP) -- correctness under G=8 and the in-step
# A/B on C3 / C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "r4u_tests_g8|200|MVAE_TILE_GROUP=8 $PT tests/test_gpu_parity.py tests/test_gpu_r3.py tests/test_gpu_r2.py" \
  "$(run r4u_c3_g0 MVAE_TILE_GROUP=0 C3)" "$(run r4u_c3_g8 MVAE_TILE_GROUP=8 C3)" "$(run r4u_c3_g4 MVAE_TILE_GROUP=4 C3)" \
  "$(run r4u_c3_g0b MVAE_TILE_GROUP=0 C3)" "$(run r4u_c2_g0 MVAE_TILE_GROUP=0 C2)" "$(run r4u_c2_g8 MVAE_TILE_GROUP=8 C2)" \
  "$(run r4u_c5_g0 MVAE_TILE_GROUP=0 C5)" "$(run r4u_c5_g8 MVAE_TILE_GROUP=8 C5)"
