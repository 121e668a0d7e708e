#!/bin/bash
# Round-4 session aj: cosine column statistics in 128-row chunks (vs 32: libmvae_cs32.so) --
# cosine tests, in-step A/B at C3 and C2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
OLD=MVAE_LIB=magic_amd/libmvae_cs32.so
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "r4aj_tests|200|$PT tests -m gpu -k 'cosine or parity or step or c3 or c2 or dp'" \
  "$(run r4aj_c3_new '' C3)" "$(run r4aj_c3_old $OLD C3)" "$(run r4aj_c3_old2 $OLD C3)" "$(run r4aj_c3_new2 '' C3)" \
  "$(run r4aj_c2_new '' C2)" "$(run r4aj_c2_old $OLD C2)"
