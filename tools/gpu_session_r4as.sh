#!/bin/bash
# Round-4 session as: the f32x head weight gradient (501 x 40 x 8192) on the ring kernel -- full
# GPU suite, in-step A/B at C2 against MVAE_THIN_RING=1 (the fp32 kernel for it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
O=MVAE_THIN_RING=1
bash tools/gpu_steps.sh \
  "r4as_tests|200|$PT tests -m gpu" \
  "$(run r4as_c2_new1 '' C2)" "$(run r4as_c2_old1 $O C2)" "$(run r4as_c2_old2 $O C2)" "$(run r4as_c2_new2 '' C2)" \
  "$(run r4as_c2_new3 '' C2)" "$(run r4as_c2_old3 $O C2)"
