#!/bin/bash
# Round-4 session ac: conv1 forward with batched stores (arg1 / n1b of 4 pooled pixels per store
# instruction) -- conv tests, C5CONV A/B against the previous kernel (libmvae_convold.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline"
OLD=MVAE_LIB=magic_amd/libmvae_convold.so
run() { echo "$1|120|$2 python bench.py --config C5CONV $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "r4ac_tests|200|$PT tests/test_gpu_conv.py" \
  "$(run r4ac_new '')" "$(run r4ac_old $OLD)" "$(run r4ac_new2 '')" "$(run r4ac_old2 $OLD)"
