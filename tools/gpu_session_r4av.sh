#!/bin/bash
# Round-4 session av: f32x short-K tall GEMMs (C2 latent-head dgrad 16384 x 500 x 40, decoder
# layer 1 forward 4096 x 500 x 21) on the fp32 MFMA kernel (MVAE_THIN_RING=3) -- in-step A/B at C2,
# the step parity tests with it on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
N=MVAE_THIN_RING=3
bash tools/gpu_steps.sh \
  "r4av_tests|200|$N $PT tests/test_gpu_parity.py -m gpu -k 'step or f32x'" \
  "$(run r4av_c2_new1 $N C2)" "$(run r4av_c2_old1 '' C2)" "$(run r4av_c2_old2 '' C2)" "$(run r4av_c2_new2 $N C2)" \
  "$(run r4av_c2_new3 $N C2)" "$(run r4av_c2_old3 '' C2)"
