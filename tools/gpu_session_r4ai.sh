#!/bin/bash
# Round-4 session ai: BCE head in whole rounds + 256x128 remainder (bce_split) -- full suite with
# its bitwise test, in-step A/B at C2 (the shape it applies to), alternating; gemm A/B of the head
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "r4ai_tests|200|$PT tests -m gpu" \
  "$(run r4ai_c2_on1 '' C2)" "$(run r4ai_c2_off1 MVAE_BCE_SPLIT=0 C2)" "$(run r4ai_c2_off2 MVAE_BCE_SPLIT=0 C2)" "$(run r4ai_c2_on2 '' C2)" \
  "$(run r4ai_c2_on3 '' C2)" "$(run r4ai_c2_off3 MVAE_BCE_SPLIT=0 C2)" \
  "r4ah_bce|200|MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --rounds 3 --iters 10 --config C2 --shapes dec_fwd_out --variants 45,47,43,44,32"
