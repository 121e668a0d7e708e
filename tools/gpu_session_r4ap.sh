#!/bin/bash
# Round-4 session ap: fork events from an empty kernel's hipExtLaunchKernel stop event instead of
# hipEventRecord (MVAE_AB_EVK=1 all waits, 2 main-stream records only) -- GPU suite with it on,
# in-step A/B at C3 / C2, a kernel trace of C3 with it on
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
RP="rocprofv3 --kernel-trace --stats -f csv"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
E1=MVAE_AB_EVK=1; E2=MVAE_AB_EVK=2
bash tools/gpu_steps.sh \
  "r4ap_tests_evk|200|$E1 $PT tests -m gpu" \
  "$(run r4ap_c3_e1a $E1 C3)" "$(run r4ap_c3_e0a '' C3)" "$(run r4ap_c3_e2a $E2 C3)" \
  "$(run r4ap_c3_e2b $E2 C3)" "$(run r4ap_c3_e0b '' C3)" "$(run r4ap_c3_e1b $E1 C3)" \
  "$(run r4ap_c2_e1a $E1 C2)" "$(run r4ap_c2_e0a '' C2)" "$(run r4ap_c2_e0b '' C2)" "$(run r4ap_c2_e1b $E1 C2)" \
  "r4ap_prof_c3|150|$E1 $RP -d gpurun_out/r4ap_prof_c3 -o c3 -- python bench.py --config C3 --no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 10 --warmup 3"
