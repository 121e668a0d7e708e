#!/bin/bash
# Round-4 session ae: early Adam in-step A/B, alternating, 3 pairs per config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "$(run r4ae_c2_on1 '' C2)" "$(run r4ae_c2_off1 MVAE_NO_EARLY_ADAM=1 C2)" \
  "$(run r4ae_c2_off2 MVAE_NO_EARLY_ADAM=1 C2)" "$(run r4ae_c2_on2 '' C2)" \
  "$(run r4ae_c2_on3 '' C2)" "$(run r4ae_c2_off3 MVAE_NO_EARLY_ADAM=1 C2)" \
  "$(run r4ae_c3_on1 '' C3)" "$(run r4ae_c3_off1 MVAE_NO_EARLY_ADAM=1 C3)" \
  "$(run r4ae_c3_off2 MVAE_NO_EARLY_ADAM=1 C3)" "$(run r4ae_c3_on2 '' C3)" \
  "$(run r4ae_c3_on3 '' C3)" "$(run r4ae_c3_off3 MVAE_NO_EARLY_ADAM=1 C3)"
