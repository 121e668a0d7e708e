#!/bin/bash
# Round-4 session aa: split-K reduction grid cap (MVAE_RED_GRID) in-step A/B, C2 and C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "$(run r4aa_c2_2k '' C2)" "$(run r4aa_c2_8k MVAE_RED_GRID=8192 C2)" "$(run r4aa_c2_64k MVAE_RED_GRID=65536 C2)" \
  "$(run r4aa_c2_2kb '' C2)" "$(run r4aa_c2_64kb MVAE_RED_GRID=65536 C2)" \
  "$(run r4aa_c3_2k '' C3)" "$(run r4aa_c3_64k MVAE_RED_GRID=65536 C3)"
