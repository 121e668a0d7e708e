#!/bin/bash
# Round-4 session aw: cost of the bench's live dominant-kernel timing (two HIP events per timed
# step) -- default line vs --no-timing at C2 / C3, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 40"
run() { echo "$1|90|python bench.py --config $3 $BQ $2 > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
T=--no-timing
bash tools/gpu_steps.sh \
  "$(run r4aw_c2_t1 '' C2)" "$(run r4aw_c2_n1 $T C2)" "$(run r4aw_c2_n2 $T C2)" "$(run r4aw_c2_t2 '' C2)" \
  "$(run r4aw_c3_t1 '' C3)" "$(run r4aw_c3_n1 $T C3)" "$(run r4aw_c3_n2 $T C3)" "$(run r4aw_c3_t2 '' C3)"
