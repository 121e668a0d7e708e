#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r6za: the round-6 tree -- adam_nt A/B (non-temporal moment stores), per-config timed-loop
# kernel traces and the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
B="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 20 --warmup 3 --mark-dominant"
p() { echo "r6za_prof_$1|240|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/prof_r6za_$1 -o run -- python3 $PWD/bench.py --config $2 $B"; }
bash tools/gpu_steps.sh \
  "r6za_c3_n0a|200|python bench.py --config C3 $A --create-opt adam_nt=0" \
  "r6za_c3_n1a|200|python bench.py --config C3 $A --create-opt adam_nt=1" \
  "r6za_c3_n0b|200|python bench.py --config C3 $A --create-opt adam_nt=0" \
  "r6za_c3_n1b|200|python bench.py --config C3 $A --create-opt adam_nt=1" \
  "r6za_c2_n0a|200|python bench.py --config C2 $A --create-opt adam_nt=0" \
  "r6za_c2_n1a|200|python bench.py --config C2 $A --create-opt adam_nt=1" \
  "$(p c2 C2)" "$(p c3 C3)" "$(p c5 C5)" \
  "r6za_bench|900|python bench.py > gpurun_out/r6za_bench.json"
