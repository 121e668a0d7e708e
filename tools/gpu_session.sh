#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r6zk: the final tree of round 6's second session (x3, cs_one) -- C2 / C3 timed-loop traces with
# the dominant region marked, the default bench line (C2 headline + configs block, PMC passes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 20 --warmup 3 --mark-dominant"
p() { echo "r6zk_prof_$1|240|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/prof_r6zk_$1 -o run -- python3 $PWD/bench.py --config $2 $B"; }
bash tools/gpu_steps.sh \
  "$(p c2 C2)" "$(p c3 C3)" \
  "r6zk_bench|900|python bench.py > gpurun_out/r6zk_bench.json"
