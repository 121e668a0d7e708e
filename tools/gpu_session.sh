#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r6m: timed-loop kernel traces with markers around the dominant region, C2 / C3 / C5 (defaults)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 20 --warmup 3 --mark-dominant"
p() { echo "r6m_prof_$1|240|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/prof_r6m_$1 -o run -- python3 $PWD/bench.py --config $2 $B"; }
bash tools/gpu_steps.sh "$(p c2 C2)" "$(p c3 C3)" "$(p c5 C5)"
