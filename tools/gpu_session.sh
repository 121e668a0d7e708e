#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r6zq: the final tree (x3=2 default) -- whole GPU suite, smoke, C2 / C3 timed-loop traces, the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
B="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 20 --warmup 3 --mark-dominant"
p() { echo "r6zq_prof_$1|240|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats --output-format csv -d $PWD/gpurun_out/prof_r6zq_$1 -o run -- python3 $PWD/bench.py --config $2 $B"; }
bash tools/gpu_steps.sh \
  "r6zq_tests|1100|$T -m gpu tests" \
  "r6zq_smoke|240|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "$(p c2 C2)" "$(p c3 C3)" \
  "r6zq_bench|900|python bench.py > gpurun_out/r6zq_bench.json"
