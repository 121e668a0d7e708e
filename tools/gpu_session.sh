#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zo: verification of the tree after the decoder chain: full GPU suite, smoke, the default bench line (CPU baseline + PMC
# traffic + configs block), per-config rocprofv3 kernel-trace runs (C2, C3, C5).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
RP="rocprofv3 --kernel-trace --stats -f csv"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 10 --warmup 3"
bash tools/gpu_steps.sh \
  "r5zo_tests|400|$PT tests -m gpu" \
  "r5zo_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r5zo_bench|500|python bench.py > gpurun_out/r5zo_bench.json 2> gpurun_out/r5zo_bench.err" \
  "r5zo_prof_c2|150|$RP -d gpurun_out/r5zo_prof_c2 -o c2 -- python bench.py --config C2 $BQ" \
  "r5zo_prof_c3|150|$RP -d gpurun_out/r5zo_prof_c3 -o c3 -- python bench.py --config C3 $BQ" \
  "r5zo_prof_c5|150|$RP -d gpurun_out/r5zo_prof_c5 -o c5 -- python bench.py --config C5 $BQ"
