#!/bin/bash
# Round-4 session o: full GPU suite and the default bench line (CPU baseline + PMC traffic) on the
# planner with the in-step kernel choices
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r4o_tests|200|$PT tests -m gpu" \
  "r4o_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r4o_bench|780|python bench.py > gpurun_out/r4o_bench.json 2> gpurun_out/r4o_bench.err"
