#!/bin/bash
# Round-4 session at (closing tree: two-slot pixel flag, head weight gradient on the ring kernel): full GPU suite, smoke, default bench line (CPU baseline + PMC
# traffic), per-config rocprofv3 kernel-trace summaries (C2, C3, C5)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
RP="rocprofv3 --kernel-trace --stats -f csv"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 10 --warmup 3"
bash tools/gpu_steps.sh \
  "r4at_tests|200|$PT tests -m gpu" \
  "r4at_smoke|120|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "r4at_bench|500|python bench.py > gpurun_out/r4at_bench.json 2> gpurun_out/r4at_bench.err" \
  "r4at_prof_c2|150|$RP -d gpurun_out/r4at_prof_c2 -o c2 -- python bench.py --config C2 $BQ" \
  "r4at_prof_c3|150|$RP -d gpurun_out/r4at_prof_c3 -o c3 -- python bench.py --config C3 $BQ" \
  "r4at_prof_c5|150|$RP -d gpurun_out/r4at_prof_c5 -o c5 -- python bench.py --config C5 $BQ"
