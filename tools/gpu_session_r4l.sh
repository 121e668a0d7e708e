#!/bin/bash
# Round-4 session l: default bench line (CPU baseline + PMC traffic) and per-config rocprofv3
# kernel-trace summaries (C2, C3, C5) of the same tree
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
RP="rocprofv3 --kernel-trace --stats -f csv"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 10 --warmup 3"
bash tools/gpu_steps.sh \
  "r4l_bench|560|python bench.py > gpurun_out/r4l_bench.json 2> gpurun_out/r4l_bench.err" \
  "r4l_prof_c2|180|$RP -d gpurun_out/r4l_prof_c2 -o c2 -- python bench.py --config C2 $BQ" \
  "r4l_prof_c3|180|$RP -d gpurun_out/r4l_prof_c3 -o c3 -- python bench.py --config C3 $BQ" \
  "r4l_prof_c5|180|$RP -d gpurun_out/r4l_prof_c5 -o c5 -- python bench.py --config C5 $BQ"
