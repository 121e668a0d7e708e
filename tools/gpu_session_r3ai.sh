#!/bin/bash
# Round-3 session ai: with this round's epilogue fixes, does the planner's twin-kernel choice
# (MVAE_TWIN=1) now win anywhere? Bench lines default vs MVAE_TWIN=1, twice each, one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python bench.py --no-cpu-baseline --pmc off"
bash tools/gpu_steps.sh \
  "r3ai_a|300|$B > gpurun_out/r3ai_a.json 2> gpurun_out/r3ai_a.err" \
  "r3ai_t|300|MVAE_TWIN=1 MVAE_PLAN_LOG=1 $B > gpurun_out/r3ai_t.json 2> gpurun_out/r3ai_t.err" \
  "r3ai_a2|300|$B > gpurun_out/r3ai_a2.json 2> gpurun_out/r3ai_a2.err" \
  "r3ai_t2|300|MVAE_TWIN=1 $B > gpurun_out/r3ai_t2.json 2> gpurun_out/r3ai_t2.err"
