#!/bin/bash
# Round-4 session j: full GPU suite with the eight-phase kernel in the plan; bench (no CPU
# baseline / PMC passes) with the C3 / C5 configs and the input-pipeline leg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r4j_tests|780|$PT tests -m gpu" \
  "r4j_bench|380|python bench.py --no-cpu-baseline --pmc off > gpurun_out/r4j_bench.json 2> gpurun_out/r4j_bench.err"
