#!/bin/bash
# Round-3 session aa: one planner pass per GEMM launch; full GPU suite
# and bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r3al_tests|900|$PT tests -m gpu" \
  "r3al_bench|300|python bench.py --no-cpu-baseline --pmc off > gpurun_out/r3al_bench.json 2> gpurun_out/r3al_bench.err"
