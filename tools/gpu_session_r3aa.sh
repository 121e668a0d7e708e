#!/bin/bash
# Round-3 session aa: cosine column statistics with batched loads (32-row chunks); full GPU suite
# and bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r3aa_tests|900|$PT tests -m gpu" \
  "r3aa_bench|300|python bench.py --no-cpu-baseline --pmc off > gpurun_out/r3aa_bench.json 2> gpurun_out/r3aa_bench.err"
