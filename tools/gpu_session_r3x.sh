#!/bin/bash
# Round-3 session x: split-K reductions with batched slab loads; parity subset and bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r3x_tests|600|$PT tests/test_gpu_parity.py tests/test_gpu_r2.py tests/test_gpu_r3.py tests/test_gpu_golden.py tests/test_gpu_dp.py" \
  "r3x_bench|300|python bench.py --no-cpu-baseline --pmc off > gpurun_out/r3x_bench.json 2> gpurun_out/r3x_bench.err"
