#!/bin/bash
# Round-3 session ab: VALU-kernel DACT operand loaded before the k-loop; parity subset, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r3ab_tests|600|$PT tests/test_gpu_parity.py tests/test_gpu_r2.py tests/test_gpu_golden.py tests/test_gpu_r3.py" \
  "r3ab_bench|300|python bench.py --no-cpu-baseline --pmc off > gpurun_out/r3ab_bench.json 2> gpurun_out/r3ab_bench.err"
