#!/bin/bash
# Round-3 session c: full GPU suite after the fused latent head, then C5 / C3 / C2 bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r3c_tests|900|$PT tests -m gpu" \
  "r3c_bench_c5|200|python bench.py --config C5 --no-cpu-baseline --pmc off" \
  "r3c_bench_c3|200|python bench.py --config C3 --no-cpu-baseline --pmc off" \
  "r3c_bench_c2|200|python bench.py --no-cpu-baseline --pmc off"
