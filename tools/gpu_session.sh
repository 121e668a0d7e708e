#!/bin/bash
# r7e: full GPU suite with x3 / cs_one defaults; smoke
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r7e_t|1100|$T -m gpu tests" \
  "r7e_smoke|200|python -c 'import __graft_entry__ as g; g.smoke()'"
