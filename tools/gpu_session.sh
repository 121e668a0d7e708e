#!/bin/bash
# r6z: the whole GPU suite and smoke on the tree with bits_reg on by default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r6z_tests|800|$T -m gpu tests" \
  "r6z_smoke|240|python -c 'import __graft_entry__ as g; g.smoke()'"
