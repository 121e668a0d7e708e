#!/bin/bash
# Round-4 session k: full GPU suite (eight-phase kernel in the plan, snake pair order)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh "r4k_tests|840|$PT tests -m gpu"
