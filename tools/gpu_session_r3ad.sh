#!/bin/bash
# Round-3 session ad: new tests (forced 192-row ring tiles, sample_latent_space on the GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh "r3ad_tests|600|$PT tests/test_gpu_r3.py -k 'tile192 or sample_latent'"
