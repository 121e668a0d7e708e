#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r6c: the B = 64 bf16 step failures with the bits path (the C/D-layout BCE epilogue read the
# target plane the bits de-interleave no longer writes): bits=0 vs bits=1 per tensor, then the
# three failing tests, then the whole suite
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh "r6c_dbg|200|python tools/dbg/bits_step.py" \
  "r6c_t3|200|$T tests/test_gpu_parity.py::test_step_bf16_documented_tolerance tests/test_gpu_r2.py::test_bce_saturation_forward_inf_gradients_finite tests/test_gpu_r5.py::test_enc_chain_step_widths" \
  "r6c_all|600|$T -m gpu tests"
