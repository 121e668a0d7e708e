#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5g: (1) k-loop time per k-tile of the template and the library's eight-phase kernel without
# stamps: the same M x N at K = 4096, 8192, 16384 (the K difference cancels prologue/epilogue);
# (2) the tests touched by the create-option refactor (no environment switches in the library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r5g_k4|120|tools/micro/gemm8p 4096 4096 4096 --rounds 5 --lib magic_amd/libmvae.so" \
  "r5g_k8|120|tools/micro/gemm8p 4096 4096 8192 --rounds 5 --lib magic_amd/libmvae.so" \
  "r5g_k16|120|tools/micro/gemm8p 4096 4096 16384 --rounds 5 --lib magic_amd/libmvae.so" \
  "r5g_tests|600|$T tests/test_gpu_r3.py tests/test_gpu_conv.py tests/test_gpu_dp.py tests/test_input_pipeline.py" \
  "r5g_smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'"
