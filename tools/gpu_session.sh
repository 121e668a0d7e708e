#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r6e: the bits path's two forms -- A images expanded once per workgroup (B) and fragments per
# wave (R) -- against the plane path on the layer-0 shapes; the whole suite (pinned chunk plans,
# the C5 DP test); the step with bits in f32x too vs off, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T="python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider"
B="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --steps 50"
bash tools/gpu_steps.sh \
  "r6e_t|300|$T -x tests/test_gpu_r6.py" \
  "r6e_c3|240|python tools/gemm_bench.py --config C3 --shapes enc_fwd_0,enc_bwd_w_0 --variants 16b,29b,16B,16R --rounds 3 --epilogues" \
  "r6e_c2|240|python tools/gemm_bench.py --config C2 --shapes enc_fwd_0,enc_bwd_w_0 --variants 32b,45b,32B,32R --rounds 3 --epilogues" \
  "r6e_all|800|$T -m gpu tests" \
  "r6e_b2|300|python bench.py $B --create-opt bits=2 > gpurun_out/r6e_b2.json" \
  "r6e_b0|300|python bench.py $B --create-opt bits=0 > gpurun_out/r6e_b0.json" \
  "r6e_b2b|300|python bench.py $B --create-opt bits=2 > gpurun_out/r6e_b2b.json" \
  "r6e_b0b|300|python bench.py $B --create-opt bits=0 > gpurun_out/r6e_b0b.json"
