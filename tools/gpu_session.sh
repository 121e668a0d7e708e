#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5u: the BCE target as one bit per pixel (written by the de-interleave for 0/1 batches): parity
# tests, then whole steps against HEAD's library (libmvae_head.so, tools/build_rev.sh), alternating;
# and the eight-phase kernel's k-loop cycles on C2's layer-0 GEMMs with DMA / fragment reads off.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 60"
r() { echo "r5u_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5u_$1.json"; }
H="MVAE_LIB=magic_amd/libmvae_head.so"
bash tools/gpu_steps.sh \
  "r5u_t|900|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_r2.py tests/test_gpu_golden.py tests/test_gpu_r5.py tests/test_gpu_r3.py" \
  "$(r c3_n1 C3)" "$(r c3_h1 C3 "$H")" "$(r c3_n2 C3)" "$(r c3_h2 C3 "$H")" "$(r c3_n3 C3)" "$(r c3_h3 C3 "$H")" \
  "$(r c2_n1 C2)" "$(r c2_h1 C2 "$H")" "$(r c2_n2 C2)" "$(r c2_h2 C2 "$H")" \
  "$(r c5_n1 C5)" "$(r c5_h1 C5 "$H")" "$(r c5_n2 C5)" "$(r c5_h2 C5 "$H")" \
  "r5u_st|300|MVAE_STAMPS=2 python tools/gemm_bench.py --config C2 --variants 45 --diag 0,1,64 --rounds 1 --iters 3 --shapes enc_bwd_w_0,enc_fwd_0,dec_bwd_w_out"
