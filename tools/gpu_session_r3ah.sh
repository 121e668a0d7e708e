#!/bin/bash
# Round-3 session ah: fp32-only unsplit GEMM outputs (latent head forward) through the LDS
# row-major epilogue (MVAE_TE_FP32=1) vs the C/D-layout epilogue: harness A/B and bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="python tools/gemm_bench.py --epilogues --shapes head_fwd,enc_bwd_w_h --rounds 3 --variants"
B="python bench.py --no-cpu-baseline --pmc off"
bash tools/gpu_steps.sh \
  "r3ah_ab|300|$S 16 --config C5 && MVAE_TE_FP32=1 $S 16 --config C5 && $S 16 --config C3 && MVAE_TE_FP32=1 $S 16 --config C3" \
  "r3ah_b0|300|$B > gpurun_out/r3ah_b0.json 2> gpurun_out/r3ah_b0.err" \
  "r3ah_b1|300|MVAE_TE_FP32=1 $B > gpurun_out/r3ah_b1.json 2> gpurun_out/r3ah_b1.err"
