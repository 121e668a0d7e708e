#!/bin/bash
# Round-3 session m: where the ring kernel's epilogue time goes. Stamps with a "stores issued"
# mark; diag 16 = no k-loop (the epilogue alone), 8 = no math, 4 = no LDS transpose.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="MVAE_BENCH_PLANES_ONLY=1 MVAE_STAMPS=1 python tools/gemm_bench.py --config C3 --shapes enc_fwd_h --epilogues --rounds 1"
bash tools/gpu_steps.sh \
  "r3m_d0|100|$S --variants 28 --diag 0" \
  "r3m_d8|100|$S --variants 28 --diag 8" \
  "r3m_d12|100|$S --variants 28 --diag 12" \
  "r3m_d16|100|$S --variants 28 --diag 16" \
  "r3m_d28|100|$S --variants 28 --diag 28" \
  "r3m_t0|100|$S --variants 27 --diag 0" \
  "r3m_t16|100|$S --variants 27 --diag 16"
for f in gpurun_out/r3m_*.log; do echo "== $f"; grep -E "stamps|enc_fwd" $f; done
