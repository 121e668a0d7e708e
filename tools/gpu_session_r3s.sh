#!/bin/bash
# Round-3 session s: the BCE head as the step runs it (binary bf16-plane target, dU planes only):
# kernel A/B (ring 256 / ring 128 / twin), stamps and ablations (diag 4 no LDS transpose, 8 no
# math, 16 no k-loop).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --epilogues --shapes dec_fwd_out"
bash tools/gpu_steps.sh \
  "r3s_ab|200|$S --config C3 --variants 28,27,29 --rounds 3 && $S --config C2 --variants 44,43,45 --rounds 3" \
  "r3s_stamps|300|MVAE_STAMPS=1 $S --config C3 --variants 28 --rounds 1 --diag 0,4,8,16,28"
