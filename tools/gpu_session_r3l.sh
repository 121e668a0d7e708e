#!/bin/bash
# Round-3 session l: epilogue band loop not unrolled (code 37.6 -> 13.6 KB for the ACT kernel):
# micro-benchmarks (cold instruction fetch, store patterns), GEMM A/B on the step shapes,
# stamps, then the three-config bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SH=enc_fwd_h,enc_bwd_d_h,dec_fwd_out,dec_bwd_d_out,head_bwd_d
GB="python tools/gemm_bench.py --shapes $SH --epilogues --rounds 3"
bash tools/gpu_steps.sh \
  "r3l_micro|100|./tools/micro/icache && ./tools/micro/store_bw" \
  "r3l_ab_c3|200|MVAE_BENCH_PLANES_ONLY=1 $GB --config C3 --variants 16" \
  "r3l_ab_c2|200|MVAE_BENCH_PLANES_ONLY=1 $GB --config C2 --variants 32" \
  "r3l_stamps|200|MVAE_BENCH_PLANES_ONLY=1 MVAE_STAMPS=1 python tools/gemm_bench.py --config C3 --shapes enc_fwd_h --variants 28 --epilogues --rounds 1" \
  "r3l_bench|300|python bench.py --no-cpu-baseline --pmc off > gpurun_out/r3l_bench.json 2> gpurun_out/r3l_bench.err"
