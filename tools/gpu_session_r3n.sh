#!/bin/bash
# Round-3 session n: whole-chunk padded epilogue stores (GemmEpi::padw). Parity subset, GEMM A/B
# on the step shapes, stamps, and the three-config bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SH=enc_fwd_h,enc_bwd_d_h,dec_fwd_out,dec_bwd_d_out,head_bwd_d
GB="python tools/gemm_bench.py --shapes $SH --epilogues --rounds 3"
bash tools/gpu_steps.sh \
  "r3n_tests|600|$PT tests/test_gpu_parity.py tests/test_gpu_r2.py tests/test_gpu_r3.py tests/test_gpu_golden.py" \
  "r3n_ab_c3|200|MVAE_BENCH_PLANES_ONLY=1 $GB --config C3 --variants 16" \
  "r3n_ab_c2|200|MVAE_BENCH_PLANES_ONLY=1 $GB --config C2 --variants 32" \
  "r3n_stamps|200|MVAE_BENCH_PLANES_ONLY=1 MVAE_STAMPS=1 python tools/gemm_bench.py --config C3 --shapes enc_fwd_h --variants 28,27 --epilogues --rounds 1" \
  "r3n_bench|300|python bench.py --no-cpu-baseline --pmc off > gpurun_out/r3n_bench.json 2> gpurun_out/r3n_bench.err"
