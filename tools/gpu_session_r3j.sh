#!/bin/bash
# Round-3 session j: branch-free epilogue math + prefetched epilogue operands: parity subset,
# stamps of the ring kernel (planes only), GEMM A/B and the three bench configurations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SH=enc_fwd_h,enc_bwd_d_h,dec_fwd_out,dec_bwd_d_out,head_bwd_d
bash tools/gpu_steps.sh \
  "r3j_tests|600|$PT tests/test_gpu_parity.py tests/test_gpu_r2.py tests/test_gpu_r3.py -k 'epilogue or step or satur or bce or c3 or c5'" \
  "r3j_stamps|200|MVAE_BENCH_PLANES_ONLY=1 MVAE_STAMPS=1 python tools/gemm_bench.py --config C3 --shapes enc_fwd_h --variants 28 --epilogues --diag 0,8 --rounds 1" \
  "r3j_ab_c3|200|MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --config C3 --shapes $SH --variants 16 --epilogues --rounds 3" \
  "r3j_ab_c2|200|MVAE_BENCH_PLANES_ONLY=1 python tools/gemm_bench.py --config C2 --shapes $SH --variants 32 --epilogues --rounds 3" \
  "r3j_bench|300|python bench.py --no-cpu-baseline --pmc off"
