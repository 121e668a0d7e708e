#!/bin/bash
# Round-3 session g: branch-free activation epilogues + 4-stage BK-32 twin kernel: parity, stamped
# timelines, GEMM A/B, C3 / C2 step benches per twin mode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
SH=enc_fwd_h,enc_bwd_d_h,enc_bwd_w_h,dec_fwd_out,head_fwd,head_bwd_d
bash tools/gpu_steps.sh \
  "r3g_tests32|600|MVAE_TWIN_BK=32 $PT tests/test_gpu_r3.py" \
  "r3g_tests|600|$PT tests/test_gpu_parity.py -k 'epilogues or layouts or wide or step_tiny'" \
  "r3g_stamps|200|for b in 64 32; do MVAE_TWIN_BK=\$b MVAE_STAMPS=1 python tools/gemm_bench.py --config C3 --shapes enc_fwd_h --variants 29 --epilogues --diag 0,8 --rounds 1; done" \
  "r3g_ab_c3_64|200|python tools/gemm_bench.py --config C3 --shapes $SH --variants 31,29 --epilogues --rounds 3" \
  "r3g_ab_c3_32|200|MVAE_TWIN_BK=32 python tools/gemm_bench.py --config C3 --shapes $SH --variants 31,29 --epilogues --rounds 3" \
  "r3g_ab_c2_32|200|MVAE_TWIN_BK=32 python tools/gemm_bench.py --config C2 --shapes $SH --variants 47,45 --epilogues --rounds 3" \
  "r3g_bench_c3_t0|200|MVAE_TWIN=0 python bench.py --config C3 --no-cpu-baseline --pmc off" \
  "r3g_bench_c3_t2|200|MVAE_TWIN=2 python bench.py --config C3 --no-cpu-baseline --pmc off" \
  "r3g_bench_c3_t2_32|200|MVAE_TWIN_BK=32 MVAE_TWIN=2 python bench.py --config C3 --no-cpu-baseline --pmc off" \
  "r3g_bench_c2_t0|200|MVAE_TWIN=0 python bench.py --no-cpu-baseline --pmc off" \
  "r3g_bench_c2_t2_32|200|MVAE_TWIN_BK=32 MVAE_TWIN=2 python bench.py --no-cpu-baseline --pmc off"
