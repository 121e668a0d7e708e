#!/bin/bash
# Round-3 session a: twin-kernel parity, GEMM A/B on the C2 / C3 shapes (planner vs ring-only vs
# twin-forced, with the step epilogues), C2 / C3 step benches per twin mode.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r3a_twin_tests|600|$PT tests/test_gpu_r3.py -k 'gemm_twin or step_twin_modes'" \
  "r3a_wide_tests|600|$PT tests/test_gpu_parity.py -k 'wide or layouts'" \
  "r3a_ab_c2|300|python tools/gemm_bench.py --config C2 --epilogues --variants 32,47,45,46 --rounds 3" \
  "r3a_ab_c3|300|python tools/gemm_bench.py --config C3 --epilogues --variants 16,31,29,30 --rounds 3" \
  "r3a_bench_c2_t0|200|MVAE_TWIN=0 python bench.py --no-cpu-baseline --pmc off" \
  "r3a_bench_c2_t1|200|MVAE_TWIN=1 python bench.py --no-cpu-baseline --pmc off" \
  "r3a_bench_c2_t2|200|MVAE_TWIN=2 python bench.py --no-cpu-baseline --pmc off" \
  "r3a_bench_c3_t0|200|MVAE_TWIN=0 python bench.py --config C3 --no-cpu-baseline --pmc off" \
  "r3a_bench_c3_t1|200|MVAE_TWIN=1 MVAE_PLAN_LOG=1 python bench.py --config C3 --no-cpu-baseline --pmc off" \
  "r3a_bench_c3_t2|200|MVAE_TWIN=2 python bench.py --config C3 --no-cpu-baseline --pmc off" \
  "r3a_step_tests|600|$PT tests/test_gpu_r3.py -k 'c3_shape or c2_f32x'"
