#!/bin/bash
# Round-3 session p: BCE row partials summed through LDS; stamps of the BCE head (fp32 target,
# harness data) and of the hidden dgrad; parity subset; bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
S="MVAE_BENCH_PLANES_ONLY=1 MVAE_STAMPS=1 python tools/gemm_bench.py --epilogues --rounds 1"
bash tools/gpu_steps.sh \
  "r3r_tests|600|$PT tests/test_gpu_parity.py tests/test_gpu_r2.py tests/test_gpu_r3.py tests/test_gpu_golden.py" \
  "r3r_stamps|200|$S --config C3 --shapes dec_fwd_out,enc_bwd_d_h --variants 28 && $S --config C2 --shapes dec_fwd_out --variants 44" \
  "r3r_bench|300|python bench.py --no-cpu-baseline --pmc off > gpurun_out/r3r_bench.json 2> gpurun_out/r3r_bench.err"
