#!/bin/bash
# Round-3 session e: stamped twin-kernel timelines of the hidden-layer forward GEMM (where does a
# short-K launch spend its time), HW-transcendental sampler check, C5 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r3e_stamps|200|for c in C2 C3; do MVAE_STAMPS=1 python tools/gemm_bench.py --config \$c --shapes enc_fwd_h --variants 29,45 --epilogues --diag 0,1,2 --rounds 1; done" \
  "r3e_tests|600|$PT tests/test_gpu_parity.py tests/test_gpu_r2.py -k 'eps or sampler or step_tiny or c5 or 8e or c3 or golden or inference'" \
  "r3e_bench_c5|200|python bench.py --config C5 --no-cpu-baseline --pmc off"
