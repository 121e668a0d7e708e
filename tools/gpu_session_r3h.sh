#!/bin/bash
# Round-3 session h: full GPU suite (chunked layer-0 gradient, ABI 4, ring-only default plan),
# stamped ring-kernel timelines, step benches, then the full default bench line (configs block,
# h2d, CPU baseline, PMC traffic).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
bash tools/gpu_steps.sh \
  "r3h_tests|900|$PT tests -m gpu" \
  "r3h_stamps|200|MVAE_STAMPS=1 python tools/gemm_bench.py --config C3 --shapes enc_fwd_h --variants 27,28 --epilogues --diag 0,1,8 --rounds 1 && MVAE_STAMPS=1 python tools/gemm_bench.py --config C2 --shapes enc_fwd_h --variants 43,44 --epilogues --diag 0,1,8 --rounds 1" \
  "r3h_bench_default|600|python bench.py > gpurun_out/r3h_default.json 2> gpurun_out/r3h_default.err"
