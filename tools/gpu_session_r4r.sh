#!/bin/bash
# Round-4 session r: f32x latent head on the ring kernel (A/B in the C2 step), full GPU suite,
# hipBLASLt yardstick on the step's GEMM shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -q --maxfail=10 --timeout 120 --timeout-method thread -p no:cacheprovider"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline"
bash tools/gpu_steps.sh \
  "r4r_tests|200|$PT tests -m gpu" \
  "r4r_c2_tr1|90|python bench.py --config C2 $BQ > gpurun_out/r4r_c2_tr1.json 2> gpurun_out/r4r_c2_tr1.err" \
  "r4r_c2_tr0|90|MVAE_THIN_RING=0 python bench.py --config C2 $BQ > gpurun_out/r4r_c2_tr0.json 2> gpurun_out/r4r_c2_tr0.err" \
  "r4r_c2_tr1b|90|python bench.py --config C2 $BQ > gpurun_out/r4r_c2_tr1b.json 2> gpurun_out/r4r_c2_tr1b.err" \
  "r4r_blas_c3|200|python tools/blas_probe.py --config C3" \
  "r4r_blas_c2|200|python tools/blas_probe.py --config C2"
