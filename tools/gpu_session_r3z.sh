#!/bin/bash
# Round-3 session z: de-interleave with 2 / 4 pixel quads per thread (MVAE_DI_U) vs the one-quad
# kernel; parity subset; bench lines with each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
B="python bench.py --no-cpu-baseline --pmc off"
bash tools/gpu_steps.sh \
  "r3z_tests|600|$PT tests/test_gpu_parity.py tests/test_input_pipeline.py tests/test_gpu_r2.py -k 'deinterleave or grey or step or batch or wide'" \
  "r3z_b2|300|$B > gpurun_out/r3z_b2.json 2> gpurun_out/r3z_b2.err" \
  "r3z_b1|300|MVAE_DI_U=1 $B > gpurun_out/r3z_b1.json 2> gpurun_out/r3z_b1.err" \
  "r3z_b4|300|MVAE_DI_U=4 $B > gpurun_out/r3z_b4.json 2> gpurun_out/r3z_b4.err"
