#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5z: events without the system-scope fence (sync events of the side stream, timing events);
# against HEAD's library, alternating, C3 / C2 / C5. Tests of the step paths first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5z_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5z_$1.json"; }
H="MVAE_LIB=magic_amd/libmvae_head.so"
bash tools/gpu_steps.sh \
  "r5z_t|600|python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_r2.py tests/test_gpu_dp.py tests/test_gpu_parity.py" \
  "$(r c3_h1 C3 "$H")" "$(r c3_n1 C3)" "$(r c3_h2 C3 "$H")" "$(r c3_n2 C3)" \
  "$(r c2_h1 C2 "$H")" "$(r c2_n1 C2)" "$(r c2_h2 C2 "$H")" "$(r c2_n2 C2)" \
  "$(r c5_h1 C5 "$H")" "$(r c5_n1 C5)"
