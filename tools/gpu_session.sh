#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5zc: the round's last changes, each against its parent commit (tools/build_rev.sh resolved
# "HEAD" inside its worktree until now, so the r5q-r5zb baselines were all commit e10f80b):
# libraries of 69aa44a (enc chain), 3f00a78 (+ BCE target bits), 590d7a3 (+ reuse walk), 91b90f1
# (+ one join), d856703 (+ events without system fence) and this tree (+ one BCE launch),
# rotated in that order, two rounds each of C2 and C3 (100 steps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline --steps 100"
r() { echo "r5zc_$1|120|$3 python bench.py --config $2 $BQ > gpurun_out/r5zc_$1.json"; }
rot() {  # config round
  for v in chain bits reuse join ev; do echo "$(r ${1}_${v}$2 $1 MVAE_LIB=magic_amd/libmvae_$v.so)"; done
  echo "$(r ${1}_tree$2 $1)"
}
mapfile -t S < <(rot C2 1; rot C3 1; rot C2 2; rot C3 2)
bash tools/gpu_steps.sh "${S[@]}"
