#!/bin/bash
# r6t: the fused workers' loaders and consumers timed apart (deint_fuse_diag 2 + 8: loaders
# only; 2 + 16: consumers only) at C3; bits_reg A/B (the bits path's A words to registers)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r6t_c3_d10|200|python bench.py --config C3 $B --create-opt deint_fuse=1,deint_fuse_diag=10" \
  "r6t_c3_d18|200|python bench.py --config C3 $B --create-opt deint_fuse=1,deint_fuse_diag=18" \
  "r6t_c3_d2|200|python bench.py --config C3 $B --create-opt deint_fuse=1,deint_fuse_diag=2" \
  "r6t_c3_r0a|200|python bench.py --config C3 $B --create-opt bits_reg=0" \
  "r6t_c3_r1a|200|python bench.py --config C3 $B --create-opt bits_reg=1" \
  "r6t_c3_r0b|200|python bench.py --config C3 $B --create-opt bits_reg=0" \
  "r6t_c3_r1b|200|python bench.py --config C3 $B --create-opt bits_reg=1" \
  "r6t_c2_r0a|200|python bench.py --config C2 $B --create-opt bits_reg=0" \
  "r6t_c2_r1a|200|python bench.py --config C2 $B --create-opt bits_reg=1" \
  "r6t_c2_r0b|200|python bench.py --config C2 $B --create-opt bits_reg=0" \
  "r6t_c2_r1b|200|python bench.py --config C2 $B --create-opt bits_reg=1" \
  "r6t_c5_r0a|200|python bench.py --config C5 $B --create-opt bits_reg=0" \
  "r6t_c5_r1a|200|python bench.py --config C5 $B --create-opt bits_reg=1"
