#!/bin/bash
# r6zd: the eight-phase kernel's s_setprio form (e8_prio: 0 flips around every MFMA quadrant,
# 1 static priority for the lagging half, 2 none), same box, alternating
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r6zd_c3_p0a|200|python bench.py --config C3 $A --create-opt e8_prio=0" \
  "r6zd_c3_p1a|200|python bench.py --config C3 $A --create-opt e8_prio=1" \
  "r6zd_c3_p2a|200|python bench.py --config C3 $A --create-opt e8_prio=2" \
  "r6zd_c3_p0b|200|python bench.py --config C3 $A --create-opt e8_prio=0" \
  "r6zd_c3_p1b|200|python bench.py --config C3 $A --create-opt e8_prio=1" \
  "r6zd_c3_p2b|200|python bench.py --config C3 $A --create-opt e8_prio=2" \
  "r6zd_c2_p0a|200|python bench.py --config C2 $A --create-opt e8_prio=0" \
  "r6zd_c2_p1a|200|python bench.py --config C2 $A --create-opt e8_prio=1" \
  "r6zd_c2_p0b|200|python bench.py --config C2 $A --create-opt e8_prio=0" \
  "r6zd_c2_p1b|200|python bench.py --config C2 $A --create-opt e8_prio=1"
