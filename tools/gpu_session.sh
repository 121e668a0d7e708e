#!/bin/bash
# r6zl: default-option re-check at C2 with x3 (same box, each against an adjacent default run)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
A="--no-cpu-baseline --pmc off --no-h2d --no-pipeline --no-configs --steps 60 --warmup 5"
bash tools/gpu_steps.sh \
  "r6zl_d1|200|python bench.py --config C2 $A" \
  "r6zl_e80|200|python bench.py --config C2 $A --create-opt e8=0" \
  "r6zl_d2|200|python bench.py --config C2 $A" \
  "r6zl_bs0|200|python bench.py --config C2 $A --create-opt bce_split=0" \
  "r6zl_d3|200|python bench.py --config C2 $A" \
  "r6zl_tr1|200|python bench.py --config C2 $A --create-opt thin_ring=1" \
  "r6zl_d4|200|python bench.py --config C2 $A" \
  "r6zl_tr0|200|python bench.py --config C2 $A --create-opt thin_ring=0" \
  "r6zl_d5|200|python bench.py --config C2 $A" \
  "r6zl_ec2|200|python bench.py --config C2 $A --opt early_chunks=2" \
  "r6zl_d6|200|python bench.py --config C2 $A" \
  "r6zl_sm1|200|python bench.py --config C2 $A --opt side_mask=1" \
  "r6zl_d7|200|python bench.py --config C2 $A"
