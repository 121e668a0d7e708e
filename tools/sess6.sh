#!/bin/bash
# step benches: C2 f32x, C3/C4/C5 bf16 (regions on stderr), each under its own limit
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for c in "C2 f32x" "C3 bf16" "C5 bf16" "C2 f32"; do
  set -- $c
  timeout -k 10 300 python bench.py --config $1 --precision $2 --no-cpu-baseline > gpurun_out/b6_$1_$2.json 2> gpurun_out/b6_$1_$2.err
  rc=$?; cat gpurun_out/b6_$1_$2.json; grep "GEMM time" gpurun_out/b6_$1_$2.err
  [ $rc -ne 0 ] && { tail -5 gpurun_out/b6_$1_$2.err; exit $rc; }
done
exit 0
