#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t7.log 2>&1
rc=$?; tail -15 gpurun_out/t7.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_bench.py --config C3 --epilogues --variants 0,20,19 --rounds 2 > gpurun_out/gemm_ab7.txt 2>&1
rc=$?; cat gpurun_out/gemm_ab7.txt; [ $rc -ne 0 ] && exit $rc
for c in "C3 bf16" "C2 f32x"; do
  set -- $c
  timeout -k 10 300 python bench.py --config $1 --precision $2 --no-cpu-baseline > gpurun_out/b7_$1_$2.json 2> gpurun_out/b7_$1_$2.err
  rc=$?; cat gpurun_out/b7_$1_$2.json; grep "\[bench\]" gpurun_out/b7_$1_$2.err | head -12
  [ $rc -ne 0 ] && { tail -5 gpurun_out/b7_$1_$2.err; exit $rc; }
done
exit 0
