#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/t8.log 2>&1
rc=$?; tail -15 gpurun_out/t8.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/gemm_bench.py --config C3 --epilogues --variants 19,35 --rounds 2 > gpurun_out/gemm_ab8.txt 2>&1
rc=$?; cat gpurun_out/gemm_ab8.txt; [ $rc -ne 0 ] && exit $rc
for c in "C3 bf16" "C2 f32x"; do
  set -- $c
  timeout -k 10 300 python bench.py --config $1 --precision $2 --no-cpu-baseline > gpurun_out/b8_$1_$2.json 2> gpurun_out/b8_$1_$2.err
  rc=$?; cat gpurun_out/b8_$1_$2.json; grep "\[bench\]" gpurun_out/b8_$1_$2.err | head -12
  [ $rc -ne 0 ] && { tail -5 gpurun_out/b8_$1_$2.err; exit $rc; }
done

cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing > $R/gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-timing > $R/gpurun_out/pmc_write.log 2>&1 || exit $?
python3 $R/tools/pmc_traffic.py --fetch $R/gpurun_out/pmc_fetch --write $R/gpurun_out/pmc_write --region enc_bwd_w_0 --config C2 --precision f32x > $R/gpurun_out/pmc_traffic.json; cat $R/gpurun_out/pmc_traffic.json
