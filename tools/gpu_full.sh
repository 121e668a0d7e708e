#!/bin/bash
# One full GPU session: parity tests, smoke, PMC traffic passes of the default bench,
# rocprofv3 kernel-trace stats, then the bench lines (default C2 with CPU baseline + C3).
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
O=$R/gpurun_out
TAG=${TAG:-r1}
mkdir -p $O
run() {  # run <name> <seconds> <cmd...>   (stdout+stderr -> $O/<name>.log)
  local n=$1 t=$2; shift 2
  echo "[gpu_full] $(date +%T) $n"
  timeout -k 10 $t "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "[gpu_full] $(date +%T) $n rc=$rc"
  [ $rc -ne 0 ] && { tail -25 $O/$n.log; exit $rc; }
  return 0
}
if [ -z "$SKIP_TESTS" ]; then
  run tests_$TAG 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
  tail -2 $O/tests_$TAG.log
  run smoke_$TAG 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
export TMPDIR=/tmp
cd /tmp
BA="--steps 3 --warmup 1 --no-cpu-baseline --no-timing ${BENCH_ARGS}"
run pmc_fetch_$TAG 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch_$TAG -o run -- python3 $R/bench.py $BA
run pmc_write_$TAG 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write_$TAG -o run -- python3 $R/bench.py $BA
python3 $R/tools/pmc_traffic.py --fetch $O/pmc_fetch_$TAG --write $O/pmc_write_$TAG --region ${REGION:-enc_bwd_w_0} \
    --config ${CFG:-C2} --precision ${PREC:-f32x} > $O/pmc_traffic_$TAG.json || exit 1
cat $O/pmc_traffic_$TAG.json
run prof_$TAG 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_$TAG -o run -- \
    python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS}
cd $R
python3 tools/summarize_prof.py "$(find $O/prof_$TAG -name "*kernel_trace.csv" | sort | tail -n 1)" > $O/prof_${TAG}_summary.md || exit 1
run bench_$TAG 600 python bench.py --traffic-json $O/pmc_traffic_$TAG.json ${BENCH_ARGS}
grep '^{' $O/bench_$TAG.log
if [ -n "$EXTRA_BENCH" ]; then
  run bench_${TAG}_extra 300 python bench.py --no-cpu-baseline $EXTRA_BENCH
  grep '^{' $O/bench_${TAG}_extra.log
fi
echo "[gpu_full] done"
