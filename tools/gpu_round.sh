#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel-trace profile.
# Stops at the first GPU fault / abort / timeout (exit >= 2 from a step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
TAG=${TAG:-r2}
mkdir -p $OUT
step() {  # step <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "[gpu_round] $(date +%T) start $name"
  timeout -k 10 $t "$@"
  local rc=$?
  echo "[gpu_round] $(date +%T) $name rc=$rc"
  return $rc
}
if [ -z "$SKIP_TESTS" ]; then
  step tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/tests_$TAG.log 2>&1
  rc=$?; tail -3 $OUT/tests_$TAG.log
  [ $rc -gt 1 ] && exit $rc
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || exit $?
fi
step bench 900 python bench.py ${BENCH_ARGS} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 3; }
cat $OUT/bench_$TAG.json
if [ -z "$SKIP_PROF" ]; then
  export TMPDIR=/tmp
  cd /tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $OUT/prof_$TAG -o run -- \
      python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > $OUT/prof_$TAG.log 2>&1 || exit $?
fi
echo "[gpu_round] done"
