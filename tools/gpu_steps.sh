#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first step that faults,
# aborts, times out or is killed (exit status >= 2; pytest's 1 = test failures continues).
#   tools/gpu_steps.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; t=${rest%%|*}; cmd=${rest#*|}
  echo "[gpu_steps] $(date +%T) start $name (limit ${t}s)"
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_steps] $(date +%T) $name rc=$rc"
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ge 2 ]; then echo "[gpu_steps] stopping after $name (rc=$rc)"; exit $rc; fi
  # a GPU fault reported as an ordinary Python error (rc 1) also ends the call
  if grep -qE "illegal memory access|Memory access fault|HSA_STATUS_ERROR|hipErrorLaunchFailure|page fault" "gpurun_out/$name.log"; then
    echo "[gpu_steps] GPU fault in $name: stopping"; exit 3
  fi
done
echo "[gpu_steps] done"
