#!/bin/bash
# wide-kernel correctness, then GEMM A/B (fp32 / bf16 128 / bf16 wide / f32x 128 / f32x wide)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -k "gemm" -x -q -p no:cacheprovider > gpurun_out/t5.log 2>&1
rc=$?; tail -15 gpurun_out/t5.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/gemm_bench.py --variants 0,20,19,36,35 --rounds 2 > gpurun_out/gemm_ab5.txt 2>&1
rc=$?; cat gpurun_out/gemm_ab5.txt; exit $rc
