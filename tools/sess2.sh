set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -k "gemm or f32x or bf16" --timeout 300 -p no:cacheprovider > $O/t2.log 2>&1; rc=$?; tail -3 $O/t2.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/gemm_bench.py > $O/gemm_ab2.txt 2>&1 || exit $?
cat $O/gemm_ab2.txt
timeout -k 10 300 python bench.py --precision f32x --no-cpu-baseline > $O/bench_f32x.json 2> $O/bench_f32x.err || { tail $O/bench_f32x.err; exit 3; }
cat $O/bench_f32x.json
timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 3; }
cat $O/bench_c3.json
