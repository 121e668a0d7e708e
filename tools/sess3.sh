set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -m pytest tests -q -m gpu --timeout 600 -p no:cacheprovider > $O/t3.log 2>&1; rc=$?; tail -5 $O/t3.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/gemm_bench.py > $O/gemm_ab3.txt 2>&1 || exit $?
cat $O/gemm_ab3.txt
for P in f32x f32; do
timeout -k 10 300 python bench.py --precision $P --no-cpu-baseline > $O/bench3_$P.json 2> $O/bench3_$P.err || { tail $O/bench3_$P.err; exit 3; }
cat $O/bench3_$P.json; grep "GEMM time" $O/bench3_$P.err
done
timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline > $O/bench3_c3.json 2> $O/bench3_c3.err || { tail $O/bench3_c3.err; exit 3; }
cat $O/bench3_c3.json; grep "GEMM time" $O/bench3_c3.err
