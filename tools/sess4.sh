set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python tools/gemm_bench.py > $O/gemm_ab4.txt 2>&1 || exit $?
cat $O/gemm_ab4.txt
timeout -k 10 900 python -m pytest tests -q -m gpu --timeout 600 -p no:cacheprovider > $O/t4.log 2>&1; rc=$?; tail -8 $O/t4.log; [ $rc -gt 1 ] && exit $rc
for P in f32x; do
timeout -k 10 300 python bench.py --precision $P --no-cpu-baseline > $O/bench4_$P.json 2> $O/bench4_$P.err || { tail $O/bench4_$P.err; exit 3; }
cat $O/bench4_$P.json; grep "GEMM time" $O/bench4_$P.err
done
timeout -k 10 300 python bench.py --config C3 --no-cpu-baseline > $O/bench4_c3.json 2> $O/bench4_c3.err || { tail $O/bench4_c3.err; exit 3; }
cat $O/bench4_c3.json; cat $O/bench4_c3.err | head -20
