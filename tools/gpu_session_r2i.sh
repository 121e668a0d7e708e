#!/bin/bash
# Round-2 closing session (after the pooling-kernel batching): full GPU tests, smoke, default bench (C2) with PMC traffic + CPU
# baseline, rocprof stats of C2, bench lines C3 / C5 / C5CONV.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
bash tools/gpu_steps.sh \
  "tests_r2i|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke_r2i|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_c2_r2i|600|python bench.py > gpurun_out/bench_c2_r2i.json 2> gpurun_out/bench_c2_r2i.err" \
  "prof_c2_r2i|300|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/prof_c2_r2i -o run -- python3 $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline --pmc off" \
  "bench_c3_r2i|300|python bench.py --config C3 --no-cpu-baseline > gpurun_out/bench_c3_r2i.json 2> gpurun_out/bench_c3_r2i.err" \
  "bench_c5_r2i|300|python bench.py --config C5 --no-cpu-baseline > gpurun_out/bench_c5_r2i.json 2> gpurun_out/bench_c5_r2i.err" \
  "bench_c5conv_r2i|300|python bench.py --config C5CONV --no-cpu-baseline > gpurun_out/bench_c5conv_r2i.json 2> gpurun_out/bench_c5conv_r2i.err"
