#!/bin/bash
# Round-2 closing session: full GPU tests, smoke, default bench (C2), C5CONV bench + rocprof stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_steps.sh \
  "tests_r2d|900|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
  "smoke_r2d|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench_c2_r2d|600|python bench.py > gpurun_out/bench_c2_r2d.json 2> gpurun_out/bench_c2_r2d.err" \
  "prof_c5conv_r2d|300|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats -T --output-format csv -d $PWD/gpurun_out/prof_c5conv_r2d -o run -- python3 $PWD/bench.py --config C5CONV --steps 5 --warmup 2 --no-cpu-baseline --pmc off --region-steps 2"
