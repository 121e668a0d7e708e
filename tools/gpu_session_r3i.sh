#!/bin/bash
# Round-3 session i: the hidden-layer GEMMs in the harness with planes-only outputs (as in the
# step) vs in the step itself: stamps, per-region PMC of the C3 step, C3 kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
G="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU,GRBM_GUI_ACTIVE"
bash tools/gpu_steps.sh \
  "r3i_stamps|200|MVAE_BENCH_PLANES_ONLY=1 MVAE_STAMPS=1 python tools/gemm_bench.py --config C3 --shapes enc_fwd_h --variants 28,27 --epilogues --diag 0,8 --rounds 1" \
  "r3i_pmc|400|python tools/pmc_regions.py --config C3 --regions enc_fwd_1,enc_bwd_d_1,enc_bwd_w_1,enc_fwd_0,enc_bwd_w_0,dec_fwd_out_bce --groups $G FETCH_SIZE WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum --out $R/gpurun_out/r3i_pmc > gpurun_out/r3i_pmc.json" \
  "r3i_trace|300|cd /tmp && TMPDIR=/tmp rocprofv3 --kernel-trace --stats -T --output-format csv -d $R/gpurun_out/r3i_trace -o run -- python3 $R/bench.py --config C3 --steps 10 --warmup 3 --no-cpu-baseline --pmc off --no-configs --no-h2d"
python3 tools/summarize_prof.py "$(find gpurun_out/r3i_trace -name '*kernel_trace.csv' | sort | tail -n 1)" > gpurun_out/r3i_trace_summary.md
