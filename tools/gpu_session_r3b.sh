#!/bin/bash
# Round-3 session b: where the hidden-layer / BCE GEMM time goes. Diagnostic ablations
# (PParams::diag: 1 no copies after the prologue, 2 no global stores, 4 no LDS transpose,
# 8 no transcendental math) and PMC passes on the ring (v31) and twin (v29) kernels, C3 shapes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
SH=enc_fwd_h,enc_bwd_d_h,dec_fwd_out,square4096
GB="python3 $R/tools/gemm_bench.py --config C3 --shapes $SH --variants 31,29 --epilogues"
steps=("r3b_diag|300|python tools/gemm_bench.py --config C3 --shapes $SH --variants 31,29 --epilogues --diag 0,1,2,8,14,15 --rounds 3")
i=0
for g in "FETCH_SIZE" "WRITE_SIZE,TCC_HIT_sum,TCC_MISS_sum" \
         "SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_VALU_MFMA_BUSY_CYCLES,SQ_INSTS_VALU,SQ_INSTS_LDS,GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  steps+=("r3b_pmc$i|120|cd /tmp && TMPDIR=/tmp rocprofv3 --pmc ${g//,/ } --kernel-trace --output-format csv -d $R/gpurun_out/r3b_pmc$i -o run -- $GB --rounds 1 --iters 5")
done
bash tools/gpu_steps.sh "${steps[@]}" && \
python3 tools/pmc_kernels.py gpurun_out/r3b_pmc1 gpurun_out/r3b_pmc2 gpurun_out/r3b_pmc3 --match gemm_bf16 > gpurun_out/r3b_pmc_summary.txt
