#!/bin/bash
# Round-3 session ac: LDS-side counters of the ring kernel on 4096^3 and the C3 layer-0 forward
# (bank conflicts, LDS instruction waits vs MFMA busy).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/r3ac_counters.txt 2>&1
GB="python3 $R/tools/gemm_bench.py --config C3 --shapes square4096,enc_fwd_0 --variants 28 --rounds 1 --iters 5"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d $R/gpurun_out/r3ac_pmc1 -o run -- $GB > $R/gpurun_out/r3ac_pmc1.log 2>&1
echo "pmc1 rc=$?"
