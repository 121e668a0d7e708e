#!/bin/bash
# Round-3 session ak: skinny GEMMs (latent head, decoder layer 1 at small L) on the fp32 VALU
# kernel (default) vs the fp32 MFMA kernel (MVAE_NO_VALU=1), bench lines twice each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
B="python bench.py --no-cpu-baseline --pmc off"
bash tools/gpu_steps.sh \
  "r3ak_a|300|$B > gpurun_out/r3ak_a.json 2> gpurun_out/r3ak_a.err" \
  "r3ak_n|300|MVAE_NO_VALU=1 $B > gpurun_out/r3ak_n.json 2> gpurun_out/r3ak_n.err" \
  "r3ak_a2|300|$B > gpurun_out/r3ak_a2.json 2> gpurun_out/r3ak_a2.err" \
  "r3ak_n2|300|MVAE_NO_VALU=1 $B > gpurun_out/r3ak_n2.json 2> gpurun_out/r3ak_n2.err"
