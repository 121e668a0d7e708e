#!/bin/bash
# Round-4 session n: in-step A/B of the GEMM kernels -- eight-phase kernel with plane-image reuse
# (current), the previous eight-phase kernel (libmvae_e8old.so), ring kernels only (MVAE_E8=0) --
# on C3 and C2, plus stamps of both eight-phase builds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
BQ="--no-cpu-baseline --pmc off --no-configs --no-h2d --no-pipeline"
OLD=MVAE_LIB=magic_amd/libmvae_e8old.so
S="MVAE_STAMPS=2 python tools/gemm_bench.py --rounds 1 --iters 3"
run() { echo "$1|90|$2 python bench.py --config $3 $BQ > gpurun_out/$1.json 2> gpurun_out/$1.err"; }
bash tools/gpu_steps.sh \
  "$(run r4n_c3_cur '' C3)" "$(run r4n_c3_ring MVAE_E8=0 C3)" "$(run r4n_c3_old $OLD C3)" "$(run r4n_c3_cur2 '' C3)" \
  "$(run r4n_c2_cur '' C2)" "$(run r4n_c2_ring MVAE_E8=0 C2)" "$(run r4n_c2_old $OLD C2)" \
  "r4n_st_cur|90|$S --config C3 --variants 22 --shapes enc_fwd_0,square4096 && $S --config C2 --variants 38 --shapes enc_fwd_0" \
  "r4n_st_old|90|$OLD $S --config C3 --variants 22 --shapes enc_fwd_0,square4096 && $OLD $S --config C2 --variants 38 --shapes enc_fwd_0"
