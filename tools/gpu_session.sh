#!/bin/bash
# The current GPU session (overwritten per session; earlier sessions are in git history):
#   tools/gpu_go.sh tools/gpu_session.sh [timeout-seconds]
# r5e: why the library's eight-phase k-loop runs ~3300 cycles per k-tile where the template runs
# ~2430 on the same NT 4096^3 shape: tile-group order (template --gm 4 / 8; library
# MVAE_TILE_GROUP 0 / 4 / 8), stamped library k-loop without DMA (diag 1) / without fragment reads
# (diag 64) / without both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
S="MVAE_STAMPS=2 python tools/gemm_bench.py --variants 29 --rounds 1 --config C3 --shapes square4096"
bash tools/gpu_steps.sh \
  "r5e_t4|120|tools/micro/gemm8p 4096 4096 4096 --rounds 3 --gm 4 --lib magic_amd/libmvae.so" \
  "r5e_t8|120|tools/micro/gemm8p 4096 4096 4096 --rounds 3 --gm 8 --lib magic_amd/libmvae.so" \
  "r5e_l4|120|MVAE_TILE_GROUP=4 tools/micro/gemm8p 4096 4096 4096 --rounds 3 --gm 4 --lib magic_amd/libmvae.so" \
  "r5e_l0|120|MVAE_TILE_GROUP=0 tools/micro/gemm8p 4096 4096 4096 --rounds 3 --gm 4 --lib magic_amd/libmvae.so" \
  "r5e_sd|200|$S --diag 0,1,64,65,128" \
  "r5e_sd4|200|MVAE_TILE_GROUP=4 $S --diag 0,1" 
