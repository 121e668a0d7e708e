#!/bin/bash
# Build an A/B variant of libmvae.so: gemm_bf16.hip recompiled with extra -D flags, linked with
# the other objects of the in-tree build (magic_amd/_build). Use it with MVAE_LIB=<out>.
#   tools/build_alt.sh magic_amd/libmvae_alt.so -DMVAE_QGAP=1
set -e
cd "$(dirname "$0")/.."
OUT=$1; shift
BID=$(cat magic_amd/_build/build_id.txt)
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value \
  -I include "$@" -c magic_amd/csrc/gemm_bf16.hip -o /tmp/gemm_bf16_alt.o
objs=$(ls magic_amd/_build/*.o | grep -v gemm_bf16.hip.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT" $objs /tmp/gemm_bf16_alt.o
echo "$OUT (build id $BID)"
