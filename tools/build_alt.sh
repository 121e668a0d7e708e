#!/bin/bash
# Build an A/B variant of libmvae.so: one kernel source recompiled -- with extra -D flags, or
# replaced by another file (e.g. the previous revision from git) -- and linked with the other
# objects of the in-tree build (magic_amd/_build). Use it with MVAE_LIB=<out>.
#   tools/build_alt.sh magic_amd/libmvae_alt.so gemm_bf16.hip -DMVAE_QGAP=1
#   git show HEAD~3:magic_amd/csrc/gemm_bf16e.hip > /tmp/old_e8.hip
#   tools/build_alt.sh magic_amd/libmvae_old.so gemm_bf16e.hip=/tmp/old_e8.hip
set -e
cd "$(dirname "$0")/.."
OUT=$1; SRC=$2; shift 2
NAME=${SRC%%=*}
FILE=magic_amd/csrc/$NAME
[ "$NAME" != "$SRC" ] && FILE=${SRC#*=}
BID=$(cat magic_amd/_build/build_id.txt)
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value \
  -I include -I magic_amd/csrc "$@" -c "$FILE" -o /tmp/alt_$NAME.o
objs=$(ls magic_amd/_build/*.o | grep -v "/$NAME.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT" $objs /tmp/alt_$NAME.o
echo "$OUT (build id $BID)"
