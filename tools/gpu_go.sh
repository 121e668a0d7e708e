#!/bin/bash
# Build libmvae.so here (the box only runs prebuilt code), then run one session script on the
# GPU box: tools/gpu_go.sh tools/gpu_session_r4X.sh [timeout-seconds]
set -e
cd "$(dirname "$0")/.."
python3 -c "import magic_amd.build as b; b.build()"
python3 -c "from magic_amd import _lib, build; import ctypes; l=ctypes.CDLL('magic_amd/libmvae.so'); l.mvae_build_id.restype=ctypes.c_char_p; assert l.mvae_build_id().decode()==build.source_hash(), 'stale'"
exec /usr/local/graft/bin/gpurun --timeout "${2:-1100}" -- "bash $1"
