#!/bin/bash
# Build libmvae.so from another git revision (A/B against the working tree) into OUT, stamped with
# the working tree's build id so magic_amd._lib accepts it under MVAE_LIB=OUT:
#   tools/build_rev.sh HEAD magic_amd/libmvae_head.so
# (the revision is checked out as a worktree in .wt_head, listed in .gitignore / .gpurunignore)
set -e
cd "$(dirname "$0")/.."
# (the revision resolved HERE: inside the worktree "HEAD" would name the worktree's own checkout)
REV=$(git rev-parse --verify "$1^{commit}"); OUT=$2
H=$(python3 -c "import magic_amd.build as b; print(b.source_hash())")
if [ -d .wt_head ]; then git -C .wt_head checkout -q --detach "$REV"; else git worktree add -f .wt_head "$REV" -q --detach; fi
(cd .wt_head && python3 -c "
import magic_amd.build as b
b.source_hash = lambda: '$H'
b.build()" > /dev/null)
cp .wt_head/magic_amd/libmvae.so "$OUT"
echo "$OUT ($REV, build id $H)"
