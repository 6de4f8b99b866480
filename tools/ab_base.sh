#!/bin/bash
# Build the committed HEAD (or a given rev) of libcbg into build/variants/base for same-box A/B sweeps:
#   tools/ab_base.sh [rev]  then  VARIANTS="tree base" tools/gpu_libab.sh (on the GPU box)
set -e
rev=${1:-HEAD}
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" worktree add -q --detach "$tmp" "$rev"
make -C "$tmp/combblas-spmm-test_amd" -s -j8 libcbg.so
mkdir -p "$root/build/variants/base"
cp "$tmp/combblas-spmm-test_amd/libcbg.so" "$root/build/variants/base/libcbg.so"
git -C "$root" worktree remove --force "$tmp"
echo "$root/build/variants/base/libcbg.so ($rev)"
