#!/bin/bash
# Build the library from a git revision (default HEAD) into snapgpu/libsnapgpu_base.so
# (scratch worktree under /tmp; the working tree is untouched).
REV=${1:-HEAD}
W=/tmp/snapgpu_base_wt
rm -rf $W && git -C /root/repo worktree prune && git -C /root/repo worktree add -f -q $W $REV || exit 1
make -s -j8 -C $W/snap-rnaseq_amd ARCH=gfx950 > /dev/null || exit 1
cp $W/snap-rnaseq_amd/snapgpu/libsnapgpu.so /root/repo/snap-rnaseq_amd/snapgpu/libsnapgpu_base.so
git -C /root/repo worktree remove --force $W
echo "base = $(git -C /root/repo rev-parse --short $REV)"
