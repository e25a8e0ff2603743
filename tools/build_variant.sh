#!/bin/bash
# Build a variant of the library from the working tree into snapgpu/libsnapgpu_<name>.so:
#   [SRC=<tree>] [DST=<tree>] [PATCH=<diff>] tools/build_variant.sh <name> "<extra hipcc flags>" ["<sed expression applied to csrc/*.hip csrc/*.h>"]
# (scratch copy of SRC's sources under /tmp, default this tree; the library lands in DST's
# snapgpu/, default /root/repo).  For tools/abn.sh.
N=$1; X=$2; S=$3
W=/tmp/snapgpu_var_$N
SRC=${SRC:-$(cd "$(dirname "$0")/.." && pwd)}
DST=${DST:-/root/repo}
rm -rf $W && mkdir -p $W && cp -r $SRC/snap-rnaseq_amd $SRC/include $W/ || exit 1
rm -rf $W/snap-rnaseq_amd/build
[ -n "$S" ] && sed -i -e "$S" $W/snap-rnaseq_amd/csrc/*.hip $W/snap-rnaseq_amd/csrc/*.h
# PATCH=<file>: a unified diff against the tree (git diff format) applied to the copy
[ -n "$PATCH" ] && { (cd $W && patch -s -p1 < $PATCH) || exit 1; }
[ -n "$MK" ] && sed -i -e "$MK" $W/snap-rnaseq_amd/Makefile
[ -n "$X" ] && sed -i -e "s|^HIPFLAGS := |HIPFLAGS := $X |" $W/snap-rnaseq_amd/Makefile
make -s -j8 -C $W/snap-rnaseq_amd ARCH=gfx950 > $W/build.log 2>&1 || { tail -5 $W/build.log; exit 1; }
cp $W/snap-rnaseq_amd/snapgpu/libsnapgpu.so $DST/snap-rnaseq_amd/snapgpu/libsnapgpu_$N.so
echo "built libsnapgpu_$N.so"
