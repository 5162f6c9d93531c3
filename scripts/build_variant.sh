#!/usr/bin/env bash
# Build a variant of the product library for same-process A/B comparisons
# (scripts/abx.py), with no experiment switch in the product sources:
#   scripts/build_variant.sh NAME REV            the package as of git REV
#   scripts/build_variant.sh NAME DIR            the working tree's package with DIR's files overlaid
#                                                (DIR mirrors gpu-accel-ofdm-ls-mrc_amd/, e.g. DIR/csrc/pk.hpp)
# -> gpu-accel-ofdm-ls-mrc_amd/lib/libofdm_lsmrc_NAME.so (loaded by abx.py next to the product one).
set -e
NAME=$1; SRC=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=gpu-accel-ofdm-ls-mrc_amd
W=$ROOT/$PKG/build/variants/$NAME
rm -rf $W && mkdir -p $W/pkg $W/include
if [ -d "$SRC" ]; then
  cp -r $ROOT/$PKG/csrc $ROOT/$PKG/Makefile $W/pkg/ && cp $ROOT/include/*.h $W/include/
  (cd $SRC && find . -type f | while read f; do mkdir -p $W/pkg/$(dirname $f); cp $f $W/pkg/$f; done)
else
  (cd $ROOT && git archive $SRC $PKG/csrc $PKG/Makefile include | tar -x -C $W)
  mv $W/$PKG/* $W/pkg/ && rmdir $W/$PKG
fi
make -C $W/pkg -j${MAKE_JOBS:-8} LIB=lib/libofdm_lsmrc.so > $W/build.log 2>&1 || { tail -20 $W/build.log; exit 1; }
mkdir -p $ROOT/$PKG/lib && cp $W/pkg/lib/libofdm_lsmrc.so $ROOT/$PKG/lib/libofdm_lsmrc_$NAME.so
rm -rf $W   # the .so is all abx.py needs; keep no source copies in the tree
echo "built $PKG/lib/libofdm_lsmrc_$NAME.so"
