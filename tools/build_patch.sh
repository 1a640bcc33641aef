#!/bin/bash
# Diagnostic builds from patch files (tools/patches/*.patch): applies the patch
# to a scratch copy of the sources it touches, builds those files, and links
# lib/libsift_hip_<name>.so with the current objects of the other files.  The
# product sources stay untouched.
# usage: tools/build_patch.sh <name> <patch> ["-Dflags"]
set -e
cd "$(dirname "$0")/../sift-gpu_amd"
make -s -j8 ARCH=gfx950 2>/dev/null
NAME=$1; PATCH=$(realpath "../$2"); DEFS=${3:-}
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -fno-gpu-rdc"
W=build/patch_$NAME
rm -rf $W && mkdir -p $W
(cd .. && git apply --include='sift-gpu_amd/csrc/*' --directory=. --check "$PATCH")
FILES=$(grep '^+++ ' "$PATCH" | sed 's#^+++ b/sift-gpu_amd/##; s#\t.*##')
for f in $FILES; do mkdir -p $W/$(dirname $f); cp $f $W/$f; done
(cd $W && patch -s -p2 < "$PATCH")
OBJS=""
for o in build/*.o; do
  keep=1
  for f in $FILES; do [ "$o" = "build/$(basename $f .hip).o" ] && keep=0; done
  [ $keep = 1 ] && OBJS="$OBJS $o"
done
for f in $FILES; do
  /opt/rocm/bin/hipcc $F $DEFS -Icsrc -Wno-inline-asm -c $W/$f -o $W/$(basename $f .hip).o
  OBJS="$OBJS $W/$(basename $f .hip).o"
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/libsift_hip_$NAME.so $OBJS
echo "built lib/libsift_hip_$NAME.so from $2"
