#!/bin/bash
# Diagnostic / A-B builds from patch files (tools/patches/*.patch): copies the
# library sources to a scratch tree, applies the patch there, builds every
# source file of the scratch tree (a patched header reaches every object) and
# links lib/libsift_hip_<name>.so.  The product sources stay untouched.
# usage: tools/build_patch.sh <name> <patch> ["-Dflags"]
set -e
cd "$(dirname "$0")/../sift-gpu_amd"
make -s -j8 ARCH=gfx950 2>/dev/null
NAME=$1; PATCH=$(realpath "../$2"); DEFS=${3:-}
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -fno-gpu-rdc"
W=build/patch_$NAME
rm -rf $W && mkdir -p $W/sift-gpu_amd/build
cp -r csrc $W/sift-gpu_amd/
cp -r ../include $W/
cp build/sym_coefs.inc $W/sift-gpu_amd/build/
(cd $W && patch -s -p1 < "$PATCH")
OBJS=""
pids=""
for f in $W/sift-gpu_amd/csrc/*.hip; do
  o=$W/$(basename $f .hip).o
  /opt/rocm/bin/hipcc $F $DEFS -Wno-inline-asm -c $f -o $o &
  pids="$pids $!"
  OBJS="$OBJS $o"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/libsift_hip_$NAME.so $OBJS -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built lib/libsift_hip_$NAME.so from $2"
