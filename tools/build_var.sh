#!/bin/bash
# Variant builds of one source file: lib/libsift_hip_<name>.so with extra
# -D flags on that file, linked with the current objects of the others.
# usage: tools/build_var.sh <file.hip> <name> "<-Dflags>" [<name> "<-Dflags>" ...]
set -e
cd "$(dirname "$0")/../sift-gpu_amd"
make -s -j8 ARCH=gfx950 2>/dev/null
SRC=$1; shift
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -fno-gpu-rdc"
base=$(basename $SRC .hip)
OBJS=$(ls build/*.o | grep -v "/$base.o")
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  /opt/rocm/bin/hipcc $F $defs -c csrc/$SRC -o build/var_$name.o.tmp 2>/dev/null
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/libsift_hip_$name.so $OBJS build/var_$name.o.tmp \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  rm build/var_$name.o.tmp
  echo "built lib/libsift_hip_$name.so ($defs)"
done
