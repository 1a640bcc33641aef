#!/bin/bash
# Ablation builds of pyramid_pair.hip: lib/libsift_hip_abl<N>.so for each N
# (PP_ABL bits, see the file), linked with the current objects.
set -e
cd "$(dirname "$0")/../sift-gpu_amd"
make -s -j8 ARCH=gfx950
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -fno-gpu-rdc"
OBJS=$(ls build/*.o | grep -v pyramid_pair)
for n in "$@"; do
  /opt/rocm/bin/hipcc $F -DPP_ABL=$n -c csrc/pyramid_pair.hip -o build/abl_$n.o.tmp
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o lib/libsift_hip_abl$n.so $OBJS build/abl_$n.o.tmp
  rm build/abl_$n.o.tmp
done
