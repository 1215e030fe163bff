#!/bin/bash
# Dev tool: build ablation variants of the split-fp16 conv kernel next to libnps_hip.so
# (libnps_x3abl_{A,MFMA,PROD}.so; select one with NPS_HIP_LIB=...).  Run on the CPU box.
set -e
cd "$(dirname "$0")/../neural-pde-surrogates_amd/csrc"
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics"
for V in A MFMA PROD; do
  /opt/rocm/bin/hipcc $FLAGS -DNPS_X3_ABL_$V -c conv2d_x3.hip -o build/conv2d_x3_$V.o &
done
wait
for V in A MFMA PROD; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/conv2d.o build/conv2d_x3_$V.o build/spectral.o \
    build/pointwise.o build/backward.o -o ../nps_hip/libnps_x3abl_$V.so
done
