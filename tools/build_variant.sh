#!/bin/bash
# Dev build: libnps_<name>.so = libnps_hip.so with conv2d_x3.hip compiled under extra -D flags
# usage: tools/build_variant.sh <name> -DFOO=1 ...   (run on the CPU host after `make`)
set -e
NAME=$1; shift
cd "$(dirname "$0")/../neural-pde-surrogates_amd/csrc"
mkdir -p build_var
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics "$@" -c conv2d_x3.hip -o build_var/conv2d_x3_$NAME.o
OBJS="build/conv2d.o build/conv1x1_res.o build/wgrad_x3.o build/spectral.o build/spectral3d.o build/data.o build/pointwise.o build/backward.o build/bf16.o build/conv3d.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS build_var/conv2d_x3_$NAME.o -o ../nps_hip/libnps_$NAME.so
