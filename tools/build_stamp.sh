#!/bin/bash
# Dev build: libnps_x3stamp.so = libnps_hip.so with per-tile s_memtime stamps in conv2d_x3_kernel and
# per-work-group stamps in conv1x1_wl_kernel (NPS_X3_STAMP), read by tools/x3_stamps.py / tools/x1_stamps.py.  Run on the CPU host after `make`.
set -e
cd "$(dirname "$0")/../neural-pde-surrogates_amd/csrc"
mkdir -p build_stamp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -DNPS_X3_STAMP \
    -c conv2d_x3.hip -o build_stamp/conv2d_x3.o
OBJS="build/conv2d.o build/wgrad_x3.o build/spectral.o build/spectral3d.o build/data.o build/pointwise.o build/backward.o build/bf16.o build/conv3d.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS build_stamp/conv2d_x3.o -o ../nps_hip/libnps_x3stamp.so
