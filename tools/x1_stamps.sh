#!/bin/bash
# GPU-box pass of tools/x1_stamps.py over the rollout's 1x1 shapes (dev; needs tools/build_stamp.sh first, its library copied to nps_hip/libnps_x1stamp.so: the x3 name is gpurun-ignored)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for A in "--cin 196 --cout 192" "--cin 81 --cout 192" "--cin 388 --cout 192"; do
  echo "== $A"
  NPS_HIP_LIB=$PWD/neural-pde-surrogates_amd/nps_hip/libnps_x1stamp.so timeout -k 10 120 python -u tools/x1_stamps.py $A 2>&1 | grep -v amdgpu.ids || exit 1
done
