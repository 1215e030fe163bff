#!/bin/bash
# Dev tool: 1x1 conv A/B, ring-free kernel (default) vs the patch-ring kernel (NPS_X3_1X1=ring).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-x1}
SHAPES=("--cin 388 --cout 192 --hw 260" "--cin 196 --cout 192 --hw 256" "--cin 84 --cout 192 --hw 256"
        "--cin 192 --cout 192 --hw 132" "--cin 192 --cout 192 --hw 256" "--cin 192 --cout 388 --hw 64"
        "--cin 20 --cout 75 --hw 64" "--cin 48 --cout 512 --hw 40")
for M in ${MODES:-direct ring}; do
  for A in "${SHAPES[@]}"; do
    echo "mode=$M $A"
    NPS_X3_WL_D=${M%%:*} NPS_X3_1X1_CFG=${M#*:} timeout -k 10 120 python -u tools/conv_bench.py --prec x3f16 --b 16 --k 1 --gn 0 $A --check || exit 1
  done
done > gpurun_out/${TAG}_1x1.log 2>&1 || { grep -v amdgpu.ids gpurun_out/${TAG}_1x1.log | tail -30; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_1x1.log | grep -v "sample [18]"
