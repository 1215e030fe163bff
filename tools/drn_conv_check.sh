#!/bin/bash
# Dev tool: the dilated-ResNet 5x5 conv shapes on the split-fp16 kernel (lattice tiling), checked against
# torch CPU conv2d, then the DRN parity tests.  Outputs: gpurun_out/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-drnc}
for A in "--cin 132 --cout 128 --dil 1 --circ 2" "--cin 128 --cout 128 --dil 2 --circ 4" \
         "--cin 128 --cout 128 --dil 4 --circ 8" "--cin 128 --cout 128 --dil 8 --circ 16"; do
  timeout -k 10 120 python -u tools/conv_bench.py --prec x3f16 --b 16 --k 5 --hw 256 --gn 0 $A --check || exit 1
done > gpurun_out/${TAG}_conv.log 2>&1 || { grep -v amdgpu.ids gpurun_out/${TAG}_conv.log | tail -20; exit 1; }
grep -v amdgpu.ids gpurun_out/${TAG}_conv.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "drn" > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
