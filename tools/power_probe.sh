#!/bin/bash
# Data-dependence of the 3x3 split-fp16 conv's speed (a power-limited clock shows as faster runs on zero /
# constant operands): the shipped library on random, zero, constant inputs and zero weights, gn=0 shape.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for d in randn zero const wzero; do
    timeout -k 10 120 python3 tools/conv_bench.py --cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn 0 --data $d 2>&1 | grep conv | sed "s/^/$d /" || exit 1
  done
done | tee gpurun_out/power_probe.txt
