#!/bin/bash
# Dev: in-kernel stamp timing of the split-fp16 3x3 conv (wide tiles), without / with the fused prologue
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export NPS_HIP_LIB=$PWD/neural-pde-surrogates_amd/nps_hip/libnps_x3stamp.so
for G in 0 1; do
  echo "== gn=$G"
  timeout -k 10 120 python3 tools/x3_stamps.py --cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn $G || exit 1
done
