#!/bin/bash
# Same-box A/B (dev): wide tiles 16x8 (default, NPS_X3_WIDE_TILE=0) vs 32x4 (=3), with a parity check of
# the 32x4 tile on the U-Net 3x3 shapes first (tools/conv_bench.py --check vs torch on the CPU).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for A in "--cin 388 --cout 192 --k 3 --hw 256 --gn 1" "--cin 192 --cout 192 --k 3 --hw 258 --gn 0" "--cin 768 --cout 192 --k 2 --hw 129 --gn 0"; do
  NPS_X3_WIDE_TILE=3 timeout -k 10 120 python -u tools/conv_bench.py --prec x3f16 --b 4 $A --check || exit 1
done > gpurun_out/tile32x4_check.log 2>&1 || { echo "check failed"; tail -20 gpurun_out/tile32x4_check.log; exit 1; }
grep -v amdgpu.ids gpurun_out/tile32x4_check.log
for round in 1 2; do
  for t in 0 3; do
    NPS_X3_WIDE_TILE=$t timeout -k 10 200 python -u bench.py --cpu-calls 0 > gpurun_out/tileb${t}_$round.log 2>&1 \
      || { echo "tile $t failed"; tail -20 gpurun_out/tileb${t}_$round.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/tileb${t}_$round.log').read().strip().splitlines()[-1]); print('tile $t', $round, d['value'], d['roofline']['avg_launch_ms'], d['roofline']['conv_classes'])"
  done
done
