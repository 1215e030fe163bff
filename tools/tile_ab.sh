#!/bin/bash
# Same-box A/B of the wide 3x3/2x2 tile shape (dev): NPS_X3_WIDE_TILE=1 (8x16, round 2 default)
# vs 0 (16x8, the default since): C3 rollout bench twice each, then one FETCH_SIZE pass each (conv class traffic per launch).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for round in 1 2; do
  for t in 1 0; do
    NPS_X3_WIDE_TILE=$t timeout -k 10 200 python -u bench.py --cpu-calls 0 > gpurun_out/tile${t}_$round.log 2>&1 \
      || { echo "tile $t failed"; tail -20 gpurun_out/tile${t}_$round.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/tile${t}_$round.log').read().strip().splitlines()[-1]); print('tile $t', $round, d['value'], d['roofline']['avg_launch_ms'], d['roofline']['conv_classes']['x3f16_9tap'])"
  done
done
CMD="python3 bench.py --steps 1 --warmup 1 --cpu-calls 0"
for t in 0 2; do
  NPS_X3_WIDE_TILE=$t timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_tile$t -o run -- $CMD > gpurun_out/pmc_tile$t.log 2>&1 || { echo "pmc tile $t failed"; tail -20 gpurun_out/pmc_tile$t.log; exit 1; }
  echo "pmc tile $t ok"
done
