#!/bin/bash
# Training step with the weight-gradient fork off / on (NPS_SIDE_WGRAD): backward / trainer / DDP parity tests
# with the fork on, then bench.py --mode train at global batch 2 and 16, two rounds.  usage: tools/side_wgrad_ab.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-sidew}
NPS_SIDE_WGRAD=1 timeout -k 10 500 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_trainer.py tests/test_gpu_ddp.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for r in 1 2; do
  for gb in 2 16; do
    for v in 0 1; do
      NPS_SIDE_WGRAD=$v timeout -k 10 400 python3 bench.py --mode train --steps 5 --warmup 2 --global-batch $gb --cpu-calls 0 \
          > gpurun_out/${TAG}_b${gb}_$v.json 2> gpurun_out/${TAG}_b${gb}_$v.err || { echo "train bench failed"; tail -5 gpurun_out/${TAG}_b${gb}_$v.err; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_b${gb}_$v.json').read().strip().splitlines()[-1]); print('train B=$gb NPS_SIDE_WGRAD=$v', 'value', d['value'], 'ms', d['ms_per_step'])"
    done
  done
done | tee gpurun_out/${TAG}_bench.txt
