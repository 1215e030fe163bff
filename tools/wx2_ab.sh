#!/bin/bash
# Same-box A/B of the 2x2 weight gradient: 128 x 128 work-groups (default) vs the 64 x 64 tiles (NPS_WX_WIDE2=0)
# on the B=16 training step (probe classes).  usage: tools/wx1_ab.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-wx1ab}
for r in 1 2; do
  for v in 0 1; do
    NPS_WX_WIDE2=$v timeout -k 10 300 python3 bench.py --mode train --steps 3 --warmup 1 --global-batch 16 --cpu-calls 0 \
      > gpurun_out/${TAG}_v$v.json 2> gpurun_out/${TAG}_v$v.err || { echo "train wide2=$v failed"; tail -5 gpurun_out/${TAG}_v$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_v$v.json').read().strip().splitlines()[-1]); c=d['roofline']['conv_classes']; print('wide2=$v', d['value'], d['ms_per_step'], {k:(v['ms'],v['tflops']) for k,v in c.items() if k.startswith('x3w')})"
  done
done | tee gpurun_out/${TAG}.txt
