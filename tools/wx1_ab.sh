#!/bin/bash
# Same-box A/B of the 1x1 weight gradient: 192 x 192 work-groups (default) vs the 64 x 64 tiles (NPS_WX_WIDE1=0)
# on the B=16 training step (probe classes).  usage: tools/wx1_ab.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-wx1ab}
for r in 1 2; do
  for v in 0 1; do
    NPS_WX_WIDE1=$v timeout -k 10 300 python3 bench.py --mode train --steps 3 --warmup 1 --global-batch 16 --cpu-calls 0 \
      > gpurun_out/${TAG}_w$v.json 2> gpurun_out/${TAG}_w$v.err || { echo "train wide1=$v failed"; tail -5 gpurun_out/${TAG}_w$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_w$v.json').read().strip().splitlines()[-1]); c=d['roofline']['conv_classes']; print('wide1=$v', d['value'], d['ms_per_step'], {k:(v['ms'],v['tflops']) for k,v in c.items() if k.startswith('x3w')})"
  done
done | tee gpurun_out/${TAG}.txt
