#!/bin/bash
# Same-box A/B of the weight-gradient work-group order (NPS_WX_REMAP=0 vs the XCD-aware default) on the B=16
# training step: the probe's x3w_* classes and the step time.  usage: tools/wx_ab.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-wxab}
for r in 1 2; do
  for v in 0 1; do
    NPS_WX_REMAP=$v timeout -k 10 300 python3 bench.py --mode train --steps 3 --warmup 1 --global-batch 16 --cpu-calls 0 \
      > gpurun_out/${TAG}_remap$v.json 2> gpurun_out/${TAG}_remap$v.err || { echo "train remap=$v failed"; tail -5 gpurun_out/${TAG}_remap$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_remap$v.json').read().strip().splitlines()[-1]); c=d['roofline']['conv_classes']; print('remap=$v', d['value'], d['ms_per_step'], {k:(v['ms'],v['tflops']) for k,v in c.items() if k.startswith('x3w')})"
  done
done | tee gpurun_out/${TAG}.txt
