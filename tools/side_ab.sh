#!/bin/bash
# Same-box A/B of the side-stream forks (ops.Fork): model parity tests with forks on, then the C3 rollout at
# B = 2 and B = 16 with the forks off / shipped (shortcut fork gated on conv1's last-round idle CUs) / every shortcut forked /
# FNO-layer fork at every size, two rounds each, plus a kernel trace
# of the B = 2 rollout with forks on.  usage: tools/side_ab.sh TAG     outputs: gpurun_out/TAG_*
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-side}
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
VARIANTS=("NPS_SIDE_STREAM=0" "NPS_SIDE_STREAM=1" "NPS_SIDE_MIN_IDLE=0" "NPS_SIDE_FNO_MAX_ELEMS=1e12")
for r in 1 2; do
  for gb in 2 16; do
    for V in "${VARIANTS[@]}"; do
      N=$(echo $V | tr ' =' '__')
      env $V timeout -k 10 200 python3 bench.py --global-batch $gb --steps 10 --warmup 2 --cpu-calls 0 \
          > gpurun_out/${TAG}_b${gb}_$N.json 2> gpurun_out/${TAG}_b${gb}_$N.err || { echo "bench $V failed"; tail -5 gpurun_out/${TAG}_b${gb}_$N.err; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_b${gb}_$N.json').read().strip().splitlines()[-1]); print('B=$gb', '$V', 'value', d['value'], 'ms', d['ms_per_step'])"
    done
  done
done | tee gpurun_out/${TAG}_bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_b2prof -o run -- python3 bench.py --global-batch 2 --steps 10 --warmup 2 --cpu-calls 0 \
    > gpurun_out/${TAG}_b2prof.log 2>&1 || { echo "b2 prof failed"; tail -20 gpurun_out/${TAG}_b2prof.log; exit 1; }
echo "b2 prof ok"
