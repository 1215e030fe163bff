#!/bin/bash
# One GPU-box pass: rocprofv3 kernel stats of the B=2 rollout (the per-GPU batch at 8 GPUs) and a
# 2-rank rehearsal of bench.py's N > 1 path on the one GPU (NPS_BENCH_REHEARSAL=1: gloo, both ranks on cuda:0).
set -o pipefail
TAG=${1:-b2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
  python3 bench.py --global-batch 2 --steps 4 --warmup 1 --cpu-calls 0 > gpurun_out/${TAG}_prof.log 2>&1 \
  || { echo "b2 prof failed"; tail -30 gpurun_out/${TAG}_prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_prof.log
NPS_BENCH_REHEARSAL=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
  > gpurun_out/${TAG}_rehearsal.log 2>&1 || { echo "rehearsal failed"; tail -40 gpurun_out/${TAG}_rehearsal.log; exit 1; }
tail -1 gpurun_out/${TAG}_rehearsal.log
