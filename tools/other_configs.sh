#!/bin/bash
# Secondary bench lines (BASELINE configs other than the headline): C4 DRN 256x256, C2 U-FNO 128x128
# (12 modes), training step; plus a rocprofv3 kernel summary of the DRN rollout.  Outputs: gpurun_out/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-oc}
timeout -k 10 300 python -u bench.py --model drn --num-c 1 --steps 5 --warmup 2 --cpu-calls 1 > gpurun_out/${TAG}_drn.log 2>&1 || { echo "drn bench failed"; tail -20 gpurun_out/${TAG}_drn.log; exit 1; }
tail -1 gpurun_out/${TAG}_drn.log
timeout -k 10 300 python -u bench.py --model ufno --res 128 --num-c 1 --fno-modes 12 --steps 10 --warmup 2 --cpu-calls 2 > gpurun_out/${TAG}_c2.log 2>&1 || { echo "c2 bench failed"; tail -20 gpurun_out/${TAG}_c2.log; exit 1; }
tail -1 gpurun_out/${TAG}_c2.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_drnprof -o run -- python3 bench.py --model drn --num-c 1 --steps 2 --warmup 1 --cpu-calls 0 > gpurun_out/${TAG}_drnprof.log 2>&1 || { echo "drn prof failed"; tail -20 gpurun_out/${TAG}_drnprof.log; exit 1; }
echo "drn prof ok"
