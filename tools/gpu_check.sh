#!/bin/bash
# One GPU-box pass: parity tests, bench, rocprofv3 kernel stats. Outputs under gpurun_out/.
# usage: tools/gpu_check.sh TAG [tests|bench|prof ...]
set -o pipefail
TAG=${1:-run}; shift
STEPS="${@:-tests bench prof}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
             > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; } ;;
    bwd)   timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py -m gpu -v --timeout 120 --timeout-method thread \
             > gpurun_out/${TAG}_bwd.log 2>&1; echo "bwd rc=$?"; grep -E "PASS|FAIL|Error|assert" gpurun_out/${TAG}_bwd.log | tail -60 ;;
    bench) timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench.log; exit 1; } ;;
    prof)  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-calls 0 \
             > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/${TAG}_prof.log; exit 1; } ;;
    train) timeout -k 10 300 python -u bench.py --mode train --steps 5 --warmup 2 --global-batch 2 > gpurun_out/${TAG}_train.log 2>&1 || { echo "train bench failed"; tail -30 gpurun_out/${TAG}_train.log; exit 1; }; tail -1 gpurun_out/${TAG}_train.log ;;
    trainprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_tprof -o run -- python3 bench.py --mode train --steps 3 --warmup 1 --global-batch 2 \
             > gpurun_out/${TAG}_tprof.log 2>&1 || { echo "train prof failed"; tail -30 gpurun_out/${TAG}_tprof.log; exit 1; } ;;
    convx3) for A in "--cin 388 --cout 192 --k 3 --hw 260 --gn 1" "--cin 192 --cout 192 --k 3 --hw 258 --gn 0" \
                     "--cin 196 --cout 192 --k 3 --hw 127 --gn 1" "--cin 388 --cout 192 --k 1 --hw 260 --gn 0" \
                     "--cin 196 --cout 192 --k 1 --hw 256 --gn 0" "--cin 81 --cout 192 --k 1 --hw 256 --gn 0" \
                     "--cin 192 --cout 75 --k 1 --hw 256 --gn 0" "--cin 768 --cout 192 --k 2 --hw 129 --gn 0" \
                     "--cin 192 --cout 192 --k 1 --hw 132 --gn 1"; do
              timeout -k 10 120 python -u tools/conv_bench.py --prec x3f16 --b 16 $A --check || exit 1
            done > gpurun_out/${TAG}_convx3.log 2>&1; cat gpurun_out/${TAG}_convx3.log | grep -v amdgpu.ids ;;
  esac
  echo "step $s ok"
done
tail -3 gpurun_out/${TAG}_tests.log 2>/dev/null; tail -1 gpurun_out/${TAG}_bench.log 2>/dev/null; true
