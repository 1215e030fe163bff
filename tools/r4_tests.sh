#!/bin/bash
# Round-4 GPU pass: the new parity tests verbose first, then the whole -m gpu suite.  Outputs under gpurun_out/.
set -o pipefail
TAG=${1:-r4}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ddp.py tests/test_gpu_conv3d.py -m gpu -v \
    --timeout 300 --timeout-method thread -k "native or c4 or ddp or gn_stats3d" > gpurun_out/${TAG}_new.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|Error|assert|passed|failed" gpurun_out/${TAG}_new.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
    --ignore=tests/test_gpu_ddp.py > gpurun_out/${TAG}_all.log 2>&1
rc2=$?; tail -15 gpurun_out/${TAG}_all.log; exit $(( rc > rc2 ? rc : rc2 ))
