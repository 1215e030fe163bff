#!/bin/bash
# C5 (3-D U-FNO, bf16 storage) with the FNO-layer fork off / on (size gate lifted): the 3-D parity tests with forks on, then the
# C5 bench line twice per setting.  usage: tools/side_c5_ab.sh TAG     outputs: gpurun_out/TAG_*
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${1:-sidec5}
timeout -k 10 400 python -u -m pytest tests/test_gpu_ufno3d.py tests/test_gpu_c5.py -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
for r in 1 2; do
  for v in 0 1; do
    NPS_SIDE_FNO=$v NPS_SIDE_FNO_MAX_ELEMS=1e12 timeout -k 10 300 python3 bench.py --model ufno3d --dtype bf16 --cpu-calls 0 > gpurun_out/${TAG}_c5_$v.json 2> gpurun_out/${TAG}_c5_$v.err \
        || { echo "c5 bench failed"; tail -5 gpurun_out/${TAG}_c5_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_c5_$v.json').read().strip().splitlines()[-1]); print('C5 NPS_SIDE_FNO=$v', 'value', d['value'], 'ms', d['ms_per_step'])"
  done
done | tee gpurun_out/${TAG}_bench.txt
