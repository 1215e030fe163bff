#!/bin/bash
# Same-box A/B of conv kernel builds (dev): the default build vs libnps_hip_<v>.so variants linked with a
# differently-defined conv2d_x3.o (VARIANTS, default "base v1 v2": round 2's NPS_X3_PRIO=1 / =2 builds),
# each the C3 rollout bench, alternated twice.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=neural-pde-surrogates_amd/nps_hip
for round in 1 2; do
  for v in ${VARIANTS:-base v1 v2}; do
    lib=$L/libnps_hip.so; [ $v != base ] && lib=$L/libnps_hip_$v.so
    NPS_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --cpu-calls 0 --steps 10 --warmup 2 > gpurun_out/ab_${v}_$round.log 2>&1 \
      || { echo "$v failed"; tail -20 gpurun_out/ab_${v}_$round.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${v}_$round.log').read().strip().splitlines()[-1]); print('$v', $round, d['value'], d['roofline']['avg_launch_ms'], d['roofline']['conv_classes'])"
  done
done
