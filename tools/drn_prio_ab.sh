set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=neural-pde-surrogates_amd/nps_hip
for round in 1 2; do
  for v in base v1; do
    lib=$L/libnps_hip.so; [ $v != base ] && lib=$L/libnps_hip_$v.so
    NPS_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --model drn --num-c 1 --steps 5 --warmup 2 --cpu-calls 0 > gpurun_out/drnab_${v}_$round.log 2>&1 || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/drnab_${v}_$round.log').read().strip().splitlines()[-1]); print('$v', $round, d['value'], d['roofline']['conv_classes'])"
  done
done
