#!/bin/bash
# Same-box A/B of dev library variants (gpurun): conv shapes, the C3 bench, parity tests on the variant.
# usage: tools/r4_ab.sh TAG VARIANT [VARIANT2 ...]
#   VARIANT = LIB[:ENV=VAL[,ENV=VAL]]: libnps_<LIB>.so (built by tools/build_variant.sh; "hip" = the in-tree
#   library) run with those environment settings.  libnps_base.so (if present) = the reference build of an
#   earlier commit, run without the s2d view.  TESTS=0 skips the parity tests, CONV_ONLY=1 the bench too.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
D=$PWD/neural-pde-surrogates_amd/nps_hip
VARS="$@"
[ -f $D/libnps_base.so ] && VARS="base $VARS"
envof() {  # VARIANT -> "NPS_HIP_LIB=... [ENV=VAL ...]"
  local lib=${1%%:*} rest=""
  [[ "$1" == *:* ]] && rest=$(echo "${1#*:}" | tr ',' ' ')
  local s2d=0; [ "$lib" = hip ] && s2d=1
  echo "NPS_S2D_VIEW=$s2d NPS_HIP_LIB=$D/libnps_$lib.so $rest"
}
for V in $VARS; do [ -f $D/libnps_${V%%:*}.so ] || { echo "missing libnps_${V%%:*}.so"; exit 2; }; done
S1="--cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn 1"
S2="--cin 388 --cout 192 --k 3 --hw 260 --b 16 --gn 1"
S3="--cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn 0"
for r in 1 2; do
  for V in $VARS; do
    for S in "$S1" "$S2" "$S3"; do
      env $(envof $V) timeout -k 10 120 python3 tools/conv_bench.py $S 2>&1 | grep conv | sed "s/^/$V /" || exit 1
    done
  done
done | tee gpurun_out/${TAG}_conv.txt
[ "${CONV_ONLY:-0}" = 1 ] && exit 0
for r in 1 2; do
  for V in $VARS; do
    N=$(echo $V | tr ':=,' '___')
    env $(envof $V) timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --cpu-calls 0 > gpurun_out/${TAG}_bench_$N.json 2>gpurun_out/${TAG}_bench_$N.err || { echo "bench $V failed"; tail -5 gpurun_out/${TAG}_bench_$N.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_bench_$N.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$V', 'value', d['value'], 'ms', d['ms_per_step'], 'x3', r['avg_launch_ms'], r['frac'], {k:v['ms'] for k,v in r['conv_classes'].items()})"
  done
done | tee gpurun_out/${TAG}_bench.txt
[ "${TESTS:-1}" = 0 ] && exit 0
for V in "$@"; do
  N=$(echo $V | tr ':=,' '___')
  env $(envof $V) timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_range.py tests/test_gpu_backward.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests_$N.log 2>&1
  echo "tests $V rc=$?"; tail -3 gpurun_out/${TAG}_tests_$N.log
done
