#!/bin/bash
# Same-box A/B of dev library variants (gpurun): conv shapes, the C3 bench, parity tests on the variant.
# usage: tools/r4_ab.sh TAG VARIANT [VARIANT2 ...]   (libnps_<VARIANT>.so built by tools/build_variant.sh; "hip" =
# the in-tree library; libnps_base.so = the reference build of an earlier commit, run without the s2d view)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
LIBS="base $@"
D=$PWD/neural-pde-surrogates_amd/nps_hip
for L in $LIBS; do [ -f $D/libnps_$L.so ] || { echo "missing $D/libnps_$L.so"; exit 2; }; done
S1="--cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn 1"
S2="--cin 388 --cout 192 --k 3 --hw 260 --b 16 --gn 1"
S3="--cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn 0"
for r in 1 2; do
  for L in $LIBS; do
    for S in "$S1" "$S2" "$S3"; do
      NPS_S2D_VIEW=$([ $L = hip ] && echo 1 || echo 0) NPS_HIP_LIB=$D/libnps_$L.so timeout -k 10 120 python3 tools/conv_bench.py $S 2>&1 | grep conv | sed "s/^/$L /" || exit 1
    done
  done
done | tee gpurun_out/${TAG}_conv.txt
for r in 1 2; do
  for L in $LIBS; do
    NPS_S2D_VIEW=$([ $L = hip ] && echo 1 || echo 0) NPS_HIP_LIB=$D/libnps_$L.so timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --cpu-calls 0 > gpurun_out/${TAG}_bench_$L.json 2>gpurun_out/${TAG}_bench_$L.err || { echo "bench $L failed"; tail -5 gpurun_out/${TAG}_bench_$L.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}_bench_$L.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$L', 'value', d['value'], 'ms', d['ms_per_step'], 'x3', r['avg_launch_ms'], r['frac'], {k:v['ms'] for k,v in r['conv_classes'].items()})"
  done
done | tee gpurun_out/${TAG}_bench.txt
for L in "$@"; do
  NPS_S2D_VIEW=$([ $L = hip ] && echo 1 || echo 0) NPS_HIP_LIB=$D/libnps_$L.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_range.py tests/test_gpu_backward.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests_$L.log 2>&1
  echo "tests $L rc=$?"; tail -3 gpurun_out/${TAG}_tests_$L.log
done
