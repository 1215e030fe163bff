# Dev A/B: store-burst stagger variants of the 3x3 wide kernel (tools/build_variant.sh)
export TMPDIR=/tmp
L=$PWD/neural-pde-surrogates_amd/nps_hip
for r in 1 2; do
for V in hip stag2 stag4; do
  echo "== $V round $r"
  NPS_HIP_LIB=$L/libnps_$V.so timeout -k 10 120 python tools/conv_bench.py --cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn 1 2>&1 | grep conv || exit 1
  NPS_HIP_LIB=$L/libnps_$V.so timeout -k 10 200 python bench.py --steps 5 --warmup 2 --cpu-calls 0 > gpurun_out/stag_$V.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/stag_$V.json')); r=d['roofline']; print(d['value'], r['avg_launch_ms'], r['conv_classes'])"
done; done
