# C5 (3-D U-FNO) pass: kernel parity tests, bench (packed-frame vs fused prologue), rocprofv3 kernel stats
export TMPDIR=/tmp
T=${1:-c}
tools/gpu_steps.sh \
 "200|gpurun_out/r3_conv3d_$T.log|python -u -m pytest tests/test_gpu_conv3d.py tests/test_gpu_ufno3d.py -q --timeout 300 --timeout-method thread" \
 "300|gpurun_out/r3_bench_ufno3d_$T.json|python bench.py --model ufno3d --dtype bf16 --steps 5 --warmup 2 --cpu-calls 0" \
 "300|gpurun_out/r3_bench_ufno3d_${T}_nopack.json|NPS_CONV3D_PACK=0 python bench.py --model ufno3d --dtype bf16 --steps 5 --warmup 2 --cpu-calls 0" \
 "300|gpurun_out/r3_prof_ufno3d_$T.log|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ufno3d_$T -o run -- python bench.py --model ufno3d --dtype bf16 --steps 2 --warmup 1 --cpu-calls 0"
