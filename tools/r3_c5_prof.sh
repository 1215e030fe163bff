export TMPDIR=/tmp
tools/gpu_steps.sh \
 "200|gpurun_out/r3_conv3d_c.log|python -u -m pytest tests/test_gpu_conv3d.py tests/test_gpu_ufno3d.py -q --timeout 300 --timeout-method thread" \
 "300|gpurun_out/r3_bench_ufno3d_c.json|python bench.py --model ufno3d --dtype bf16 --steps 5 --warmup 2 --cpu-calls 0" \
 "300|gpurun_out/r3_prof_ufno3d_c.log|rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ufno3d_c -o run -- python bench.py --model ufno3d --dtype bf16 --steps 2 --warmup 1 --cpu-calls 0"
