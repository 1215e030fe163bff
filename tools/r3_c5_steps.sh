tools/gpu_steps.sh \
 "200|gpurun_out/r3_conv3d_b.log|python -u -m pytest tests/test_gpu_conv3d.py -v --timeout 120 --timeout-method thread" \
 "400|gpurun_out/r3_ufno3d_b.log|python -u -m pytest tests/test_gpu_ufno3d.py -v -s --timeout 300 --timeout-method thread" \
 "200|gpurun_out/r3_c1_b.log|python -u -m pytest tests/test_gpu_parity.py -v -k c1 --timeout 120 --timeout-method thread" \
 "300|gpurun_out/r3_bench_ufno3d_b.json|python bench.py --model ufno3d --dtype bf16 --steps 5 --warmup 2"
