export TMPDIR=/tmp
tools/gpu_steps.sh \
 "200|gpurun_out/r3_x3stamps_m.log|bash tools/stamps_ab.sh" \
 "600|gpurun_out/r3_gpu_tests_m.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300|gpurun_out/r3_bench_m.log|python bench.py --cpu-calls 0 --steps 6 && python bench.py --cpu-calls 0 --steps 6"
