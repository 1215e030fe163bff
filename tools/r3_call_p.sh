export TMPDIR=/tmp
tools/gpu_steps.sh \
 "600|gpurun_out/r3_gpu_tests_p.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "400|gpurun_out/r3_train_p.json|python bench.py --mode train"
