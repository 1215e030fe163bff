export TMPDIR=/tmp
L=$PWD/neural-pde-surrogates_amd/nps_hip
export L
tools/gpu_steps.sh \
 "200|gpurun_out/r3_x3stamps_n.log|bash tools/stamps_ab.sh" \
 "600|gpurun_out/r3_gpu_tests_n.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "400|gpurun_out/r3_ab_n.log|for r in 1 2; do for V in hip head; do echo == \$V; NPS_HIP_LIB=\$L/libnps_\$V.so python bench.py --cpu-calls 0 --steps 6 2>/dev/null | python -c \"import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['avg_launch_ms'], r['conv_classes'])\"; done; done"
