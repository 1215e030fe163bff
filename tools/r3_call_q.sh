export TMPDIR=/tmp
L=$PWD/neural-pde-surrogates_amd/nps_hip
export L
tools/gpu_steps.sh \
 "600|gpurun_out/r3_gpu_tests_q.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "500|gpurun_out/r3_ab_q.log|for r in 1 2; do for V in hip head; do echo == \$V; NPS_HIP_LIB=\$L/libnps_\$V.so python bench.py --cpu-calls 0 --steps 6 2>/dev/null | python -c \"import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['avg_launch_ms'], r['conv_classes'])\"; done; done; for V in hip head; do echo == \$V B=2; NPS_HIP_LIB=\$L/libnps_\$V.so python bench.py --cpu-calls 0 --steps 8 --global-batch 2 2>/dev/null | python -c \"import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['avg_launch_ms'], r['conv_classes'])\"; done" \
 "300|gpurun_out/r3_shapes_q.log|python tools/call_shapes.py"
