export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900|gpurun_out/r3_gpu_tests_k.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "300|gpurun_out/r3_ab_k.log|for r in 1 2; do for M in 1 0; do echo == merge=\$M; NPS_CONVT_MERGE=\$M python bench.py --cpu-calls 0 --steps 6 2>/dev/null | python -c \"import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['conv_classes'])\"; done; done" \
 "300|gpurun_out/r3_b2_k.log|for M in 1 0; do echo == merge=\$M B=2; NPS_CONVT_MERGE=\$M python bench.py --cpu-calls 0 --global-batch 2 --steps 10 2>/dev/null | python -c \"import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], r['conv_classes'])\"; done" \
 "120|gpurun_out/r3_calib_k.log|bash tools/calib/run.sh"
