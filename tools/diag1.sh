cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|FAILED|Error" > gpurun_out/diag1_x3.log
echo "x3 rc=$?"
NPS_CONV_PRECISION=f32 timeout -k 10 300 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | grep -E "passed|failed|FAILED|Error" > gpurun_out/diag1_f32.log
echo "f32 rc=$?"
cat gpurun_out/diag1_x3.log gpurun_out/diag1_f32.log
