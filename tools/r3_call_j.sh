export TMPDIR=/tmp
tools/gpu_steps.sh \
 "200|gpurun_out/r3_x3stamps_j.log|bash tools/stamps_ab.sh" \
 "300|gpurun_out/r3_shapes_j.log|NPS_X1_DMA=1 python tools/call_shapes.py && echo ==== wl && NPS_X1_DMA=0 python tools/call_shapes.py" \
 "200|gpurun_out/r3_store_bw_j.log|./tools/calib/store_bw" \
 "120|gpurun_out/r3_calib_j.log|bash tools/calib/run.sh" \
 "400|gpurun_out/r3_gpu_tests_j.log|python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_range.py -x -q --timeout 300 --timeout-method thread" \
 "300|gpurun_out/r3_bench_j.json|python bench.py --cpu-calls 0"
