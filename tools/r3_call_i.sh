export TMPDIR=/tmp
L=$PWD/neural-pde-surrogates_amd/nps_hip
export L
tools/gpu_steps.sh \
 "900|gpurun_out/r3_gpu_tests_i.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200|gpurun_out/r3_x3stamps_i.log|bash tools/stamps_ab.sh" \
 "200|gpurun_out/r3_spec_w4.log|NPS_SPEC_W4=0 python tools/spectral_bench.py && NPS_SPEC_W4=1 python tools/spectral_bench.py" \
 "300|gpurun_out/r3_bench_i.json|python bench.py --cpu-calls 0"
