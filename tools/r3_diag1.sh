export TMPDIR=/tmp
tools/gpu_steps.sh \
 "200|gpurun_out/r3_shapes_c3.log|python tools/call_shapes.py" \
 "200|gpurun_out/r3_x3stamps.log|bash tools/stamps_ab.sh"
