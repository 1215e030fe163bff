export TMPDIR=/tmp
tools/gpu_steps.sh "200|gpurun_out/r3_x3stamps2.log|bash tools/stamps_ab.sh"
