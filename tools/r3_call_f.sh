export TMPDIR=/tmp
tools/gpu_steps.sh "300|gpurun_out/r3_x1dma_b.log|bash tools/r3_x1dma.sh" "600|gpurun_out/r3_stag_ab.log|bash tools/r3_stag_ab.sh"
