export TMPDIR=/tmp
L=$PWD/neural-pde-surrogates_amd/nps_hip
tools/gpu_steps.sh "120|gpurun_out/r3_x1d_stamps.log|NPS_HIP_LIB=$L/libnps_x3stamp.so python tools/x1d_stamps.py && NPS_HIP_LIB=$L/libnps_x3stamp.so python tools/x1d_stamps.py --cin 196 --hw 256" \
  "300|gpurun_out/r3_x1dma_c.log|bash tools/r3_x1dma.sh" \
  "600|gpurun_out/r3_stag_ab.log|bash tools/r3_stag_ab.sh"
