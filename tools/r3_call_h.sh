export TMPDIR=/tmp
L=$PWD/neural-pde-surrogates_amd/nps_hip
tools/gpu_steps.sh "120|gpurun_out/r3_store_bw.log|./tools/calib/store_bw" \
  "300|gpurun_out/r3_aring_ab.log|for r in 1 2; do for V in hip aring3; do echo == \$V; NPS_HIP_LIB=\$L/libnps_\$V.so python tools/conv_bench.py --cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn 1 --check 2>&1 | grep -v amdgpu; done; done"
