#!/bin/bash
# Short round-3 closing pass: GPU tests, smoke, C3 bench, rocprofv3 kernel stats.  Output: gpurun_out/fin4_*
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "600|gpurun_out/fin4_gpu_tests.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200|gpurun_out/fin4_smoke.log|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "400|gpurun_out/fin4_bench.json|python bench.py" \
 "300|gpurun_out/fin4_prof.log|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin4_prof -o run -- python bench.py --steps 3 --warmup 1 --cpu-calls 0"
