#!/bin/bash
# Round-3 final GPU pass: tests, smoke, benches (C3 B=16 with CPU baseline, B=2, training, C5), rocprofv3 kernel
# stats (B=16 and B=2), PMC FETCH/WRITE passes, and the 2-rank N>1 rehearsal.  Output: gpurun_out/fin_*
export TMPDIR=/tmp
tools/gpu_steps.sh \
 "900|gpurun_out/fin_gpu_tests.log|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
 "200|gpurun_out/fin_smoke.log|python -c 'import __graft_entry__ as g; g.smoke()'" \
 "400|gpurun_out/fin_bench.json|python bench.py" \
 "300|gpurun_out/fin_bench_b2.json|python bench.py --global-batch 2 --steps 10 --cpu-calls 0" \
 "300|gpurun_out/fin_prof.log|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof -o run -- python bench.py --steps 3 --warmup 1 --cpu-calls 0" \
 "300|gpurun_out/fin_prof_b2.log|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin_prof_b2 -o run -- python bench.py --global-batch 2 --steps 4 --warmup 1 --cpu-calls 0" \
 "600|gpurun_out/fin_pmc.log|bash tools/pmc_traffic.sh" \
 "400|gpurun_out/fin_train.json|python bench.py --mode train" \
 "400|gpurun_out/fin_c5.json|python bench.py --model ufno3d --dtype bf16 --steps 5 --warmup 2" \
 "300|gpurun_out/fin_rehearsal.log|NPS_BENCH_REHEARSAL=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1"
