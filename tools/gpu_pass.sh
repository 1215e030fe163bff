#!/bin/bash
# One GPU-box pass (gpurun): parity suite, C3 bench + rocprof, B=2 line, training lines + rocprof, C5 line +
# rocprof, and the N=2 rehearsals of `bench.py --gpus 2` (the driver's own command form; ranks share cuda:0
# over gloo: NPS_BENCH_REHEARSAL=1, never a reported number).  Outputs: gpurun_out/${TAG}_*.
# usage: tools/gpu_pass.sh TAG [steps...]
#   steps: tests sel($TESTSEL) pmc bench prof b2 b2prof train trainprof tb2prof c2 c4 c5 c5prof reh rehroll smoke
set -o pipefail
TAG=${1:-r5}; shift
STEPS="${@:-tests bench prof b2 train c5 reh}"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
O=gpurun_out/$TAG
for s in $STEPS; do
  case $s in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > ${O}_tests.log 2>&1 \
             || { echo "tests failed"; tail -30 ${O}_tests.log; exit 1; }; tail -2 ${O}_tests.log ;;
    sel)   timeout -k 10 600 python -u -m pytest $TESTSEL -m gpu -q -x --timeout 200 --timeout-method thread > ${O}_sel.log 2>&1 \
             || { echo "selected tests failed"; tail -30 ${O}_sel.log; exit 1; }; tail -2 ${O}_sel.log ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.log 2>&1 \
             || { echo "smoke failed"; tail -20 ${O}_smoke.log; exit 1; }; tail -3 ${O}_smoke.log ;;
    pmc)   timeout -k 10 900 bash tools/pmc_traffic.sh > ${O}_pmc.log 2>&1 || { echo "pmc failed"; tail -20 ${O}_pmc.log; exit 1; }; cp gpurun_out/pmc_traffic.json ${O}_pmc_traffic.json ;;
    bench) timeout -k 10 400 python -u bench.py > ${O}_bench.json 2> ${O}_bench.err || { echo "bench failed"; tail -20 ${O}_bench.err; exit 1; }; tail -c 600 ${O}_bench.json ;;
    prof)  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_prof -o run -- python3 bench.py --steps 3 --warmup 1 --cpu-calls 0 \
             > ${O}_prof.log 2>&1 || { echo "prof failed"; tail -20 ${O}_prof.log; exit 1; } ;;
    b2)    timeout -k 10 300 python -u bench.py --global-batch 2 --cpu-calls 0 > ${O}_b2.json 2> ${O}_b2.err || { echo "b2 failed"; tail -20 ${O}_b2.err; exit 1; }; tail -c 300 ${O}_b2.json ;;
    b2prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_b2prof -o run -- python3 bench.py --global-batch 2 --steps 10 --warmup 2 --cpu-calls 0 \
             > ${O}_b2prof.log 2>&1 || { echo "b2 prof failed"; tail -20 ${O}_b2prof.log; exit 1; } ;;
    train) for gb in 2 16; do timeout -k 10 400 python -u bench.py --mode train --steps 5 --warmup 2 --global-batch $gb > ${O}_train_b$gb.json 2> ${O}_train_b$gb.err \
             || { echo "train $gb failed"; tail -20 ${O}_train_b$gb.err; exit 1; }; tail -c 300 ${O}_train_b$gb.json; done ;;
    trainprof) timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_tprof -o run -- python3 bench.py --mode train --steps 3 --warmup 1 --global-batch 16 --cpu-calls 0 \
             > ${O}_tprof.log 2>&1 || { echo "train prof failed"; tail -20 ${O}_tprof.log; exit 1; } ;;
    tb2prof) timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d ${O}_tb2prof -o run -- python3 bench.py --mode train --steps 5 --warmup 2 --global-batch 2 --cpu-calls 0 \
             > ${O}_tb2prof.log 2>&1 || { echo "train b2 prof failed"; tail -20 ${O}_tb2prof.log; exit 1; } ;;
    c2)    timeout -k 10 300 python -u bench.py --res 128 --num-c 1 --fno-modes 12 --cpu-calls 0 > ${O}_c2.json 2> ${O}_c2.err || { echo "c2 failed"; tail -20 ${O}_c2.err; exit 1; }; tail -c 300 ${O}_c2.json ;;
    c4)    timeout -k 10 300 python -u bench.py --model drn --num-c 1 --cpu-calls 0 > ${O}_c4.json 2> ${O}_c4.err || { echo "c4 failed"; tail -20 ${O}_c4.err; exit 1; }; tail -c 300 ${O}_c4.json ;;
    c5)    timeout -k 10 400 python -u bench.py --model ufno3d --dtype bf16 > ${O}_c5.json 2> ${O}_c5.err || { echo "c5 failed"; tail -20 ${O}_c5.err; exit 1; }; tail -c 300 ${O}_c5.json ;;
    c5prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d ${O}_c5prof -o run -- python3 bench.py --model ufno3d --dtype bf16 --steps 3 --warmup 1 --cpu-calls 0 \
             > ${O}_c5prof.log 2>&1 || { echo "c5 prof failed"; tail -20 ${O}_c5prof.log; exit 1; } ;;
    reh)   NPS_BENCH_REHEARSAL=1 timeout -k 10 400 python3 bench.py --gpus 2 --mode train --steps 3 --warmup 1 --global-batch 4 --cpu-calls 0 \
             > ${O}_reh_train.json 2> ${O}_reh_train.err || { echo "train rehearsal failed"; tail -20 ${O}_reh_train.err; exit 1; }; tail -c 400 ${O}_reh_train.json ;;
    rehroll) NPS_BENCH_REHEARSAL=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 1 --cpu-calls 0 \
             > ${O}_reh_roll.json 2> ${O}_reh_roll.err || { echo "rollout rehearsal failed"; tail -20 ${O}_reh_roll.err; exit 1; }; tail -c 400 ${O}_reh_roll.json ;;
  esac
  echo "step $s ok"
done
