#!/bin/bash
# HBM traffic of the rollout's conv kernels from rocprofv3 PMC counters, one counter set per pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass).  Output: gpurun_out/pmc_*/
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
CMD="python3 bench.py --steps 1 --warmup 1 --cpu-calls 0"
i=0
for P in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_$i -o run -- $CMD > gpurun_out/pmc_$i.log 2>&1 || { echo "pmc pass $i ($P) failed"; tail -20 gpurun_out/pmc_$i.log; exit 1; }
  echo "pmc pass $i ($P) ok"
done
python3 tools/pmc_summary.py gpurun_out/pmc_1 gpurun_out/pmc_2 "$CMD" > gpurun_out/pmc_traffic.json && cat gpurun_out/pmc_traffic.json | head -40
