#!/bin/bash
# Dev tool: PMC passes over one 1x1 conv shape (tools/conv_bench.py), one counter set per pass.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
CMD="python3 tools/conv_bench.py --prec x3f16 --b 16 --k 1 --gn 0 --cin 196 --cout 192 --hw 256 --iters 5"
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc1x1_list.txt 2>&1 || true
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES" \
         "FETCH_SIZE" "WRITE_SIZE" "TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc1x1_$i -o run -- $CMD > gpurun_out/pmc1x1_$i.log 2>&1 || { echo "pass $i ($P) failed"; tail -5 gpurun_out/pmc1x1_$i.log; }
done
echo done
