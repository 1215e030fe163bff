#!/bin/bash
# PMC passes on one conv launch shape (args forwarded to tools/conv_bench.py, or $PMCC_BENCH), one counter set per pass
# (MI355X_MICROARCH.md per-block limits); pass 1 also records the kernel trace (durations -> effective
# clock).  Results under gpurun_out/pmcc_*; summary: python tools/pmc_conv_summary.py gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="$@"
T=${PMCC_TAG:-pmcc}   # output prefix (NPS_HIP_LIB selects the library build)
BENCH=${PMCC_BENCH:-tools/conv_bench.py}   # tools/conv3d_bench.py for the 3-D convs
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
         "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  KT=""; [ $i -eq 1 ] && KT="--kernel-trace"
  timeout -s KILL 120 rocprofv3 --pmc $P $KT --output-format csv -d gpurun_out/${T}_$i -o run -- python3 $BENCH --iters 3 $ARGS > gpurun_out/${T}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${T}_$i.log; exit 1; }
done
echo pmc done
