#!/bin/bash
# Dev tool (GPU box): 3x3 main-loop ablations (NPS_X3_ABL builds, speed only) + cache counters.
# Output: gpurun_out/x3abl_*
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S1="--cin 192 --cout 192 --k 3 --hw 258 --b 16 --gn 0"
S2="--cin 388 --cout 192 --k 3 --hw 260 --b 16 --gn 1"
for L in libnps_hip libnps_x3abl1 libnps_x3abl2 libnps_x3abl4 libnps_hip; do
  echo "== $L"
  for S in "$S1" "$S2"; do
    NPS_HIP_LIB=$PWD/neural-pde-surrogates_amd/nps_hip/$L.so timeout -k 10 120 python3 tools/conv_bench.py $S 2>&1 | grep conv || exit 1
  done
done
timeout -s KILL 60 rocprofv3 -L > gpurun_out/x3abl_counters_list.txt 2>&1
i=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum" \
         "TA_BUSY_avr TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --output-format csv -d gpurun_out/x3abl_pmc$i -o run -- python3 tools/conv_bench.py $S1 --iters 3 > gpurun_out/x3abl_pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 gpurun_out/x3abl_pmc$i.log; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/x3abl_pmc*/**/*counter_collection.csv", recursive=True)):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        if "x3" not in k: continue
        print(k, {c: round(sum(v) / len(v), 1) for c, v in d.items()})
PY
