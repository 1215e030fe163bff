"""Summarise tools/pmc_conv.sh passes for the conv kernel of the shape (the longest-running kernel).

Effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration (MI355X_MICROARCH.md 'DVFS give-back');
MFMA pipe busy = SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles x 4 SIMDs x CUs).
usage: python tools/pmc_conv_summary.py gpurun_out [n_cu] [prefix (default pmcc)]
"""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1]
ncu = int(sys.argv[2]) if len(sys.argv) > 2 else 256
pre = sys.argv[3] if len(sys.argv) > 3 else "pmcc"
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/{pre}_*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = defaultdict(list)
for f in glob.glob(f"{root}/{pre}_1/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
name = max(dur, key=lambda k: sum(dur[k]))
d = sum(dur[name]) / len(dur[name])
c = {k: sum(v) / len(v) for k, v in vals[name].items()}
out = {"kernel": name[:120], "avg_duration_ms": d * 1e3, "counters_per_launch": c}
if "GRBM_GUI_ACTIVE" in c:
    clk = c["GRBM_GUI_ACTIVE"] / 8 / d
    out["effective_clock_GHz"] = clk / 1e9
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        out["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * d * 4 * ncu)
if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
    out["hbm_bytes"] = 2 * 1024 * c["FETCH_SIZE"] + 1024 * c["WRITE_SIZE"]
print(json.dumps(out, indent=1))
