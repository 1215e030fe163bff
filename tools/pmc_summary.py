"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per conv kernel class (dev tool).

FETCH_SIZE is doubled: on gfx950 it reports exactly half the bytes of wide coalesced reads
(MI355X_MICROARCH.md § HBM).  Both counters are in KB (rocprofv3 derived metrics).
usage: python tools/pmc_summary.py <fetch_dir> <write_dir> "<command>"
"""
import csv
import glob
import json
import re
import sys


def load(d, counter):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = {}
    for r in csv.DictReader(open(f[0])):
        if r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"]
        per.setdefault(name, []).append(float(r["Counter_Value"]))
    return per


def klass(name):
    m = re.search(r"conv2d_x3_kernel<(\d+), \d+(?:, (?:true|false))*>", name)
    if m:
        return f"x3f16_{m.group(1)}tap"
    if re.search(r"conv1x1_(?:x3|wl)_kernel<", name):
        return "x3f16_1tap"
    m = re.search(r"conv2d_pc_kernel<(\d+), \d+, \d+, \d+, \d+>", name)
    if m:
        return f"f32_{m.group(1)}tap"
    return None


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {"command": sys.argv[3], "unit": "bytes per launch",
           "note": "FETCH_SIZE x 2 (gfx950 half-count of 16 B/lane reads) + WRITE_SIZE, KB -> bytes; "
                   "Infinity-Cache hits are counted by these fabric-side counters",
           "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        fv, wv = fetch.get(name, []), write.get(name, [])
        if not fv or not wv:
            continue
        fb = 2 * 1024 * sum(fv) / len(fv)
        wb = 1024 * sum(wv) / len(wv)
        out["kernels"][name[:160]] = dict(launches=len(fv), fetch_bytes_per_launch=fb, write_bytes_per_launch=wb,
                                          hbm_bytes_per_launch=fb + wb, **({"class": klass(name)} if klass(name) else {}))
    classes = {}
    for rec in out["kernels"].values():
        if "class" in rec:
            c = classes.setdefault(rec["class"], dict(launches=0, hbm_bytes=0.0))
            c["launches"] += rec["launches"]
            c["hbm_bytes"] += rec["hbm_bytes_per_launch"] * rec["launches"]
    out["classes"] = {k: dict(launches=v["launches"], hbm_bytes_per_launch=v["hbm_bytes"] / v["launches"])
                      for k, v in classes.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
