"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per conv kernel class (dev tool).

FETCH_SIZE scale per access shape, calibrated on each access pattern (tools/calib/pmc_calib.hip,
profiles/r3/pmc_calib.txt): a wide coalesced 16 B/lane sweep reads 1 GiB and FETCH_SIZE reports 0.5 GiB
(MI355X_MICROARCH.md § HBM: x 2); so do LDS-DMA full-line reads and the 1x1 kernels' B operand (both 64-B
halves of a line in one instruction); the 2x2/3x3/5x5 producers read ONE 64-B half of a pixel's line per
stage and for that shape FETCH_SIZE reports the bytes 1:1.  WRITE_SIZE is 1:1 for coalesced and for
MFMA-fragment stores.  Both counters are in KB (rocprofv3 derived metrics).
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
    if re.search(r"conv1x1_(?:x3|wl|dma)_kernel<", name):
        return "x3f16_1tap"
    m = re.search(r"conv2d_pc_kernel<(\d+), \d+, \d+, \d+, \d+>", name)
    if m:
        return f"f32_{m.group(1)}tap"
    return None


def fetch_scale(name):
    """FETCH_SIZE -> bytes per access shape (tools/calib/pmc_calib.hip, profiles/r3/pmc_calib.txt): x 1 for the
    patch producers of the 2x2 / 3x3 / 5x5 ring kernels (each stage reads one 64-B half of a pixel's 128-B
    line, the other half a stage later: 1 GiB read, 1 GiB reported); x 2 for full 128-B lines read by one
    instruction — 16 B/lane sweeps, LDS-DMA lines (conv1x1_dma_kernel) and the register-staged 1x1's B
    operand (lane halves read both 64-B halves of a line in one instruction: 1 GiB read, 0.5 GiB reported)."""
    c = klass(name)
    if c is not None and c.startswith("x3f16_") and c != "x3f16_1tap":
        return 1
    if "timeconv_fast_kernel" in name:
        # each block stages PX = 16 pixels of every planar pre-decoder row: 64-B halves of 128-B lines, the
        # other half read by the neighbouring block — the producers' counted-1:1 shape (round 4: the x 2 here
        # made the kernel read as 3.4x its algorithmic bytes; it reads them once)
        return 1
    return 2


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    out = {"command": sys.argv[3], "unit": "bytes per launch",
           "note": "FETCH_SIZE x 1 for the 2x2/3x3/5x5 ring-kernel producers (64-B halves of 128-B lines read a "
                   "stage apart, counted 1:1), x 2 for full-line reads by one instruction (16 B/lane sweeps, the "
                   "1x1 kernels' B operand, LDS-DMA: half-counted), WRITE_SIZE x 1 (coalesced and MFMA-fragment "
                   "stores both counted 1:1) — tools/calib/pmc_calib.hip, profiles/r3/pmc_calib.txt; KB -> bytes; "
                   "Infinity-Cache hits are counted by these fabric-side counters",
           "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        fv, wv = fetch.get(name, []), write.get(name, [])
        if not fv or not wv:
            continue
        fb = fetch_scale(name) * 1024 * sum(fv) / len(fv)
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
