"""GPU busy fraction of a rocprofv3 --kernel-trace run: union of kernel intervals over the span of the last
`--window` ms of the trace (the timed steps), plus the inter-kernel gap distribution and the top kernels by time.
A busy fraction near 1 means the step is device-bound and HIP graphs / fewer launches cannot buy much.

usage: python tools/busy_frac.py gpurun_out/<dir>/run_kernel_trace.csv [--window MS] [--top N]
"""
import argparse
import csv
import re
import statistics
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=float, default=0.0, help="analyse only the last MS of the trace (0 = all)")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if a.window > 0:
        t_end = max(e for _, e, _ in iv)
        iv = [x for x in iv if x[0] >= t_end - a.window * 1e6]
    span = max(e for _, e, _ in iv) - iv[0][0]
    busy, gaps, cur_s, cur_e = 0, [], iv[0][0], iv[0][1]
    for s, e, _ in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = defaultdict(lambda: [0, 0])
    for s, e, n in iv:
        k = re.sub(r"^void |\(anonymous namespace\)::", "", n)
        k = k[:100] if k.startswith("at::native") else re.split(r"[<(]", k)[0]
        per[k][0] += 1
        per[k][1] += e - s
    print(f"kernels {len(iv)}  span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  busy_fraction {busy / span:.4f}")
    if gaps:
        gs = sorted(gaps)
        print(f"gaps {len(gaps)}  total {sum(gaps) / 1e6:.2f} ms  median {statistics.median(gs) / 1e3:.2f} us  "
              f"p90 {gs[int(0.9 * len(gs))] / 1e3:.2f} us  max {gs[-1] / 1e3:.1f} us")
    print(f"top {a.top} kernels by time:")
    for k, (n, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {t / 1e6:8.2f} ms  {n:6d}  {k}")


if __name__ == "__main__":
    main()
