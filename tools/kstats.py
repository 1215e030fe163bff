"""Per-model-call kernel table from a rocprofv3 --stats CSV: python tools/kstats.py CSV [calls] [top]."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
calls = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / calls:8.2f} ms/call {int(r['Calls']) / calls:6.1f} "
          f"{float(r['AverageNs']) / 1e3:9.1f} us  {r['Name'][:100]}")
print(f"total {tot / 1e6 / calls:.2f} ms/call")
