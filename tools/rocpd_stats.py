"""Kernel-time table from a rocprofv3 sqlite output (run_results.db) — the --stats summary when the CSV
was not requested: python tools/rocpd_stats.py DB [calls] [top] [csv_out]."""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
calls = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = db.execute("""select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start)
                     from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
                     group by s.kernel_name order by sum(d.end - d.start) desc""").fetchall()
tot = sum(r[2] for r in rows)
for name, n, t, avg in rows[:top]:
    print(f"{t / 1e6 / calls:8.2f} ms/call {n / calls:7.1f} {avg / 1e3:9.1f} us {100 * t / tot:5.1f}%  {name[:110]}")
print(f"total {tot / 1e6 / calls:.2f} ms/call")
if len(sys.argv) > 4:
    with open(sys.argv[4], "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
        for name, n, t, avg in rows:
            w.writerow([name, n, t, avg, 100 * t / tot])
