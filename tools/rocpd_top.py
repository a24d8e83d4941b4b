"""Per-kernel summary (name, calls, total and average ns) from a rocprofv3 rocpd database:
python tools/rocpd_top.py RUN_results.db > kernel_stats.csv"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage"])
for name, calls, total, avg, pct in db.execute(
        "select name, total_calls, total_duration, average, percentage from top_kernels"):
    # top_kernels reports durations in microseconds
    w.writerow([name, calls, round(float(total) * 1e3), round(float(avg) * 1e3), round(float(pct), 3)])
