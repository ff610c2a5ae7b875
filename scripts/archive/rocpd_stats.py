#!/usr/bin/env python3
"""rocprofv3 writes its kernel trace as a rocpd SQLite database (run_results.db)
on this ROCm; this prints the same per-kernel summary `--stats` gives
(name, calls, total/average/min/max ns, percentage) as CSV.

    python3 scripts/rocpd_stats.py gpurun_out/r02_prof/run_results.db > profiles/r02/x.csv
"""
import csv
import sqlite3
import sys


def main(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "name" if "name" in cols else "kernel_name"
    rows = c.execute(
        f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), "
        f"max(end - start) from kernels group by {name} order by sum(end - start) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for n, calls, tot, avg, mn, mx in rows:
        w.writerow([n, calls, tot, round(avg, 1), mn, mx, round(100.0 * tot / total, 3)])


if __name__ == "__main__":
    main(sys.argv[1])
