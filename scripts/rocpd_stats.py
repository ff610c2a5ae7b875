"""Summarise a rocprofv3 rocpd database (``*_results.db``) as a kernel-stats CSV.

rocprofv3 in ROCm 7 writes its trace as a SQLite "rocpd" database unless
``--output-format csv`` is given.  This reproduces the columns of the CSV
``--stats`` summary (durations in ns) from the database's dispatch table, so
profiles captured either way are committed in one format.

    python scripts/rocpd_stats.py gpurun_out/prof/run_results.db > profiles/X_kernel_stats.csv
"""
import csv
import sqlite3
import statistics
import sys


def main(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, start, end from kernels").fetchall()
    per = {}
    for name, start, end in rows:
        per.setdefault(name, []).append(end - start)
    total = sum(sum(v) for v in per.values()) or 1
    w = csv.writer(sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
    for name, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        sd = statistics.pstdev(d) if len(d) > 1 else 0.0
        w.writerow([name, len(d), sum(d), round(sum(d) / len(d), 3), round(100.0 * sum(d) / total, 2),
                    min(d), max(d), round(sd, 3)])


if __name__ == "__main__":
    main(sys.argv[1])
