"""The last N kernel dispatches of a rocprofv3 kernel trace as a timeline
(start and end in us relative to the first of them, duration, queue):
    python scripts/ktimeline.py <run_kernel_trace.csv> [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    q = r.get("Queue_Id", r.get("Stream_Id", ""))
    print(f'{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3}  {r["Kernel_Name"][:70]}')
