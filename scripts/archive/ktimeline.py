"""The last N kernel dispatches of a rocprofv3 kernel trace as a timeline
(start and end in us relative to the first of them, duration, queue), with
the memory copies of a memory-copy trace merged in when one is given:
    python scripts/ktimeline.py <run_kernel_trace.csv> [N] [run_memory_copy_trace.csv]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
for r in rows:
    r["_name"] = r["Kernel_Name"]
if len(sys.argv) > 3:
    try:
        for r in csv.DictReader(open(sys.argv[3])):
            kind = r.get("Direction") or r.get("Operation") or r.get("Kind") or "copy"
            size = r.get("Bytes") or r.get("Size") or ""
            r["_name"] = f"COPY {kind} {size} B"
            rows.append(r)
    except FileNotFoundError:
        pass
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    q = r.get("Queue_Id", r.get("Stream_Id", ""))
    print(f'{s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3}  {r["_name"][:70]}')
