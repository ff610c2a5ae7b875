"""Per-(kernel, grid size) call count, mean and median duration from a
rocprofv3 --kernel-trace CSV: bench.py launches the same kernels at several
sizes (C1/C2 steps, the other_configs lines, one-group drop-in calls), so the
per-name averages of the stats CSV mix them.
    python scripts/kstats_grid.py <run_kernel_trace.csv> [name-substring]"""
import collections, csv, statistics, sys

rows = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if len(sys.argv) > 2 and sys.argv[2] not in r["Kernel_Name"]:
        continue
    rows[(r["Kernel_Name"][:60], int(r["Grid_Size_X"]))].append(
        int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print(f"{'kernel':62s} {'grid':>9s} {'calls':>5s} {'avg_ns':>10s} {'median_ns':>10s}")
for (k, g), v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:62s} {g:9d} {len(v):5d} {statistics.mean(v):10.0f} {statistics.median(v):10.0f}")
