"""Per-kernel launch statistics from rocprofv3 output.

    python scripts/kstats.py <run_kernel_stats.csv>     name / calls / average ns
    python scripts/kstats.py <run_kernel_trace.csv>     the same per (kernel, grid size):
        one bench process launches k_bs_20_30 both over 65,536 groups and once
        per rs_encode2 call (dropin_latency), so the whole-kernel average of
        --stats mixes the two; this separates them.
"""
import csv
import statistics
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    if rows and "Grid_Size_X" in rows[0]:
        by = {}
        for r in rows:
            key = (r["Kernel_Name"], int(r["Grid_Size_X"]))
            by.setdefault(key, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        print(f'{"kernel":60s} {"grid":>9s} {"calls":>5s} {"avg_ns":>10s} {"median_ns":>10s}')
        for (name, grid), d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            print(f'{name[:60]:60s} {grid:9d} {len(d):5d} {statistics.mean(d):10.0f} '
                  f'{statistics.median(d):10.0f}')
        return
    for r in rows:
        print(f'{r["Name"][:60]:60s} {r["Calls"]:>5s} {float(r["AverageNs"]):12.0f}')


if __name__ == "__main__":
    main(sys.argv[1])
