"""Print name / calls / average ns of a rocprofv3 kernel_stats.csv."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    print(f'{r["Name"][:60]:60s} {r["Calls"]:>5s} {float(r["AverageNs"]):12.0f}')
