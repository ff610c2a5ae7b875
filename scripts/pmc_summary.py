"""Average PMC counters per dispatch for kernels matching a substring:
    python scripts/pmc_summary.py gpurun_out/pmc_cook cook decook"""
import collections
import csv
import glob
import sys

root, names = sys.argv[1], sys.argv[2:]
for p in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for row in csv.DictReader(open(p)):
        k = row["Kernel_Name"].replace("(anonymous namespace)", "anon")
        hit = [n for n in names if ("::" + n + "(") in k or ("::" + n + "<") in k
               or k.startswith(n + "(") or k.startswith(n + "<")]
        if not hit:
            continue
        # template instances (k_decode_ragged_cls<5, 5>) are kept apart
        short = k.split("(")[0].split("::")[-1] if "<" not in k.split("(")[0] else \
            k[k.find(hit[-1]):k.find(">", k.find(hit[-1])) + 1]
        agg[short][(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
    for kn, d in agg.items():
        per = collections.defaultdict(list)
        for (disp, c), v in d.items():
            per[c].append(v)
        print(p.split("/")[-2], kn, {c: round(sum(v) / len(v)) for c, v in per.items()})
