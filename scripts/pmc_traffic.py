"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into per-launch HBM bytes.

gfx950 corrections (MI355X_MICROARCH.md section HBM): FETCH_SIZE (KiB) reports
half the bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE
(KiB) is exact for 16-B-per-lane stores.  Usage:
  python scripts/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> \
      <kernel-substring> <groups> <alg_bytes_per_launch> [encode|decode] > profiles/traffic.json
With the last argument the JSON carries the digest of that kernel's sources
(bench.py KERNEL_SOURCES), which bench.py checks before it reports the bytes.
"""
import csv, json, os, statistics, sys


def per_dispatch(path, kernel, counter):
    vals = {}
    for row in csv.DictReader(open(path)):
        if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
            vals.setdefault(row["Dispatch_Id"], 0.0)
            vals[row["Dispatch_Id"]] += float(row["Counter_Value"])
    return list(vals.values())


fetch_csv, write_csv, kernel, groups, alg = sys.argv[1:6]
which = sys.argv[6] if len(sys.argv) > 6 else None
f = per_dispatch(fetch_csv, kernel, "FETCH_SIZE")
w = per_dispatch(write_csv, kernel, "WRITE_SIZE")
fb = statistics.median(f) * 1024 * 2
wb = statistics.median(w) * 1024
out = {"kernel": kernel, "groups": int(groups), "dispatches": [len(f), len(w)],
       "fetch_bytes_per_launch": fb, "write_bytes_per_launch": wb,
       "hbm_bytes_per_launch": fb + wb, "alg_bytes_per_launch": int(alg),
       "ratio_to_alg": (fb + wb) / int(alg),
       "correction": "FETCH_SIZE x2 (gfx950 wide-read half count), WRITE_SIZE x1; KiB->B"}
if which:
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_source_sha
    out["source_sha256"] = kernel_source_sha(which)
print(json.dumps(out, indent=1))
