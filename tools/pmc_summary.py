"""Summarise rocprofv3 counter CSVs for one kernel (per-dispatch average of the last N dispatches)."""
import csv, collections, sys
kern = sys.argv[1]
for d in sys.argv[2:]:
    rows = list(csv.DictReader(open(d)))
    agg = collections.defaultdict(list)
    for r in rows:
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(f"{k:28s} n={len(v):3d} last={v[-1]:.6g}")
