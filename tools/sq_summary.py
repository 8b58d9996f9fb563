#!/usr/bin/env python3
"""Per-kernel averages of rocprofv3 --pmc csv files (gpurun_out/sq/*_counter_collection.csv)."""
import collections, csv, glob, sys
root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f"{root}/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    if not k.startswith("rsk::"):
        continue
    print(k)
    for c, xs in sorted(v.items()):
        print(f"    {c:34s} {sum(xs) / len(xs):16.1f}")
