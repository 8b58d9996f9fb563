#!/usr/bin/env python3
"""Per-kernel FETCH_SIZE / WRITE_SIZE averages of a tools/gpu_r06.sh pmc:* step:
the bytes per launch as tools/pmc_summary.py counts them ((2 x FETCH + WRITE) x
1 KiB; FETCH doubled for gfx950's coalesced reads, MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(root, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != c:
                continue
            m = re.search(r"rsk::(\w+?)(?:<|\()", r["Kernel_Name"])
            k = m.group(1) if m else r["Kernel_Name"][:40]
            vals[k][c].append(float(r["Counter_Value"]))
for k, d in sorted(vals.items()):
    f = sum(d["FETCH_SIZE"]) / max(1, len(d["FETCH_SIZE"]))
    w = sum(d["WRITE_SIZE"]) / max(1, len(d["WRITE_SIZE"]))
    print(f"{k:32s} launches {len(d['FETCH_SIZE']):4d}  read {2 * f * 1024 / 1e9:8.4f} GB  write {w * 1024 / 1e9:8.4f} GB  "
          f"traffic {(2 * f + w) * 1024 / 1e9:8.4f} GB")
