#!/usr/bin/env python3
"""Summarise a gpu_check.sh session (gpurun_out/) into profiles/.

Reads the rocprofv3 kernel-trace stats (prof/run_kernel_stats.csv,
prof/run_kernel_trace.csv) and the separate PMC passes (pmc/fetch_*,
pmc/write_*, pmc/l2_*), and writes:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (copied)
  profiles/<tag>_summary.json       per-kernel: launches, avg duration (trace),
                                    FETCH_SIZE / WRITE_SIZE / TCC hit+miss per launch
  profiles/pmc_headline.json        hbm_bytes_per_launch per kernel for bench.py

HBM bytes = (FETCH_SIZE + WRITE_SIZE) * 1024 per launch.  The microarch guide's
x2 FETCH correction applies to 16-B-per-lane streaming reads; these kernels
read 4 B per lane (dword loads / global_load_lds_dword), for which the raw
FETCH_SIZE matched the known image bytes (391 tiles x 272 rows x 64 chunks x
256 B = 1.74 GB vs 1.78 GB measured), so it is reported uncorrected, with the
x2 figure alongside.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import os
import re
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    m = re.search(r"rsk::(\w+?)(?:<|\()", name)
    return m.group(1).replace("_kernel", "") if m else name[:40]


def read_pmc(path, counter):
    out = collections.defaultdict(list)
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            out[(short(r["Kernel_Name"]), r["Grid_Size"])].append(float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--src", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--config", default="headline")
    ap.add_argument("--S", type=int, default=4096)
    args = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(args.src, "prof", "run_kernel_stats.csv"),
                os.path.join(prof, f"{args.tag}_kernel_stats.csv"))
    trace = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(args.src, "prof", "run_kernel_trace.csv"))):
        trace[(short(r["Kernel_Name"]), r["Grid_Size_X"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    pmc = {c: read_pmc(os.path.join(args.src, "pmc", f"{f}_counter_collection.csv"), c)
           for f, c in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE"), ("l2", "TCC_HIT_sum"),
                        ("l2", "TCC_MISS_sum"))}
    summary = {}
    for (k, grid), durs in sorted(trace.items()):
        if not k.startswith("car") and k not in ("pick_node", "node_reduce"):
            continue
        e = {"grid": int(grid), "launches": len(durs), "avg_us": round(sum(durs) / len(durs) / 1e3, 2)}
        for c, d in pmc.items():
            v = d.get((k, grid))
            if v:
                e[c] = round(sum(v) / len(v), 1)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes_per_launch"] = int((e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024)
            e["hbm_bytes_per_launch_fetch_x2"] = int((2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024)
            e["hbm_GBps"] = round(e["hbm_bytes_per_launch"] / (e["avg_us"] * 1e3), 1)
        summary[f"{k}@{grid}"] = e
    with open(os.path.join(prof, f"{args.tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    # per kernel name: launch-weighted traffic for bench.py's roofline.traffic
    by_kernel = collections.defaultdict(lambda: [0, 0, 0.0])
    for key, e in summary.items():
        if "hbm_bytes_per_launch" in e:
            b = by_kernel[key.split("@")[0]]
            b[0] += e["hbm_bytes_per_launch"]
            b[1] += 1
            b[2] += e["avg_us"]
    head = {"source": f"profiles/{args.tag}_summary.json", args.config: {}}
    for k, (bytes_, n, us) in by_kernel.items():
        head[args.config][f"car_{k[4:]}" if k.startswith("car_") else k] = {
            "S": args.S, "hbm_bytes_per_launch": bytes_ // max(n, 1), "avg_us": round(us / max(n, 1), 2)}
    with open(os.path.join(prof, "pmc_headline.json"), "w") as f:
        json.dump(head, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
