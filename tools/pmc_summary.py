#!/usr/bin/env python3
"""Summarise a tools/gpu_prof.sh session into profiles/.

Reads the rocprofv3 kernel-trace stats (<src>/prof/run_kernel_stats.csv,
<src>/prof/run_kernel_trace.csv) and the separate PMC passes
(<src>/pmc/fetch_*, write_*, l2_*), and writes:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary (copied)
  profiles/<tag>_summary.json       per kernel: launches, avg duration (trace),
                                    FETCH_SIZE / WRITE_SIZE / TCC hit+miss per launch
  profiles/pmc_traffic.json         {"configs": {config: {kernel: {S,
                                    hbm_bytes_per_launch, ...}}}} for bench.py

HBM bytes per launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: on gfx950
FETCH_SIZE reports half the bytes of coalesced streaming reads
(MI355X_MICROARCH.md, HBM section), and these kernels' bulk reads are
coalesced 128-/256-B rows (lane = scenario).  Infinity-Cache hits are counted
too (the same section), so the figure is an upper bound on DRAM bytes.
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


# kernel symbol -> the timer name bench.py reports (librsk ScopedTimer names)
BENCH_NAME = {"car_tile16": "car_tile", "car_fused16": "car_tile", "car_hub": "car_heavy", "car_side16": "car_side"}
# bench timers that bracket several launches of one step (car_tile: the lean and
# the heavy tile launch, two grid sizes of car_tile16): their per-"launch"
# traffic is the sum over the grids, not the mean
SUM_GRIDS = {"car_tile"}
# kernel 3 (bench.py's "kernel3" leg): the launches of one librsk call, summed per call
KERNEL3 = ("node_reduce", "nr_", "cut_cost", "cut_bins", "std_")
KERNEL3_CALL = {"node_reduce": ("nr_scan", "nr_colscan", "nr_place", "nr_sum", "nr_spill"),
                "load_std": ("std_partial", "std_merge"), "cut_cost": ("cut_cost_wave", "cut_bins_sum")}


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
    ap.add_argument("--src", required=True, help="a tools/gpu_prof.sh output directory")
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
        if not k.startswith("car") and not k.startswith(KERNEL3) and k not in ("pick_node",):
            continue
        e = {"grid": int(grid), "launches": len(durs), "avg_us": round(sum(durs) / len(durs) / 1e3, 2)}
        for c, d in pmc.items():
            v = d.get((k, grid))
            if v:
                e[c] = round(sum(v) / len(v), 1)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["read_bytes_per_launch"] = int(2 * e["FETCH_SIZE"] * 1024)   # x2: gfx950 FETCH_SIZE correction
            e["write_bytes_per_launch"] = int(e["WRITE_SIZE"] * 1024)
            e["hbm_bytes_per_launch"] = e["read_bytes_per_launch"] + e["write_bytes_per_launch"]
            e["hbm_bytes_per_launch_fetch_raw"] = int((e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024)
            e["hbm_GBps"] = round(e["hbm_bytes_per_launch"] / (e["avg_us"] * 1e3), 1)
        summary[f"{k}@{grid}"] = e
    with open(os.path.join(prof, f"{args.tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    # per kernel name: launch-weighted traffic for bench.py's roofline.traffic
    by_kernel = collections.defaultdict(lambda: [0, 0, 0.0])
    for key, e in summary.items():
        if "hbm_bytes_per_launch" in e:
            k = key.split("@")[0]
            name = BENCH_NAME.get(k, k)
            b = by_kernel[name]
            b[0] += e["hbm_bytes_per_launch"]
            b[1] = 1 if name in SUM_GRIDS else b[1] + 1
            b[2] += e["avg_us"]
    path = os.path.join(prof, "pmc_traffic.json")
    try:
        with open(path) as f:
            traffic = json.load(f)
    except (OSError, ValueError):
        traffic = {}
    traffic.setdefault("note", "hbm_bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE) x 1024, per launch "
                               "(tools/pmc_summary.py); bench.py reads configs[config][kernel]")
    entry = traffic.setdefault("configs", {}).setdefault(args.config, {})
    entry.clear()
    for k, (bytes_, n, us) in by_kernel.items():
        entry[k] = {"S": args.S, "hbm_bytes_per_launch": bytes_ // max(n, 1), "avg_us": round(us / max(n, 1), 2),
                    "source": f"profiles/{args.tag}_summary.json"}
    # kernel 3: every launch of one call summed (durations and PMC bytes per call)
    k3 = {}
    for call, parts in KERNEL3_CALL.items():
        tot_b, tot_us, seen = 0, 0.0, []
        for key, e in summary.items():
            k = key.split("@")[0]
            if k in parts and "hbm_bytes_per_launch" in e:
                tot_b += e["hbm_bytes_per_launch"]
                tot_us += e["avg_us"]
                seen.append(k)
        if seen:
            k3[call] = {"S": args.S, "hbm_bytes_per_call": tot_b, "kernels_us_per_call": round(tot_us, 2),
                        "launches": sorted(seen), "source": f"profiles/{args.tag}_summary.json"}
    if k3:
        traffic.setdefault("kernel3", {})[args.config] = k3
    with open(path, "w") as f:
        json.dump(traffic, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
