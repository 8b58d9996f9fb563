#!/usr/bin/env python3
"""End-to-end latency of the drop-in placement calls.

Times ``rescheduling.communication`` / ``spread`` / ``binpack`` exactly as
main.py:78-91 calls them — cluster_monitoring dict in, created Deployment body
out through the test-side stub kubernetes client (tests/stubs; the API call
itself is out of scope) — on the synthetic 2k/64 and 100k/5k clusters, hazard
= nodes at >= 30 % CPU (harzard_detect.py).  Each call includes the
marshalling of the dict (rsk/cluster.py) and the librsk call on the GPU.

Beside each figure: the reference's own functions timed in the build container
through the same stub (SURVEY.md §6, 1 core of an 8-vCPU Xeon — a different
host CPU than the GPU box's).

    python tools/dropin_latency.py [--calls 50] [--out gpurun_out/dropin.json]
"""
import argparse
import copy
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests", "stubs"), os.path.join(REPO, "kubernetes-rescheduling_amd")]

SURVEY_MS = {  # SURVEY.md §6 "Measured this session": reference ms per call
    "2k64": {"communication": 0.147, "spread": 0.039, "binpack": 0.038},
    "100k5k": {"communication": 106.9, "spread": 30.5, "binpack": 40.3},
}
CONFIGS = {"2k64": (2000, 64), "100k5k": (100_000, 5_000)}


def info_for(name):
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": name, "namespace": "default", "labels": {"app": name}},
            "spec": {"replicas": 1, "template": {"metadata": {"labels": {"app": name}},
                                                 "spec": {"containers": [{"name": name}], "affinity": None}}}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import numpy as np
    import rescheduling as R
    from kubernetes import client
    from rsk import synth
    rows = []
    for cfg, (P, N) in CONFIGS.items():
        c = synth.make_cluster(P, N, S=1, seed=0)
        names, cm, rel = synth.to_cluster_monitoring(c, 0)
        hz = [n for n in names if cm[n]["cpu_pct"] >= 30]
        rng = np.random.default_rng(0)
        deps = [f"d{int(p)}" for p in rng.choice(P, args.calls + 3, replace=False)]
        for algo in ("communication", "spread", "binpack"):
            times = []
            for k, d in enumerate(deps):
                info = info_for(d)
                client.CREATED.clear()
                t0 = time.perf_counter()
                if algo == "communication":
                    R.communication(info, hz, cm, rel, names)
                elif algo == "spread":
                    R.spread(info, hz, cm)
                else:
                    R.binpack(info, hz, cm)
                dt = (time.perf_counter() - t0) * 1e3
                assert client.CREATED, "no Deployment created"
                if k >= 3:  # first calls: library load, context, caches
                    times.append(dt)
            t = np.array(times)
            row = {"config": cfg, "algo": algo, "calls": len(t), "median_ms": round(float(np.median(t)), 4),
                   "p90_ms": round(float(np.percentile(t, 90)), 4), "hazard_nodes": len(hz),
                   "reference_ms_survey": SURVEY_MS[cfg][algo]}
            row["speedup_vs_survey"] = round(row["reference_ms_survey"] / row["median_ms"], 2)
            rows.append(row)
            print(json.dumps(row), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
