#!/usr/bin/env python3
"""End-to-end latency of the drop-in placement calls.

Times ``rescheduling.communication`` / ``spread`` / ``binpack`` / ``random``
exactly as main.py:78-91 calls them — cluster_monitoring dict in, created
Deployment body out through the test-side stub kubernetes client (tests/stubs;
the API call itself is out of scope).  Each call includes the marshalling of the
dict (rsk/cluster.py) and the librsk call on the GPU.  Configs:

* ``wm3``    — the reference's operating point (README.md:44-48, BASELINE
  config 1): the µBench workmodelC services on 3 workers, the 103 three-worker
  snapshots of tests/golden/wm_snapshots.json replayed in turn;
* ``2k64``, ``100k5k`` — the synthetic clusters, hazard = nodes
  at >= 30 % CPU (harzard_detect.py).

Beside each figure: the reference's own functions timed the same way in the
build container (tools/ref_latency.py -> profiles/ref_latency_container.json;
a different host CPU than the GPU box's), and the part of the drop-in call
spent outside librsk (``host_ms``: marshalling + affinity patch + create).

    python tools/dropin_latency.py [--calls 50] [--out gpurun_out/dropin.json]
"""
import argparse
import copy
import json
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests", "stubs"), os.path.join(REPO, "kubernetes-rescheduling_amd")]

SURVEY_MS = {  # SURVEY.md §6 "Measured this session": reference ms per call
    "2k64": {"communication": 0.147, "spread": 0.039, "binpack": 0.038, "random": 0.023},
    "100k5k": {"communication": 106.9, "spread": 30.5, "binpack": 40.3, "random": 44.3},
}
SYNTH = {"2k64": (2000, 64), "100k5k": (100_000, 5_000)}
ALGOS = ("communication", "spread", "binpack", "random")


def info_for(name):
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": name, "namespace": "default", "labels": {"app": name}},
            "spec": {"replicas": 1, "template": {"metadata": {"labels": {"app": name}},
                                                 "spec": {"containers": [{"name": name}], "affinity": None}}}}


def cases(calls):
    """(config, factory) pairs; factory() yields calls + 3 argument tuples
    (deployment_info, hazard list, cluster_monitoring, relation, nodes_name)."""
    import numpy as np
    from rsk import synth
    with open(os.path.join(REPO, "tests", "golden", "wm_snapshots.json")) as f:
        wm = json.load(f)
    snaps = [s for s in wm["snapshots"] if len(s["nodes_name"]) == 3]
    rel = wm["relation"]

    def wm3():
        for k in range(calls + 3):
            s = snaps[k % len(snaps)]
            yield (copy.deepcopy(s["deployment_info"]), list(s["hazard"]), s["cluster_monitoring"], rel,
                   list(s["nodes_name"]))
    out = [("wm3", wm3)]
    for cfg, (P, N) in SYNTH.items():
        c = synth.make_cluster(P, N, S=1, seed=0)
        names, cm, srel = synth.to_cluster_monitoring(c, 0)
        hz = [n for n in names if cm[n]["cpu_pct"] >= 30]
        deps = [f"d{int(p)}" for p in np.random.default_rng(0).choice(P, calls + 3, replace=False)]

        def synth_iter(deps=deps, hz=hz, cm=cm, srel=srel, names=names):
            for d in deps:
                yield info_for(d), hz, cm, srel, names
        out.append((cfg, synth_iter))
    return out


def call(R, algo, args):
    info, hz, cm, rel, names = args
    if algo == "communication":
        return R.communication(info, hz, cm, rel, names)
    if algo == "spread":
        return R.spread(info, hz, cm)
    if algo == "binpack":
        return R.binpack(info, hz, cm)
    return R.random(info, hz, names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=50)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import numpy as np
    import rescheduling as R
    from kubernetes import client
    from rsk import _lib
    ref = {}
    try:
        with open(os.path.join(REPO, "profiles", "ref_latency_container.json")) as f:
            for r in json.load(f)["rows"]:
                ref[(r["config"], r["algo"])] = r["median_ms"]
    except (OSError, ValueError, KeyError):
        pass
    ctx = _lib.default_context()
    rows = []
    for cfg, factory in cases(args.calls):
        for algo in ALGOS:
            times, dev = [], []
            for k, a in enumerate(factory()):
                client.CREATED.clear()
                random.seed(k)
                ctx.reset_profiling()
                ctx.set_profiling(True)
                t0 = time.perf_counter()
                try:
                    call(R, algo, a)
                except (RuntimeError, ValueError):
                    pass
                dt = (time.perf_counter() - t0) * 1e3
                ctx.set_profiling(False)
                kern = sum(ctx.kernel_time(n)[0] for n in ("car_row", "car_tile", "car_prep", "car_side", "spread",
                                                            "binpack", "random_candidates"))
                if k >= 3:  # first calls: library load, context, caches
                    times.append(dt)
                    dev.append(kern)
            t = np.array(times)
            row = {"config": cfg, "algo": algo, "calls": len(t), "median_ms": round(float(np.median(t)), 4),
                   "p90_ms": round(float(np.percentile(t, 90)), 4),
                   "kernel_ms_median": round(float(np.median(dev)), 4)}
            r = ref.get((cfg, algo))
            if r is not None:
                row["reference_ms_container"] = r
                row["speedup_vs_reference_container"] = round(r / row["median_ms"], 2)
            s = SURVEY_MS.get(cfg, {}).get(algo)
            if s is not None:
                row["reference_ms_survey"] = s
            rows.append(row)
            print(json.dumps(row), flush=True)
    if args.out:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
