#!/usr/bin/env python3
"""Generate tests/golden/snapshots.json and tests/golden/quantities.json from the
REFERENCE itself (snapshot replay and harness metrics).

Run ONLY in the build container (the reference does not travel to the GPU box):

    python -B tests/golden/make_snapshots.py [--reference /root/reference]

Like make_golden.py it puts the test-side ``kubernetes`` stub (tests/stubs)
ahead of the unmodified reference modules, fills the stub's in-memory cluster
with seeded random state (quantity strings in every unit the metrics server and
node status use, missing metrics, nodes missing from the node list, malformed
quantities, pods without owners or outside ``default``) and records, as plain
data, that state and what the reference computes from it:

* ``podmonitor.monitor()`` -> nodes_name, the default-namespace pod names and
  cluster_monitoring (or the exception type it raises);
* ``nodemonitor.node_resorce_std()``;
* ``communicationcost.communication_cost(relation)`` with main.py's relation.

``quantities.json`` holds unit_convertion.cpu_conversion / mem_conversion of
hand-picked corner spellings and seeded random ones (value or exception name).
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import random
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402  (stub path setup + reference loader)


def conv(f, s):
    try:
        return f(s)
    except Exception as e:  # noqa: BLE001
        return {"error": type(e).__name__}


CPU_CORNERS = ["53m", " 53m ", "53.9m", "-1.5m", "0m", "123456789n", "999999n", "1500000n", "2500000n",
               "500000n", "499u", "500u", "1500u", "2500u", "20", "0.5", "0.0005", "0.0015", "0.0025",
               "1e3m", "1E-3", "+2", "-0.5", ".5", "5.", "1_000m", "inf", "nan", "m", "", "  ", "1Mi",
               "5mm", "1e400", "12 m", "1.5e2n", "3\t", "0x10", "1e19", "9.3e18m", "４m", "1 m",
               "None", "1.", "-0", "123456789012345678n"]
MEM_CORNERS = ["536Mi", "1Gi", "16318712Ki", "7.5Gi", "0.1Ki", "8000000000", "1e3", "1K", "1M", "1G",
               "Ki", "1Ei", "8Ei", "1.5Pi", " 2Ti ", "-1Mi", "12.9", "1_024Ki", "nan", "1e400", "",
               "100Mi\n", "1ki", "1KiB", "3Zi", "None", "1e20", "9.2e18"]


def quantities(rng):
    out = {"cpu": [], "mem": []}
    for s in CPU_CORNERS:
        out["cpu"].append([s, conv(REF.UC.cpu_conversion, s)])
    for s in MEM_CORNERS:
        out["mem"].append([s, conv(REF.UC.mem_conversion, s)])
    for _ in range(600):
        k = rng.randrange(6)
        x = rng.choice([rng.randrange(0, 10 ** rng.randrange(1, 13)), round(rng.uniform(0, 64), rng.randrange(0, 7))])
        s = [f"{x}n", f"{x}u", f"{x}m", f"{x}", f"{x}e{rng.randrange(-3, 4)}", f"{rng.randrange(10**9)}n"][k]
        out["cpu"].append([s, conv(REF.UC.cpu_conversion, s)])
    for _ in range(600):
        k = rng.randrange(4)
        x = rng.choice([rng.randrange(0, 10 ** rng.randrange(1, 11)), round(rng.uniform(0, 4096), rng.randrange(0, 5))])
        s = [f"{x}{rng.choice(['Ki', 'Mi', 'Gi', 'Ti'])}", f"{x}", f"{int(x)}Ki", f"{x}Mi"][k]
        out["mem"].append([s, conv(REF.UC.mem_conversion, s)])
    return out


def cpu_str(rng, millis):
    k = rng.randrange(4)
    if k == 0:
        return f"{millis * 1_000_000 + rng.randrange(-499_999, 500_000)}n"
    if k == 1:
        return f"{millis * 1000 + rng.randrange(-500, 500)}u"
    if k == 2:
        return f"{millis}m"
    return f"{millis / 1000}"


def mem_str(rng, b):
    k = rng.randrange(3)
    if k == 0:
        return f"{b // 1024}Ki"
    if k == 1:
        return f"{b // 2**20}Mi"
    return f"{b}"


def fake_cluster(rng, case):
    nw = rng.randrange(1, 13)
    workers = [rng.choice(["worker", "node-", "w"]) + str(i + 1) for i in range(nw)]
    workers = list(dict.fromkeys(workers))
    caps = {n: rng.choice(["2", "4", "8", "16", "0.5", "3500m", "0"] if case % 7 == 3 else ["2", "4", "8", "16", "3500m"])
            for n in workers}
    nodes = [{"name": "master", "cpu_capacity": "4", "mem_capacity": "8Gi"}] if rng.random() < 0.7 else []
    for n in workers:
        nodes.append({"name": n, "cpu_capacity": caps[n],
                      "mem_capacity": rng.choice(["32Gi", "16318712Ki", "8000000000", "7.5Gi"])})
    rng.shuffle(nodes)
    node_usage = {}
    for nd in nodes:
        if nd["name"] != "master" and rng.random() < (0.15 if case % 5 == 1 else 0.0):
            continue  # no metrics for this node
        node_usage[nd["name"]] = {"cpu": cpu_str(rng, rng.randrange(0, 6000)),
                                  "memory": mem_str(rng, rng.randrange(2**28, 2**34))}
    if case % 11 == 4:
        node_usage["ghost"] = {"cpu": "100m", "memory": "1Gi"}  # not in the node list
    if case % 13 == 6 and node_usage:
        node_usage[rng.choice(list(node_usage))]["cpu"] = rng.choice(["abc", "1Mi", "inf"])
    pods, pod_usage = [], {"default": {}}
    for i in range(rng.randrange(0, 41)):
        dep = rng.choice([f"s{rng.randrange(20)}"] * 9 + [None])
        ns = "default" if rng.random() < 0.9 else "kube-system"
        on = rng.choice(workers + [None] * (1 if case % 3 == 0 else 0)) if workers else None
        name = f"{dep or 'bare'}-{case}-{i}"
        pods.append({"name": name, "namespace": ns, "node_name": on, "deployment": dep, "pod_ip": f"10.0.0.{i}"})
        if ns == "default" and rng.random() < 0.9:
            pod_usage["default"][name] = [{"cpu": cpu_str(rng, rng.randrange(0, 900)),
                                           "memory": mem_str(rng, rng.randrange(2**20, 2**30))}
                                          for _ in range(rng.randrange(1, 4))]
    if case % 17 == 8 and pod_usage["default"]:
        k = rng.choice(list(pod_usage["default"]))
        pod_usage["default"][k][0]["memory"] = "12XB"
    if case % 19 == 2:
        pod_usage = {"default": {}}
    return {"nodes": nodes, "node_usage": node_usage, "pods": pods, "pod_usage": pod_usage}


def run_reference(state, relation):
    from kubernetes import client as kc
    kc.reset()
    kc.FAKE.nodes = state["nodes"]
    kc.FAKE.node_usage = state["node_usage"]
    kc.FAKE.pods = state["pods"]
    kc.FAKE.pod_usage = state["pod_usage"]
    with contextlib.redirect_stdout(io.StringIO()):
        try:
            nodes_name, spods, cm = REF.PM.monitor()
            mon = {"nodes_name": nodes_name, "spods": [p.metadata.name for p in spods], "cluster_monitoring": cm}
        except Exception as e:  # noqa: BLE001
            mon = {"error": type(e).__name__}
        std = REF.NM.node_resorce_std()
        cost = REF.CC.communication_cost(relation)
    return {"monitor": mon, "std": None if std is None else float(std), "cost": cost}


def main():
    global REF
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    args = ap.parse_args()
    pkg = os.path.join(MG.REPO, "kubernetes-rescheduling_amd")
    sys.path[:] = [x for x in sys.path if os.path.abspath(x) != pkg]  # the drop-in would shadow the reference
    REF = MG.load_reference(args.reference)
    relation = MG.reference_relation(args.reference)
    rng = random.Random(20261016)
    with open(os.path.join(HERE, "quantities.json"), "w") as f:
        json.dump(quantities(rng), f, separators=(",", ":"))
    cases = []
    for case in range(120):
        state = fake_cluster(rng, case)
        cases.append({"state": state, "expect": run_reference(state, relation)})
    with open(os.path.join(HERE, "snapshots.json"), "w") as f:
        json.dump({"relation": relation, "cases": cases}, f, separators=(",", ":"))
    errs = sum("error" in c["expect"]["monitor"] for c in cases)
    print(f"wrote {len(cases)} snapshot cases ({errs} where monitor raises)")


REF = None
if __name__ == "__main__":
    main()
