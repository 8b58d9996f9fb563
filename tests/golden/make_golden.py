#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run ONLY in the build container (the reference does not travel to the GPU box):

    python -B tests/golden/make_golden.py [--reference /root/reference]

It puts a test-side stub ``kubernetes`` package (tests/stubs) ahead of the
reference on ``sys.path``, imports the reference modules unmodified, drives
them against an in-memory fake cluster, and writes plain-JSON inputs and
expected outputs:

* ``wm_snapshots.json`` — 256 monitor→detect→evict→place snapshots of the µBench
  workmodelC services on 2-12 workers, every algorithm's created body (or
  exception); plus the reference's hard-coded relation (main.py:31-52, read with
  ``ast.literal_eval`` as data) and the workmodel's call graph.
* ``edge_cases.json`` — hand-built inputs for every tie / error corner of §8a.
* ``synth.json`` — CAR targets for sampled pods of the 2k/64 (S=8) and 100k/5k
  synthetic clusters, spread/binpack/random decisions, and input checksums.
* ``metrics.json`` — communication_cost, node_resorce_std, cpu_pct and
  detection/pick_max_pod values.

Nothing from the reference's source is copied: only values it computes (and the
relation dict / workmodel graph, which are data) are stored.
"""
from __future__ import annotations

import argparse
import ast
import copy
import hashlib
import json
import os
import random as pyrandom
import sys
from types import SimpleNamespace as NS

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests", "stubs"))
sys.path.insert(0, os.path.join(REPO, "kubernetes-rescheduling_amd"))

ALGOS = ["spread", "binpack", "random", "kubescheduling", "communication"]


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:16]


def load_reference(ref_dir):
    sys.path.insert(0, ref_dir)  # ahead of the package dir (its rescheduling.py is the drop-in)
    import rescheduling as R  # noqa: E402  (the reference module)
    import main as M
    import harzard_detect as H
    import delete_replaced_pod as D
    import podmonitor as PM
    import communicationcost as CC
    import nodemonitor as NM
    import get_resource_usage as GRU
    import unit_convertion as UC
    for mod in (R, M, H, D, PM, CC, NM, GRU, UC):
        assert os.path.dirname(os.path.abspath(mod.__file__)) == os.path.abspath(ref_dir), mod
    return NS(R=R, M=M, H=H, D=D, PM=PM, CC=CC, NM=NM, GRU=GRU, UC=UC)


def reference_relation(ref_dir):
    """The relation dict literal assigned in main.main (main.py:31-52), as data."""
    with open(os.path.join(ref_dir, "main.py"), "r", encoding="utf-8") as f:
        tree = ast.parse(f.read())
    for node in ast.walk(tree):
        if isinstance(node, ast.Assign) and any(getattr(t, "id", None) == "relation" for t in node.targets):
            return ast.literal_eval(node.value)
    raise RuntimeError("relation literal not found")


class Quiet:
    """Silence the reference's prints while it runs."""

    def __enter__(self):
        self._o = sys.stdout
        sys.stdout = open(os.devnull, "w")

    def __exit__(self, *a):
        sys.stdout.close()
        sys.stdout = self._o


def run_algo(ref, client, algo, info, hazard, cm, relation, nodes_name, seed):
    info = copy.deepcopy(info)
    cm = copy.deepcopy(cm)
    client.CREATED.clear()
    out = {"exception": None, "body": None, "returned": None}
    try:
        with Quiet():
            if algo == "spread":
                r = ref.R.spread(info, list(hazard), cm)
            elif algo == "binpack":
                r = ref.R.binpack(info, list(hazard), cm)
            elif algo == "random":
                pyrandom.seed(seed)
                r = ref.R.random(info, list(hazard), list(nodes_name))
            elif algo == "kubescheduling":
                r = ref.R.kubescheduling(info, list(hazard))
            else:
                r = ref.R.communication(info, list(hazard), cm, relation, list(nodes_name))
        out["returned"] = r
    except Exception as e:  # noqa: BLE001 - the reference's own error behaviour is the fixture
        out["exception"] = [type(e).__name__, str(e)]
    out["body"] = client.CREATED[-1][1] if client.CREATED else None
    if out["body"] is None:
        out["info_after"] = info  # the reference mutates deployment_info in place (even on error)
    return out


# ----------------------------------------------------------------------------------
# workmodelC snapshots through monitor → detection → pod_delete → edit_cluster
# ----------------------------------------------------------------------------------

def _deployment_obj(name, affinity):
    cont = NS(name=name, image=f"msvcbench/microservice:{name}", imagePullPolicy="Always",
              ports=[{"containerPort": 8080, "name": "http", "protocol": "TCP"}],
              env=None, resources={"requests": {"cpu": "100m"}}, volumeMounts=None, args=["--x"])
    tmpl_spec = NS(containers=[cont], volumes=None, termination_grace_period_seconds=30,
                   node_selector=None, affinity=affinity)
    return NS(api_version="apps/v1", kind="Deployment",
              metadata=NS(name=name, namespace="default", labels={"app": name}),
              spec=NS(replicas=1, selector=NS(match_labels={"app": name}, match_expressions=None),
                      strategy={"type": "RollingUpdate"},
                      template=NS(metadata=NS(labels={"app": name}, annotations=None), spec=tmpl_spec)))


def _cpu_str(m, rng):
    k = rng.integers(0, 3)
    if k == 0:
        return f"{m}m"
    if k == 1:
        return f"{m * 1_000_000 + int(rng.integers(0, 999_999))}n"
    return f"{m * 1000 + int(rng.integers(0, 999))}u"


def workmodel_snapshots(ref, client, relation, n_snap=256, seed=1234):
    services = list(relation.keys())
    rng = np.random.default_rng(seed)
    snaps = []
    skipped = 0
    i = 0
    while len(snaps) < n_snap:
        i += 1
        client.reset() if hasattr(client, "reset") else None
        K = int(rng.choice([2, 3, 3, 3, 4, 5, 8, 12]))
        names = [f"worker{j + 1}" for j in range(K)]
        if rng.random() < 0.3:
            rng.shuffle(names)
        nodes = [{"name": n, "cpu_capacity": str(int(rng.choice([4, 8, 8, 16]))), "mem_capacity": "16Gi"}
                 for n in names]
        if rng.random() < 0.3:
            nodes.insert(int(rng.integers(0, len(nodes) + 1)), {"name": "master", "cpu_capacity": "4", "mem_capacity": "8Gi"})
        cap_m = {n["name"]: int(n["cpu_capacity"]) * 1000 for n in nodes}
        pods = []
        pod_usage = {}
        node_cpu = {n: 0 for n in cap_m}
        for svc in services:
            reps = 1 if rng.random() < 0.9 else 2
            for r in range(reps):
                node = names[int(rng.integers(0, K))]
                pname = f"{svc}-{int(rng.integers(0, 1 << 30)):08x}"
                cpu = int(rng.integers(1, 400)) if rng.random() < 0.8 else int(rng.choice([100, 200]))
                pods.append({"name": pname, "namespace": "default", "node_name": node, "deployment": svc})
                pod_usage[pname] = [{"cpu": _cpu_str(cpu, rng), "memory": f"{int(rng.integers(10, 200))}Mi"}]
                node_cpu[node] += cpu
        if rng.random() < 0.2:  # a pod outside the default namespace is invisible to the loop
            pods.append({"name": "coredns-x", "namespace": "kube-system", "node_name": names[0], "deployment": "coredns"})
        node_usage = {}
        for n in cap_m:
            bg = int(rng.integers(0, int(cap_m[n] * 0.36)))
            if rng.random() < 0.15:
                bg = int(cap_m[n] * 0.30) - node_cpu[n]  # land exactly on the threshold
                bg = max(bg, 0)
            node_usage[n] = {"cpu": _cpu_str(bg + node_cpu[n], rng), "memory": f"{int(rng.integers(1000, 9000))}Mi"}
        client.FAKE.reset()
        client.FAKE.nodes = nodes
        client.FAKE.node_usage = node_usage
        client.FAKE.pods = pods
        client.FAKE.pod_usage = {"default": pod_usage}
        for svc in services:
            aff = None
            if rng.random() < 0.25:
                aff = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                    "nodeSelectorTerms": [{"matchExpressions": [{"key": "disk", "operator": "In", "values": ["ssd"]}]}]}}}
            elif rng.random() < 0.1:
                aff = {"podAntiAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": []}}
            client.FAKE.deployments[("default", svc)] = _deployment_obj(svc, aff)
        with Quiet():
            nodes_name, spods, cm = ref.PM.monitor()
            most, hazard = ref.H.detection(nodes_name, cm)
        if not most:
            skipped += 1
            continue
        with Quiet():
            res = ref.D.pod_delete(most, spods, "default", relation)
        if res is None:
            skipped += 1
            continue
        info, dpodname = res
        if not info:
            skipped += 1
            continue
        cm = ref.M.edit_cluster(cm, dpodname, most)
        seed_k = 1000 + len(snaps)
        outs = {a: run_algo(ref, client, a, info, hazard, cm, relation, nodes_name, seed_k) for a in ALGOS}
        snaps.append({"nodes_name": nodes_name, "hazard": hazard, "most": most, "evicted": dpodname,
                      "cluster_monitoring": cm, "deployment_info": info, "random_seed": seed_k,
                      "results": outs})
    return snaps, skipped


# ----------------------------------------------------------------------------------
# hand-built edge cases
# ----------------------------------------------------------------------------------

def _node(cap, use, pods, pct=None):
    if pct is None:
        pct = int(round(use / cap * 100)) if cap else -1
    return {"node_cpu_capacity": cap, "node_cpu_usage": use, "cpu_pct": pct,
            "node_mem_capacity": 1 << 34, "node_mem_usage": 1 << 30, "mem_pct": 6, "pods": pods}


def _pod(name, dep, cpu=10):
    return {"podname": name, "deploymentname": dep, "pod_cpu_usage": cpu, "pod_mem_usage": 1 << 20}


def _info(name, affinity=None):
    return {"apiVersion": "apps/v1", "kind": "Deployment",
            "metadata": {"name": name, "namespace": "default", "labels": {"app": name}},
            "spec": {"replicas": 1, "template": {"metadata": {"labels": {"app": name}},
                                                 "spec": {"containers": [{"name": name}], "affinity": affinity}}}}


def edge_cases(ref, client):
    rel = {"a": ["b", "c"], "b": ["a"], "c": ["a"], "x": ["b", "b", "c"], "lonely": []}
    cases = []

    def add(name, info, hazard, cm, nodes_name, relation=rel, seed=7):
        outs = {a: run_algo(ref, client, a, info, hazard, cm, relation, nodes_name, seed) for a in ALGOS}
        cases.append({"name": name, "deployment_info": info, "hazard": hazard, "cluster_monitoring": cm,
                      "nodes_name": nodes_name, "relations": relation, "random_seed": seed, "results": outs})

    cm = {"w1": _node(4000, 3000, [_pod("b-1", "b")]), "w2": _node(4000, 3500, [_pod("c-1", "c")])}
    add("all_hazard", _info("a"), ["w1", "w2"], cm, ["w1", "w2"])
    # CAR: two best nodes, both overloaded (rem <= -1) -> nodeName None
    cm = {"w1": _node(4000, 4001, [_pod("b-1", "b")]), "w2": _node(4000, 4500, [_pod("c-1", "c")]),
          "w3": _node(4000, 100, [])}
    add("car_overloaded_tie_none", _info("a"), [], cm, ["w1", "w2", "w3"])
    # rem exactly -1 and 0
    cm = {"w1": _node(4000, 4001, [_pod("b-1", "b")]), "w2": _node(4000, 4000, [_pod("c-1", "c")])}
    add("car_rem_minus1_vs_0", _info("a"), [], cm, ["w1", "w2"])
    cm = {"w1": _node(4000, 4001, [_pod("b-1", "b")]), "w2": _node(4000, 4001, [_pod("c-1", "c")])}
    add("car_rem_all_minus1", _info("a"), [], cm, ["w1", "w2"])
    # CAR: single best overloaded -> still chosen
    cm = {"w1": _node(4000, 9000, [_pod("b-1", "b"), _pod("c-1", "c")]), "w2": _node(4000, 10, [])}
    add("car_single_best_overloaded", _info("a"), [], cm, ["w1", "w2"])
    # CAR: no related pods anywhere -> every candidate scores 0 -> max remaining CPU
    cm = {"w1": _node(4000, 1000, [_pod("z-1", "z")]), "w2": _node(4000, 500, []),
          "w3": _node(4000, 500, [])}
    add("car_all_zero_scores", _info("lonely"), [], cm, ["w1", "w2", "w3"])
    add("car_unknown_deployment", _info("nope"), ["w2"], cm, ["w1", "w2", "w3"])
    # equal remaining CPU among tied best -> first in nodes_name order
    cm = {"w1": _node(4000, 1000, [_pod("b-1", "b")]), "w2": _node(4000, 1000, [_pod("c-1", "c")])}
    add("car_tie_equal_rem_order", _info("a"), [], cm, ["w2", "w1"])
    # duplicate rel entries do not double count; None deployment never matches
    cm = {"w1": _node(4000, 1000, [_pod("b-1", "b"), _pod("n-1", None)]),
          "w2": _node(4000, 10, [_pod("c-1", "c"), _pod("c-2", "c")])}
    add("car_duplicate_rel", _info("x"), [], cm, ["w1", "w2"])
    # name-order ties: 'w10' < 'w2' in str order
    cm = {"w2": _node(4000, 1000, [_pod("p1", "q")]), "w10": _node(4000, 1000, [_pod("p2", "q")]),
          "w1": _node(4000, 1000, [_pod("p3", "q")]), "w9": _node(4000, 1000, [_pod("p4", "q")])}
    add("name_order_ties", _info("a"), ["w1"], cm, ["w2", "w10", "w1", "w9"])
    cm = {"w2": _node(4000, 1000, []), "w10": _node(4000, 1000, []), "w3": _node(4000, 2000, [])}
    add("binpack_pct_then_name", _info("a"), [], cm, ["w2", "w10", "w3"])
    # hazard list naming unknown nodes; affinity already carrying nodeSelectorTerms (extend)
    aff = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": [{"matchExpressions": [{"key": "zone", "operator": "In", "values": ["a"]}]}]}}}
    cm = {"w1": _node(4000, 100, [_pod("b-1", "b")]), "w2": _node(4000, 100, [])}
    add("affinity_extend_and_unknown_hazard", _info("a", aff), ["ghost", "w2"], cm, ["w1", "w2"])
    aff2 = {"nodeAffinity": {"preferredDuringSchedulingIgnoredDuringExecution": [{"weight": 1}]},
            "podAffinity": {"x": 1}}
    add("affinity_merge_other_keys", _info("a", aff2), ["w2"], cm, ["w1", "w2"])
    # single candidate
    add("single_candidate", _info("a"), ["w1"], cm, ["w1", "w2"])
    # nodes_name with a node absent from hazard but pods only on hazard nodes
    cm = {"w1": _node(4000, 3900, [_pod("b-1", "b"), _pod("c-1", "c")]), "w2": _node(4000, 200, []),
          "w3": _node(8000, 200, [])}
    add("related_only_on_hazard", _info("a"), ["w1"], cm, ["w1", "w2", "w3"])
    # replicas of the moving deployment itself are counted when it relates to itself
    rel2 = dict(rel)
    rel2["self"] = ["self", "b"]
    cm = {"w1": _node(4000, 100, [_pod("self-1", "self")]), "w2": _node(4000, 100, [_pod("b-1", "b")]),
          "w3": _node(4000, 50, [])}
    add("self_relation_replica", _info("self"), [], cm, ["w1", "w2", "w3"], relation=rel2)
    # larger random name-collision stress for spread/binpack on 12 workers
    rng = np.random.default_rng(99)
    for t in range(24):
        K = 12
        names = [f"w{j + 1}" for j in range(K)]
        rng.shuffle(names)
        cm = {}
        for n in names:
            npods = int(rng.integers(0, 3))
            cm[n] = _node(4000, int(rng.choice([1000, 1200, 1200, 4100])),
                          [_pod(f"{n}-p{k}", str(rng.choice(["a", "b", "c", "q"]))) for k in range(npods)])
        hz = [n for n in names if rng.random() < 0.3]
        add(f"stress_{t}", _info(str(rng.choice(["a", "b", "c", "x"]))), hz, cm, list(names), seed=100 + t)
    return cases


# ----------------------------------------------------------------------------------
# synthetic clusters (rsk.synth) through the reference
# ----------------------------------------------------------------------------------

def synth_car(ref, client, c, s, pods, relations, names, cm_base):
    """Reference CAR decision for pod p of scenario s: evict p from its node
    (edit_cluster, main.py:73) then communication() (rescheduling.py:174)."""
    with Quiet():
        _, hazard = ref.H.detection(names, cm_base)
    out = []
    S = c.S
    for p in pods:
        node = names[int(c.assign[p * S + s])]
        cm = cm_base
        pod_entry = next(x for x in cm[node]["pods"] if x["deploymentname"] == f"d{p}")
        saved = list(cm[node]["pods"])
        ref.M.edit_cluster(cm, pod_entry["podname"], node)
        assert len(cm[node]["pods"]) == len(saved) - 1
        client.CREATED.clear()
        info = _info(f"d{p}")
        try:
            with Quiet():
                ref.R.communication(info, hazard, cm, relations, names)
            tgt = client.CREATED[-1][1]["spec"]["template"]["spec"]["nodeName"]
            out.append(names.index(tgt) if tgt is not None else -1)
        except ValueError:
            out.append(-2)
        cm[node]["pods"][:] = saved
    return out, hazard


def synth_fixtures(ref, client):
    from rsk import synth
    res = {}
    for tag, P, N, S, npods, per_s in [("2k64", 2000, 64, 8, 512, 64), ("100k5k", 100000, 5000, 1, 64, 64)]:
        c = synth.make_cluster(P, N, S=S, seed=0)
        rng = np.random.default_rng(4242)
        entry = {"P": P, "N": N, "S": S, "seed": 0, "nnz": c.nnz, "max_degree": int(np.diff(c.row_ptr).max()),
                 "checksums": {k: sha(getattr(c, k)) for k in ("row_ptr", "col_idx", "assign", "use_cpu", "hazard", "cpu_pct")},
                 "scenarios": []}
        for s in range(S):
            names, cm, relations = synth.to_cluster_monitoring(c, s)
            if s == 0:
                pods = sorted(set(rng.choice(P, npods, replace=False).tolist())
                              | {int(np.argmax(np.diff(c.row_ptr)))} | {0, P - 1})
            else:
                pods = sorted(rng.choice(P, per_s, replace=False).tolist())
            tg, hazard = synth_car(ref, client, c, s, pods, relations, names, cm)
            sc = {"s": s, "pods": pods, "car_target": tg, "n_hazard": len(hazard)}
            for a in ("spread", "binpack", "random"):
                o = run_algo(ref, client, a, _info("d0"), hazard, cm, relations, names, 77 + s)
                spec = o["body"]["spec"]["template"]["spec"] if o["body"] else None
                if a == "random":
                    sc[a] = names.index(spec["nodeName"]) if spec else -2
                else:
                    sc[a] = names.index(spec["nodeSelector"]["kubernetes.io/hostname"]) if spec else -2
            sc["random_seed"] = 77 + s
            entry["scenarios"].append(sc)
            print(f"  synth {tag} s={s}: {len(pods)} pods, {len(hazard)} hazard", file=sys.stderr)
        res[tag] = entry
    return res


# ----------------------------------------------------------------------------------
# metrics: communication_cost, node_resorce_std, cpu_pct, detection, pick_max_pod
# ----------------------------------------------------------------------------------

def metric_fixtures(ref, client, relation):
    out = {"communication_cost": [], "node_std": [], "cpu_pct": [], "detection": [], "pick_max_pod": [],
           "unit": []}
    rng = np.random.default_rng(555)
    services = list(relation.keys())
    for t in range(48):
        client.FAKE.reset()
        K = int(rng.choice([2, 3, 5]))
        names = [f"worker{j + 1}" for j in range(K)]
        pods = []
        for svc in services:
            if t % 6 == 5 and rng.random() < 0.15:
                continue  # deployment missing entirely -> relation lookups give None (x.5 costs)
            for r in range(1 if rng.random() < 0.85 else 2):
                node = names[int(rng.integers(0, K))] if rng.random() > 0.05 else None
                pods.append({"name": f"{svc}-{t}-{r}", "namespace": "default", "node_name": node, "deployment": svc})
        client.FAKE.pods = pods
        with Quiet():
            cost = ref.CC.communication_cost(relation)
        out["communication_cost"].append({"pods": pods, "relation": relation, "cost": cost})
    # synthetic 2k64 base assignment: deployment-level cut cost
    from rsk import synth
    c = synth.make_cluster(2000, 64, S=1, seed=0)
    names, cm, relations = synth.to_cluster_monitoring(c, 0)
    client.FAKE.reset()
    client.FAKE.pods = [{"name": f"pod-{p}", "namespace": "default", "node_name": names[int(c.assign[p])],
                         "deployment": f"d{p}"} for p in range(c.P)]
    with Quiet():
        out["synth_2k64_cost"] = ref.CC.communication_cost(relations)
    out["synth_2k64_checksum"] = sha(c.assign)

    for t in range(40):
        client.FAKE.reset()
        K = int(rng.integers(1, 9))
        nodes, usage = [], {}
        for j in range(K):
            nm = f"n{j}" if not (t % 7 == 3 and j == 0) else "master"
            capc = str(int(rng.choice([1, 2, 4, 8, 16, 0]))) if t % 5 == 4 else str(int(rng.choice([2, 4, 8])))
            nodes.append({"name": nm, "cpu_capacity": capc, "mem_capacity": "32Gi"})
            usage[nm] = {"cpu": _cpu_str(int(rng.integers(0, 8000)), rng), "memory": "1Gi"}
        client.FAKE.nodes = nodes
        client.FAKE.node_usage = usage
        with Quiet():
            v = ref.NM.node_resorce_std()
            nu = ref.GRU.get_nodes_usage(client.CoreV1Api())
        out["node_std"].append({"nodes": nodes, "usage": usage, "std": None if v is None else float(v)})
        out["cpu_pct"].append({"nodes": nodes, "usage": usage,
                               "node_res_usage": {k: list(v2) for k, v2 in nu.items()}})
    # cpu_pct rounding corner cases: exact .5 boundaries (round half even)
    corner = []
    for cap in (1000, 2000, 4000, 64000, 3):
        for use in range(0, 2 * cap + 1, max(1, cap // 200)):
            corner.append([use, cap])
    corner += [[5, 1000], [15, 1000], [25, 1000], [35, 1000], [1, 3], [2, 3], [7, 8], [5, 0]]
    vals = []
    for use, cap in corner:
        client.FAKE.reset()
        client.FAKE.nodes = [{"name": "n", "cpu_capacity": f"{cap}m", "mem_capacity": "1Gi"}]
        client.FAKE.node_usage = {"n": {"cpu": f"{use}m", "memory": "1Mi"}}
        with Quiet():
            nu = ref.GRU.get_nodes_usage(client.CoreV1Api())
        vals.append(nu["n"][1] if "n" in nu else None)
    out["cpu_pct_corner"] = {"pairs": corner, "pct": vals}
    for t in range(64):
        K = int(rng.integers(1, 8))
        names = [f"n{j}" for j in range(K)]
        cm = {n: {"cpu_pct": int(rng.choice([10, 29, 30, 31, 55, 55, 80]))} for n in names}
        most, hz = ref.H.detection(names, cm)
        out["detection"].append({"nodes_name": names, "cpu_pct": [cm[n]["cpu_pct"] for n in names],
                                 "most": most, "hazard": hz})
    for t in range(64):
        K = int(rng.integers(1, 4))
        spods = []
        usage = {}
        for k in range(int(rng.integers(0, 10))):
            nm = f"p{k}"
            node = f"n{int(rng.integers(0, K))}"
            spods.append(NS(metadata=NS(name=nm), spec=NS(node_name=node)))
            usage[nm] = (int(rng.choice([5, 10, 10, 300])), 1)
        most = f"n{int(rng.integers(0, K))}"
        p = ref.D.pick_max_pod(most, spods, usage)
        out["pick_max_pod"].append({"pods": [[x.metadata.name, x.spec.node_name, usage[x.metadata.name][0]] for x in spods],
                                    "most": most, "picked": None if p is None else p.metadata.name})
    for s in ["53m", "123456789n", "250u", "20", "0.5", "1500m", "999999n", "1500000n", "2500000n", "499u", "500u", "1500u"]:
        out["unit"].append(["cpu", s, ref.UC.cpu_conversion(s)])
    for s in ["536Mi", "1Gi", "1.5Gi", "1024Ki", "100", "3Ti"]:
        out["unit"].append(["mem", s, ref.UC.mem_conversion(s)])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    ref = load_reference(args.reference)
    from kubernetes import client
    relation = reference_relation(args.reference)
    with open(os.path.join(args.reference, "workmodelC.json"), "r", encoding="utf-8") as f:
        wm = json.load(f)
    calls = {s: [t for g in spec.get("external_services", []) for t in g.get("services", [])]
             for s, spec in wm.items()}
    only = set(args.only.split(",")) if args.only else None

    def dump(name, obj):
        with open(os.path.join(HERE, name), "w", encoding="utf-8") as f:
            json.dump(obj, f, separators=(",", ":"), sort_keys=False)
        print(f"wrote {name} ({os.path.getsize(os.path.join(HERE, name))} B)", file=sys.stderr)

    if not only or "workmodel" in only:
        snaps, skipped = workmodel_snapshots(ref, client, relation)
        dump("wm_snapshots.json", {"relation": relation, "workmodel_calls": calls, "snapshots": snaps,
                                 "skipped_stable_rounds": skipped})
    if not only or "edge" in only:
        dump("edge_cases.json", {"cases": edge_cases(ref, client)})
    if not only or "metrics" in only:
        dump("metrics.json", metric_fixtures(ref, client, relation))
    if not only or "synth" in only:
        dump("synth.json", synth_fixtures(ref, client))


if __name__ == "__main__":
    main()
