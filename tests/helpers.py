"""Shared helpers for the parity tests.

``oracle_decision`` marshals one golden snapshot with the product's host
marshaller (rsk.cluster) and decides with the CPU oracle; ``dropin_decision``
calls our drop-in ``rescheduling`` module exactly as main.py does and reads the
created body back from the stub kubernetes client.  Both are compared with what
the reference itself produced (tests/golden/*.json).
"""
from __future__ import annotations

import copy
import random as pyrandom

ALGOS = ["spread", "binpack", "random", "kubescheduling", "communication"]


def golden_decision(res):
    """(exception type or None, nodeName, nodeSelector) of a golden result."""
    if res["exception"]:
        return (res["exception"][0], None, None)
    spec = res["body"]["spec"]["template"]["spec"]
    return (None, spec.get("nodeName"), spec.get("nodeSelector"))


def oracle_decision(algo, case, relations):
    from oracle import oracle as orc
    from rsk import cluster

    hz, cm, nodes_name = case["hazard"], case["cluster_monitoring"], case["nodes_name"]
    info = case["deployment_info"]
    if algo == "kubescheduling":
        return (None, None, None)
    if algo == "communication":
        req = cluster.car_request(info["metadata"]["name"], hz, cm, relations, nodes_name)
        N = len(req.nodes)
        if N == 0 or req.hazard.all():
            return ("ValueError", None, None)
        t, _ = orc.car(req.row_ptr, req.col_idx, req.assign, 1, req.cap_cpu, req.use_cpu, req.hazard, N, rows=[0])
        t = int(t[0])
        assert t != -2
        return (None, None if t < 0 else req.nodes[t], None)
    if algo in ("spread", "binpack"):
        tab = cluster.node_table(hz, cm, "pods" if algo == "spread" else "cpu_pct")
        if not tab.names or tab.hazard.all():
            return ("RuntimeError", None, None)
        f = orc.spread if algo == "spread" else orc.binpack
        n = int(f(tab.value, tab.name_rank, tab.hazard, len(tab.names), 1)[0])
        return (None, None, {"kubernetes.io/hostname": tab.names[n]})
    # random: candidates[Random(seed)._randbelow(len)] (main.py seeds nothing; the
    # fixture generator called random.seed(seed) right before the call)
    mask = cluster.candidate_mask(hz, nodes_name)
    cnt = int((mask == 0).sum())
    if cnt == 0:
        return ("RuntimeError", None, None)
    r = orc.py_randbelow(case["random_seed"], cnt)
    cands = [n for n, h in zip(nodes_name, mask) if not h]
    return (None, cands[r], None)


def dropin_decision(algo, case, relations):
    """Run our drop-in like main.py:78-91; return (exc, body, info_after)."""
    import rescheduling as R
    from kubernetes import client

    info = copy.deepcopy(case["deployment_info"])
    cm = copy.deepcopy(case["cluster_monitoring"])
    hz = list(case["hazard"])
    nodes_name = list(case["nodes_name"])
    client.CREATED.clear()
    exc = None
    try:
        if algo == "spread":
            R.spread(info, hz, cm)
        elif algo == "binpack":
            R.binpack(info, hz, cm)
        elif algo == "random":
            pyrandom.seed(case["random_seed"])
            R.random(info, hz, nodes_name)
        elif algo == "kubescheduling":
            R.kubescheduling(info, hz)
        else:
            R.communication(info, hz, cm, relations, nodes_name)
    except Exception as e:  # noqa: BLE001 - compared with the reference's own exception
        exc = [type(e).__name__, str(e)]
    body = client.CREATED[-1][1] if client.CREATED else None
    return exc, body, info


def assert_dropin_matches(algo, case, relations, label=""):
    res = case["results"][algo]
    exc, body, info = dropin_decision(algo, case, relations)
    assert (exc[0] if exc else None) == (res["exception"][0] if res["exception"] else None), \
        f"{label} {algo}: exception {exc} vs {res['exception']}"
    if res["exception"]:
        assert exc[1] == res["exception"][1], f"{label} {algo}: message {exc[1]!r} vs {res['exception'][1]!r}"
        assert body is None
        assert info == res["info_after"], f"{label} {algo}: deployment_info after the error differs"
    else:
        assert body == res["body"], f"{label} {algo}: created body differs\n ours={body}\n ref={res['body']}"
