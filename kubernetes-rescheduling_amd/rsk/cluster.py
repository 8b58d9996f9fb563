"""``cluster_monitoring`` dict → flat arrays for one drop-in placement call.

The reference's placement functions read the snapshot that podmonitor.monitor()
builds (schema podmonitor.py:72-84, 114-121):

    {node: {node_cpu_capacity, node_cpu_usage, cpu_pct, node_mem_capacity,
            node_mem_usage, mem_pct, pods: [{podname, deploymentname,
            pod_cpu_usage, pod_mem_usage}]}}

Each flattener below touches exactly the dict entries the corresponding
reference function touches for candidate (non-hazard) nodes, so a malformed
snapshot fails with the same KeyError; it never reads hazard nodes' entries.
The resulting int32/uint8 arrays follow include/rsk.h with S = 1.
"""
from __future__ import annotations

from dataclasses import dataclass
from operator import itemgetter
from typing import List

import numpy as np

INT32_MAX = 2**31 - 1


def _members(seq):
    """Fast membership test with the semantics of ``x in seq`` for a list of names."""
    try:
        return set(seq).__contains__
    except TypeError:  # unhashable entries: use the sequence's own ==
        return seq.__contains__


def _i32(v, what: str) -> int:
    iv = int(v)
    if not 0 <= iv <= INT32_MAX:
        raise ValueError(f"{what}={v!r} outside the ABI range [0, 2^31-1] of librsk")
    return iv


def _i32_array(vals, names, field: str) -> np.ndarray:
    """int32 array of the values, _i32's range check (and message) on the first bad one."""
    try:
        a = np.array(vals, np.int64)
        if a.size == 0 or (a.min() >= 0 and a.max() <= INT32_MAX):
            return a.astype(np.int32)
    except (OverflowError, TypeError, ValueError):
        pass
    return np.array([_i32(v, f"{n}.{field}") for v, n in zip(vals, names)], np.int32)


@dataclass
class CarRequest:
    nodes: List[str]        # candidate order: nodes_name, first occurrence kept
    row_ptr: np.ndarray     # int32 [P+1]; row 0 = the moving deployment
    col_idx: np.ndarray     # int32 [nnz]
    assign: np.ndarray      # int32 [P]; pod 0 (the moving one) is off-cluster (-1)
    cap_cpu: np.ndarray     # int32 [N]
    use_cpu: np.ndarray     # int32 [N]
    hazard: np.ndarray      # uint8 [N]


def car_request(name, harzard_node, cluster_monitoring, relations, nodes_name) -> CarRequest:
    """Inputs of `communication` (rescheduling.py:183-195) as a one-row CSR.

    Row 0 is the moving deployment; its neighbours are every pod on a candidate
    node whose deploymentname is in ``relations.get(name, [])`` (list
    membership, so duplicates in the relation count once and ``None`` never
    matches).  The score dict of the reference keeps the first occurrence of a
    repeated node name, hence ``dict.fromkeys``.
    """
    nodes = list(dict.fromkeys(nodes_name))
    N = len(nodes)
    member = _members(relations.get(name, []))
    is_haz = _members(harzard_node)
    dep = itemgetter("deploymentname")
    hz = [1 if is_haz(n) else 0 for n in nodes]
    cnt = [0] * N
    capl = [0] * N
    usel = [0] * N
    for i, n in enumerate(nodes):
        if hz[i]:
            continue
        info = cluster_monitoring[n]
        # the per-pod membership test runs in C (map over the pod list), with the
        # reference's KeyError for a pod without "deploymentname"
        cnt[i] = sum(map(member, map(dep, info["pods"])))
        capl[i] = info["node_cpu_capacity"]
        usel[i] = info["node_cpu_usage"]
    haz = np.array(hz, np.uint8)
    cap = _i32_array(capl, nodes, "node_cpu_capacity")
    use = _i32_array(usel, nodes, "node_cpu_usage")
    nb = np.repeat(np.arange(N, dtype=np.int32), cnt)   # one neighbour entry per related pod, on its node
    k = int(nb.size)
    row_ptr = np.full(k + 2, k, np.int32)
    row_ptr[0] = 0
    col_idx = np.arange(1, k + 1, dtype=np.int32)
    assign = np.empty(k + 1, np.int32)
    assign[0] = -1
    assign[1:] = nb
    return CarRequest(nodes, row_ptr, col_idx, assign, cap, use, haz)


@dataclass
class NodeTable:
    names: List[str]
    value: np.ndarray       # int32 [N]: pod count (spread) or cpu_pct (binpack)
    name_rank: np.ndarray   # int32 [N]: rank in Python str order
    hazard: np.ndarray      # uint8 [N]


def node_table(harzard_node, cluster_monitoring, field: str) -> NodeTable:
    """Candidates of spread (rescheduling.py:91-96, field='pods' -> len) or
    binpack (:123-128, field='cpu_pct'), in cluster_monitoring key order."""
    names = list(cluster_monitoring.keys())
    N = len(names)
    val = np.zeros(N, np.int32)
    haz = np.zeros(N, np.uint8)
    is_haz = _members(harzard_node)
    for i, n in enumerate(names):
        if is_haz(n):
            haz[i] = 1
            continue
        info = cluster_monitoring[n]
        v = len(info["pods"]) if field == "pods" else int(info[field])
        if not -2**31 <= v <= INT32_MAX:
            raise ValueError(f"{n}.{field}={v!r} outside int32")
        val[i] = v
    order = sorted(range(N), key=names.__getitem__)
    rank = np.empty(N, np.int32)
    rank[order] = np.arange(N, dtype=np.int32)
    return NodeTable(names, val, rank, haz)


def candidate_mask(harzard_node, nodes_name) -> np.ndarray:
    """hazard flags over nodes_name as given (rescheduling.py:149, duplicates kept)."""
    is_haz = _members(harzard_node)
    return np.fromiter((1 if is_haz(n) else 0 for n in nodes_name), np.uint8, len(nodes_name))
