"""``cluster_monitoring`` snapshot replay and the harness metrics (SURVEY.md §8f
items 3 and 4).

The reference builds its cluster snapshot live from the Kubernetes API
(``podmonitor.monitor``, podmonitor.py:7-125) and measures the two experiment
metrics the same way (``nodemonitor.node_resorce_std``, nodemonitor.py:9-56;
``communicationcost.communication_cost``, communicationcost.py:6-49).  This
module replays all three from JSON dumps of the same API objects, so recorded
snapshots can be re-scored offline and at scale:

=====================  ====================================================
dump                   what ``kubectl`` prints it as
=====================  ====================================================
``nodes``              ``kubectl get nodes -o json``
``node_metrics``       ``kubectl get --raw /apis/metrics.k8s.io/v1beta1/nodes``
``pods``               ``kubectl get pods -A -o json``
``pod_metrics``        ``kubectl get --raw /apis/metrics.k8s.io/v1beta1/namespaces/default/pods``
``replicasets``        ``kubectl get rs -n default -o json``
=====================  ====================================================

Quantity strings are converted in bulk by the native parser
(``rsk_parse_quantities``, csrc/rsk_snapshot.cpp); :func:`cpu_conversion` and
:func:`mem_conversion` restate unit_convertion.py:1-32 for the spellings the
native grammar leaves to Python (and raise the reference's exceptions for
malformed text).  The metrics run on the GPU through the C ABI (``rsk_load_std``,
``rsk_cut_cost``).  Control flow, warnings-then-partial-results and error
returns follow the reference function by function; each cites its lines.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

QTY_CPU, QTY_MEM = 0, 1

_MEM_UNITS = {"Ki": 1024, "Mi": 1024 ** 2, "Gi": 1024 ** 3, "Ti": 1024 ** 4, "Pi": 1024 ** 5, "Ei": 1024 ** 6}


# ---------------------------------------------------------------------------
# unit_convertion.py
# ---------------------------------------------------------------------------
def cpu_conversion(cpu_usage) -> int:
    """Millicores (unit_convertion.py:1-13): 'Xm' truncates, 'Xn' / 'Xu' and bare
    cores round half-even."""
    s = str(cpu_usage).strip()
    if s.endswith("m"):
        return int(float(s[:-1]))
    if s.endswith("n"):
        return int(round(float(s[:-1]) / 1_000_000))
    if s.endswith("u"):
        return int(round(float(s[:-1]) / 1000))
    return int(round(float(s) * 1000))


def mem_conversion(mem_usage) -> int:
    """Bytes (unit_convertion.py:15-32): binary suffixes only, truncating."""
    s = str(mem_usage).strip()
    unit = s[-2:]
    if unit in _MEM_UNITS:
        return int(float(s[:-len(unit)]) * _MEM_UNITS[unit])
    return int(float(s))


def parse_quantities(values: Sequence, kind: int) -> np.ndarray:
    """Bulk :func:`cpu_conversion` (kind 0) / :func:`mem_conversion` (kind 1) into
    int64 via librsk's native parser.  Elements it flags go through the Python
    restatement in order, so the first malformed value raises exactly what the
    reference raises for it.  Host-only: needs librsk.so, not a GPU."""
    from . import _lib

    n = len(values)
    out = np.zeros(n, np.int64)
    if n == 0:
        return out
    strs = [v if type(v) is str else str(v) for v in values]
    joined = "".join(strs)
    buf = joined.encode("utf-8")
    if len(buf) == len(joined):  # ASCII: byte offsets are character offsets
        lens = np.fromiter(map(len, strs), np.int64, n)
    else:
        lens = np.fromiter((len(x.encode("utf-8")) for x in strs), np.int64, n)
    offs = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=offs[1:])
    buf = buf or b"\0"
    status = np.zeros(n, np.uint8)
    lib = _lib.load_library()
    _lib.check(lib.rsk_parse_quantities(buf, offs.ctypes.data, n, kind, out.ctypes.data, status.ctypes.data))
    conv = cpu_conversion if kind == QTY_CPU else mem_conversion
    for i in np.flatnonzero(status):
        v = conv(values[i])
        if not -2 ** 63 <= v < 2 ** 63:
            raise OverflowError(f"quantity {values[i]!r} = {v} outside int64")
        out[i] = v
    return out


def _try_parse(values, kind):
    """(parsed int64 array, index of the first value the reference fails on or
    len(values), that exception or None) -- for the reference's loops that stop
    at the first error and keep what they had."""
    try:
        return parse_quantities(values, kind), len(values), None
    except (ValueError, TypeError, OverflowError) as e:
        conv = cpu_conversion if kind == QTY_CPU else mem_conversion
        out = np.zeros(len(values), np.int64)
        for i, v in enumerate(values):
            try:
                out[i] = conv(v)
            except (ValueError, TypeError, OverflowError) as e2:
                return out, i, e2
        return out, len(values), e


def _pct(u: int, c: int) -> int:
    """get_resource_usage.py:37-38: int(round(u / c * 100)), -1 if c is 0."""
    return int(round(u / c * 100)) if c else -1


# ---------------------------------------------------------------------------
# get_resource_usage.py
# ---------------------------------------------------------------------------
def node_capacity_table(nodes: dict) -> Dict[str, Tuple[int, int]]:
    """name -> (cpu millicores, memory bytes) over every node (get_resource_usage.py:5-16).
    A node without a capacity converts ``str(None)`` and raises, as there."""
    items = nodes.get("items", [])
    names = [it["metadata"]["name"] for it in items]
    caps = [(it.get("status") or {}).get("capacity") or {} for it in items]
    cpu = parse_quantities([str(c.get("cpu")) for c in caps], QTY_CPU)
    mem = parse_quantities([str(c.get("memory")) for c in caps], QTY_MEM)
    return {n: (int(cpu[i]), int(mem[i])) for i, n in enumerate(names)}


def get_nodes_usage(nodes: dict, node_metrics: dict, warn=print) -> Dict[str, tuple]:
    """name -> (cpu_use, cpu_pct, mem_use, mem_pct, cpu_cap, mem_cap), 'master'
    skipped (get_resource_usage.py:19-45).  The first failing item ends the scan
    with a warning and the entries gathered so far, as the reference's try does."""
    capacity = node_capacity_table(nodes)
    items = [it for it in node_metrics.get("items", [])]
    out: Dict[str, tuple] = {}
    try:
        keep = [it for it in items if it["metadata"]["name"] != "master"]
        cpu, bad_c, err_c = _try_parse([it["usage"]["cpu"] for it in keep], QTY_CPU)
        mem, bad_m, err_m = _try_parse([it["usage"]["memory"] for it in keep], QTY_MEM)
        for i, it in enumerate(keep):
            name = it["metadata"]["name"]
            if i == bad_c:
                raise err_c
            if i == bad_m:
                raise err_m
            cap = capacity.get(name)
            if cap is None:
                raise TypeError("cannot unpack non-iterable NoneType object")
            cc, mc = cap
            u, m = int(cpu[i]), int(mem[i])
            out[name] = (u, _pct(u, cc), m, _pct(m, mc), cc, mc)
    except Exception as e:  # noqa: BLE001  (get_resource_usage.py:42-43)
        warn(f"[warn] node metrics query failed: {e}")
    return out


def get_pods_usage(pod_metrics: dict, warn=print) -> Dict[str, Tuple[int, int]]:
    """podname -> (cpu, mem) summed over containers (get_resource_usage.py:48-69);
    stops at the first failing item with the entries so far."""
    out: Dict[str, Tuple[int, int]] = {}
    try:
        items = pod_metrics.get("items", [])
        flat_c, flat_m, owner = [], [], []
        for k, it in enumerate(items):
            for c in it.get("containers", []):
                flat_c.append(c["usage"]["cpu"])
                flat_m.append(c["usage"]["memory"])
                owner.append(k)
        cpu, bad_c, err_c = _try_parse(flat_c, QTY_CPU)
        mem, bad_m, err_m = _try_parse(flat_m, QTY_MEM)
        j = 0
        for k, it in enumerate(items):
            podname = it["metadata"]["name"]
            pc = pm = 0
            while j < len(owner) and owner[j] == k:
                if j == bad_c:
                    raise err_c
                pc += int(cpu[j])
                if j == bad_m:
                    raise err_m
                pm += int(mem[j])
                j += 1
            out[podname] = (pc, pm)
    except Exception as e:  # noqa: BLE001  (get_resource_usage.py:66-67)
        warn(f"[warn] pod metrics query failed: {e}")
    return out


# ---------------------------------------------------------------------------
# delete_replaced_pod.py / podmonitor.py
# ---------------------------------------------------------------------------
def _replicaset_index(replicasets: Optional[dict]) -> Dict[str, dict]:
    return {rs["metadata"]["name"]: rs for rs in (replicasets or {}).get("items", [])}


def deployment_for_pod(pod: dict, rs_index: Dict[str, dict]) -> Optional[str]:
    """Pod -> ReplicaSet -> Deployment (delete_replaced_pod.py:25-38).  A
    ReplicaSet missing from the dump raises KeyError where the reference's
    read_namespaced_replica_set raises its 404."""
    for o in pod["metadata"].get("ownerReferences") or []:
        if o.get("kind") == "Deployment":
            return o["name"]
        if o.get("kind") == "ReplicaSet":
            rs = rs_index[o["name"]]
            for ro in rs["metadata"].get("ownerReferences") or []:
                if ro.get("kind") == "Deployment":
                    return ro["name"]
    return None


def monitor(nodes: dict, node_metrics: dict, pods: dict, pod_metrics: dict,
            replicasets: Optional[dict] = None, namespace: str = "default", warn=print):
    """``(nodes_name, spods, cluster_monitoring)`` as podmonitor.monitor() returns
    them (podmonitor.py:7-125), from API dumps.  ``spods`` are the pod objects
    of ``namespace`` in API order.  A node without metrics keeps an empty entry,
    so a pod on it fails with the same KeyError('pods') as the reference."""
    nodes_name = [it["metadata"]["name"] for it in nodes.get("items", []) if it["metadata"]["name"] != "master"]
    cm: Dict[str, dict] = {n: {} for n in nodes_name}
    usage = get_nodes_usage(nodes, node_metrics, warn=warn)
    if usage:
        for name in nodes_name:
            if name in usage:
                u, p, m, mp, cc, mc = usage[name]
                cm[name] = {"node_cpu_capacity": cc, "node_cpu_usage": u, "cpu_pct": p,
                            "node_mem_capacity": mc, "node_mem_usage": m, "mem_pct": mp, "pods": []}
    else:
        warn("metrics-server is missing or metrics.k8s.io cannot be queried")
    spods = [p for p in pods.get("items", []) if p["metadata"].get("namespace") == namespace]
    pod_usage = get_pods_usage(pod_metrics, warn=warn)
    if pod_usage:
        rs_index = _replicaset_index(replicasets)
        by_node: Dict[str, List[dict]] = {}
        for p in spods:
            by_node.setdefault((p.get("spec") or {}).get("nodeName"), []).append(p)
        for node_name in nodes_name:
            for p in by_node.get(node_name, []):
                podname = p["metadata"]["name"]
                pc, pm = pod_usage.get(podname, ("-", "-"))
                cm[node_name]["pods"].append({"podname": podname,
                                              "deploymentname": deployment_for_pod(p, rs_index),
                                              "pod_cpu_usage": pc, "pod_mem_usage": pm})
    return nodes_name, spods, cm


# ---------------------------------------------------------------------------
# cluster_monitoring -> flat arrays (the layout include/rsk.h takes, S = 1)
# ---------------------------------------------------------------------------
@dataclass
class ClusterArrays:
    nodes: List[str]            # nodes_name order
    cap_cpu: np.ndarray         # int32 [N] millicores
    use_cpu: np.ndarray         # int32 [N]
    cap_mem: np.ndarray         # int64 [N] bytes
    use_mem: np.ndarray         # int64 [N]
    cpu_pct: np.ndarray         # int32 [N]
    pods: List[str]             # pod names, node by node in nodes_name order
    deployments: List[Optional[str]]
    assign: np.ndarray          # int32 [P] node index
    pod_cpu: np.ndarray         # int32 [P]; -1 where metrics gave "-"
    pod_mem: np.ndarray         # int64 [P]; -1 where metrics gave "-"


def cluster_arrays(nodes_name, cluster_monitoring) -> ClusterArrays:
    """Flatten a snapshot for the device kernels (node_reduce, detect,
    pick_max_pod, rounds).  Nodes without metrics get capacity 0 (cpu_pct -1)."""
    from .cluster import _i32

    N = len(nodes_name)
    cap = np.zeros(N, np.int32)
    use = np.zeros(N, np.int32)
    capm = np.zeros(N, np.int64)
    usem = np.zeros(N, np.int64)
    pct = np.full(N, -1, np.int32)
    pods: List[str] = []
    deps: List[Optional[str]] = []
    assign: List[int] = []
    pcpu: List[int] = []
    pmem: List[int] = []
    for i, n in enumerate(nodes_name):
        info = cluster_monitoring.get(n) or {}
        if not info:
            continue
        cap[i] = _i32(info["node_cpu_capacity"], f"{n}.node_cpu_capacity")
        use[i] = _i32(info["node_cpu_usage"], f"{n}.node_cpu_usage")
        capm[i], usem[i], pct[i] = info["node_mem_capacity"], info["node_mem_usage"], info["cpu_pct"]
        for p in info["pods"]:
            pods.append(p["podname"])
            deps.append(p["deploymentname"])
            assign.append(i)
            c, m = p["pod_cpu_usage"], p["pod_mem_usage"]
            pcpu.append(-1 if c == "-" else _i32(c, f"{p['podname']}.pod_cpu_usage"))
            pmem.append(-1 if m == "-" else int(m))
    return ClusterArrays(list(nodes_name), cap, use, capm, usem, pct, pods, deps,
                         np.asarray(assign, np.int32), np.asarray(pcpu, np.int32), np.asarray(pmem, np.int64))


# ---------------------------------------------------------------------------
# the harness metrics, on the GPU
# ---------------------------------------------------------------------------
def node_resorce_std(nodes: dict, node_metrics: dict, ctx=None, warn=print) -> Optional[float]:
    """Population std of node CPU % (nodemonitor.py:9-56): 'master' and nodes
    without capacity skipped, capacity 0 excluded, 0.0 when nothing is left,
    None on a failure.  The std itself runs on the device (rsk_load_std, fp64)."""
    from . import api

    try:
        capacity = node_capacity_table(nodes)
        use, cap = [], []
        items = [it for it in node_metrics.get("items", []) if it["metadata"]["name"] != "master"]
        known = [it for it in items if it["metadata"]["name"] in capacity]
        for it in items:
            if it["metadata"]["name"] not in capacity:
                warn(f"[warn] node {it['metadata']['name']!r} has no capacity; skipped")
        cpu = parse_quantities([it["usage"]["cpu"] for it in known], QTY_CPU)
        for i, it in enumerate(known):
            c = capacity[it["metadata"]["name"]][0]
            if c > 0:
                use.append(int(cpu[i]))
                cap.append(c)
            else:
                warn(f"[warn] node {it['metadata']['name']!r} has CPU capacity 0; skipped")
        if not use:
            return 0.0
        u, c = np.asarray(use, np.int64), np.asarray(cap, np.int64)
        if u.min() < 0 or u.max() > 2**31 - 1 or c.max() > 2**31 - 1:
            raise ValueError("CPU quantities outside the int32 millicore ABI range")
        return float(api.load_std(u.astype(np.int32), c.astype(np.int32), len(use), 1, ctx=ctx)[0])
    except Exception as e:  # noqa: BLE001  (nodemonitor.py:54-56)
        warn(f"[warn] node metrics query/compute failed: {e}")
        return None


def communication_cost(pods: dict, relation: dict, replicasets: Optional[dict] = None, ctx=None,
                       namespace: str = "default", warn=print):
    """Cross-node relation count / 2 (communicationcost.py:6-49): the last pod of
    a deployment decides its node; a related deployment with no pod, or an
    unscheduled pod, compares as None; -1 on any failure.  Like the reference
    the deployment name carries over from the previous pod when a pod has no
    Deployment owner.  The pair count runs on the device (rsk_cut_cost)."""
    from . import api
    from .workmodel import relation_csr

    try:
        rs_index = _replicaset_index(replicasets)
        inf: Dict[str, Optional[str]] = {}
        deployment_name = _UNBOUND = object()
        for pod in pods.get("items", []):
            if pod["metadata"].get("namespace") != namespace:
                continue
            node_name = (pod.get("spec") or {}).get("nodeName")
            for o in pod["metadata"].get("ownerReferences") or []:
                if o.get("kind") == "Deployment":
                    deployment_name = o["name"]
                elif o.get("kind") == "ReplicaSet":
                    rs = rs_index[o["name"]]
                    for ro in rs["metadata"].get("ownerReferences") or []:
                        if ro.get("kind") == "Deployment":
                            deployment_name = ro["name"]
            if deployment_name is _UNBOUND:
                raise NameError("deployment_name is unbound")
            inf[deployment_name] = node_name
        names = list(inf)
        node_ix: Dict[str, int] = {}
        assign = np.array([-1 if inf[d] is None else node_ix.setdefault(inf[d], len(node_ix)) for d in names],
                          np.int32)
        rp, ci, miss = relation_csr(relation, names, dedup=False)
        directed = int(api.cut_cost(rp, ci, assign, len(names), 1, miss, ctx=ctx)[0]) if names else 0
        return directed / 2
    except Exception as e:  # noqa: BLE001  (communicationcost.py:47-49)
        warn(f"[ERROR] communication cost failed: {e}")
        return -1
