"""Synthetic clusters for the placement-scoring path.

The reference only ever runs against a live 3-worker cluster; its scale configs
(2k/64, 100k/5k, 1M/50k) are synthetic.  This generator is the one the survey
timed the reference with, so its seed-0 statistics are pinned:

* graph: preferential-attachment tree (m=1, µBench-like; workmodelC.json is a
  20-service tree), symmetrised, ``nnz = 2(P-1)``.  Seed 0 at P=100k gives max
  degree 531; at P=2k, 61.
* ``assign = rng.integers(0, N, P)``, ``pod_cpu = rng.integers(50, 500, P)`` m,
  ``cap_cpu = 64000`` m, ``bg = rng.integers(0, 16000, N)``, drawn in that order
  after the tree; ``use_cpu = bg + bincount(assign, pod_cpu)``.
* ``cpu_pct = int(round(use / cap * 100))`` (get_resource_usage.py:37) and
  ``hazard = cpu_pct >= 30`` (harzard_detect.py:7,12).  Seed 0 → 18 hazard nodes at
  2k/64 and 764 at 100k/5k.
* scenario ``s``: the base assignment with ``P // 100`` pods redrawn by
  ``default_rng(1 + s)``; use / pct / hazard recomputed per scenario.

All arrays use the batched ABI layouts of ``include/rsk.h``: per-scenario arrays
are scenario-minor (``assign[p*S + s]``, ``use_cpu[n*S + s]``).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

CAP_CPU_M = 64000
HAZARD_THRESHOLD = 30  # harzard_detect.py:7


def pa_tree_parents(P: int, rng: np.random.Generator) -> np.ndarray:
    """Parent of every pod in a preferential-attachment tree (parent[0] = -1).

    Pod i attaches to an endpoint drawn uniformly from the multiset of edge
    endpoints so far (probability proportional to degree), one ``rng.integers``
    call per pod, in pod order.
    """
    rep = np.empty(max(2 * P, 1), dtype=np.int64)
    rep[0] = 0
    L = 1
    parent = np.empty(P, dtype=np.int64)
    parent[0] = -1
    draws = rng.integers  # bound method; one call per pod keeps the stream pinned
    for i in range(1, P):
        t = rep[draws(0, L)]
        parent[i] = t
        rep[L] = i
        rep[L + 1] = t
        L += 2
    return parent


def tree_csr(parent: np.ndarray):
    """Symmetrised CSR (row_ptr[P+1], col_idx[nnz]) of a parent array, rows sorted."""
    P = parent.shape[0]
    child = np.arange(1, P, dtype=np.int64)
    par = parent[1:]
    src = np.concatenate([child, par])
    dst = np.concatenate([par, child])
    order = np.lexsort((dst, src))
    src, dst = src[order], dst[order]
    row_ptr = np.zeros(P + 1, dtype=np.int64)
    np.cumsum(np.bincount(src, minlength=P), out=row_ptr[1:])
    return row_ptr.astype(np.int32), dst.astype(np.int32)


def cpu_pct(use: np.ndarray, cap) -> np.ndarray:
    """``int(round(u / c * 100))`` elementwise in fp64, -1 where c == 0
    (get_resource_usage.py:37).  numpy's rint is round-half-even like Python's round."""
    use = np.asarray(use, dtype=np.float64)
    cap = np.broadcast_to(np.asarray(cap, dtype=np.float64), use.shape)
    with np.errstate(divide="ignore", invalid="ignore"):
        pct = np.rint((use / cap) * 100.0)
    pct = np.where(cap != 0, pct, -1.0)
    return pct.astype(np.int32)


@dataclass
class SynthCluster:
    P: int
    N: int
    S: int
    row_ptr: np.ndarray          # int32 [P+1]
    col_idx: np.ndarray          # int32 [nnz]
    assign: np.ndarray           # int32 [P*S]  scenario-minor
    pod_cpu: np.ndarray          # int32 [P]
    pod_mem: np.ndarray          # int64 [P]
    cap_cpu: np.ndarray          # int32 [N]
    bg_cpu: np.ndarray           # int32 [N]
    use_cpu: np.ndarray          # int32 [N*S]  scenario-minor
    cpu_pct: np.ndarray          # int32 [N*S]
    hazard: np.ndarray           # uint8 [N*S]
    extra: dict = field(default_factory=dict)

    @property
    def nnz(self) -> int:
        return int(self.col_idx.shape[0])

    def node_names(self):
        return [f"node-{n:05d}" for n in range(self.N)]


def make_cluster(P: int, N: int, S: int = 1, seed: int = 0, redraw_frac: float = 0.01,
                 graph: str = "pa", s0: int = 0) -> SynthCluster:
    """Build the synthetic cluster of SURVEY.md §8d (see module docstring).

    ``s0`` offsets the global scenario ids: local scenario j is global scenario
    ``s0 + j`` (its redraws come from ``default_rng(1 + s0 + j)``; global scenario 0
    is the unperturbed base).  Ranks of a scenario-sharded run use disjoint ``s0``.
    """
    rng = np.random.default_rng(seed)
    if graph == "pa":
        parent = pa_tree_parents(P, rng)
        row_ptr, col_idx = tree_csr(parent)
    else:
        raise ValueError(f"unknown graph kind {graph!r}")
    base = rng.integers(0, N, P).astype(np.int32)
    pod_cpu = rng.integers(50, 500, P).astype(np.int32)
    bg = rng.integers(0, 16000, N).astype(np.int32)
    pod_mem = (pod_cpu.astype(np.int64) * (1 << 20))  # 1 MiB per millicore: deterministic, int64
    cap = np.full(N, CAP_CPU_M, dtype=np.int32)

    k = P // 100 if redraw_frac == 0.01 else int(P * redraw_frac)
    w = pod_cpu.astype(np.int64)
    base_use = bg.astype(np.int64) + np.bincount(base, weights=w, minlength=N).astype(np.int64)
    # scenario-minor layouts built in place: assign[p, s], use[n, s]
    assign = np.empty((P, S), dtype=np.int32)
    assign[:] = base[:, None]
    use = np.empty((N, S), dtype=np.int64)
    use[:] = base_use[:, None]
    for j in range(S):
        g = s0 + j
        if g == 0 or k == 0:
            continue
        r = np.random.default_rng(1 + g)
        idx = r.integers(0, P, k)
        new = r.integers(0, N, k).astype(np.int32)
        changed = np.unique(idx)
        tmp = base[changed].copy()
        # fancy assignment with repeated indices keeps the last value, as a[idx] = new does
        last = np.empty(P, dtype=np.int32)
        last[idx] = new
        newv = last[changed]
        assign[changed, j] = newv
        ww = w[changed]
        use[:, j] += np.bincount(newv, weights=ww, minlength=N).astype(np.int64)
        use[:, j] -= np.bincount(tmp, weights=ww, minlength=N).astype(np.int64)
    use32 = use.astype(np.int32)
    pct = cpu_pct(use32, cap[:, None])
    haz = (pct >= HAZARD_THRESHOLD).astype(np.uint8)
    return SynthCluster(
        P=P, N=N, S=S, row_ptr=row_ptr, col_idx=col_idx,
        assign=assign.reshape(-1), pod_cpu=pod_cpu, pod_mem=pod_mem, cap_cpu=cap, bg_cpu=bg,
        use_cpu=use32.reshape(-1), cpu_pct=pct.reshape(-1), hazard=haz.reshape(-1),
    )


def to_cluster_monitoring(c: SynthCluster, s: int = 0):
    """The reference's ``(nodes_name, cluster_monitoring, relations)`` for scenario ``s``.

    Pod p is deployment ``d{p}`` with pod name ``pod-{p}``; ``relations[d{p}]`` lists
    the deployments of p's CSR neighbours.  Schema: podmonitor.py:72-84,114-121.
    """
    names = c.node_names()
    S = c.S
    cm = {}
    for n, name in enumerate(names):
        u = int(c.use_cpu[n * S + s])
        cm[name] = {
            "node_cpu_capacity": int(c.cap_cpu[n]),
            "node_cpu_usage": u,
            "cpu_pct": int(c.cpu_pct[n * S + s]),
            "node_mem_capacity": 256 << 30,
            "node_mem_usage": 0,
            "mem_pct": 0,
            "pods": [],
        }
    a = c.assign.reshape(c.P, S)[:, s]
    for p in range(c.P):
        cm[names[a[p]]]["pods"].append({
            "podname": f"pod-{p}", "deploymentname": f"d{p}",
            "pod_cpu_usage": int(c.pod_cpu[p]), "pod_mem_usage": int(c.pod_mem[p]),
        })
    rp, ci = c.row_ptr, c.col_idx
    relations = {f"d{p}": [f"d{q}" for q in ci[rp[p]:rp[p + 1]]] for p in range(c.P)}
    return names, cm, relations
