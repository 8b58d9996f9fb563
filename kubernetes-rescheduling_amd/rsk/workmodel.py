"""µBench workmodel JSON → service relation graph.

``workmodelC.json`` lists, per service, ``external_services[*].services`` (the
services it calls).  The reference hard-codes the symmetrised graph in
``main.py:31-52`` (and again in ``communicationcost.py:69-88``):
``rel(s) = {services s calls} ∪ {services that call s}``.  This module derives that
relation from the workmodel itself and lays it out as a deduplicated CSR.
"""
from __future__ import annotations

import json
from typing import Dict, List

import numpy as np


def load_workmodel(path_or_obj) -> dict:
    if isinstance(path_or_obj, dict):
        return path_or_obj
    with open(path_or_obj, "r", encoding="utf-8") as f:
        return json.load(f)


def relation_from_workmodel(workmodel) -> Dict[str, List[str]]:
    """Symmetrised service relation: parents first (in discovery order), then callees
    in ``external_services`` order; duplicates and self-edges dropped.

    Membership is all the placement path uses (rescheduling.py:194), and the cost
    metric sums over it (communicationcost.py:40-43), so list order is cosmetic.
    """
    wm = load_workmodel(workmodel)
    callees: Dict[str, List[str]] = {}
    callers: Dict[str, List[str]] = {s: [] for s in wm}
    for svc, spec in wm.items():
        out: List[str] = []
        for group in spec.get("external_services", []) or []:
            for t in group.get("services", []) or []:
                if t != svc and t not in out:
                    out.append(t)
        callees[svc] = out
        for t in out:
            callers.setdefault(t, [])
            if svc not in callers[t]:
                callers[t].append(svc)
    rel: Dict[str, List[str]] = {}
    for svc in list(wm.keys()) + [t for t in callers if t not in wm]:
        seen: List[str] = []
        for t in callers.get(svc, []) + callees.get(svc, []):
            if t not in seen:
                seen.append(t)
        rel[svc] = seen
    return rel


def relation_csr(relations: Dict[str, List[str]], names: List[str], dedup: bool = True):
    """CSR over ``names`` (a deployment per row): row i lists the indices of the
    deployments in ``relations[names[i]]`` that appear in ``names``.  Unknown names
    are skipped and counted in ``missing_counts``.

    ``dedup=True`` (placement): duplicates and self-edges dropped, since CAR only
    tests membership (rescheduling.py:194).  ``dedup=False`` (cost metric): every
    list entry is an edge, as ``communicationcost.py:41`` iterates the list itself.
    Returns (row_ptr int32[P+1], col_idx int32[nnz], missing_counts int32[P])."""
    index = {}
    for i, n in enumerate(names):
        index.setdefault(n, i)
    row_ptr = [0]
    cols: List[int] = []
    missing = []
    for i, n in enumerate(names):
        seen = set()
        miss = 0
        rels = relations.get(n, [])
        for r in (dict.fromkeys(rels) if dedup else rels):  # dict.fromkeys: ordered dedup
            j = index.get(r)
            if j is None:
                miss += 1
                continue
            if dedup and (j == i or j in seen):
                continue
            seen.add(j)
            cols.append(j)
        row_ptr.append(len(cols))
        missing.append(miss)
    return (np.asarray(row_ptr, dtype=np.int32), np.asarray(cols, dtype=np.int32),
            np.asarray(missing, dtype=np.int32))
