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


# ---------------------------------------------------------------------------
# Native streaming reader (librsk.so, csrc/rsk_workmodel.cpp) and a synthetic
# µBench workmodel writer for 100k-1M services.
# ---------------------------------------------------------------------------
def read_workmodel(src):
    """Parse a µBench workmodel with the native one-pass reader.

    ``src``: a path, or the JSON text as ``bytes``/``str``.  Returns
    ``(names, row_ptr int32[P+1], col_idx int32[nnz])``: the symmetrised relation
    of ``relation_from_workmodel`` over ``names`` (defined services in file order,
    then never-defined callees in order of first mention), self calls dropped,
    deduplicated, columns ascending.  Malformed JSON raises ``RskError``.
    Host-only: needs librsk.so, not a GPU."""
    import ctypes as C

    from . import _lib

    lib = _lib.load_library()
    h = C.c_void_p()
    text = isinstance(src, (bytes, bytearray)) or (isinstance(src, str) and src.lstrip().startswith("{"))
    if text:
        buf = src.encode() if isinstance(src, str) else bytes(src)
        _lib.check(lib.rsk_workmodel_parse(buf, len(buf), C.byref(h)))
    else:
        _lib.check(lib.rsk_workmodel_load(str(src).encode(), C.byref(h)))
    try:
        P, nnz, nb = C.c_int32(), C.c_int64(), C.c_int64()
        _lib.check(lib.rsk_workmodel_sizes(h, C.byref(P), C.byref(nnz), C.byref(nb)))
        row_ptr = np.empty(P.value + 1, dtype=np.int32)
        col_idx = np.empty(max(nnz.value, 1), dtype=np.int32)
        _lib.check(lib.rsk_workmodel_csr(h, row_ptr.ctypes.data, col_idx.ctypes.data))
        raw = C.create_string_buffer(max(nb.value, 1))
        _lib.check(lib.rsk_workmodel_names(h, raw))
        names = raw.raw[: nb.value].decode("utf-8").split("\0")[:-1] if nb.value else []
    finally:
        lib.rsk_workmodel_destroy(h)
    return names, row_ptr, col_idx[: nnz.value]


_LOADER = ('{"loader": {"cpu_stress": {"run": true, "range_complexity": [100, 100], "thread_pool_size": 1, '
           '"trials": 10}, "mean_response_size": 11, "function_id": "f2"}}')


def write_synth_workmodel(path: str, P: int, seed: int = 0, chunk: int = 65536) -> None:
    """Write a µBench-style workmodel of ``P`` services ``s0..s{P-1}`` whose call
    graph is the preferential-attachment tree of ``synth.pa_tree_parents`` (each
    parent calls its children, as workmodelC.json's tree does), streamed to
    ``path`` in chunks so 1M services never build a dict.  Its relation CSR
    equals ``synth.tree_csr`` of the same parents."""
    from .synth import pa_tree_parents

    parent = pa_tree_parents(P, np.random.default_rng(seed))
    order = np.argsort(parent[1:], kind="stable") + 1          # children grouped by parent
    starts = np.searchsorted(parent[order], np.arange(P + 1))
    with open(path, "w", encoding="utf-8") as f:
        f.write("{\n")
        buf = []
        for i in range(P):
            kids = order[starts[i]:starts[i + 1]]
            ext = ('[{"seq_len": 100, "services": [' + ", ".join(f'"s{k}"' for k in kids) + "]}]") if len(kids) else "[]"
            buf.append(f'  "s{i}": {{"external_services": {ext}, "internal_service": {_LOADER}, '
                       f'"request_method": "rest", "workers": 8, "threads": 128, "cpu-requests": "100m"}}'
                       + (",\n" if i + 1 < P else "\n"))
            if len(buf) >= chunk:
                f.write("".join(buf))
                buf.clear()
        f.write("".join(buf))
        f.write("}\n")
