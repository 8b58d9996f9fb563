"""CPU restatements of CAR in Python — TEST / BASELINE INFRASTRUCTURE ONLY.

Two single-core restatements of `communication`'s score loop and argmax
(reference rescheduling.py:183-214), timed as bench.py's extra cpu_baseline
legs and pinned by tests/test_oracle_golden.py
against the C oracle (rsk_oracle.c) and the reference's own fixtures:

* ``car_literal`` keeps the reference's data structures and control flow: a
  per-node loop over the pods on each node with list-membership tests against
  the relation list (:188-195) and the hazard list (:189), ``max`` over the
  score dict (:199), the best-node list (:200) and the remaining-CPU
  tie-break loop (:203-212).
* ``car_numpy`` is the vectorized form: a bincount of the related pods' nodes,
  hazard nodes masked out, then the same tie rules.

Neither is ever called by the product path (librsk.so); only tests/ and
bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import numpy as np

NONE = -1          # nodeName=None (rescheduling.py:203-212, every tied rem <= -1)
NO_CANDIDATE = -2  # max() of an empty sequence raises ValueError (:199)


def pods_by_node(assign_s, N):
    """The per-node pod lists of one scenario (cluster_monitoring[n]['pods'],
    podmonitor.py:114-121), pods in id order; assignments outside [0, N) are
    on no node."""
    out = [[] for _ in range(N)]
    for q, n in enumerate(assign_s.tolist()):
        if 0 <= n < N:
            out[n].append(q)
    return out


def car_literal(rel, by_node, hazard_list, cap, use):
    """rescheduling.py:183-214 on flat ids: ``rel`` is the moving pod's related
    pods (a list, membership by ``in`` as :193), ``by_node[n]`` the pods on node
    n, ``hazard_list`` a list of hazard node ids (:189), cap / use per node."""
    scores = {}
    for n in range(len(by_node)):
        if n in hazard_list:
            continue
        score = 0
        for q in by_node[n]:
            if q in rel:
                score += 1
        scores[n] = score
    if not scores:
        return NO_CANDIDATE
    max_score = max(scores.values())
    best_nodes = [n for n, s in scores.items() if s == max_score]
    if len(best_nodes) == 1:
        return best_nodes[0]
    target, remaining = None, -1
    for n in best_nodes:
        rem = cap[n] - use[n]
        if rem > remaining:
            remaining = rem
            target = n
    return NONE if target is None else target


def car_numpy(nbrs, assign_s, cap, use_s, haz_s, N):
    """Vectorized rescheduling.py:183-214 for one (pod, scenario): ``nbrs`` the
    deduplicated related pods (no self edge), ``assign_s`` / ``use_s`` /
    ``haz_s`` that scenario's arrays."""
    nodes = assign_s[nbrs]
    nodes = nodes[(nodes >= 0) & (nodes < N)]
    score = np.bincount(nodes, minlength=N)
    cand = haz_s == 0
    if not cand.any():
        return NO_CANDIDATE
    m = score[cand].max()
    best = np.flatnonzero((score == m) & cand)
    if best.size == 1:
        return int(best[0])
    rem = cap[best].astype(np.int64) - use_s[best]
    i = int(np.argmax(rem))
    return int(best[i]) if rem[i] > -1 else NONE


def dedup_rows(row_ptr, col_idx, rows):
    """Deduplicated neighbour arrays without the self edge, per requested row."""
    out = []
    for p in rows:
        nb = np.unique(col_idx[row_ptr[p]:row_ptr[p + 1]])
        out.append(nb[nb != p].astype(np.int64))
    return out


def scenario_view(assign, use, hazard, P, N, S, s):
    """Scenario s of the scenario-minor batched arrays."""
    return (np.ascontiguousarray(assign.reshape(P, S)[:, s]), np.ascontiguousarray(use.reshape(N, S)[:, s]),
            np.ascontiguousarray(hazard.reshape(N, S)[:, s]))
