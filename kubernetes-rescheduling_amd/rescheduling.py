"""Drop-in replacement for the reference's ``rescheduling.py`` (MI355X path).

Put this directory ahead of the reference on ``sys.path`` (or PYTHONPATH) and
``main.py`` — ``from rescheduling import spread, binpack, random,
kubescheduling, communication`` (reference main.py:7) — runs unchanged.  The
five entry points keep the reference's names, arguments, in-place mutation of
``deployment_info``, return values (``create()``'s True/False) and exceptions;
the node choice inside spread / binpack / random / communication is computed by
librsk.so's gfx950 kernels.  Kubernetes I/O (affinity patch, create) stays on
the host exactly as in the reference.

Reference map: affinity merge rescheduling.py:21-40, hazard NotIn term :42-55,
create :57-73, spread :77-105, binpack :107-137, random :140-157,
kubescheduling :159-171, communication :174-218.
"""
from __future__ import annotations

import copy
import random as _pyrandom
import time

from kubernetes import client, config
from kubernetes.client import ApiException

from rsk import api as _api
from rsk import cluster as _cluster
from rsk._lib import TARGET_NO_CANDIDATE

_NO_CANDIDATES = "No candidate nodes available (all nodes are hazardous)."
_HOSTNAME = "kubernetes.io/hostname"


def _wait_deleted(apps_v1, namespace, name, timeout=120):
    """Poll until the Deployment is gone (404); False on timeout (reference :8-19)."""
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            apps_v1.read_namespaced_deployment(name=name, namespace=namespace)
        except ApiException as exc:
            if exc.status != 404:
                raise
            return True
        time.sleep(1)
    return False


def _merge_into(dst, src, depth):
    # Levels 0 and 1 recurse into dict/dict pairs; level 2 extends list/list
    # pairs; anything else is replaced by the patch value (shared, not copied).
    for key, val in src.items():
        cur = dst.get(key)
        if depth < 2 and isinstance(cur, dict) and isinstance(val, dict):
            _merge_into(cur, val, depth + 1)
        elif depth == 2 and isinstance(cur, list) and isinstance(val, list):
            cur.extend(val)
        else:
            dst[key] = val


def _merge_affinity(orig, patch):
    """Merge ``patch`` into a deep copy of ``orig`` (None/{} -> {})."""
    merged = copy.deepcopy(orig) if orig else {}
    _merge_into(merged, patch, 0)
    return merged


def exclude_hazard_nodes(hazard_nodes):
    """Required node affinity: hostname NotIn the hazard nodes."""
    term = {"matchExpressions": [{"key": _HOSTNAME, "operator": "NotIn", "values": hazard_nodes}]}
    return {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [term]}}}


def create(apps_v1, namespace, body, wait_if_exists: bool = False):
    """create_namespaced_deployment; True on success, False (logged) on ApiException."""
    name = body["metadata"]["name"]
    if wait_if_exists:
        _wait_deleted(apps_v1, namespace, name)
    try:
        apps_v1.create_namespaced_deployment(namespace=namespace, body=body)
    except ApiException as exc:
        print(f"[error] create {name}: {exc.status} {exc.reason}")
        try:
            print(exc.body)
        except Exception:  # noqa: BLE001 - logging only
            pass
        return False
    print(f"[success] New Deployment {name} created in ns={namespace}.")
    return True


def _pod_spec(deployment_info):
    return deployment_info["spec"]["template"]["spec"]


def _setup(deployment_info, harzard_node, patch_affinity: bool):
    config.load_kube_config()
    apps_v1 = client.AppsV1Api()
    namespace = deployment_info["metadata"].get("namespace", "default")
    if patch_affinity:
        spec = _pod_spec(deployment_info)
        spec["affinity"] = _merge_affinity(spec["affinity"], exclude_hazard_nodes(harzard_node))
    return apps_v1, namespace


def _pick_node_table(harzard_node, cluster_monitoring, field, place):
    tab = _cluster.node_table(harzard_node, cluster_monitoring, field)
    if not tab.names or tab.hazard.all():
        raise RuntimeError(_NO_CANDIDATES)
    out = place(tab.value, tab.name_rank, tab.hazard, len(tab.names), 1)
    if int(out[0]) == TARGET_NO_CANDIDATE:
        raise RuntimeError(_NO_CANDIDATES)
    return tab.names[int(out[0])]


def spread(deployment_info, harzard_node, cluster_monitoring):
    """Least-loaded (fewest pods) non-hazard node, ties to the smallest name."""
    apps_v1, namespace = _setup(deployment_info, harzard_node, True)
    node = _pick_node_table(harzard_node, cluster_monitoring, "pods", _api.spread_place)
    _pod_spec(deployment_info)["nodeSelector"] = {_HOSTNAME: node}
    return create(apps_v1, namespace, deployment_info)


def binpack(deployment_info, harzard_node, cluster_monitoring):
    """Most-utilised (highest cpu_pct) non-hazard node, ties to the largest name."""
    apps_v1, namespace = _setup(deployment_info, harzard_node, True)
    node = _pick_node_table(harzard_node, cluster_monitoring, "cpu_pct", _api.binpack_place)
    _pod_spec(deployment_info)["nodeSelector"] = {_HOSTNAME: node}
    return create(apps_v1, namespace, deployment_info)


def random(deployment_info, harzard_node, nodes_name):
    """Uniform non-hazard node drawn from Python's global ``random`` state."""
    apps_v1, namespace = _setup(deployment_info, harzard_node, False)
    nodes = list(nodes_name)
    haz = _cluster.candidate_mask(harzard_node, nodes)
    cand = _api.random_candidates(haz, len(nodes)) if nodes else ()
    if len(cand) == 0:
        raise RuntimeError(_NO_CANDIDATES)
    # random.choice(seq) is seq[_randbelow(len(seq))]: draw the same index.
    r = _pyrandom.choice(range(len(cand)))
    _pod_spec(deployment_info)["nodeName"] = nodes[int(cand[r])]
    return create(apps_v1, namespace, deployment_info)


def kubescheduling(deployment_info, harzard_node):
    """Hazard NotIn affinity only; kube-scheduler picks the node."""
    apps_v1, namespace = _setup(deployment_info, harzard_node, True)
    return create(apps_v1, namespace, deployment_info)


def communication(deployment_info, harzard_node, cluster_monitoring, relations, nodes_name):
    """CAR: the non-hazard node hosting most related pods; ties to the most free
    CPU (first in nodes_name order), None when every tied node is overloaded."""
    apps_v1, namespace = _setup(deployment_info, harzard_node, True)
    name = deployment_info["metadata"]["name"]
    req = _cluster.car_request(name, harzard_node, cluster_monitoring, relations, nodes_name)
    N = len(req.nodes)
    if N == 0 or req.hazard.all():
        raise ValueError("max() arg is an empty sequence")
    if N <= _api.ROW_MAX_N:  # one launch: the related pods' nodes -> histogram -> argmax
        t, _ = _api.car_row(req.assign[1:], req.cap_cpu, req.use_cpu, req.hazard, N)
    else:
        tgt, _ = _api.car_place(req.row_ptr, req.col_idx, req.assign, 1, req.cap_cpu, req.use_cpu, req.hazard, N,
                                rows=[0])
        t = int(tgt[0])
    if t == TARGET_NO_CANDIDATE:
        raise ValueError("max() arg is an empty sequence")
    _pod_spec(deployment_info)["nodeName"] = None if t < 0 else req.nodes[t]
    return create(apps_v1, namespace, deployment_info)
