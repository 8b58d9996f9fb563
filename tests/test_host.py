"""CPU: host-side logic and the C-ABI boundary (no GPU compute calls)."""
import os
import re

import numpy as np
import pytest

from conftest import REPO
from helpers import assert_dropin_matches

HEADER = os.path.join(REPO, "include", "rsk.h")


def declared_symbols():
    txt = open(HEADER, encoding="utf-8").read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(rsk_\w+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from rsk import _lib
    lib = _lib.load_library()
    syms = declared_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), f"librsk.so does not export {s}"
    assert set(syms) == set(_lib.SIGNATURES), "ctypes signature table out of sync with include/rsk.h"
    assert lib.rsk_version() >= 104


def test_rows_blk_bytes_host_only():
    """rsk_rows_blk_bytes (host arithmetic, no device): the row-sharded loop's
    detect scratch = S x ceil(N / 64) blocks x 20 B (two u64 maxima and a count)."""
    from rsk import _lib
    lib = _lib.load_library()
    for N, S in ((1, 1), (64, 1), (65, 3), (50_000, 64), (5_000, 1024)):
        assert lib.rsk_rows_blk_bytes(N, S) == S * -(-N // 64) * 20
    assert lib.rsk_rows_blk_bytes(0, 8) == 0 and lib.rsk_rows_blk_bytes(8, 0) == 0


def test_u64_workspace_slices_aligned_for_every_s():
    """The r04p2 fault class (a 64-bit atomic on a misaligned workspace word):
    rsk_check_ws_layout runs the layout arithmetic every entry point checks
    before it launches (the plan's zero-case halves, the rounds keys, the block
    maxima, the move tables and the persistent loop's LDS block row) for
    S = 1..4,100 at several node counts and move-table sizes: every u64 slice
    starts on an 8-B boundary.  Host arithmetic only (no device)."""
    from rsk import _lib
    lib = _lib.load_library()
    for N in (1, 63, 64, 65, 5_000, 50_000):
        for H in (0, 2, 4, 1024, 1 << 16):
            bad = [S for S in range(1, 4101) if lib.rsk_check_ws_layout(N, S, H) != 0]
            assert not bad, f"N={N} H={H}: misaligned at S={bad[:5]}: {lib.rsk_last_error().decode()}"
    assert lib.rsk_check_ws_layout(0, 1, 2) != 0 and lib.rsk_check_ws_layout(5, 0, 2) != 0


def test_library_is_gfx950_code_object():
    """The embedded device code object targets gfx950 (and nothing else)."""
    so = os.path.join(REPO, "kubernetes-rescheduling_amd", "rsk", "librsk.so")
    blob = open(so, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    assert not re.search(rb"amdgcn-amd-amdhsa--gfx9(0|4)\d", blob)


def test_randbelow_host_mt_matches_cpython():
    import random as pyrandom
    from rsk import api
    for seed in (0, 1, 7, 2**32 + 5, 123456789):
        for n in (1, 2, 3, 17, 1000, 99991):
            assert api.py_randbelow(seed, n) == pyrandom.Random(seed)._randbelow(n)


def test_kubescheduling_dropin_matches_reference(wm_golden, edge_golden):
    """kubescheduling is host-only (affinity merge + create): checkable without a GPU."""
    for k, snap in enumerate(wm_golden["snapshots"]):
        assert_dropin_matches("kubescheduling", snap, wm_golden["relation"], f"snapshot {k}")
    for case in edge_golden["cases"]:
        assert_dropin_matches("kubescheduling", case, case["relations"], case["name"])


def test_merge_affinity_levels():
    import rescheduling as R
    orig = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [{"a": 1}]},
                             "preferred": [1]},
            "podAffinity": {"x": 1}}
    patch = R.exclude_hazard_nodes(["w1"])
    out = R._merge_affinity(orig, patch)
    terms = out["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"]["nodeSelectorTerms"]
    assert terms[0] == {"a": 1} and terms[1]["matchExpressions"][0]["values"] == ["w1"]
    assert orig["nodeAffinity"]["requiredDuringSchedulingIgnoredDuringExecution"]["nodeSelectorTerms"] == [{"a": 1}]
    assert out["podAffinity"] == {"x": 1} and out["nodeAffinity"]["preferred"] == [1]
    assert R._merge_affinity(None, patch) == patch
    assert R._merge_affinity({}, {"k": 1}) == {"k": 1}
    # level-3 dicts are replaced, not merged
    a = {"x": {"y": {"z": {"old": 1}}}}
    assert R._merge_affinity(a, {"x": {"y": {"z": {"new": 2}}}}) == {"x": {"y": {"z": {"new": 2}}}}


def test_workmodel_relation_matches_reference(wm_golden):
    from rsk import workmodel
    calls = wm_golden["workmodel_calls"]
    wm = {s: {"external_services": [{"services": v}]} for s, v in calls.items()}
    ours = workmodel.relation_from_workmodel(wm)
    ref = wm_golden["relation"]
    assert set(ours) == set(ref)
    for k in ref:
        assert set(ours[k]) == set(ref[k]), k
        assert len(ours[k]) == len(set(ours[k]))
    rp, ci, miss = workmodel.relation_csr(ref, list(ref))
    assert rp[-1] == 38 and miss.sum() == 0  # 19 undirected edges, symmetrised


def test_synth_generator_pins():
    from rsk import synth
    c = synth.make_cluster(2000, 64, S=3, seed=0)
    assert c.nnz == 2 * (c.P - 1)
    assert int(np.diff(c.row_ptr).max()) == 61
    assert int(c.hazard.reshape(c.N, c.S)[:, 0].sum()) == 18
    # scenario-minor layout and recomputed per-scenario usage
    a = c.assign.reshape(c.P, c.S)
    assert (a[:, 1] != a[:, 0]).sum() <= c.P // 100
    use = c.use_cpu.reshape(c.N, c.S)
    for s in range(c.S):
        exp = c.bg_cpu + np.bincount(a[:, s], weights=c.pod_cpu, minlength=c.N)
        assert np.array_equal(use[:, s], exp.astype(np.int32))


def test_car_request_marshalling():
    from rsk import cluster
    cm = {"w1": {"node_cpu_capacity": 4000, "node_cpu_usage": 100, "pods": [
        {"podname": "b", "deploymentname": "b"}, {"podname": "z", "deploymentname": None}]},
          "w2": {"node_cpu_capacity": 4000, "node_cpu_usage": 200, "pods": [{"podname": "c", "deploymentname": "c"}]}}
    req = cluster.car_request("a", ["w2"], cm, {"a": ["b", "c", "b"]}, ["w1", "w2", "w1"])
    assert req.nodes == ["w1", "w2"]
    assert req.hazard.tolist() == [0, 1]
    assert req.assign.tolist() == [-1, 0]          # c sits on a hazard node: not scanned
    assert req.row_ptr.tolist() == [0, 1, 1]
    with pytest.raises(KeyError):
        cluster.car_request("a", [], {"w1": cm["w1"]}, {}, ["w1", "w3"])


def test_product_path_fails_loudly_without_gpu():
    """No silent CPU fallback: without a device the drop-in raises RskError."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("GPU present")
    import rescheduling as R
    from rsk._lib import RskError
    cm = {"w1": {"node_cpu_capacity": 4000, "node_cpu_usage": 100, "cpu_pct": 3, "pods": []}}
    info = {"metadata": {"name": "a"}, "spec": {"template": {"spec": {"affinity": None}}}}
    with pytest.raises(RskError):
        R.communication(info, [], cm, {}, ["w1"])
    for f in (R.spread, R.binpack):   # the single-launch S = 1 paths too
        with pytest.raises(RskError):
            f(dict(info), [], cm)


def test_stream_ordered_backend_rejects_default_stream(monkeypatch):
    """The row-sharded loop's stream-ordered backend binds librsk to the current
    torch stream; handle 0 (the legacy default stream) would read as "the
    context's own stream" and leave librsk and torch unordered — the cause of
    round 2's faulting gather.  It must refuse before any call."""
    torch = pytest.importorskip("torch")
    from rsk import dist as rdist

    class _Default:
        cuda_stream = 0

    monkeypatch.setattr(torch.cuda, "current_stream", lambda *a, **k: _Default())
    rp = np.array([0, 1, 2], np.int32)
    ci = np.array([1, 0], np.int32)
    with pytest.raises(ValueError, match="non-default"):
        rdist.LibrskRoundsBackend(rp, ci, np.array([100, 200], np.int32), device="cuda:0", stream_ordered=True)
