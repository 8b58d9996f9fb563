"""Snapshot replay and harness metrics (rsk/snapshot.py, csrc/rsk_snapshot.cpp;
SURVEY §8f items 3-4), pinned to fixtures the reference itself produced
(tests/golden/make_snapshots.py drives podmonitor.monitor, nodemonitor.node_resorce_std,
communicationcost.communication_cost and unit_convertion against the test stub).

CPU tests: the native quantity parser (host code in librsk.so), the Python
restatement, and the monitor() replay.  The two metrics run on the device; on
CPU their host logic is checked with the C oracle standing in for the two
kernels, and the ``gpu`` tests call the real kernels."""
import json
import math
import os

import numpy as np
import pytest

from conftest import load_golden

QTY = load_golden("quantities.json")
SNAP = load_golden("snapshots.json")


def _lib_or_skip():
    from rsk import _lib
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("librsk.so not built")


def dumps(state):
    """The stub cluster's state as the kubectl / metrics-API JSON dumps rsk.snapshot reads."""
    nodes = {"items": [{"metadata": {"name": n["name"]},
                        "status": {"capacity": {"cpu": n["cpu_capacity"], "memory": n["mem_capacity"]}}}
                       for n in state["nodes"]]}
    node_metrics = {"items": [{"metadata": {"name": k}, "usage": dict(v)} for k, v in state["node_usage"].items()]}
    pods = {"items": []}
    rs = {}
    for p in state["pods"]:
        owners = []
        if p.get("deployment"):
            owners = [{"kind": "ReplicaSet", "name": f"{p['deployment']}-rs"}]
            rs[f"{p['deployment']}-rs"] = p["deployment"]
        pods["items"].append({"metadata": {"name": p["name"], "namespace": p["namespace"], "ownerReferences": owners},
                              "spec": {"nodeName": p["node_name"]}})
    replicasets = {"items": [{"metadata": {"name": k, "ownerReferences": [{"kind": "Deployment", "name": v}]}}
                             for k, v in rs.items()]}
    pod_metrics = {"items": [{"metadata": {"name": k}, "containers": [{"usage": dict(c)} for c in v]}
                             for k, v in state["pod_usage"].get("default", {}).items()]}
    return nodes, node_metrics, pods, pod_metrics, replicasets


def _expect_conv(f, s, exp):
    if isinstance(exp, dict):
        with pytest.raises(Exception) as ei:
            f(s)
        assert type(ei.value).__name__ == exp["error"], (s, ei.value)
    else:
        assert f(s) == exp, s


@pytest.mark.parametrize("kind", ["cpu", "mem"])
def test_python_restatement_matches_reference(kind):
    from rsk import snapshot
    f = snapshot.cpu_conversion if kind == "cpu" else snapshot.mem_conversion
    for s, exp in QTY[kind]:
        _expect_conv(f, s, exp)


@pytest.mark.parametrize("kind", ["cpu", "mem"])
def test_native_parser_matches_reference(kind):
    _lib_or_skip()
    from rsk import snapshot
    k = snapshot.QTY_CPU if kind == "cpu" else snapshot.QTY_MEM
    i64 = [(s, e) for s, e in QTY[kind] if not isinstance(e, dict) and -2**63 <= e < 2**63]
    got = snapshot.parse_quantities([s for s, _ in i64], k)
    assert got.tolist() == [e for _, e in i64]
    for s, exp in QTY[kind]:
        if not isinstance(exp, dict) and not -2**63 <= exp < 2**63:
            exp = {"error": "OverflowError"}  # documented: the arrays are int64, Python's int is unbounded
        _expect_conv(lambda x: int(snapshot.parse_quantities([x], k)[0]), s, exp)


def test_native_parser_takes_the_common_spellings_itself():
    """The plain decimal grammar never falls back to Python (status 0)."""
    _lib_or_skip()
    import ctypes as C  # noqa: F401
    from rsk import _lib
    vals = [b"123456789n", b"250u", b"1500m", b"0.5", b"16318712Ki", b"7.5Gi", b"8000000000", b" 3 "]
    offs = np.zeros(len(vals) + 1, np.int64)
    np.cumsum([len(v) for v in vals], out=offs[1:])
    out = np.zeros(len(vals), np.int64)
    st = np.ones(len(vals), np.uint8)
    lib = _lib.load_library()
    assert lib.rsk_parse_quantities(b"".join(vals), offs.ctypes.data, len(vals), 0, out.ctypes.data,
                                    st.ctypes.data) == 0
    assert st[[0, 1, 2, 3, 7]].tolist() == [0] * 5
    assert out[[0, 1, 2, 3, 7]].tolist() == [123, 0, 1500, 500, 3000]
    assert lib.rsk_parse_quantities(b"".join(vals), offs.ctypes.data, len(vals), 1, out.ctypes.data,
                                    st.ctypes.data) == 0
    assert st[4:7].tolist() == [0, 0, 0] and out[4:7].tolist() == [16318712 * 1024, int(7.5 * 2**30), 8000000000]
    assert lib.rsk_parse_quantities(b"x", offs.ctypes.data, 1, 7, out.ctypes.data, st.ctypes.data) == 2


def _norm(x):
    return json.loads(json.dumps(x))


@pytest.mark.parametrize("i", range(len(SNAP["cases"])))
def test_monitor_replay_matches_reference(i):
    _lib_or_skip()
    from rsk import snapshot
    case = SNAP["cases"][i]
    exp = case["expect"]["monitor"]
    args = dumps(case["state"])
    if "error" in exp:
        with pytest.raises(Exception) as ei:
            snapshot.monitor(*args, warn=lambda *_: None)
        assert type(ei.value).__name__ == exp["error"]
        return
    nodes_name, spods, cm = snapshot.monitor(*args, warn=lambda *_: None)
    assert nodes_name == exp["nodes_name"]
    assert [p["metadata"]["name"] for p in spods] == exp["spods"]
    assert _norm(cm) == exp["cluster_monitoring"]
    if all(cm[n] for n in nodes_name):
        arr = snapshot.cluster_arrays(nodes_name, cm)
        assert len(arr.pods) == sum(len(cm[n]["pods"]) for n in nodes_name)
        assert np.array_equal(np.bincount(arr.assign, minlength=len(nodes_name)),
                              [len(cm[n]["pods"]) for n in nodes_name])


def _check_metrics(case, ctx=None):
    from rsk import snapshot
    nodes, node_metrics, pods, _, replicasets = dumps(case["state"])
    std = snapshot.node_resorce_std(nodes, node_metrics, ctx=ctx, warn=lambda *_: None)
    exp = case["expect"]["std"]
    if exp is None:
        assert std is None
    else:
        assert std is not None and math.isclose(std, exp, rel_tol=1e-12, abs_tol=1e-12), (std, exp)
    cost = snapshot.communication_cost(pods, SNAP["relation"], replicasets, ctx=ctx, warn=lambda *_: None)
    assert cost == case["expect"]["cost"]


def test_metrics_host_logic_with_oracle_kernels(monkeypatch):
    """The metric functions' host logic, with the oracle standing in for the two
    device kernels (CPU; the gpu test below runs the real kernels)."""
    _lib_or_skip()
    from oracle import oracle as orc
    from rsk import api
    monkeypatch.setattr(api, "load_std", lambda u, c, N, S, ctx=None: orc.load_std(u, c, N, S))
    monkeypatch.setattr(api, "cut_cost",
                        lambda rp, ci, a, P, S, missing=None, ctx=None: orc.cut_cost(rp, ci, a, P, S, missing))
    for case in SNAP["cases"]:
        _check_metrics(case)


@pytest.mark.gpu
def test_metrics_on_device_match_reference():
    from rsk import _lib
    ctx = _lib.default_context()
    for case in SNAP["cases"]:
        _check_metrics(case, ctx=ctx)


@pytest.mark.gpu
def test_monitors_cli_writes_reference_csv(tmp_path):
    """rsk.monitors on one recorded snapshot: the printed metrics and the CSV rows
    the reference's save_to_csv would append."""
    import csv
    from rsk import monitors
    case = next(c for c in SNAP["cases"] if c["expect"]["std"] is not None and c["expect"]["cost"] != -1)
    nodes, node_metrics, pods, _, rs = dumps(case["state"])
    d = tmp_path / "dump"
    d.mkdir()
    for name, obj in [("nodes", nodes), ("node_metrics", node_metrics), ("pods", pods), ("replicasets", rs),
                      ("relation", SNAP["relation"])]:
        (d / f"{name}.json").write_text(json.dumps(obj))
    out = tmp_path / "csv"
    assert monitors.main([str(d), "--csv-dir", str(out)]) == 0
    assert monitors.main([str(d), "--csv-dir", str(out)]) == 0
    rows = list(csv.reader(open(out / "communication_cost.csv")))
    assert rows[0] == ["timestamp", "cost"] and len(rows) == 3
    assert float(rows[1][1]) == case["expect"]["cost"]
    rows = list(csv.reader(open(out / "node_std.csv")))
    assert rows[0] == ["timestamp", "cpu_std"] and math.isclose(float(rows[2][1]), case["expect"]["std"],
                                                                rel_tol=1e-12, abs_tol=1e-12)
