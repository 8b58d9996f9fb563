"""CPU: pin the oracle (and the host marshalling it shares with the product)
against the reference's own outputs in tests/golden/ (SURVEY.md §8c).

No GPU, no reference import: everything here reads committed fixtures.
"""
import random as pyrandom

import numpy as np
import pytest

from helpers import ALGOS, golden_decision, oracle_decision


@pytest.mark.parametrize("algo", ALGOS)
def test_workmodel_snapshots_oracle(wm_golden, algo):
    rel = wm_golden["relation"]
    n = 0
    for k, snap in enumerate(wm_golden["snapshots"]):
        want = golden_decision(snap["results"][algo])
        got = oracle_decision(algo, snap, rel)
        assert got == want, f"snapshot {k} {algo}: oracle {got} vs reference {want}"
        n += 1
    assert n == 256


@pytest.mark.parametrize("algo", ALGOS)
def test_edge_cases_oracle(edge_golden, algo):
    for case in edge_golden["cases"]:
        want = golden_decision(case["results"][algo])
        got = oracle_decision(algo, case, case["relations"])
        assert got == want, f"{case['name']} {algo}: oracle {got} vs reference {want}"


def test_edge_case_coverage(edge_golden):
    by = {c["name"]: c for c in edge_golden["cases"]}
    car = {k: golden_decision(v["results"]["communication"]) for k, v in by.items()}
    assert car["all_hazard"][0] == "ValueError"
    assert car["car_overloaded_tie_none"] == (None, None, None)
    assert car["car_rem_all_minus1"] == (None, None, None)
    assert car["car_single_best_overloaded"][1] == "w1"
    assert golden_decision(by["all_hazard"]["results"]["spread"])[0] == "RuntimeError"
    assert golden_decision(by["name_order_ties"]["results"]["spread"])[2] == {"kubernetes.io/hostname": "w10"}


def test_synth_checksums_match_generator(synth_golden):
    """rsk.synth regenerates exactly the clusters the reference was run on."""
    import hashlib
    from rsk import synth
    for tag in ("2k64",):
        g = synth_golden[tag]
        c = synth.make_cluster(g["P"], g["N"], S=g["S"], seed=g["seed"])
        for k, h in g["checksums"].items():
            assert hashlib.sha256(np.ascontiguousarray(getattr(c, k)).tobytes()).hexdigest()[:16] == h, k
        assert int(np.diff(c.row_ptr).max()) == g["max_degree"]


def test_synth_2k64_car_oracle(synth_golden):
    from oracle import oracle as orc
    from rsk import synth
    g = synth_golden["2k64"]
    c = synth.make_cluster(g["P"], g["N"], S=g["S"], seed=g["seed"])
    names = c.node_names()
    order = sorted(range(c.N), key=names.__getitem__)
    rank = np.empty(c.N, np.int32)
    rank[order] = np.arange(c.N)
    cnt, _, _ = orc.node_reduce(c.assign, c.P, c.S, c.pod_cpu, c.pod_mem, c.N)
    for sc in g["scenarios"]:
        s = sc["s"]
        sub = lambda a: np.ascontiguousarray(a.reshape(-1, c.S)[:, s])  # noqa: E731
        t, _ = orc.car(c.row_ptr, c.col_idx, sub(c.assign), 1, c.cap_cpu, sub(c.use_cpu), sub(c.hazard), c.N,
                       rows=sc["pods"])
        assert t.tolist() == sc["car_target"], f"scenario {s}"
        haz = sub(c.hazard)
        assert int(haz.sum()) == sc["n_hazard"]
        assert int(orc.spread(sub(cnt), rank, haz, c.N, 1)[0]) == sc["spread"]
        assert int(orc.binpack(sub(c.cpu_pct), rank, haz, c.N, 1)[0]) == sc["binpack"]
        out, _ = orc.random(haz, c.N, 1, [sc["random_seed"]])
        assert int(out[0]) == sc["random"]


def test_synth_100k_car_oracle(synth_golden):
    """64+ sampled pods of the headline 100k/5k cluster (scenario 0)."""
    from oracle import oracle as orc
    from rsk import synth
    g = synth_golden["100k5k"]
    c = synth.make_cluster(g["P"], g["N"], S=1, seed=0)
    assert int(np.diff(c.row_ptr).max()) == g["max_degree"] == 531
    sc = g["scenarios"][0]
    assert int(c.hazard.sum()) == sc["n_hazard"] == 764
    t, _ = orc.car(c.row_ptr, c.col_idx, c.assign, 1, c.cap_cpu, c.use_cpu, c.hazard, c.N, rows=sc["pods"])
    assert t.tolist() == sc["car_target"]


def test_metrics_oracle(metrics_golden):
    from oracle import oracle as orc
    from rsk import workmodel
    m = metrics_golden
    # communication_cost (communicationcost.py:22-45): deployment -> node of its last pod
    for case in m["communication_cost"]:
        inf = {}
        for p in case["pods"]:
            if p["namespace"] == "default":
                inf[p["deployment"]] = p["node_name"]
        names = list(inf.keys())
        nodes = {n: i for i, n in enumerate(sorted({v for v in inf.values() if v is not None}))}
        assign = np.array([nodes[inf[d]] if inf[d] is not None else -1 for d in names], np.int32)
        rp, ci, miss = workmodel.relation_csr(case["relation"], names, dedup=False)
        d = int(orc.cut_cost(rp, ci, assign, len(names), 1, miss)[0])
        assert d / 2 == case["cost"]
    # node_resorce_std (nodemonitor.py:24-50)
    for case in m["node_std"]:
        if case["std"] is None:
            continue
        caps, uses = [], []
        cap_by = {}
        for n in case["nodes"]:
            cap_by[n["name"]] = int(round(float(n["cpu_capacity"]) * 1000))
        for name, u in case["usage"].items():
            if name == "master" or name not in cap_by:
                continue
            caps.append(cap_by[name])
            uses.append(_cpu_m(u["cpu"]))
        if not caps:
            assert case["std"] == 0.0
            continue
        v = float(orc.load_std(np.array(uses), np.array(caps), len(caps), 1)[0])
        assert v == pytest.approx(case["std"], rel=1e-12, abs=1e-12)
    # cpu_pct (get_resource_usage.py:37), including exact .5 boundaries
    pairs = np.array(m["cpu_pct_corner"]["pairs"], np.int64)
    want = m["cpu_pct_corner"]["pct"]
    got = orc.cpu_pct(pairs[:, 0].astype(np.int32), pairs[:, 1].astype(np.int32), len(pairs), 1)
    assert got.tolist() == want
    # detection (harzard_detect.py)
    for case in m["detection"]:
        names = case["nodes_name"]
        haz, most = orc.detect(case["cpu_pct"], len(names), 1)
        assert [n for n, h in zip(names, haz) if h] == case["hazard"]
        assert (names[most[0]] if most[0] >= 0 else "") == case["most"]
    # pick_max_pod (delete_replaced_pod.py:41-61)
    for case in m["pick_max_pod"]:
        pods = case["pods"]
        nodes = sorted({p[1] for p in pods} | {case["most"]})
        idx = {n: i for i, n in enumerate(nodes)}
        assign = np.array([idx[p[1]] for p in pods], np.int32)
        cpu = np.array([p[2] for p in pods], np.int32)
        r = int(orc.pick_max_pod(assign, cpu, len(pods), 1, [idx[case["most"]]])[0])
        assert (pods[r][0] if r >= 0 else None) == case["picked"]


def _cpu_m(s):
    """unit_convertion.cpu_conversion semantics (pinned by metrics.json['unit'])."""
    s = str(s).strip()
    if s.endswith("m"):
        return int(float(s[:-1]))
    if s.endswith("n"):
        return int(round(float(s[:-1]) / 1_000_000))
    if s.endswith("u"):
        return int(round(float(s[:-1]) / 1000))
    return int(round(float(s) * 1000))


def test_unit_conversion_pins(metrics_golden):
    for kind, s, v in metrics_golden["unit"]:
        if kind == "cpu":
            assert _cpu_m(s) == v


def test_py_randbelow_matches_cpython():
    from oracle import oracle as orc
    rng = np.random.default_rng(3)
    for _ in range(400):
        seed = int(rng.integers(0, 2**40)) if rng.random() < 0.5 else int(rng.integers(0, 1000))
        n = int(rng.integers(1, 100000))
        assert orc.py_randbelow(seed, n) == pyrandom.Random(seed)._randbelow(n)
    assert orc.py_randbelow(0, 7) == pyrandom.Random(0)._randbelow(7)


def test_python_restatements_match_golden_and_c_oracle(synth_golden):
    """oracle/car_py.py's literal and numpy CAR restatements (bench.py's extra
    CPU legs) against the reference's 2k/64 decisions and, on
    random tie-heavy cases, against the C oracle."""
    from oracle import car_py
    from oracle import oracle as orc
    from rsk import synth
    g = synth_golden["2k64"]
    c = synth.make_cluster(g["P"], g["N"], S=g["S"], seed=g["seed"])
    for sc in g["scenarios"]:
        s = sc["s"]
        a, u, h = car_py.scenario_view(c.assign, c.use_cpu, c.hazard, c.P, c.N, c.S, s)
        by_node = car_py.pods_by_node(a, c.N)
        haz_list = [n for n in range(c.N) if h[n]]
        nbrs = car_py.dedup_rows(c.row_ptr, c.col_idx, sc["pods"])
        lit = [car_py.car_literal(nb.tolist(), by_node, haz_list, c.cap_cpu, u) for nb in nbrs]
        vec = [car_py.car_numpy(nb, a, c.cap_cpu, u, h, c.N) for nb in nbrs]
        assert lit == sc["car_target"] and vec == sc["car_target"], f"scenario {s}"
    rng = np.random.default_rng(12)
    for trial in range(40):
        N, P = int(rng.integers(1, 9)), int(rng.integers(2, 40))
        rows = [rng.integers(0, P, int(rng.integers(0, 6))) for _ in range(P)]
        rp = np.zeros(P + 1, np.int32)
        rp[1:] = np.cumsum([len(r) for r in rows])
        ci = np.concatenate(rows + [np.zeros(0, np.int64)]).astype(np.int32)
        a = rng.integers(-1, N, P).astype(np.int32)
        cap = rng.choice([1000, 2000], N).astype(np.int32)
        use = rng.choice([0, 1000, 1500, 2000, 2500], N).astype(np.int32)
        h = (rng.random(N) < 0.3).astype(np.uint8)
        drp, dci = orc.dedup_csr(rp, ci)  # the C oracle takes relation sets (rows deduplicated)
        exp, _ = orc.car(drp, dci, a, 1, cap, use, h, N)
        by_node = car_py.pods_by_node(a, N)
        haz_list = [n for n in range(N) if h[n]]
        for p, nb in enumerate(car_py.dedup_rows(rp, ci, range(P))):
            assert car_py.car_literal(nb.tolist(), by_node, haz_list, cap, use) == exp[p], (trial, p)
            assert car_py.car_numpy(nb, a, cap, use, h, N) == exp[p], (trial, p)


def _pick_edge_arrays(case):
    pods = case["pods"]
    nodes = sorted({p[1] for p in pods} | {case["most"]})
    idx = {n: i for i, n in enumerate(nodes)}
    assign = np.array([idx[p[1]] for p in pods], np.int32)
    cpu = np.array([-1 if p[2] is None else p[2] for p in pods], np.int32)   # no metrics -> -1 (rsk/snapshot.py)
    return pods, assign, cpu, idx[case["most"]]


def pick_edge_expected(case):
    """The build's documented answer: the reference's pick where
    it returns; where it raises TypeError (a pod without metrics on the hazard node
    meets the ("0", "0") default), the first max-CPU pod among those with metrics."""
    if "picked" in case:
        return case["picked"]
    assert case["raises"] == "TypeError"
    best, name = -1, None
    for n, node, c in case["pods"]:
        if node == case["most"] and c is not None and c > best:
            best, name = c, n
    return name


def test_pick_max_pod_metric_edges_vs_reference():
    """pick_edges.json (tests/golden/make_pick_edges.py, the reference run here):
    0-CPU pods, ties and missing-elsewhere pods match the reference exactly; the
    16 cases where the reference raises TypeError get the documented divergence."""
    import json
    import os
    from oracle import oracle as orc
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pick_edges.json")) as f:
        cases = json.load(f)["cases"]
    raised = 0
    for case in cases:
        pods, assign, cpu, most = _pick_edge_arrays(case)
        r = int(orc.pick_max_pod(assign, cpu, len(pods), 1, [most])[0])
        assert (pods[r][0] if r >= 0 else None) == pick_edge_expected(case), case
        raised += "raises" in case
    assert raised >= 10 and any(c.get("picked") and any(p[2] == 0 for p in c["pods"]) for c in cases)


def _sparse_as_car(monkeypatch):
    from oracle import oracle as orc
    monkeypatch.setattr(orc, "car", orc.car_sparse)


@pytest.mark.parametrize("fixture", ["wm", "edge"])
def test_car_sparse_against_reference_fixtures(monkeypatch, wm_golden, edge_golden, fixture):
    """The sparse CAR restatement (oracle_car_sparse, the full-batch checker of
    tests/test_gpu_headline.py) decides the reference's own 256 workmodel
    snapshots and 40 edge cases exactly as the reference did."""
    _sparse_as_car(monkeypatch)
    if fixture == "wm":
        for k, snap in enumerate(wm_golden["snapshots"]):
            assert oracle_decision("communication", snap, wm_golden["relation"]) == \
                golden_decision(snap["results"]["communication"]), k
    else:
        for case in edge_golden["cases"]:
            assert oracle_decision("communication", case, case["relations"]) == \
                golden_decision(case["results"]["communication"]), case["name"]


def test_car_sparse_synth_golden(synth_golden):
    """... and the reference's 2k/64 (8 scenarios) and 100k/5k decisions."""
    from oracle import oracle as orc
    from rsk import synth
    g = synth_golden["2k64"]
    c = synth.make_cluster(g["P"], g["N"], S=g["S"], seed=g["seed"])
    t, _ = orc.car_sparse(c.row_ptr, c.col_idx, c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N, threads=4)
    t = t.reshape(c.P, c.S)
    for sc in g["scenarios"]:
        assert t[sc["pods"], sc["s"]].tolist() == sc["car_target"], sc["s"]
    g = synth_golden["100k5k"]
    c = synth.make_cluster(g["P"], g["N"], S=1, seed=0)
    sc = g["scenarios"][0]
    t, _ = orc.car_sparse(c.row_ptr, c.col_idx, c.assign, 1, c.cap_cpu, c.use_cpu, c.hazard, c.N, rows=sc["pods"])
    assert t.tolist() == sc["car_target"]


@pytest.mark.parametrize("seed", range(6))
def test_car_sparse_equals_car_one(seed):
    """oracle_car_sparse == oracle_car (the literal per-cell restatement) on
    random graphs built to hit every branch: duplicate entries and self edges
    (the literal one counts entries as given), assignments outside [0, N),
    hazard densities up to all-hazard, crowded ties with rem < 0 (None), a
    single non-hazard node (the zero case's outright winner), empty rows, hubs,
    row subsets and S not a multiple of the 16-scenario block."""
    from oracle import oracle as orc
    rng = np.random.default_rng(900 + seed)
    seen = set()
    for trial in range(12):
        N = int(rng.choice([1, 2, 3, 7, 40, 300]))
        P = int(rng.integers(2, 400))
        S = int(rng.choice([1, 5, 16, 17, 40]))
        lens = rng.integers(0, 7, P)
        lens[rng.integers(0, P, 3)] = rng.integers(20, 120, 3)
        rp = np.zeros(P + 1, np.int32)
        rp[1:] = np.cumsum(lens)
        ci = rng.integers(0, P, int(rp[-1])).astype(np.int32)
        a = rng.integers(-2, N + 2, P * S).astype(np.int32)
        cap = rng.choice([1000, 2000, 4000], N).astype(np.int32)
        use = rng.choice([0, 999, 1000, 1001, 2000, 2500, 5000], N * S).astype(np.int32)
        p_h = float(rng.choice([0.0, 0.3, 0.9, 1.0]))
        h = (rng.random(N * S) < p_h).astype(np.uint8)
        if trial % 4 == 3:            # exactly one non-hazard node in every scenario
            h[:] = 1
            h.reshape(N, S)[rng.integers(0, N), :] = 0
        rows = None if trial % 2 else np.sort(rng.choice(P, min(P, 50), replace=False)).astype(np.int32)
        et, es = orc.car(rp, ci, a, S, cap, use, h, N, rows=rows)
        gt, gs = orc.car_sparse(rp, ci, a, S, cap, use, h, N, rows=rows, threads=3)
        assert np.array_equal(gt, et), (seed, trial, int((gt != et).sum()))
        assert np.array_equal(gs, es), (seed, trial)
        seen.update(np.unique(np.minimum(et, 0)).tolist())
    assert seen == {-2, -1, 0}, seen    # no candidate, None and real targets all occurred
