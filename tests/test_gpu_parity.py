"""GPU parity: librsk.so (gfx950) against the reference fixtures and the oracle.

Bit-exact for every placement / integer output; fp64 metrics within 1e-9 rel
(north_star allows 1e-5).  All calls go through the C-ABI (ctypes).
"""
import os

import numpy as np
import pytest

from helpers import ALGOS, assert_dropin_matches

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from rsk import _lib
    return _lib.default_context()


# ---------------------------------------------------------------------------
# drop-in module vs the reference's own decisions
# ---------------------------------------------------------------------------

@pytest.mark.parametrize("algo", ALGOS)
def test_dropin_workmodel_snapshots(ctx, wm_golden, algo):
    for k, snap in enumerate(wm_golden["snapshots"]):
        assert_dropin_matches(algo, snap, wm_golden["relation"], f"snapshot {k}")


@pytest.mark.parametrize("algo", ALGOS)
def test_dropin_edge_cases(ctx, edge_golden, algo):
    for case in edge_golden["cases"]:
        assert_dropin_matches(algo, case, case["relations"], case["name"])


# ---------------------------------------------------------------------------
# batched CAR vs golden and oracle
# ---------------------------------------------------------------------------

def _dedup_csr(row_ptr, col_idx):
    rp, ci = [0], []
    for p in range(len(row_ptr) - 1):
        nb = sorted(set(int(q) for q in col_idx[row_ptr[p]:row_ptr[p + 1]]) - {p})
        ci += nb
        rp.append(len(ci))
    return np.array(rp, np.int32), np.array(ci, np.int32)


def _check_car(ctx, row_ptr, col_idx, assign, S, cap, use, haz, N, rows=None, label=""):
    from oracle import oracle as orc
    from rsk import api
    tgt, sc = api.car_place(row_ptr, col_idx, assign, S, cap, use, haz, N, rows=rows, ctx=ctx, want_score=True)
    rp, ci = _dedup_csr(row_ptr, col_idx)
    ot, osc = orc.car(rp, ci, assign, S, cap, use, haz, N, rows=rows)
    bad = np.nonzero(tgt != ot)[0]
    assert bad.size == 0, f"{label}: {bad.size} targets differ, first cell {bad[0]}: gpu {tgt[bad[0]]} oracle {ot[bad[0]]}"
    assert np.array_equal(sc, osc), f"{label}: scores differ"
    return tgt


def test_car_synth_2k64_golden(ctx, synth_golden):
    from rsk import api, synth
    g = synth_golden["2k64"]
    c = synth.make_cluster(g["P"], g["N"], S=g["S"], seed=0)
    tgt, _ = api.car_place(c.row_ptr, c.col_idx, c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N, ctx=ctx)
    t = tgt.reshape(c.P, c.S)
    for sc in g["scenarios"]:
        assert t[sc["pods"], sc["s"]].tolist() == sc["car_target"], f"scenario {sc['s']}"
    _check_car(ctx, c.row_ptr, c.col_idx, c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N, label="2k64 all rows")


def test_car_synth_100k_golden(ctx, synth_golden):
    from rsk import api, synth
    g = synth_golden["100k5k"]
    c = synth.make_cluster(g["P"], g["N"], S=1, seed=0)
    sc = g["scenarios"][0]
    tgt, _ = api.car_place(c.row_ptr, c.col_idx, c.assign, 1, c.cap_cpu, c.use_cpu, c.hazard, c.N, ctx=ctx)
    assert tgt[sc["pods"]].tolist() == sc["car_target"]


def test_car_synth_100k_s64_sampled(ctx):
    """Headline cluster with 64 scenarios; oracle on 1500 sampled rows incl. every heavy row."""
    from oracle import oracle as orc
    from rsk import api, synth
    c = synth.make_cluster(100000, 5000, S=64, seed=0)
    plan = api.CarPlan(c.row_ptr, c.col_idx, ctx=ctx)
    tgt, sc = plan.execute(c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N, want_score=True)
    deg = np.diff(c.row_ptr)
    rng = np.random.default_rng(5)
    rows = np.unique(np.concatenate([np.nonzero(deg > 16)[0], rng.choice(c.P, 1500, replace=False)]))
    ot, osc = orc.car(c.row_ptr, c.col_idx, c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N, rows=rows, threads=8)
    t = tgt.reshape(c.P, c.S)[rows].reshape(-1)
    assert np.array_equal(t, ot)
    assert np.array_equal(sc.reshape(c.P, c.S)[rows].reshape(-1), osc)


def _random_case(rng, P, N, S, max_deg, hub_deg=(), p_haz=0.3, overload=0.2, tie_heavy=False):
    rows = [[] for _ in range(P)]
    for p in range(P):
        d = int(rng.integers(0, max_deg + 1))
        rows[p] = rng.integers(0, P, d).tolist()
    for k, hd in enumerate(hub_deg):
        if k < P:
            rows[k] = rng.integers(0, P, hd).tolist() + [k, k]  # duplicates + self loop
    row_ptr = np.zeros(P + 1, np.int32)
    row_ptr[1:] = np.cumsum([len(r) for r in rows])
    col_idx = np.array([q for r in rows for q in r], np.int32)
    nn = max(1, N // 4) if tie_heavy else N
    assign = rng.integers(-1, nn, P * S).astype(np.int32)
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    if tie_heavy:
        use = np.repeat(rng.choice([1000, 3000], N).astype(np.int32), S)
    else:
        use = rng.integers(0, 8000, N * S).astype(np.int32)
    over = rng.random(N * S) < overload
    use[over] = (np.repeat(cap, S)[over] + rng.integers(0, 3, over.sum())).astype(np.int32)
    haz = (rng.random(N * S) < p_haz).astype(np.uint8)
    return row_ptr, col_idx, assign, cap, use, haz


@pytest.mark.parametrize("S", [1, 3, 64, 100, 130])
def test_car_random_graphs(ctx, S):
    rng = np.random.default_rng(100 + S)
    for trial in range(4):
        N = int(rng.choice([1, 2, 5, 40, 300]))
        P = int(rng.integers(20, 400))
        hubs = [17, 65, 300, 1100] if trial == 3 else [20, 70]
        rp, ci, a, cap, use, haz = _random_case(rng, P, N, S, max_deg=int(rng.choice([2, 8, 16])), hub_deg=hubs,
                                                p_haz=float(rng.choice([0.0, 0.3, 0.95])),
                                                tie_heavy=bool(trial % 2))
        _check_car(ctx, rp, ci, a, S, cap, use, haz, N, label=f"S={S} trial={trial} N={N} P={P}")


@pytest.mark.parametrize("S", [1, 64, 65])
def test_car_degree_bucket_boundaries(ctx, S):
    """Rows at every routing boundary: tile classes 1/2/4/8/16/32 < mid 64 < hub classes 128/256/512/1024."""
    rng = np.random.default_rng(300 + S)
    hubs = [2, 3, 4, 5, 8, 9, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 511, 512, 513]
    P, N = 1400, 60
    rp, ci, a, cap, use, haz = _random_case(rng, P, N, S, max_deg=3, hub_deg=hubs, p_haz=0.2)
    _check_car(ctx, rp, ci, a, S, cap, use, haz, N, label=f"boundaries S={S}")
    from rsk import api
    info = api.CarPlan(rp, ci, ctx=ctx).info()
    # 17..32 in the tiles (sorted class), 33..64 and > 64 side rows
    assert info["sorted_rows"] >= 3, info
    assert info["mid_rows"] >= 3 and info["heavy_rows"] >= 5 and info["tile_rows"] > 0, info


@pytest.mark.parametrize("S", [1, 40])
def test_car_hub_exact_degrees_and_counter_limits(ctx, S):
    """Hub rows of exact degree at the hub class edges (u8 counters up to 255,
    u16 from 256, register entries up to 1024, LDS re-reads beyond), with
    scenarios that pile every neighbour onto one node (count == degree)."""
    rng = np.random.default_rng(400 + S)
    degs = [65, 127, 128, 129, 254, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 2049]
    P, N = 2200, 30
    rows = [rng.choice(P, d, replace=False).tolist() for d in degs]
    rows = [[q for q in r if q != k] for k, r in enumerate(rows)]
    rows += [rng.integers(0, P, int(rng.integers(0, 4))).tolist() for _ in range(P - len(degs))]
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.array([q for r in rows for q in r], np.int32)
    a = rng.integers(-1, N, (P, S)).astype(np.int32)
    a[:, 0] = 7                      # scenario 0: every pod on node 7 -> count == degree
    if S > 1:
        a[:, 1] = rng.integers(0, 2, P)  # two nodes, near-ties
    a = a.reshape(-1)
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    use = rng.integers(0, 8000, N * S).astype(np.int32)
    haz = (rng.random(N * S) < 0.1).astype(np.uint8)
    haz.reshape(N, S)[7, 0] = 0
    qrows = np.arange(0, len(degs) + 20, dtype=np.int32)
    tgt = _check_car(ctx, rp, ci, a, S, cap, use, haz, N, rows=qrows, label=f"hub degrees S={S}")
    assert (tgt.reshape(len(qrows), S)[:len(degs), 0] == 7).all()


def test_car_heavy_hash_path_large_n(ctx):
    """N > 16384 switches heavy rows from direct LDS count tables to the LDS hash."""
    rng = np.random.default_rng(21)
    for S in (1, 5, 64):
        P, N = 600, 20000
        rp, ci, a, cap, use, haz = _random_case(rng, P, N, S, max_deg=4, hub_deg=[40, 200, 700], p_haz=0.2)
        a[:] = rng.integers(-1, 300, P * S)  # crowd the neighbours onto few nodes -> real counts and ties
        _check_car(ctx, rp, ci, a, S, cap, use, haz, N, rows=np.arange(0, 60, dtype=np.int32), label=f"hash S={S}")


def test_car_huge_n_alt_plan(ctx):
    """N >= 2^24 - 1: node ids no longer fit the tiles' packed (node << 8 | row)
    sort words, so the plan's N >= kPackMaxN variant sends rows 17..64 to the
    mid kernel.  Neighbours crowd onto node ids around 2^24 for real counts."""
    rng = np.random.default_rng(31)
    N, S, P = (1 << 24) + 5, 2, 500
    hubs = [17, 20, 31, 32, 33, 40, 63, 64, 65, 100]
    rp, ci, a, cap, use, haz = _random_case(rng, P, N, S, max_deg=12, hub_deg=hubs, p_haz=0.2)
    pool = np.array([0, 5, (1 << 24) - 2, (1 << 24) - 1, 1 << 24, N - 1], np.int32)
    a[:] = rng.choice(pool, P * S)
    a[rng.random(P * S) < 0.05] = -1
    haz.reshape(N, S)[pool] = 0
    _check_car(ctx, rp, ci, a, S, cap, use, haz, N, label="N >= 2^24")


def test_car_all_hazard_and_rows_subset(ctx):
    rng = np.random.default_rng(7)
    P, N, S = 300, 12, 70
    rp, ci, a, cap, use, haz = _random_case(rng, P, N, S, max_deg=6, hub_deg=[40])
    haz.reshape(N, S)[:, 5] = 1          # scenario 5: every node hazard -> ValueError cells
    haz.reshape(N, S)[:, 6] = 1
    haz.reshape(N, S)[3, 6] = 0          # scenario 6: exactly one candidate
    rows = np.array([0, 5, 5, 299, 17, 0], np.int32)
    tgt = _check_car(ctx, rp, ci, a, S, cap, use, haz, N, rows=rows, label="subset")
    t = tgt.reshape(len(rows), S)
    assert (t[:, 5] == -2).all()
    assert (t[:, 6] == 3).all()


def test_car_device_mode_matches_host(ctx):
    import torch
    from rsk import api, synth
    c = synth.make_cluster(2000, 64, S=96, seed=3)
    plan = api.CarPlan(c.row_ptr, c.col_idx, ctx=ctx)
    host_t, host_s = plan.execute(c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N, want_score=True)
    dev = torch.device("cuda", ctx.device)
    T = {k: torch.from_numpy(getattr(c, k)).to(dev) for k in ("assign", "cap_cpu", "use_cpu", "hazard")}
    out_t = torch.empty(c.P * c.S, dtype=torch.int32, device=dev)
    out_s = torch.empty_like(out_t)
    ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    try:
        plan.execute(T["assign"], c.S, T["cap_cpu"], T["use_cpu"], T["hazard"], c.N, out_t, out_s, device=True)
        torch.cuda.synchronize(dev)
    finally:
        ctx.set_stream(None)
    assert np.array_equal(out_t.cpu().numpy(), host_t)
    assert np.array_equal(out_s.cpu().numpy(), host_s)


# ---------------------------------------------------------------------------
# spread / binpack / random / kernel-3 reductions vs oracle
# ---------------------------------------------------------------------------

def test_baselines_vs_oracle(ctx, synth_golden):
    from oracle import oracle as orc
    from rsk import api, synth
    c = synth.make_cluster(2000, 64, S=8, seed=0)
    names = c.node_names()
    rank = np.argsort(np.argsort(np.array(names))).astype(np.int32)
    cnt, cpu, mem = api.node_reduce(c.assign, c.P, c.S, c.pod_cpu, c.pod_mem, c.N, ctx=ctx)
    ocnt, ocpu, omem = orc.node_reduce(c.assign, c.P, c.S, c.pod_cpu, c.pod_mem, c.N)
    assert np.array_equal(cnt, ocnt) and np.array_equal(cpu, ocpu) and np.array_equal(mem, omem)
    assert np.array_equal(cpu.reshape(c.N, c.S) + c.bg_cpu[:, None], c.use_cpu.reshape(c.N, c.S))
    sp = api.spread_place(cnt, rank, c.hazard, c.N, c.S, ctx=ctx)
    bp = api.binpack_place(c.cpu_pct, rank, c.hazard, c.N, c.S, ctx=ctx)
    assert np.array_equal(sp, orc.spread(cnt, rank, c.hazard, c.N, c.S))
    assert np.array_equal(bp, orc.binpack(c.cpu_pct, rank, c.hazard, c.N, c.S))
    seeds = np.array([sc["random_seed"] for sc in synth_golden["2k64"]["scenarios"]], np.uint64)
    rd = api.random_place(c.hazard, c.N, c.S, seeds, ctx=ctx)
    ord_, ocnt2 = orc.random(c.hazard, c.N, c.S, seeds)
    assert np.array_equal(rd, ord_)
    assert np.array_equal(api.random_count(c.hazard, c.N, c.S, ctx=ctx), ocnt2)
    for sc in synth_golden["2k64"]["scenarios"]:
        s = sc["s"]
        assert (sp[s], bp[s], rd[s]) == (sc["spread"], sc["binpack"], sc["random"])


def test_baselines_ties_and_empty(ctx):
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(11)
    for N, S in [(1, 1), (5, 7), (37, 64), (300, 129)]:
        val = rng.integers(-1, 3, N * S).astype(np.int32)
        rank = rng.permutation(N).astype(np.int32)
        haz = (rng.random(N * S) < 0.4).astype(np.uint8)
        haz.reshape(N, S)[:, 0] = 1
        assert np.array_equal(api.spread_place(val, rank, haz, N, S, ctx=ctx), orc.spread(val, rank, haz, N, S))
        assert np.array_equal(api.binpack_place(val, rank, haz, N, S, ctx=ctx), orc.binpack(val, rank, haz, N, S))
        r = rng.integers(-1, N + 1, S).astype(np.int32)
        got = api.random_select(haz, N, S, r, ctx=ctx)
        for s in range(S):
            free = [n for n in range(N) if not haz[n * S + s]]
            exp = free[r[s]] if 0 <= r[s] < len(free) else -2
            assert got[s] == exp
    # extreme values on the S = 1 single-workgroup path: binpack's
    # key for cpu_pct == INT32_MIN on name rank 0 is the all-zero word
    for val0 in (np.iinfo(np.int32).min, np.iinfo(np.int32).max):
        for N in (1, 3, 70):
            val = np.full(N, val0, np.int32)
            rank = np.arange(N, dtype=np.int32)[::-1].copy()
            rank[0], rank[-1] = rank[-1], rank[0]
            haz = np.zeros(N, np.uint8)
            assert api.binpack_place(val, rank, haz, N, 1, ctx=ctx)[0] == orc.binpack(val, rank, haz, N, 1)[0]
            assert api.spread_place(val, rank, haz, N, 1, ctx=ctx)[0] == orc.spread(val, rank, haz, N, 1)[0]


@pytest.mark.parametrize("N,S", [(1, 1), (5, 2), (40_000, 1), (3_001, 8), (20_000, 64), (777, 128), (9_000, 256),
                                 (1_500, 12), (2_000, 300), (600, 4096)])
def test_load_std_shapes(ctx, N, S):
    """rsk_load_std over the partial-kernel shapes: S dividing 256 (a workgroup
    folds 256 / S whole chunks before writing), S = 256 and S that does not
    divide it (one partial per chunk), S not a multiple of 8 (the merge's
    XCD-grouped scenario order falls back to the identity), ragged last
    chunks and a partly filled last workgroup, cap <= 0 nodes skipped
    (nodemonitor.py:38-43); within 1e-9 relative of the oracle."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(N * 7 + S)
    cap = rng.integers(1_000, 64_000, N).astype(np.int32)
    if N > 4:
        cap[rng.choice(N, N // 5, replace=False)] = 0
        cap[rng.choice(N, N // 9, replace=False)] = -3
    use = rng.integers(0, 64_000, (N, S)).astype(np.int32).reshape(-1)
    std = api.load_std(use, cap, N, S, ctx=ctx)
    ostd = orc.load_std(use, cap, N, S)
    np.testing.assert_allclose(std, ostd, rtol=1e-9, atol=1e-12)


def test_metrics_vs_oracle(ctx):
    from oracle import oracle as orc
    from rsk import api, synth
    c = synth.make_cluster(3000, 97, S=33, seed=9)
    pct = api.cpu_pct(c.use_cpu, c.cap_cpu, c.N, c.S, ctx=ctx)
    assert np.array_equal(pct, orc.cpu_pct(c.use_cpu, c.cap_cpu, c.N, c.S))
    assert np.array_equal(pct, c.cpu_pct)
    haz, most = api.detect(pct, c.N, c.S, ctx=ctx)
    oh, om = orc.detect(pct, c.N, c.S)
    assert np.array_equal(haz, oh) and np.array_equal(most, om)
    std = api.load_std(c.use_cpu, c.cap_cpu, c.N, c.S, ctx=ctx)
    ostd = orc.load_std(c.use_cpu, c.cap_cpu, c.N, c.S)
    np.testing.assert_allclose(std, ostd, rtol=1e-9, atol=1e-12)
    npstd = np.std(c.use_cpu.reshape(c.N, c.S) / c.cap_cpu[:, None] * 100, axis=0)
    np.testing.assert_allclose(std, npstd, rtol=1e-9)
    cut = api.cut_cost(c.row_ptr, c.col_idx, c.assign, c.P, c.S, ctx=ctx)
    assert np.array_equal(cut, orc.cut_cost(c.row_ptr, c.col_idx, c.assign, c.P, c.S))
    pm = api.pick_max_pod(c.assign, c.pod_cpu, c.P, c.S, most, ctx=ctx)
    assert np.array_equal(pm, orc.pick_max_pod(c.assign, c.pod_cpu, c.P, c.S, most))


def test_cpu_pct_round_half_even(ctx, metrics_golden):
    from rsk import api
    pairs = np.array(metrics_golden["cpu_pct_corner"]["pairs"], np.int64)
    got = api.cpu_pct(pairs[:, 0].astype(np.int32), pairs[:, 1].astype(np.int32), len(pairs), 1, ctx=ctx)
    # N = len(pairs), S = 1: cap is per node, one node per pair
    assert got.tolist() == metrics_golden["cpu_pct_corner"]["pct"]


def test_cut_cost_golden(ctx, metrics_golden):
    from rsk import api, workmodel
    for case in metrics_golden["communication_cost"]:
        inf = {}
        for p in case["pods"]:
            if p["namespace"] == "default":
                inf[p["deployment"]] = p["node_name"]
        names = list(inf)
        nodes = {n: i for i, n in enumerate(sorted({v for v in inf.values() if v is not None}))}
        assign = np.array([nodes[inf[d]] if inf[d] is not None else -1 for d in names], np.int32)
        rp, ci, miss = workmodel.relation_csr(case["relation"], names, dedup=False)
        d = int(api.cut_cost(rp, ci, assign, len(names), 1, miss, ctx=ctx)[0])
        assert d / 2 == case["cost"]


# ---------------------------------------------------------------------------
# compact path (N <= 65535): 16-bit node codes + exact resolution of equal codes
# ---------------------------------------------------------------------------

def _crowded_rem_case(rng, P, N, S, hubs, neg_frac=0.1):
    """Remaining CPU crowded into single 16-bit code buckets (spacing 1 below
    2^14, 2..32 up to 2^19, one bucket above): ties between distinct nodes that
    only the exact cap - use comparison can order."""
    rp, ci, a, _, _, haz = _random_case(rng, P, N, S, max_deg=int(rng.choice([4, 12, 30])), hub_deg=hubs, p_haz=0.1)
    a[:] = rng.integers(-1, min(N, 24), P * S)  # neighbours on few nodes: real counts and many-way ties
    base = rng.choice([3000, 20000, 100000, 300000, 600000, 1 << 29], N).astype(np.int64)
    cap = (base + 5000).astype(np.int32)
    rem = base[:, None] + rng.integers(0, 4, (N, S))         # within one code bucket above 2^14
    neg = rng.random((N, S)) < neg_frac
    rem[neg] = -rng.integers(1, 5, neg.sum())                  # rem < 0: all one code
    use = (cap.astype(np.int64)[:, None] - rem).astype(np.int32).reshape(-1)
    return rp, ci, a, cap, use, haz


@pytest.mark.parametrize("S", [1, 7, 64, 100])
def test_car_code_collisions_exact(ctx, S):
    rng = np.random.default_rng(500 + S)
    hubs = [3, 5, 9, 16, 17, 20, 31, 32, 33, 40, 64, 65, 130, 300]
    for N in (7, 300, 5000):
        rp, ci, a, cap, use, haz = _crowded_rem_case(rng, 900, N, S, hubs)
        _check_car(ctx, rp, ci, a, S, cap, use, haz, N, label=f"collisions S={S} N={N}")


@pytest.mark.parametrize("S", [1, 64, 70])
def test_car_invalid_assign_values_never_alias(ctx, S):
    """Assignments outside [0, N) mean "on no node" (include/rsk.h): values that
    truncate to a real 16-bit node id (65536 + x, -2 = 0xfffe) must not add to
    that node's score."""
    rng = np.random.default_rng(600 + S)
    P, N = 1200, 300
    rp, ci, a, cap, use, haz = _random_case(rng, P, N, S, max_deg=16, hub_deg=[20, 40, 70], p_haz=0.1)
    x = rng.integers(0, 8, P * S)
    bad = rng.random(P * S) < 0.4
    pool = np.array([-2, -1, -65536, 65536, 65536 + 3, 131072 + 5, N, N + 5, 2 ** 31 - 1], np.int64)
    a = np.where(bad, rng.choice(pool, P * S), x).astype(np.int32)
    _check_car(ctx, rp, ci, a, S, cap, use, haz, N, label=f"invalid S={S}")


def test_car_wide_path_n_above_u16(ctx):
    """65535 < N < 2^24: the wide tile kernel (int2 {node, key} image)."""
    rng = np.random.default_rng(41)
    N, P = 70000, 800
    for S in (1, 33):
        rp, ci, a, cap, use, haz = _random_case(rng, P, N, S, max_deg=12, hub_deg=[17, 33, 65, 200], p_haz=0.2)
        pool = np.array([0, 3, 65534, 65535, 65536, 65537, N - 1], np.int32)
        a[:] = rng.choice(pool, P * S)
        a[rng.random(P * S) < 0.05] = -1
        haz.reshape(N, S)[pool] = 0
        _check_car(ctx, rp, ci, a, S, cap, use, haz, N, label=f"wide S={S}")


def test_car_score_variant_matches(ctx):
    """want_score=False (the bench's template instance) gives the same targets."""
    from rsk import api, synth
    c = synth.make_cluster(5000, 300, S=128, seed=4)
    plan = api.CarPlan(c.row_ptr, c.col_idx, ctx=ctx)
    t0, _ = plan.execute(c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N)
    t1, _ = plan.execute(c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N, want_score=True)
    assert np.array_equal(t0, t1)


@pytest.mark.parametrize("S", [1, 64])
def test_car_row_above_4096_neighbours(ctx, S):
    """A deployment related to more than 4096 others: the compact
    path scores it with the side kernel (any degree with min(deg, N) distinct
    nodes within its LDS table)."""
    rng = np.random.default_rng(700 + S)
    P, N = 9000, 300
    rows = [rng.integers(0, P, int(rng.integers(0, 4))).tolist() for _ in range(P)]
    rows[0] = rng.choice(np.arange(1, P), 6000, replace=False).tolist()
    rows[1] = rng.choice(np.arange(2, P), 4500, replace=False).tolist()
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.array([q for r in rows for q in r], np.int32)
    a = rng.integers(-1, 40, (P, S)).astype(np.int32).reshape(-1)
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    use = rng.integers(0, 8000, N * S).astype(np.int32)
    haz = (rng.random(N * S) < 0.2).astype(np.uint8)
    _check_car(ctx, rp, ci, a, S, cap, use, haz, N, rows=np.arange(0, 40, dtype=np.int32), label=f"deg>4096 S={S}")


@pytest.mark.parametrize("S", [1, 64])
def test_car_row_5000_distinct_nodes(ctx, S):
    """A row of degree 5000 over N = 6000 nodes: 5000 distinct
    neighbour nodes, the side kernel's largest table (one team per workgroup),
    with per-scenario random placements (every lane overflows its deviation
    list: the exact per-scenario recount)."""
    rng = np.random.default_rng(900 + S)
    P, N = 7000, 6000
    rows = [rng.integers(0, P, int(rng.integers(0, 3))).tolist() for _ in range(P)]
    rows[0] = rng.choice(np.arange(1, P), 5000, replace=False).tolist()
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.array([q for r in rows for q in r], np.int32)
    base = rng.permutation(P) % N
    a = np.repeat(base[:, None], S, axis=1).astype(np.int32)
    flip = rng.random((P, S)) < 0.3
    a[flip] = rng.integers(-1, N, flip.sum())
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    use = rng.integers(0, 8000, N * S).astype(np.int32)
    haz = (rng.random(N * S) < 0.2).astype(np.uint8)
    _check_car(ctx, rp, ci, a.reshape(-1), S, cap, use, haz, N, rows=np.arange(0, 16, dtype=np.int32),
               label=f"deg 5000 N {N} S={S}")


@pytest.mark.parametrize("P,N,deg,S", [(23000, 21845, 21000, 1), (23000, 21845, 21000, 64), (13000, 3000, 12000, 64),
                                       (32000, 30000, 26000, 1), (32000, 30000, 26000, 64)])
def test_car_row_largest_tables(ctx, P, N, deg, S):
    """The side kernel's table limits: a row with 21,000 distinct neighbour
    nodes (the largest table the LDS holds, 32,768 words), a degree-12,000 row
    over 3,000 nodes whose ~2,900 nodes counted twice overflow the 2,048-entry
    list (every lane takes the exact recount), and a degree-26,000 row over
    30,000 nodes whose table (65,536 words) lives in global memory.  1 % of
    placements redrawn per scenario, as in the synthetic what-if batches."""
    rng = np.random.default_rng(deg + S)
    rows = [rng.integers(0, P, int(rng.integers(0, 3))).tolist() for _ in range(P)]
    rows[0] = rng.choice(np.arange(1, P), deg, replace=False).tolist()
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.array([q for r in rows for q in r], np.int32)
    base = rng.permutation(P) % N
    a = np.repeat(base[:, None], S, axis=1).astype(np.int32)
    flip = rng.random((P, S)) < 0.01
    a[flip] = rng.integers(-1, N, flip.sum())
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    use = rng.integers(0, 8000, N * S).astype(np.int32)
    haz = (rng.random(N * S) < 0.2).astype(np.uint8)
    _check_car(ctx, rp, ci, a.reshape(-1), S, cap, use, haz, N, rows=np.arange(0, 8, dtype=np.int32),
               label=f"deg {deg} N {N} S={S}")


@pytest.mark.parametrize("S", [1, 64])
def test_car_wide_path_rows_above_4096(ctx, S):
    """N > 65535 (the wide path, 32-bit node ids): rows of degree 5,000 and
    9,000 (above the hub kernel's 4096) through car_bigrow_kernel, with
    neighbours piled onto few nodes in some scenarios (counts in the
    thousands), hazards, unassigned pods and overloaded ties."""
    rng = np.random.default_rng(4100 + S)
    P, N = 12000, 70000
    rows = [rng.integers(0, P, int(rng.integers(0, 4))).tolist() for _ in range(P)]
    rows[0] = rng.choice(np.arange(1, P), 5000, replace=False).tolist()
    rows[1] = rng.choice(np.arange(2, P), 9000, replace=False).tolist()
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.array([q for r in rows for q in r], np.int32)
    a = rng.integers(-1, N, (P, S)).astype(np.int32)
    crowd = rng.random((P, S)) < 0.5
    a[crowd] = rng.integers(0, 40, crowd.sum())           # half the placements on 40 nodes
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    use = rng.integers(0, 8000, N * S).astype(np.int32)
    haz = (rng.random(N * S) < 0.2).astype(np.uint8)
    _check_car(ctx, rp, ci, a.reshape(-1), S, cap, use, haz, N, rows=np.arange(0, 6, dtype=np.int32),
               label=f"wide path deg > 4096 S={S}")


def test_car_global_table_exact_recount(ctx):
    """The global-memory work area with every lane's deviation list
    overflowing (30 % of placements redrawn per scenario): each of the 64
    scenarios of a degree-26,000 row over 30,000 nodes is recounted exactly
    through the global table."""
    rng = np.random.default_rng(2600)
    P, N, S, deg = 32000, 30000, 64, 26000
    rows = [rng.integers(0, P, int(rng.integers(0, 3))).tolist() for _ in range(P)]
    rows[0] = rng.choice(np.arange(1, P), deg, replace=False).tolist()
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.array([q for r in rows for q in r], np.int32)
    base = rng.permutation(P) % N
    a = np.repeat(base[:, None], S, axis=1).astype(np.int32)
    flip = rng.random((P, S)) < 0.3
    a[flip] = rng.integers(-1, N, flip.sum())
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    use = rng.integers(0, 8000, N * S).astype(np.int32)
    haz = (rng.random(N * S) < 0.2).astype(np.uint8)
    _check_car(ctx, rp, ci, a.reshape(-1), S, cap, use, haz, N, rows=np.arange(0, 4, dtype=np.int32),
               label="global table, exact recount")


@pytest.mark.parametrize("S", [64, 200])
def test_car_fused_side_rows_outnumber_tiles(ctx, S):
    """The fused tile + side launch when the side rows (33..128 and above)
    outnumber what the tile periods hold: 2,600 rows of degree 33..300 against
    ~400 tile rows (the side rows left over run after the tiles)."""
    rng = np.random.default_rng(1300 + S)
    P, N = 3000, 400
    deg = np.where(rng.random(P) < 0.86, rng.integers(33, 130, P), rng.integers(0, 5, P))
    deg[:20] = rng.integers(129, 300, 20)
    rows = [rng.integers(0, P, int(d)).tolist() for d in deg]
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.array([q for r in rows for q in r], np.int32)
    base = rng.integers(0, N, P)
    a = np.repeat(base[:, None], S, axis=1).astype(np.int32)
    flip = rng.random((P, S)) < 0.02
    a[flip] = rng.integers(-1, N, flip.sum())
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    use = rng.integers(0, 8000, N * S).astype(np.int32)
    haz = (rng.random(N * S) < 0.15).astype(np.uint8)
    _check_car(ctx, rp, ci, a.reshape(-1), S, cap, use, haz, N, label=f"side rows > tiles S={S}")


def test_dropin_communication_5000_related_above_row_max_n(ctx):
    """The drop-in's `communication` with N > 32768 nodes goes through
    car_place; a deployment related to 5000 others gets the
    oracle's node."""
    import rescheduling as R
    from kubernetes import client
    from oracle import oracle as orc
    from rsk import synth
    c = synth.make_cluster(8000, 33000, S=1, seed=3)
    rng = np.random.default_rng(3)
    rows = [c.col_idx[c.row_ptr[p]:c.row_ptr[p + 1]].tolist() for p in range(c.P)]
    rows[0] = rng.choice(np.arange(1, c.P), 5000, replace=False).tolist()
    c.row_ptr = np.zeros(c.P + 1, np.int32)
    c.row_ptr[1:] = np.cumsum([len(r) for r in rows])
    c.col_idx = np.array([q for r in rows for q in r], np.int32)
    names, cm, rel = synth.to_cluster_monitoring(c, 0)
    hz = [n for n in names if cm[n]["cpu_pct"] >= 30]
    info = {"metadata": {"name": "d0", "namespace": "default"},
            "spec": {"template": {"spec": {"affinity": None}}}}
    client.CREATED.clear()
    R.communication(info, hz, cm, rel, names)
    t, _ = orc.car(c.row_ptr, c.col_idx, c.assign, 1, c.cap_cpu, c.use_cpu, c.hazard, c.N,
                   rows=np.array([0], np.int32))
    got = client.CREATED[-1][1]["spec"]["template"]["spec"]["nodeName"]
    assert got == (names[int(t[0])] if t[0] >= 0 else None)


def test_car_side_rows_fresh_nodes(ctx):
    """Rows of degree 33..255 at S >= 64 with every scenario drawing fresh
    nodes out of 5000: thousands of distinct nodes per row and 64-scenario
    chunk, so the side kernel's per-lane deviation lists overflow and every
    lane takes the exact recount; then half the scenarios sharing scenario 0's
    nodes (mixed pivots and deviations)."""
    rng = np.random.default_rng(800)
    P, N, S = 3000, 5000, 128
    rp, ci, a, cap, use, haz = _random_case(rng, P, N, S, max_deg=3,
                                            hub_deg=[33, 50, 64, 65, 100, 128, 129, 200, 254, 255], p_haz=0.1)
    _check_car(ctx, rp, ci, a, S, cap, use, haz, N, rows=np.arange(0, 40, dtype=np.int32), label="fresh nodes")
    a2 = a.reshape(P, S).copy()
    a2[:, ::2] = a2[:, :1]            # half the scenarios share scenario 0's nodes: tables near the degree
    _check_car(ctx, rp, ci, a2.reshape(-1), S, cap, use, haz, N, rows=np.arange(0, 40, dtype=np.int32),
               label="mixed")


@pytest.mark.parametrize("S", [9, 40, 64, 100])
def test_cut_cost_rows_partition_sums_to_full(ctx, S):
    """rsk_cut_cost_rows over a partition of the rows sums to rsk_cut_cost and
    to the oracle (the row-sharded cut-cost partials); S >= 32
    runs the lane = scenario kernel, with and without the missing term."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(900 + S)
    P, N = 700, 40
    rp, ci, a, _, _, _ = _random_case(rng, P, N, S, max_deg=6, hub_deg=[30, 90, 600])
    full = api.cut_cost(rp, ci, a, P, S, ctx=ctx)
    assert np.array_equal(full, orc.cut_cost(rp, ci, a, P, S))
    miss = rng.integers(0, 3, P).astype(np.int32)
    assert np.array_equal(api.cut_cost(rp, ci, a, P, S, miss, ctx=ctx), orc.cut_cost(rp, ci, a, P, S, miss))
    cuts = [0, 1, 250, 251, 699, 700]
    parts = sum(api.cut_cost_rows(rp, ci, a, P, S, cuts[k], cuts[k + 1], ctx=ctx) for k in range(len(cuts) - 1))
    assert np.array_equal(parts, full)


def test_pick_max_pod_metric_edges_gpu(ctx):
    """librsk's pick on the reference's metric-edge fixtures (pick_edges.json):
    equal to the reference where it returns, the documented divergence where it
    raises TypeError."""
    import json
    import os
    from rsk import api
    from test_oracle_golden import _pick_edge_arrays, pick_edge_expected
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "pick_edges.json")) as f:
        cases = json.load(f)["cases"]
    for case in cases:
        pods, assign, cpu, most = _pick_edge_arrays(case)
        if not pods:
            continue
        r = int(api.pick_max_pod(assign, cpu, len(pods), 1, [most], ctx=ctx)[0])
        assert (pods[r][0] if r >= 0 else None) == pick_edge_expected(case), case


def test_car_row_single_launch_vs_oracle(ctx):
    """rsk_car_row (the drop-in's one-launch CAR for S = 1) against the oracle's
    one-row CSR: random node multisets with ties, overloaded nodes, zero
    scores, invalid node ids, every node hazard, and N up to 32768."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(1200)
    for trial in range(60):
        N = int(rng.choice([1, 2, 3, 7, 64, 5000, 32768]))
        k = int(rng.choice([0, 1, 2, 5, 40, 300, 3000]))
        spread = max(1, N // int(rng.choice([1, 4, 50])))
        node_of = rng.integers(-1, spread + 1, k).astype(np.int32)
        cap = rng.choice([4000, 8000], N).astype(np.int32)
        use = rng.integers(0, 9000, N).astype(np.int32)
        if trial % 3 == 0:
            use[:] = cap - rng.integers(-2, 3, N)  # rem around 0: None vs node
        haz = (rng.random(N) < float(rng.choice([0.0, 0.3, 1.0]))).astype(np.uint8)
        rp = np.array([0, k] + [k] * k, np.int32)
        ci = np.arange(1, k + 1, dtype=np.int32)
        assign = np.concatenate([[-1], node_of]).astype(np.int32)
        t, sc = api.car_row(node_of, cap, use, haz, N, ctx=ctx)
        ot, osc = orc.car(rp, ci, assign, 1, cap, use, haz, N, rows=np.array([0], np.int32))
        assert t == int(ot[0]), f"trial {trial}: N={N} k={k} target {t} != {int(ot[0])}"
        if int(ot[0]) != -2:
            assert sc == int(osc[0]), f"trial {trial}: score {sc} != {int(osc[0])}"


def _check_car_sparse(ctx, row_ptr, col_idx, assign, S, cap, use, haz, N, rows=None, label=""):
    """_check_car against the sparse oracle (pinned to the literal one in
    tests/test_oracle_golden.py), multi-threaded, for the big cases."""
    from oracle import oracle as orc
    from rsk import api
    tgt, sc = api.car_place(row_ptr, col_idx, assign, S, cap, use, haz, N, rows=rows, ctx=ctx, want_score=True)
    rp, ci = _dedup_csr(row_ptr, col_idx)
    ot, osc = orc.car_sparse(rp, ci, assign, S, cap, use, haz, N, rows=rows, threads=min(16, os.cpu_count() or 1))
    bad = np.nonzero(tgt != ot)[0]
    assert bad.size == 0, f"{label}: {bad.size} targets differ, first cell {bad[0]}: gpu {tgt[bad[0]]} oracle {ot[bad[0]]}"
    assert np.array_equal(sc, osc), f"{label}: scores differ"


def test_car_many_global_table_rows_s768(ctx):
    """80 rows of degree 22,000 over 30,000 nodes at S = 768 — 960
    work items whose tables live in global memory, more than the capped grid
    of resident work areas holds, so the workgroups stride over the items and
    reuse their areas."""
    rng = np.random.default_rng(2200)
    P, N, S, deg, nbig = 30000, 30000, 768, 22000, 80
    lens = rng.integers(0, 3, P)
    lens[:nbig] = deg
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum(lens)
    ci = np.empty(int(rp[-1]), np.int32)
    for p in range(P):
        if lens[p] == deg:
            ci[rp[p]:rp[p + 1]] = rng.choice(np.arange(nbig, P), deg, replace=False)
        else:
            ci[rp[p]:rp[p + 1]] = rng.integers(0, P, lens[p])
    base = rng.permutation(P) % N
    a = np.repeat(base[:, None], S, axis=1).astype(np.int32)
    flip = rng.random((P, S)) < 0.01
    a[flip] = rng.integers(-1, N, flip.sum())
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    use = rng.integers(0, 8000, N * S).astype(np.int32)
    haz = (rng.random(N * S) < 0.2).astype(np.uint8)
    _check_car_sparse(ctx, rp, ci, a.reshape(-1), S, cap, use, haz, N, rows=np.arange(0, nbig + 40, dtype=np.int32),
                      label="80 global-table rows, S=768")


@pytest.mark.parametrize("S", [1, 3])
def test_car_row_above_65535_neighbours(ctx, S):
    """a row of degree 69,000 (beyond the side tables' 16-bit
    counts) over a compact-sized node set: the plan is accepted and runs the
    wide path (car_bigrow, 32-bit counts); a pile-up scenario puts every
    neighbour on one node (count 69,000)."""
    rng = np.random.default_rng(6900 + S)
    P, N, deg = 70000, 50, 69000
    lens = rng.integers(0, 3, P)
    lens[0] = deg
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum(lens)
    ci = rng.integers(0, P, int(rp[-1])).astype(np.int32)
    ci[:deg] = rng.choice(np.arange(1, P), deg, replace=False)
    a = rng.integers(-1, N, (P, S)).astype(np.int32)
    a[:, 0] = 7
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    use = rng.integers(0, 8000, N * S).astype(np.int32)
    haz = (rng.random(N * S) < 0.2).astype(np.uint8)
    haz.reshape(N, S)[7, 0] = 0
    from rsk import api
    plan = api.CarPlan(rp, ci, ctx=ctx)
    assert plan.info()["max_degree"] == deg
    plan.close()
    _check_car_sparse(ctx, rp, ci, a.reshape(-1), S, cap, use, haz, N, rows=np.arange(0, 64, dtype=np.int32),
                      label=f"deg 69000 S={S}")


@pytest.mark.parametrize("N", [1, 63, 1023, 1024, 1025, 4097, 70000])
def test_random_candidates_order_and_count(ctx, N):
    """rsk_random_candidates (the drop-in random's candidate list)
    equals the reference's `[n for n in nodes_name if n not in hazard]`
    (rescheduling.py:149-150) in order and count, across the multi-chunk
    compaction (N > 1024) and the inputs above 64 KB, at several hazard
    densities (none, some, all but one, all)."""
    from rsk import api
    rng = np.random.default_rng(N)
    for p in (0.0, 0.1, 0.5, 0.97, 1.0):
        h = (rng.random(N) < p).astype(np.uint8)
        got = api.random_candidates(h, N, ctx=ctx)
        assert np.array_equal(got, np.nonzero(h == 0)[0].astype(np.int32)), (N, p)
    h = np.ones(N, np.uint8)
    h[N - 1] = 0
    assert api.random_candidates(h, N, ctx=ctx).tolist() == [N - 1]


@pytest.mark.parametrize("seed", [0, 1, 7, 12345])
def test_dropin_random_matches_reference_choice(ctx, seed):
    """The drop-in random() picks what the reference's `rd.choice(candidates)`
    (rescheduling.py:149-153, CPython's global Random) picks after the same
    random.seed, on a 3,000-node cluster with hazards, and it leaves the global
    state where the reference leaves it."""
    import random as pyrandom

    import rescheduling as R
    from kubernetes import client
    rng = np.random.default_rng(seed)
    nodes = [f"node-{i:05d}" for i in range(3000)]
    haz = [n for n in nodes if rng.random() < 0.3]
    hs = set(haz)
    pyrandom.seed(seed)
    want = pyrandom.choice([n for n in nodes if n not in hs])
    after = pyrandom.random()
    info = {"metadata": {"name": "d0", "namespace": "default"},
            "spec": {"template": {"spec": {"affinity": None}}}}
    client.CREATED.clear()
    pyrandom.seed(seed)
    R.random(info, haz, nodes)
    assert client.CREATED[-1][1]["spec"]["template"]["spec"]["nodeName"] == want
    assert pyrandom.random() == after


@pytest.mark.parametrize("P,N,S,p_flip", [(3000, 97, 33, 0.01), (5000, 300, 64, 0.3), (20000, 2000, 130, 0.01),
                                          (4000, 50, 1, 0.0), (1_000_000, 50_000, 64, 0.01),
                                          (100_000, 2_000, 64, 0.6), (3000, 70_000, 40, 0.05)])
def test_node_reduce_segmented_vs_oracle(ctx, P, N, S, p_flip):
    """Kernel 3's per-node count / CPU / memory sums (podmonitor.py:104-121,
    nodemonitor.py:24-46) against the oracle: the segmented kernel (S >= 32:
    pods bucketed by key node, register sums per key) on perturbed batches,
    heavily perturbed ones (30 % of placements redrawn: most lanes off the key),
    a partial last chunk (S = 130), assignments outside [0, N) (skipped), and
    the atomic kernel at S = 1; config 4's size; 60 % redrawn over 6.4 M cells
    (most cells off their key node); more nodes than pods (most nodes' cells
    zeros)."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(P + S)
    base = rng.integers(0, N, P)
    a = np.repeat(base[:, None], S, axis=1).astype(np.int32)
    flip = rng.random((P, S)) < p_flip
    a[flip] = rng.integers(-2, N + 2, int(flip.sum()))
    a[rng.integers(0, P, 50), :] = -1          # unscheduled pods
    pod_cpu = rng.integers(50, 500, P).astype(np.int32)
    pod_mem = rng.integers(1 << 20, 1 << 31, P).astype(np.int64)
    got = api.node_reduce(a.reshape(-1), P, S, pod_cpu, pod_mem, N, ctx=ctx)
    exp = orc.node_reduce(a.reshape(-1), P, S, pod_cpu, pod_mem, N)
    for g, e, name in zip(got, exp, ("count", "cpu", "mem")):
        assert np.array_equal(g, e), name


@pytest.mark.parametrize("P,N,S", [(20_000, 3_000, 64), (9_000, 500, 4096), (12_000, 1_000, 100)])
def test_node_reduce_deviation_form_edges(ctx, P, N, S):
    """The deviation form of kernel 3's node sums (out = base[key node] +
    per-scenario deviations, podmonitor.py:104-121) against the oracle where
    its bookkeeping branches: pods 4096-8191 — block 1 of the scan's
    4,096-pod blocks — with 40 % of their cells redrawn (its entry region
    overflows: its deviations go through the spill launch) beside blocks that
    list theirs; pods whose scenario-0 node is
    redrawn (the key is the majority of scenarios 0 / 21 / 42), pods with no
    key (unscheduled in two of the three), pods unscheduled in scenario 0 only,
    assignments equal to N; 64 chunks per pod (S = 4096) and a partial chunk
    (S = 100)."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(P * 7 + S)
    base = rng.integers(0, N, P)
    a = np.repeat(base[:, None], S, axis=1).astype(np.int32)
    flip = rng.random((P, S)) < 0.01
    flip[4096:8192] = rng.random((4096, S)) < 0.4         # block 1 (4,096 pods) overflows
    a[flip] = rng.integers(-2, N + 2, int(flip.sum()))
    q = rng.integers(0, P, 300)
    a[q, 0] = rng.integers(0, N, 300)                      # scenario 0 redrawn: key from 21 / 42
    q = rng.integers(0, P, 100)
    a[q, 0] = -1                                           # unscheduled in scenario 0 only
    q = rng.integers(0, P, 100)
    a[q, 0] = -1
    a[q, 21] = N                                           # no key node
    a[rng.integers(0, P, 50), :] = -1
    pod_cpu = rng.integers(-500, 500, P).astype(np.int32)
    pod_mem = rng.integers(-(1 << 40), 1 << 40, P).astype(np.int64)
    for mem in (pod_mem, None):
        got = api.node_reduce(a.reshape(-1), P, S, pod_cpu, mem, N, ctx=ctx)
        exp = orc.node_reduce(a.reshape(-1), P, S, pod_cpu, pod_mem, N)
        assert np.array_equal(got[0], exp[0]), "count"
        assert np.array_equal(got[1], exp[1]), "cpu"
        if mem is not None:
            assert np.array_equal(got[2], exp[2]), "mem"


@pytest.mark.parametrize("S", [64, 130])
def test_car_early_side_rows_on_the_fly_codes(ctx, S):
    """Rows too big for the fused grid's 20 KB teams (degree 1,200-2,000 over
    30,000 nodes) run on the side stream from the start with their node codes
    computed on the fly (car_prep0's max(cap) only) and, where a scenario's row
    reaches no candidate node, the zero case scanned by the wave: one row whose
    neighbours all sit on nodes that are hazards in every scenario, one whose
    neighbours are all unscheduled, crowded overloaded ties (None) and the
    rest, against the oracle at S = 64 and a partial second chunk."""
    rng = np.random.default_rng(1500 + S)
    P, N = 30000, 30000
    lens = rng.integers(0, 4, P)
    big = np.arange(10, 22)
    lens[big] = rng.integers(1200, 2000, big.size)
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum(lens)
    ci = rng.integers(0, P, int(rp[-1])).astype(np.int32)
    base = rng.integers(0, N, P)
    a = np.repeat(base[:, None], S, axis=1)
    flip = rng.random((P, S)) < 0.02
    a[flip] = rng.integers(-1, N, int(flip.sum()))
    haz = (rng.random((N, S)) < 0.1).astype(np.uint8)
    # row 10: every neighbour on nodes 0..99, hazard everywhere -> zero case
    a[ci[rp[10]:rp[11]], :] = rng.integers(0, 100, (int(lens[10]), 1))
    haz[:100, :] = 1
    # row 11: every neighbour unscheduled -> zero case
    a[ci[rp[11]:rp[12]], :] = -1
    # row 12: neighbours piled on 40 overloaded nodes (ties at rem < 0 -> None)
    nb12 = ci[rp[12]:rp[13]]
    a[nb12, :] = 200 + (np.arange(nb12.size) % 40)[:, None]
    cap = rng.choice([4000, 8000], N).astype(np.int32)
    use = rng.integers(0, 8000, (N, S)).astype(np.int32)
    use[200:240, :] = 9000
    cap[200:240] = 4000
    haz[200:240, :] = 0
    rows = np.concatenate([big, rng.choice(P, 300, replace=False)]).astype(np.int32)
    _check_car_sparse(ctx, rp, ci, a.astype(np.int32).reshape(-1), S, cap, use.reshape(-1), haz.reshape(-1), N,
                      rows=np.unique(rows), label=f"early side rows S={S}")
    from rsk import api
    plan = api.CarPlan(rp, ci, ctx=ctx)
    tgt, _ = plan.execute(a.astype(np.int32).reshape(-1), S, cap, use.reshape(-1), haz.reshape(-1), N)
    plan.close()
    from oracle import oracle as orc
    drp, dci = _dedup_csr(rp, ci)
    exp, _ = orc.car_sparse(drp, dci, a.astype(np.int32).reshape(-1), S, cap, use.reshape(-1), haz.reshape(-1), N,
                            threads=min(16, os.cpu_count() or 1), want_score=False)
    assert np.array_equal(tgt, exp), f"plan path: {(tgt != exp).sum()} cells differ"
    t = tgt.reshape(P, S)
    assert (t[11] >= 0).all() or (t[11] == -1).any()
    assert (t[12] == -1).sum() > 0


def test_car_big_side_rows_plan_reuse(ctx):
    """Side rows of degree 800 to 9,000 over 40,000 nodes (beyond the fused
    grid's teams: on the side stream from the start, codes on the fly), one
    plan executed four times — two batches at S = 128 (two chunks), one at S =
    64, the first batch again — each against the oracle, so state a launch
    leaves behind in the plan's work areas would show in the next."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(9000)
    P, N = 20000, 40000
    lens = rng.integers(0, 4, P)
    lens[:6] = [800, 1500, 3000, 5000, 7000, 9000]
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum(lens)
    ci = rng.integers(0, P, int(rp[-1])).astype(np.int32)
    for r in range(6):
        ci[rp[r]:rp[r + 1]] = rng.choice(np.arange(6, P), lens[r], replace=False)
    drp, dci = _dedup_csr(rp, ci)
    plan = api.CarPlan(rp, ci, ctx=ctx)

    def batch(seed, S):
        g = np.random.default_rng(seed)
        base = g.integers(0, N, P)
        a = np.repeat(base[:, None], S, axis=1)
        flip = g.random((P, S)) < 0.03
        a[flip] = g.integers(-1, N, int(flip.sum()))
        cap = g.choice([4000, 8000], N).astype(np.int32)
        use = g.integers(0, 8000, N * S).astype(np.int32)
        haz = (g.random(N * S) < 0.2).astype(np.uint8)
        return a.astype(np.int32).reshape(-1), cap, use, haz

    for k, (seed, S) in enumerate([(1, 128), (2, 128), (3, 64), (1, 128)]):
        a, cap, use, haz = batch(seed, S)
        tgt, _ = plan.execute(a, S, cap, use, haz, N)
        exp, _ = orc.car_sparse(drp, dci, a, S, cap, use, haz, N, threads=min(16, os.cpu_count() or 1),
                                want_score=False)
        bad = np.nonzero(tgt != exp)[0]
        assert bad.size == 0, f"execute {k}: {bad.size} cells differ, first row {bad[0] // S}"
    plan.close()


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1, 3, 4])
def test_car_direct_small_batches(ctx, S):
    """The one-launch path of small batches (S <= 4, Q*S <= 65536, no scores
    requested: a workgroup per (row, scenario)) against the oracle: rows with
    duplicates and a self edge, unassigned pods, an all-hazard scenario (no
    candidate), a row subset in shuffled order, and a hub row whose distinct
    nodes overflow an LDS table (global work areas)."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(40 + S)
    P, N = 12000, 10000
    rows_l = [rng.integers(0, P, int(rng.integers(0, 6))).tolist() for _ in range(P)]
    rows_l[0] = rng.choice(P, 9000, replace=False).tolist()   # ~5,900 distinct nodes: beyond the LDS
    rows_l[1] = [1, 1, 2, 2, 3]                               # a self edge and duplicates
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows_l])
    ci = np.array([q for r in rows_l for q in r], np.int32)
    assign = rng.integers(0, N, P * S).astype(np.int32)
    assign[rng.random(P * S) < 0.01] = -1
    cap = np.full(N, 50000, np.int32)
    use = rng.integers(0, 60000, N * S).astype(np.int32)
    haz = (rng.random(N * S) < 0.2).astype(np.uint8)
    haz.reshape(N, S)[:, S - 1] = 1                           # the last scenario: every node hazardous
    rpd, cid = _dedup_csr(rp, ci)
    subset = rng.permutation(P)[:7000].astype(np.int32)
    for rows in (None, subset):
        tgt, _ = api.car_place(rp, ci, assign, S, cap, use, haz, N, rows=rows, ctx=ctx)
        ot, _ = orc.car(rpd, cid, assign, S, cap, use, haz, N, rows=rows)
        bad = np.nonzero(tgt != ot)[0]
        assert bad.size == 0, f"S={S}: {bad.size} differ, first {bad[0]}: gpu {tgt[bad[0]]} oracle {ot[bad[0]]}"
        assert (tgt.reshape(-1, S)[:, S - 1] == -2).all()     # no candidate anywhere in the last scenario


@pytest.mark.gpu
@pytest.mark.parametrize("S", [1, 4])
def test_car_direct_one_wave_rows_boundary(ctx, S):
    """Round 6's one-wave path of car_move_one (rows of <= 64 neighbours: a
    ballot per distinct node instead of the LDS hash) through the small-batch
    launch, at its boundary: rows of 63, 64 and 65 entries with duplicates and
    self edges, rows whose every neighbour sits on a hazard node in some
    scenario (max score 0 with no zero-case words: the workgroup's scan of
    every node), overloaded single candidates and None ties; every cell against
    the oracle."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(640 + S)
    P, N = 3000, 40
    rows_l = [rng.integers(0, P, int(rng.integers(0, 5))).tolist() for _ in range(P)]
    for k in range(300):
        d = (63, 64, 65)[k % 3]
        r = rng.integers(0, P, d).tolist()
        r[0] = k                 # a self edge
        r[1] = r[2]              # a duplicate
        rows_l[k] = r
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows_l])
    ci = np.array([q for r in rows_l for q in r], np.int32)
    assign = rng.integers(0, N, (P, S)).astype(np.int32)
    haz = (rng.random((N, S)) < 0.15).astype(np.uint8)
    for k in range(0, 300, 7):   # every neighbour of row k on a hazard node in scenario k % S
        s = k % S
        hn = int(np.nonzero(haz[:, s])[0][0]) if haz[:, s].any() else 0
        haz[hn, s] = 1
        assign[[q for q in rows_l[k] if q != k], s] = hn
    cap = np.full(N, 40000, np.int32)
    use = rng.integers(20000, 45000, (N, S)).astype(np.int32)   # some rem < 0: None ties and overloaded singles
    assign, haz, use = assign.reshape(-1), haz.reshape(-1), use.reshape(-1)
    rpd, cid = _dedup_csr(rp, ci)
    tgt, _ = api.car_place(rp, ci, assign, S, cap, use, haz, N, ctx=ctx)
    ot, _ = orc.car(rpd, cid, assign, S, cap, use, haz, N)
    bad = np.nonzero(tgt != ot)[0]
    assert bad.size == 0, f"S={S}: {bad.size} differ, first {bad[0]}: gpu {tgt[bad[0]]} oracle {ot[bad[0]]}"
    assert (ot == -1).any() and (ot >= 0).any()


@pytest.mark.parametrize("S,n_hubs", [(64, 6), (256, 40)])
def test_car_big_rows_beyond_the_fused_grid(ctx, S, n_hubs):
    """Rows whose tables exceed the fused grid's LDS (degree 1,200-1,900 over
    5,000 nodes): as one workgroup per (row, scenario) at the front of the fused
    grid when they make few cells (S = 64, 6 rows: 384 cells, targets only) and
    as on-the-fly pivot teams on the side stream beside car_prep otherwise
    (S = 256, 40 rows: 10,240 cells; and whenever scores are requested).  Both
    against the oracle, every cell, with and without scores."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(900 + S)
    P, N = 4000, 5000
    hubs = rng.integers(1200, 1900, n_hubs).tolist()
    rp, ci, a, cap, use, haz = _random_case(rng, P, N, S, max_deg=6, hub_deg=hubs, p_haz=0.1)
    A = a.reshape(P, S)   # what-if scenarios: mostly one base assignment
    base = rng.integers(0, N, P)
    keep = rng.random((P, S)) < 0.97
    A[keep] = np.repeat(base[:, None], S, axis=1)[keep]
    a = A.reshape(-1).astype(np.int32)
    plan = api.CarPlan(rp, ci, ctx=ctx)
    assert plan.info()["max_degree"] >= 1200
    t0, _ = plan.execute(a, S, cap, use, haz, N)                    # targets only
    t1, sc = plan.execute(a, S, cap, use, haz, N, want_score=True)  # pivot teams (scores)
    plan.close()
    rp2, ci2 = _dedup_csr(rp, ci)
    ot, osc = orc.car_sparse(rp2, ci2, a, S, cap, use, haz, N, threads=min(16, os.cpu_count() or 1))
    for t, label in ((t0, "targets only"), (t1, "with scores")):
        bad = np.nonzero(t != ot)[0]
        assert bad.size == 0, f"{label}: {bad.size} cells differ, first {bad[0]}: gpu {t[bad[0]]} oracle {ot[bad[0]]}"
    assert np.array_equal(sc, osc)


def test_car_big_rows_direct_cells_edge_cases(ctx):
    """The big rows as direct cells at the front of the fused grid (S = 64, 6
    rows of 1,200-1,900 neighbours, targets only: no side launch) through every
    branch of the rule (rescheduling.py:183-214), each in its own scenario:
    every neighbour node hazardous (max score 0: the prep kernel's zero case
    over 5 free nodes with equal remaining CPU: the lowest index), every node
    hazardous (no candidate), all neighbours on one overloaded node (the single
    best), neighbours split over two nodes with equal remaining CPU, fitting and
    overloaded, every neighbour unassigned.  Every cell against the oracle."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(4242)
    P, N, S = 4000, 5000, 64
    hubs = rng.integers(1200, 1900, 6).tolist()
    rp, ci, a, cap, use, haz = _random_case(rng, P, N, S, max_deg=6, hub_deg=hubs, p_haz=0.05)
    A, U, Hz = a.reshape(P, S), use.reshape(N, S), haz.reshape(N, S)
    A[:] = rng.integers(0, N, P)[:, None]
    nb = np.unique(np.concatenate([ci[rp[k]:rp[k + 1]] for k in range(6)]))
    nb = nb[nb >= 6]   # the hubs' neighbours (rows 0-5 keep their own nodes)
    free = np.setdiff1d(np.arange(N), A[:, 1])[:5]
    Hz[:, 1] = 1
    Hz[free, 1] = 0                                   # s = 1: zero case over the free nodes, tied
    U[free, 1] = cap[free] - 100
    Hz[:, 2] = 1                                      # s = 2: no candidate
    A[nb, 3] = 7
    Hz[7, 3] = 0
    U[7, 3] = cap[7] + 5                              # s = 3: one overloaded best
    for s, over in ((4, False), (5, True)):           # s = 4 / 5: a two-node tie, fitting / overloaded
        A[nb, s] = np.where(np.arange(nb.size) % 2 == 0, 10, 11)
        Hz[[10, 11], s] = 0
        U[10, s] = cap[10] + (3 if over else -100)
        U[11, s] = cap[11] + (3 if over else -100)
    A[nb, 6] = -1                                     # s = 6: every neighbour unassigned
    a, use, haz = A.reshape(-1).copy(), U.reshape(-1).copy(), Hz.reshape(-1).copy()
    plan = api.CarPlan(rp, ci, ctx=ctx)
    ctx.reset_profiling()
    ctx.set_profiling(True)
    t0, _ = plan.execute(a, S, cap, use, haz, N)
    ctx.set_profiling(False)
    assert ctx.kernel_time("car_side")[1] == 0 and ctx.kernel_time("car_tile")[1] == 1   # one fused launch
    plan.close()
    rp2, ci2 = _dedup_csr(rp, ci)
    ot, _ = orc.car_sparse(rp2, ci2, a, S, cap, use, haz, N, threads=min(16, os.cpu_count() or 1))
    bad = np.nonzero(t0 != ot)[0]
    assert bad.size == 0, f"{bad.size} cells differ, first {bad[0]}: gpu {t0[bad[0]]} oracle {ot[bad[0]]}"
    T = t0.reshape(P, S)
    assert (T[:6, 2] == -2).all() and (T[:6, 3] == 7).all() and np.isin(T[:6, 4:6], (10, 11)).all()
    assert (T[:6, 1] == free.min()).all()


def test_node_reduce_rejects_misaligned_u64_outputs(ctx):
    """rsk_node_reduce stores (and, for an overflowing block, atomically adds)
    64-bit sums: a cpu_sum / mem_sum / pod_mem device pointer that is not 8-B
    aligned is an argument error naming the buffer, before any launch (the
    r04p2 fault class); the aligned call still matches the oracle."""
    import torch
    from oracle import oracle as orc
    from rsk import _lib
    dev = torch.device("cuda:0")
    P, N, S = 3000, 100, 64
    rng = np.random.default_rng(11)
    a = np.repeat(rng.integers(0, N, P)[:, None], S, axis=1).astype(np.int32)
    pc = rng.integers(1, 500, P).astype(np.int32)
    pm = rng.integers(1, 1 << 30, P).astype(np.int64)
    T = lambda x: torch.from_numpy(x).to(dev)  # noqa: E731
    ta, tpc, tpm = T(a.reshape(-1)), T(pc), T(pm)
    cnt = torch.empty(N * S, dtype=torch.int32, device=dev)
    big = torch.empty(N * S + 1, dtype=torch.int64, device=dev)   # + 4 B: misaligned views
    mem = torch.empty(N * S, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)  # (the context's own stream reads what torch's stream wrote)
    L, h = ctx.lib, ctx.handle
    for bad, name in ((0, "cpu_sum"), (1, "mem_sum")):
        cs = big.data_ptr() + 4 if bad == 0 else big.data_ptr()
        ms = big.data_ptr() + 4 if bad == 1 else mem.data_ptr()
        rc = L.rsk_node_reduce(h, ta.data_ptr(), P, S, tpc.data_ptr(), tpm.data_ptr(), N, cnt.data_ptr(), cs, ms,
                               _lib.RSK_F_DEVICE)
        assert rc != 0 and name in _lib.last_error()
    cs = torch.empty(N * S, dtype=torch.int64, device=dev)
    _lib.check(L.rsk_node_reduce(h, ta.data_ptr(), P, S, tpc.data_ptr(), tpm.data_ptr(), N, cnt.data_ptr(),
                                 cs.data_ptr(), mem.data_ptr(), _lib.RSK_F_DEVICE))
    torch.cuda.synchronize(dev)
    exp = orc.node_reduce(a.reshape(-1), P, S, pc, pm, N)
    assert np.array_equal(cnt.cpu().numpy(), exp[0]) and np.array_equal(cs.cpu().numpy(), exp[1])
    assert np.array_equal(mem.cpu().numpy(), exp[2])


@pytest.mark.parametrize("P,N,S", [(20_000, 50_000, 512), (30_000, 150_000, 64)])
def test_node_reduce_counters_beyond_64k_lds(ctx, P, N, S):
    """The deviation form with more than 8,192 per-block counters (key buckets
    + entry bins, nh = ceil(N / 32) * (1 + S / 64)): nh = 14,067 at N = 50k,
    S = 512 and 9,376 at N = 150k, S = 64, so nr_place's dynamic LDS (4 nh +
    8 + 2048 * 16 B with memory sums) is 88 KB / 70 KB — above the 64 KB that
    a launch gets without hipFuncAttributeMaxDynamicSharedMemorySize (ADVICE
    round 5).  Count / CPU / memory sums against the oracle, with and without
    memory (podmonitor.py:104-121, nodemonitor.py:24-46)."""
    from oracle import oracle as orc
    from rsk import api
    rng = np.random.default_rng(P + N + S)
    a = np.repeat(rng.integers(0, N, P)[:, None], S, axis=1).astype(np.int32)
    flip = rng.random((P, S)) < 0.02
    a[flip] = rng.integers(-1, N + 1, int(flip.sum()))
    pod_cpu = rng.integers(1, 900, P).astype(np.int32)
    pod_mem = rng.integers(1 << 20, 1 << 34, P).astype(np.int64)
    exp = orc.node_reduce(a.reshape(-1), P, S, pod_cpu, pod_mem, N)
    for mem in (pod_mem, None):
        got = api.node_reduce(a.reshape(-1), P, S, pod_cpu, mem, N, ctx=ctx)
        assert np.array_equal(got[0], exp[0]), "count"
        assert np.array_equal(got[1], exp[1]), "cpu"
        if mem is not None:
            assert np.array_equal(got[2], exp[2]), "mem"


def test_write_guard_reports_an_overflowing_scatter(ctx):
    """The r05v fault class: nr_place writes records at offsets
    built from nr_scan's counts.  rsk_selftest_write_guard runs node_reduce
    with the record capacity lowered below the batch's pod count: the guarded
    stores are skipped (no fault) and the device error word comes back as
    RSK_EHIP naming nr_place.  The word is cleared once reported: the next call
    on the same context runs and matches the oracle."""
    from oracle import oracle as orc
    from rsk import _lib, api
    rc = ctx.lib.rsk_selftest_write_guard(ctx.handle)
    assert rc == _lib.RSK_EHIP, (rc, _lib.last_error())
    assert "nr_place" in _lib.last_error()
    P, N, S = 5000, 300, 64
    rng = np.random.default_rng(5)
    a = np.repeat(rng.integers(0, N, P)[:, None], S, axis=1).astype(np.int32)
    a[rng.random((P, S)) < 0.02] = 7
    pc = rng.integers(1, 500, P).astype(np.int32)
    got = api.node_reduce(a.reshape(-1), P, S, pc, None, N, ctx=ctx)
    exp = orc.node_reduce(a.reshape(-1), P, S, pc, np.zeros(P, np.int64), N)
    assert np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1])
