"""GPU parity at the benchmark shapes (BASELINE.json configs 3-5).

Each test runs librsk at the size bench.py times and checks EVERY cell
against the oracle's sparse restatement (oracle_car_sparse, pinned to the
literal per-cell oracle and to the reference's fixtures in
tests/test_oracle_golden.py), bit-exactly; the literal oracle re-checks the
hard rows.  The kernels' template instances are the ones the bench runs: no
score output, S >= 64 (64-scenario tiles); config 2 at S = 1.
"""
import os
from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

THREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def ctx():
    from rsk import _lib
    return _lib.default_context()


def _rows_to_check(c, n_sample, seed):
    deg = np.diff(c.row_ptr)
    rng = np.random.default_rng(seed)
    hard = np.nonzero(deg > 16)[0]                       # every heavy-tile (17..32), mid and hub row
    sample = rng.choice(c.P, n_sample, replace=False)
    return np.unique(np.concatenate([hard, sample])).astype(np.int32), hard


def _all_cells(c, S, t, label):
    """Every (row, scenario) cell of t [P, S] against oracle_car_sparse."""
    from oracle import oracle as orc
    exp, _ = orc.car_sparse(c.row_ptr, c.col_idx, c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, c.N,
                            threads=THREADS, want_score=False)
    exp = exp.reshape(c.P, S)
    bad = np.argwhere(t != exp)
    assert bad.size == 0, f"{label}: {len(bad)} of {t.size} cells differ; first row {bad[0][0]} s {bad[0][1]}: " \
                          f"gpu {t[bad[0][0], bad[0][1]]} oracle {exp[bad[0][0], bad[0][1]]}"
    return t.size


def test_config2_2k64_s1_all_rows(ctx, synth_golden):
    """Config 2 exactly as bench.py runs it: 2k pods x 64 nodes, S = 1 (the
    generic-tile instance), every row through CarPlan, plus the reference's
    own decisions for scenario 0 of its golden 2k/64 batch."""
    from rsk import api, synth
    g = synth_golden["2k64"]
    c = synth.make_cluster(2_000, 64, S=1, seed=0)
    plan = api.CarPlan(c.row_ptr, c.col_idx, ctx=ctx)
    tgt, _ = plan.execute(c.assign, 1, c.cap_cpu, c.use_cpu, c.hazard, c.N)   # one launch (small batch)
    tt, _ = plan.execute(c.assign, 1, c.cap_cpu, c.use_cpu, c.hazard, c.N, tiled=True)   # tiles + side rows
    plan.close()
    assert _all_cells(c, 1, tgt.reshape(c.P, 1), "config 2") == 2_000
    assert _all_cells(c, 1, tt.reshape(c.P, 1), "config 2 tiled") == 2_000
    g0 = [sc for sc in g["scenarios"] if sc["s"] == 0][0]
    assert tgt[g0["pods"]].tolist() == g0["car_target"]
    assert tt[g0["pods"]].tolist() == g0["car_target"]


def test_config3_headline_s4096(ctx, synth_golden):
    """100k pods x 5k nodes x 4096 scenarios (the headline batch): all
    409.6 M cells against the sparse oracle, every row of degree > 16 plus
    200 sampled rows against the literal one, and the reference's own 66
    golden pods in the unperturbed scenario 0."""
    from oracle import oracle as orc
    from rsk import api, synth
    P, N, S = 100_000, 5_000, 4096
    c = synth.make_cluster(P, N, S=S, seed=0)
    plan = api.CarPlan(c.row_ptr, c.col_idx, ctx=ctx)
    info = plan.info()
    tgt, sc = plan.execute(c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, N)
    assert sc is None
    plan.close()
    t = tgt.reshape(P, S)
    g = synth_golden["100k5k"]["scenarios"][0]
    assert t[g["pods"], 0].tolist() == g["car_target"]
    assert _all_cells(c, S, t, "config 3") == 409_600_000
    rows, hard = _rows_to_check(c, 200, 7)
    assert hard.size == 640 and info["mid_rows"] + info["heavy_rows"] == 201
    assert info["light_max"] == 32 and info["side_rows"] == 201 and info["sorted_rows"] == 439
    exp, _ = orc.car(c.row_ptr, c.col_idx, c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, N, rows=rows,
                     threads=THREADS)
    got = t[rows].reshape(-1)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} cells differ; first row {rows[bad[0] // S]} s {bad[0] % S}"


def test_config4_1m50k_s64(ctx):
    """1M pods x 50k nodes x 64 scenarios: all 64 M cells against the sparse
    oracle, all hub and mid rows (max degree 1,756) plus 200 sampled rows
    against the literal one; also the row-sharded plans of 2 ranks (the rows
    each rank owns) give the same targets."""
    from oracle import oracle as orc
    from rsk import api, synth
    from rsk import dist as rdist
    P, N, S = 1_000_000, 50_000, 64
    c = synth.make_cluster(P, N, S=S, seed=0)
    plan = api.CarPlan(c.row_ptr, c.col_idx, ctx=ctx)
    tgt, _ = plan.execute(c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, N)
    plan.close()
    t = tgt.reshape(P, S)
    assert _all_cells(c, S, t, "config 4") == 64_000_000
    rows, hard = _rows_to_check(c, 200, 8)
    assert hard.size > 1000 and int(np.diff(c.row_ptr).max()) > 1000
    exp, _ = orc.car(c.row_ptr, c.col_idx, c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, N, rows=rows,
                     threads=THREADS)
    bad = np.nonzero(t[rows].reshape(-1) != exp)[0]
    assert bad.size == 0, f"{bad.size} cells differ; first row {rows[bad[0] // S]}"
    for r in range(2):
        sh = rdist.row_shard_for(r, 2, c.row_ptr)
        p2 = api.CarPlan(c.row_ptr, c.col_idx, rows=sh.rows, ctx=ctx)
        t2, _ = p2.execute(c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, N)
        p2.close()
        assert np.array_equal(t2.reshape(sh.q, S), t[sh.rows]), f"row shard {r}"


def _rounds_vs_oracle(ctx, c, S, R, k, threshold=30):
    """rsk_rounds_run over all S scenarios for R rounds; its first k scenarios
    (k = S: all of them) against oracle_rounds (final state, evictions and
    targets of every round), the scenarios split over THREADS oracle threads."""
    from oracle import oracle as orc
    from rsk import api
    P, N = c.P, c.N
    a0 = c.assign.reshape(P, S)[:, :k].copy().reshape(-1)
    u0 = c.use_cpu.reshape(N, S)[:, :k].copy().reshape(-1)
    rounds = api.Rounds(c.row_ptr, c.col_idx, c.pod_cpu, ctx=ctx)
    a, u = c.assign.copy(), c.use_cpu.copy()
    ev, tg = rounds.run(a, S, c.cap_cpu, u, N, R, threshold=threshold)
    rounds.close()
    ea, eu, eev, etg = orc.rounds(c.row_ptr, c.col_idx, c.pod_cpu, a0, k, c.cap_cpu, u0, N, R, threshold=threshold,
                                  threads=THREADS)
    got_t = tg.reshape(R, S)[:, :k]
    bad = np.argwhere(got_t != etg.reshape(R, k))
    assert bad.size == 0, f"targets differ first at round {bad[0][0]} scenario {bad[0][1]}"
    assert np.array_equal(ev.reshape(R, S)[:, :k].reshape(-1), eev)
    assert np.array_equal(a.reshape(P, S)[:, :k].reshape(-1), ea)
    assert np.array_equal(u.reshape(N, S)[:, :k].reshape(-1), eu)
    return etg


@pytest.mark.parametrize("R", [10, 256])
def test_config5_rounds_100k_s1024(ctx, R):
    """100k/5k x 1024 scenarios, R rounds of detect -> evict -> CAR -> update on
    the device: R = 10 is the reference's MAX_ROUNDS (main.py:28), R = 256
    config 5's loop length; ALL 1,024 scenarios against oracle_rounds (every
    round's eviction and target, the final assign and use)."""
    from rsk import synth
    c = synth.make_cluster(100_000, 5_000, S=1024, seed=0)
    etg = _rounds_vs_oracle(ctx, c, 1024, R, 1024)
    assert (etg >= 0).sum() > R * 1024 // 2  # real moves happened


def test_rounds_none_and_no_candidate_mid_run(ctx):
    """A loop whose scenarios run into every outcome mid-run: threshold 120 %
    lets overloaded nodes (rem < 0) stay candidates, so ties among them give
    None (rescheduling.py:203-212); scenarios with a heavy background load turn
    every node hazardous, so CAR has no candidate (the reference's ValueError,
    main.py:97-98) — next to real moves, 60 rounds against oracle_rounds."""
    from rsk import synth
    rng = np.random.default_rng(5)
    P, N, S, R = 3000, 40, 64, 60
    par = synth.pa_tree_parents(P, rng)
    rp, ci = synth.tree_csr(par)
    pod_cpu = rng.integers(50, 500, P).astype(np.int32)
    a = rng.integers(0, N, P * S).astype(np.int32)
    cap = rng.integers(14000, 28000, N).astype(np.int32)
    A = a.reshape(P, S)
    use = np.zeros((N, S), np.int64)
    for s in range(S):
        use[:, s] = np.bincount(A[:, s], weights=pod_cpu, minlength=N) + (s % 4) * 9000
    c = SimpleNamespace(P=P, N=N, row_ptr=rp, col_idx=ci, pod_cpu=pod_cpu, assign=a, cap_cpu=cap,
                        use_cpu=use.astype(np.int32).reshape(-1))
    etg = _rounds_vs_oracle(ctx, c, S, R, S, threshold=120)
    assert (etg == -1).sum() > 100 and (etg == -2).sum() > 100 and (etg >= 0).sum() > 100


@pytest.mark.parametrize("P,N,deg", [(12_000, 3_000, 5_000), (26_000, 30_000, 20_000)])
def test_rounds_hub_above_4096_neighbours(ctx, P, N, deg):
    """The loop takes any row CAR takes: a hub pod of degree 5,000
    (its count table in the LDS) or 20,000 over 30,000 nodes (20,000 distinct
    candidates: the table in global work areas).  The hub carries the largest
    CPU, so every round evicts it from the hazard node it lands on and scores
    it again; 24 rounds x 16 scenarios against oracle_rounds."""
    rng = np.random.default_rng(deg)
    S, R = 16, 24
    lens = rng.integers(0, 3, P)
    lens[5] = deg
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum(lens)
    ci = rng.integers(0, P, int(rp[-1])).astype(np.int32)
    ci[rp[5]:rp[6]] = rng.choice(np.delete(np.arange(P), 5), deg, replace=False)
    pod_cpu = rng.integers(50, 500, P).astype(np.int32)
    pod_cpu[5] = 900_000
    base = rng.integers(0, N, P)
    a = np.repeat(base[:, None], S, axis=1)
    flip = rng.random((P, S)) < 0.05
    a[flip] = rng.integers(0, N, int(flip.sum()))
    a = a.astype(np.int32)
    cap = np.full(N, 2_000_000, np.int32)
    use = np.zeros((N, S), np.int64)
    for s in range(S):
        use[:, s] = np.bincount(a[:, s], weights=pod_cpu, minlength=N) + rng.integers(0, 200_000, N)
    c = SimpleNamespace(P=P, N=N, row_ptr=rp, col_idx=ci, pod_cpu=pod_cpu, assign=a.reshape(-1), cap_cpu=cap,
                        use_cpu=use.astype(np.int32).reshape(-1))
    from oracle import oracle as orc
    _, _, eev, _ = orc.rounds(rp, ci, pod_cpu, c.assign, S, cap, c.use_cpu, N, R)
    assert (eev == 5).sum() > R * S // 2      # the hub is the evicted pod in most rounds
    etg = _rounds_vs_oracle(ctx, c, S, R, S)
    assert (etg >= 0).sum() > R * S // 2


def test_kernel3_config4_1m50k_s64(ctx):
    """North-star kernel 3 at config 4's shape (1M pods x 50k nodes x 64
    scenarios): rsk_load_std (3,125 node chunks of 16 nodes per scenario,
    folded four to a workgroup into 782 partials, up to four per merge lane
    before the butterfly) with 700 nodes of cap <= 0
    mixed in, and a near-constant-pct batch that stresses the shifted sums;
    rsk_cut_cost over all 1M rows (with and without `missing`) and
    rsk_node_reduce over all 64 M cells, against the oracle
    (nodemonitor.py:24-46, communicationcost.py:37-45, podmonitor.py:104-121).
    The std within 1e-9 relative (north star: 1e-5), the rest exact."""
    from oracle import oracle as orc
    from rsk import api, synth
    P, N, S = 1_000_000, 50_000, 64
    c = synth.make_cluster(P, N, S=S, seed=0)
    rng = np.random.default_rng(11)
    cap = c.cap_cpu.copy()
    cap[rng.choice(N, 500, replace=False)] = 0
    cap[rng.choice(N, 200, replace=False)] = -7
    std = api.load_std(c.use_cpu, cap, N, S, ctx=ctx)
    ostd = orc.load_std(c.use_cpu, cap, N, S)
    assert np.allclose(std, ostd, rtol=1e-9, atol=0), f"max rel {np.max(np.abs(std / ostd - 1))}"
    # near-constant pct: every node at ~37 % with a +-1-millicore jitter
    base = (cap.astype(np.int64) * 37 // 100).clip(0)
    use2 = (base[:, None] + rng.integers(-1, 2, (N, S))).clip(0).astype(np.int32).reshape(-1)
    std2 = api.load_std(use2, cap, N, S, ctx=ctx)
    ostd2 = orc.load_std(use2, cap, N, S)
    assert (ostd2 < 0.05).all() and (ostd2 > 0).all()
    assert np.allclose(std2, ostd2, rtol=1e-9, atol=1e-12), f"max rel {np.max(np.abs(std2 / ostd2 - 1))}"
    # every pct equal (use = cap / 2 on even caps): std 0 on both sides, to rounding
    cap3 = (cap // 2) * 2
    use3 = np.repeat((cap3 // 2).clip(0)[:, None], S, axis=1).astype(np.int32).reshape(-1)
    assert np.allclose(api.load_std(use3, cap3, N, S, ctx=ctx), orc.load_std(use3, cap3, N, S), rtol=0, atol=1e-12)
    cut = api.cut_cost(c.row_ptr, c.col_idx, c.assign, P, S, ctx=ctx)
    assert np.array_equal(cut, orc.cut_cost(c.row_ptr, c.col_idx, c.assign, P, S))
    miss = rng.integers(0, 3, P).astype(np.int32)
    a2 = c.assign.copy()
    a2[rng.choice(P * S, 100_000, replace=False)] = -1
    assert np.array_equal(api.cut_cost(c.row_ptr, c.col_idx, a2, P, S, miss, ctx=ctx),
                          orc.cut_cost(c.row_ptr, c.col_idx, a2, P, S, miss))
    got = api.node_reduce(c.assign, P, S, c.pod_cpu, c.pod_mem, N, ctx=ctx)
    exp = orc.node_reduce(c.assign, P, S, c.pod_cpu, c.pod_mem.astype(np.int64), N)
    for g, e, name in zip(got, exp, ("count", "cpu", "mem")):
        assert np.array_equal(g, e), name
