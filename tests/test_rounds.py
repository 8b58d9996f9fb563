"""The multi-round loop: detect -> evict -> CAR -> update.

CPU: the oracle's C loop (oracle_rounds) equals a round-by-round composition
of the single-step oracle functions, which tests/test_oracle_golden.py pins
against the reference's own fixtures.  The update rule (the pod's CPU moves
with it) is build-defined: the reference re-measures the live cluster each
round, so beyond one round the loop is "parity unpinned" against the
reference and pinned against this restatement only.
GPU: librsk's rsk_rounds_run against oracle_rounds, bit-exact.
"""
import numpy as np
import pytest


def _case(seed, P=400, N=12, S=6):
    """A synthetic cluster whose hottest nodes sit around the threshold."""
    from rsk import synth
    rng = np.random.default_rng(seed)
    c = synth.make_cluster(P, N, S=S, seed=seed)
    pod_cpu = c.pod_cpu.astype(np.int32).copy()
    pod_cpu[rng.random(P) < 0.05] = -1  # never picked (strict '>' from -1)
    a = c.assign.reshape(P, S)
    load = np.stack([np.bincount(a[:, s][a[:, s] >= 0], weights=np.maximum(pod_cpu[a[:, s] >= 0], 0),
                                 minlength=N) for s in range(S)], axis=1)
    cap = np.full(N, int(load.mean() * 100 / 30) + 1, np.int32)  # mean node at ~30 %
    use = (load + rng.integers(0, cap[0] // 10, (N, 1))).astype(np.int32).reshape(-1)
    return c, pod_cpu, cap, use


def _compose(c, pod_cpu, cap, use, N, S, R, thr):
    """Round by round from the pinned single-step oracles."""
    from oracle import oracle as orc
    rp, ci = orc.dedup_csr(c.row_ptr, c.col_idx)
    a, u = c.assign.copy(), use.copy()
    evs, tgs = [], []
    for _ in range(R):
        pct = orc.cpu_pct(u, cap, N, S)
        haz, most = orc.detect(pct, N, S, thr)
        ev = orc.pick_max_pod(a, pod_cpu, c.P, S, most)
        tg = np.full(S, -3, np.int32)
        for s in range(S):
            p = int(ev[s])
            if p < 0:
                continue
            t, _ = orc.car(rp, ci, a, S, cap, u, haz, N, rows=np.array([p], np.int32))
            tg[s] = t.reshape(S)[s]
            if tg[s] >= 0:
                old = a[p * S + s]
                if 0 <= old < N:
                    u[old * S + s] -= pod_cpu[p]
                u[tg[s] * S + s] += pod_cpu[p]
                a[p * S + s] = tg[s]
        evs.append(ev)
        tgs.append(tg)
    return a, u, np.concatenate(evs), np.concatenate(tgs)


@pytest.mark.parametrize("seed,thr,moves", [(1, 30, True), (2, 34, True), (3, 10, False)])
def test_oracle_rounds_equals_composition(seed, thr, moves):
    """thr 10: every node is hazard, every move raises (target -2)."""
    from oracle import oracle as orc
    c, pod_cpu, cap, use = _case(seed)
    R = 12
    got = orc.rounds(c.row_ptr, c.col_idx, pod_cpu, c.assign, c.S, cap, use, c.N, R, thr)
    exp = _compose(c, pod_cpu, cap, use, c.N, c.S, R, thr)
    for g, e, name in zip(got, exp, ("assign", "use", "evict", "target")):
        assert np.array_equal(g, e), name
    if moves:
        assert (got[2] >= 0).any() and (got[3] >= 0).any()  # the loop really moved pods
    else:
        assert (got[3][got[2] >= 0] == -2).all()


@pytest.mark.parametrize("seed,thr,S,threads", [(1, 30, 6, 3), (2, 34, 37, 8), (3, 10, 5, 2), (4, 45, 64, 1)])
def test_oracle_rounds_par_equals_serial(seed, thr, S, threads):
    """oracle_rounds_par (each scenario an S = 1 run on its own columns, the
    scenarios split over threads) gives oracle_rounds' results; its numpy
    CSR dedup gives dedup_csr's rows (duplicates and self edges included)."""
    from oracle import oracle as orc
    c, pod_cpu, cap, use = _case(seed, P=600, N=20, S=S)
    rng = np.random.default_rng(seed)
    extra = rng.integers(0, c.P, 200).astype(np.int32)           # duplicate edges and self edges
    rows = rng.integers(0, c.P, 200)
    rp, ci = c.row_ptr.astype(np.int64), c.col_idx[:c.row_ptr[-1]].astype(np.int64)
    lists = [list(ci[rp[p]:rp[p + 1]]) for p in range(c.P)]
    for r, q in zip(rows, extra):
        lists[r] += [q, q, r]
    rp2 = np.zeros(c.P + 1, np.int32)
    rp2[1:] = np.cumsum([len(x) for x in lists])
    ci2 = np.array([q for x in lists for q in x], np.int32)
    a1, b1 = orc.dedup_csr(rp2, ci2)
    a2, b2 = orc.dedup_csr_fast(rp2, ci2)
    assert np.array_equal(a1, a2) and np.array_equal(b1[:a1[-1]], b2[:a2[-1]])
    R = 20
    ser = orc.rounds(rp2, ci2, pod_cpu, c.assign, S, cap, use, c.N, R, thr)
    par = orc.rounds(rp2, ci2, pod_cpu, c.assign, S, cap, use, c.N, R, thr, threads=threads)
    for g, e, name in zip(par, ser, ("assign", "use", "evict", "target")):
        assert np.array_equal(g, e), name
    if thr != 10:
        assert (ser[3] >= 0).any()  # real moves


@pytest.mark.gpu
@pytest.mark.parametrize("seed,thr,S", [(1, 30, 6), (2, 45, 64), (3, 10, 65), (4, 30, 1)])
def test_gpu_rounds_match_oracle(seed, thr, S):
    from oracle import oracle as orc
    from rsk import _lib, api
    c, pod_cpu, cap, use = _case(seed, S=S)
    R = 16
    exp = orc.rounds(c.row_ptr, c.col_idx, pod_cpu, c.assign, c.S, cap, use, c.N, R, thr)
    rounds = api.Rounds(c.row_ptr, c.col_idx, pod_cpu, ctx=_lib.default_context())
    a, u = c.assign.copy(), use.copy()
    ev, tg = rounds.run(a, c.S, cap, u, c.N, R, threshold=thr)
    rounds.close()
    for g, e, name in zip((a, u, ev, tg), exp, ("assign", "use", "evict", "target")):
        bad = np.nonzero(g != e)[0]
        assert bad.size == 0, f"{name}: {bad.size} differ, first {bad[0]}: gpu {g[bad[0]]} oracle {e[bad[0]]}"


@pytest.mark.gpu
def test_gpu_rounds_hub_rows_and_hash():
    """An evicted hub pod (degree up to 700) and N = 20000 (large hash spread)."""
    from oracle import oracle as orc
    from rsk import _lib, api
    rng = np.random.default_rng(9)
    P, N, S, R = 1500, 20000, 8, 6
    rows = [rng.integers(0, P, int(rng.integers(0, 4))).tolist() for _ in range(P)]
    for k, d in enumerate([700, 300, 90]):
        rows[k] = rng.choice(P, d, replace=False).tolist()
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.array([q for r in rows for q in r], np.int32)
    assign = rng.integers(0, 40, P * S).astype(np.int32)  # crowded: real counts and ties
    assign.reshape(P, S)[:3] = 0                           # the hubs sit on node 0, the hottest
    pod_cpu = rng.integers(1, 500, P).astype(np.int32)
    pod_cpu[:3] = 100000
    cap = np.full(N, 50000, np.int32)
    use = rng.integers(0, 20000, N * S).astype(np.int32)
    use.reshape(N, S)[0] = 49000
    exp = orc.rounds(rp, ci, pod_cpu, assign, S, cap, use, N, R)
    rounds = api.Rounds(rp, ci, pod_cpu, ctx=_lib.default_context())
    a, u = assign.copy(), use.copy()
    ev, tg = rounds.run(a, S, cap, u, N, R)
    rounds.close()
    assert (exp[2][:S] <= 2).all()  # the first round evicts a hub pod
    for g, e, name in zip((a, u, ev, tg), exp, ("assign", "use", "evict", "target")):
        assert np.array_equal(g, e), name


@pytest.mark.gpu
def test_gpu_rounds_pod_lists_overflow_mid_run():
    """The eviction pick's pod lists (rsk_rounds_run): scenarios whose list of
    pods off their base node (scenario 0's node) starts just under the list's
    capacity (max(256, P/16) = 256 here) and overflows while pods move (the
    full-scan fallback), one far beyond it from the start, and unassigned pods
    (-1) in the base and in the scenarios."""
    from oracle import oracle as orc
    from rsk import _lib, api
    rng = np.random.default_rng(21)
    P, N, S, R = 4096, 64, 8, 24
    rows = [rng.integers(0, P, int(rng.integers(0, 6))).tolist() for _ in range(P)]
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.array([q for r in rows for q in r], np.int32)
    base = rng.integers(0, N, P).astype(np.int32)
    base[rng.random(P) < 0.01] = -1
    a = np.repeat(base[:, None], S, axis=1)
    for s in range(1, S):
        k = {1: 0, 2: 240, 3: 250, 4: 255, 5: 256, 6: 3000}.get(s, 100)
        idx = rng.choice(P, k, replace=False)
        a[idx, s] = (a[idx, s] + 1 + rng.integers(0, N - 1, k)) % N   # another node (or -1 -> a node)
    a[rng.random((P, S)) < 0.002] = -1
    assign = a.reshape(-1).astype(np.int32)
    pod_cpu = rng.integers(1, 500, P).astype(np.int32)
    pod_cpu[rng.random(P) < 0.03] = -1
    load = np.stack([np.bincount(a[:, s][a[:, s] >= 0], weights=np.maximum(pod_cpu[a[:, s] >= 0], 0), minlength=N)
                     for s in range(S)], axis=1)
    cap = np.full(N, int(load.mean() * 100 / 30) + 1, np.int32)
    use = (load + rng.integers(0, cap[0] // 10, (N, 1))).astype(np.int32).reshape(-1)
    exp = orc.rounds(rp, ci, pod_cpu, assign, S, cap, use, N, R)
    rounds = api.Rounds(rp, ci, pod_cpu, ctx=_lib.default_context())
    g_a, g_u = assign.copy(), use.copy()
    ev, tg = rounds.run(g_a, S, cap, g_u, N, R)
    rounds.close()
    assert (exp[3] >= 0).sum() > R * S // 2   # pods really move (lists grow)
    for g, e, name in zip((g_a, g_u, ev, tg), exp, ("assign", "use", "evict", "target")):
        bad = np.nonzero(g != e)[0]
        assert bad.size == 0, f"{name}: {bad.size} differ, first {bad[0]}: gpu {g[bad[0]]} oracle {e[bad[0]]}"


@pytest.mark.gpu
def test_gpu_rounds_one_wave_rows_boundary():
    """Round 6's one-wave path of car_move_one (rows of <= 64 neighbours: a
    ballot per distinct node, no hash, no barrier) at its boundary: evicted
    pods whose rows have 63, 64 and 65 entries (drawn with duplicates, self
    edges included, so the distinct count differs from the entry count), a row
    whose neighbours all sit on the hazard node in one scenario (max score 0:
    the zero case from the loop's LDS detect state) and pods with one or no
    neighbour; against oracle_rounds, every scenario and round."""
    from oracle import oracle as orc
    from rsk import _lib, api
    rng = np.random.default_rng(64)
    P, N, S, R = 700, 30, 8, 14
    rows = [rng.integers(0, P, int(rng.integers(0, 4))).tolist() for _ in range(P)]
    for k, d in enumerate([63, 64, 65, 64, 65, 1, 0]):
        r = rng.integers(0, P, d).tolist()
        if d >= 2:
            r[0] = k               # a self edge
            r[1] = r[2 % d]        # a duplicate
        rows[k] = r
    rp = np.zeros(P + 1, np.int32)
    rp[1:] = np.cumsum([len(r) for r in rows])
    ci = np.array([q for r in rows for q in r], np.int32)
    assign = rng.integers(1, N, (P, S)).astype(np.int32)
    assign[:7] = 0                                    # the boundary rows' pods on node 0, the hottest
    assign[[q for q in rows[1] if q >= 7], 2] = 0     # scenario 2: row 1's neighbours on the hazard node too
    pod_cpu = rng.integers(1, 400, P).astype(np.int32)
    pod_cpu[:7] = 50000 - np.arange(7) * 1000         # evicted first, in row order
    cap = np.full(N, 60000, np.int32)
    load = np.stack([np.bincount(assign[:, s], weights=pod_cpu, minlength=N) for s in range(S)], axis=1)
    use = (load + rng.integers(0, 3000, (N, 1))).astype(np.int32).reshape(-1)
    assign = assign.reshape(-1)
    exp = orc.rounds(rp, ci, pod_cpu, assign, S, cap, use, N, R, 40)
    rounds = api.Rounds(rp, ci, pod_cpu, ctx=_lib.default_context())
    a, u = assign.copy(), use.copy()
    ev, tg = rounds.run(a, S, cap, u, N, R, threshold=40)
    rounds.close()
    assert set(range(5)) <= set(exp[2].tolist())     # the 63 / 64 / 65-entry rows are evicted
    for g, e, name in zip((a, u, ev, tg), exp, ("assign", "use", "evict", "target")):
        bad = np.nonzero(g != e)[0]
        assert bad.size == 0, f"{name}: {bad.size} differ, first {bad[0]}: gpu {g[bad[0]]} oracle {e[bad[0]]}"
