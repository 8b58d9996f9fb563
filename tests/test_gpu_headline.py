"""GPU parity at the benchmark shapes (BASELINE.json configs 3-5).

Each test runs librsk at the size bench.py times and checks it against the
oracle (oracle/rsk_oracle.c, pinned by the reference's own fixtures) on every
hard row plus a random sample, bit-exactly.  The kernels' template instances
are the ones the bench runs: no score output, S >= 64 (64-scenario tiles).
"""
import os

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


def test_config3_headline_s4096(ctx, synth_golden):
    """100k pods x 5k nodes x 4096 scenarios (the headline batch): every
    mid / hub row and 1000 sampled rows against the oracle, and the reference's
    own 66 golden pods in the unperturbed scenario 0."""
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
    rows, hard = _rows_to_check(c, 1000, 7)
    assert hard.size == 640 and info["mid_rows"] + info["heavy_rows"] == 201 and info["sorted_rows"] == 439
    exp, _ = orc.car(c.row_ptr, c.col_idx, c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, N, rows=rows,
                     threads=THREADS)
    got = t[rows].reshape(-1)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} cells differ; first row {rows[bad[0] // S]} s {bad[0] % S}"


def test_config4_1m50k_s64(ctx):
    """1M pods x 50k nodes x 64 scenarios: all hub and mid rows (max degree
    1,756) plus 1000 sampled rows; also the row-sharded plans of 2 ranks
    (the rows each rank owns) give the same targets."""
    from oracle import oracle as orc
    from rsk import api, synth
    from rsk import dist as rdist
    P, N, S = 1_000_000, 50_000, 64
    c = synth.make_cluster(P, N, S=S, seed=0)
    plan = api.CarPlan(c.row_ptr, c.col_idx, ctx=ctx)
    tgt, _ = plan.execute(c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, N)
    plan.close()
    t = tgt.reshape(P, S)
    rows, hard = _rows_to_check(c, 1000, 8)
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


def test_config5_rounds_100k_s1024(ctx):
    """100k/5k x 1024 scenarios, 8 rounds of detect -> evict -> CAR -> update
    on the device; the first 16 scenarios against oracle_rounds (state,
    evictions and targets of every round)."""
    from oracle import oracle as orc
    from rsk import api, synth
    P, N, S, R, k = 100_000, 5_000, 1024, 8, 16
    c = synth.make_cluster(P, N, S=S, seed=0)
    a0 = c.assign.reshape(P, S)[:, :k].copy().reshape(-1)
    u0 = c.use_cpu.reshape(N, S)[:, :k].copy().reshape(-1)
    rounds = api.Rounds(c.row_ptr, c.col_idx, c.pod_cpu, ctx=ctx)
    a, u = c.assign.copy(), c.use_cpu.copy()
    ev, tg = rounds.run(a, S, c.cap_cpu, u, N, R)
    rounds.close()
    ea, eu, eev, etg = orc.rounds(c.row_ptr, c.col_idx, c.pod_cpu, a0, k, c.cap_cpu, u0, N, R)
    assert np.array_equal(a.reshape(P, S)[:, :k].reshape(-1), ea)
    assert np.array_equal(u.reshape(N, S)[:, :k].reshape(-1), eu)
    assert np.array_equal(ev.reshape(R, S)[:, :k].reshape(-1), eev)
    assert np.array_equal(tg.reshape(R, S)[:, :k].reshape(-1), etg)
    assert (tg >= 0).sum() > R * S // 2  # real moves happened
