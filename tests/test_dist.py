"""CPU: the scenario-sharded multi-GPU layout, rehearsed with gloo at world size 2.

Each rank builds only its own scenario range (synth.make_cluster(..., s0=rank·S)),
scores it (oracle here; librsk on the GPU box), and the optional exchanges
(all-gather of per-scenario results, all-reduce of metrics) reassemble exactly
what a single process scoring all scenarios produces.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, S, out_q):
    import sys
    sys.path[:0] = [PKG, REPO]
    import torch
    import torch.distributed as dist

    from oracle import oracle as orc
    from rsk import dist as rdist
    from rsk import synth

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = rdist.shard_for(rank, world, S)
        c = synth.make_cluster(600, 24, S=S, seed=1, s0=sh.s0)
        rows = np.arange(0, 600, 37, dtype=np.int32)
        tgt, _ = orc.car(c.row_ptr, c.col_idx, c.assign, S, c.cap_cpu, c.use_cpu, c.hazard, c.N, rows=rows)
        full = rdist.gather_scenarios(torch.from_numpy(tgt.reshape(len(rows), S)))
        cut = torch.from_numpy(orc.cut_cost(c.row_ptr, c.col_idx, c.assign, c.P, S)).sum().reshape(1)
        rdist.allreduce_sum(cut)
        if rank == 0:
            out_q.put((full.numpy(), int(cut.item())))
    finally:
        dist.destroy_process_group()


def test_scenario_sharding_world2_matches_single_process():
    from oracle import oracle as orc
    from rsk import synth
    world, S = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, cut = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = synth.make_cluster(600, 24, S=world * S, seed=1)
    rows = np.arange(0, 600, 37, dtype=np.int32)
    tgt, _ = orc.car(c.row_ptr, c.col_idx, c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N, rows=rows)
    assert np.array_equal(full, tgt.reshape(len(rows), c.S))
    assert cut == int(orc.cut_cost(c.row_ptr, c.col_idx, c.assign, c.P, c.S).sum())


def test_shard_ids():
    from rsk import dist as rdist
    sh = rdist.shard_for(3, 8, 1024)
    assert sh.s0 == 3072 and sh.s_total == 8192 and list(sh.global_ids())[:2] == [3072, 3073]
    with pytest.raises(ValueError):
        rdist.shard_for(8, 8, 1)


def _row_worker(rank, world, port, out_q):
    import sys
    sys.path[:0] = [PKG, REPO]
    import torch
    import torch.distributed as dist

    from oracle import oracle as orc
    from rsk import dist as rdist
    from rsk import synth

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = synth.make_cluster(900, 30, S=3, seed=4)  # every rank holds the full assign replica
        sh = rdist.row_shard_for(rank, world, c.row_ptr)
        tgt, _ = orc.car(c.row_ptr, c.col_idx, c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N, rows=sh.rows)
        full = rdist.gather_rows(torch.from_numpy(tgt), sh, c.S)
        if rank == 0:
            out_q.put(full.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharding_matches_single_process(world):
    from oracle import oracle as orc
    from rsk import synth
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_row_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    full = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    c = synth.make_cluster(900, 30, S=3, seed=4)
    tgt, _ = orc.car(c.row_ptr, c.col_idx, c.assign, c.S, c.cap_cpu, c.use_cpu, c.hazard, c.N)
    assert np.array_equal(full, tgt)


def test_row_shard_bounds_balance_nnz():
    from rsk import dist as rdist
    from rsk import synth
    c = synth.make_cluster(20000, 50, S=1, seed=0)
    deg = np.diff(c.row_ptr)
    for world in (1, 2, 4, 8):
        shards = [rdist.row_shard_for(r, world, c.row_ptr) for r in range(world)]
        assert shards[0].r0 == 0 and shards[-1].r1 == c.P
        assert all(shards[k].r1 == shards[k + 1].r0 for k in range(world - 1))
        cost = [int(deg[s.r0:s.r1].sum()) + s.q for s in shards]
        # the PA root (degree ~ sqrt-scale hub) is the only indivisible lump
        assert max(cost) - min(cost) <= int(deg.max()) + 2, (world, cost)
    rp = np.array([0, 0, 0], np.int32)  # more ranks than rows: empty ranges are fine
    s = [rdist.row_shard_for(r, 4, rp) for r in range(4)]
    assert sum(x.q for x in s) == 2
