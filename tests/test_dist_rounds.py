"""The pod-row-sharded multi-round loop (rsk/dist.py RowShardedRounds; SURVEY.md
§8e pod-row sharding x §8f item 1): int64 all-reduce of per-node CPU / mem
partials, MAX all-reduce of the packed eviction key, all-gather of the changed
assignment slices, SUM all-reduce of the cut cost — rehearsed with gloo at
world sizes 2 and 3 on CPU and checked bit-equal against the single-process
oracle_rounds (oracle/rsk_oracle.c), round by round.

On CPU the per-rank compute is a numpy backend over the oracle (this file; the
exchange logic is what these tests pin).  The GPU test runs the same driver on
librsk (LibrskRoundsBackend, device pointers) in two processes sharing the
box's one GPU, gloo carrying the collectives.
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


class OracleRoundsBackend:
    """CPU backend of RowShardedRounds over the C oracle (test infrastructure)."""

    def __init__(self, row_ptr, col_idx):
        from oracle import oracle as orc
        self.orc = orc
        self.rp, self.ci = np.asarray(row_ptr, np.int32), np.asarray(col_idx, np.int32)
        self.drp, self.dci = orc.dedup_csr(self.rp, self.ci)
        self.P = len(self.rp) - 1
        self.rev = [[] for _ in range(self.P)]   # rows holding each pod (the CSR's transpose)
        for p in range(self.P):
            for q in self.ci[self.rp[p]:self.rp[p + 1]]:
                self.rev[int(q)].append(p)

    @staticmethod
    def _t(a):
        import torch
        return torch.from_numpy(np.ascontiguousarray(a))

    def node_partials(self, assign_rows, pod_cpu_rows, pod_mem_rows, q, N, S):
        _, cpu, mem = self.orc.node_reduce(assign_rows.numpy(), q, S, pod_cpu_rows.numpy(), pod_mem_rows.numpy(), N)
        return self._t(cpu), self._t(mem)

    def detect(self, use, cap, N, S, threshold):
        pct = self.orc.cpu_pct(use.numpy(), cap.numpy(), N, S)
        haz, most = self.orc.detect(pct, N, S, threshold)
        return self._t(haz), self._t(most)

    def pick_rows(self, assign_rows, pod_cpu_rows, q, S, most):
        return self._t(self.orc.pick_max_pod(assign_rows.numpy(), pod_cpu_rows.numpy(), q, S, most.numpy()))

    def place(self, assign, S, cap, use, haz, N, evict):
        a, u, h, e = assign.numpy().reshape(-1, S), use.numpy().reshape(N, S), haz.numpy().reshape(N, S), evict.numpy()
        out = np.full(S, -3, np.int32)
        for s in np.nonzero(e >= 0)[0]:
            t, _ = self.orc.car(self.drp, self.dci, np.ascontiguousarray(a[:, s]), 1, cap.numpy(),
                                np.ascontiguousarray(u[:, s]), np.ascontiguousarray(h[:, s]), N,
                                rows=np.array([e[s]], np.int32))
            out[s] = t[0]
        return self._t(out)

    def cut_delta(self, assign, S, evict, target, r0, r1, N, cut):
        """cut[s] += the change of the directed cut over rows [r0, r1) that
        scenario s's move makes (assign still holds the old node)."""
        a, ev, tg, out = assign.numpy().reshape(-1, S), evict.numpy(), target.numpy(), cut.numpy()
        for s in range(S):
            e, t = int(ev[s]), int(tg[s])
            if e < 0 or e >= self.P or t < 0 or t >= N:
                continue
            o, d = a[e, s], 0
            if r0 <= e < r1:
                for q in self.ci[self.rp[e]:self.rp[e + 1]]:
                    if q != e:
                        d += int(t != a[q, s]) - int(o != a[q, s])
            for q in self.rev[e]:
                if q != e and r0 <= q < r1:
                    d += int(a[q, s] != t) - int(a[q, s] != o)
            out[s] += d

    def cut_rows(self, assign, S, r0, r1):
        deg = np.diff(self.rp)
        deg[:r0] = 0
        deg[r1:] = 0
        rp = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
        ci = np.concatenate([self.ci[self.rp[p]:self.rp[p + 1]] for p in range(r0, r1)] + [np.zeros(0, np.int32)])
        return self._t(self.orc.cut_cost(rp, ci.astype(np.int32), assign.numpy(), self.P, S))


def _case(seed=5, P=900, N=12, S=6):
    """A synthetic cluster whose hottest nodes sit around the 30 % threshold
    (as tests/test_rounds.py), plus per-pod memory for the mem partials."""
    from rsk import synth
    c = synth.make_cluster(P, N, S=S, seed=seed)
    rng = np.random.default_rng(seed)
    pod_mem = rng.integers(1 << 20, 1 << 30, P).astype(np.int64)
    pod_cpu = c.pod_cpu.astype(np.int32).copy()
    pod_cpu[rng.random(P) < 0.02] = -1            # pods without metrics: never evicted
    a = c.assign.reshape(P, S)
    load = np.stack([np.bincount(a[:, s][a[:, s] >= 0], weights=np.maximum(pod_cpu[a[:, s] >= 0], 0),
                                 minlength=N) for s in range(S)], axis=1)
    c.cap_cpu = np.full(N, int(load.mean() * 100 / 30) + 1, np.int32)
    c.use_cpu = (load + rng.integers(0, c.cap_cpu[0] // 10, (N, 1))).astype(np.int32).reshape(-1)
    return c, pod_cpu, pod_mem


def _expected(c, pod_cpu, R):
    """oracle_rounds one round at a time: per-round evict / target / directed cut, final state."""
    from oracle import oracle as orc
    a, u = c.assign.copy(), c.use_cpu.copy()
    ev, tg, cut = [], [], []
    for _ in range(R):
        a, u, e, t = orc.rounds(c.row_ptr, c.col_idx, pod_cpu, a, c.S, c.cap_cpu, u, c.N, 1)
        ev.append(e)
        tg.append(t)
        cut.append(orc.cut_cost(c.row_ptr, c.col_idx, a, c.P, c.S))
    return np.array(ev), np.array(tg), np.array(cut), a, u


def _worker(rank, world, port, R, out_q, use_gpu, pg="gloo", ordered=False, fused=True, case=None):
    import sys
    sys.path[:0] = [PKG, REPO]
    import torch
    import torch.distributed as dist

    from rsk import dist as rdist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if use_gpu:
        import faulthandler
        os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
        fh = open(os.path.join(REPO, "gpurun_out", f"dist_rounds_rank{rank}.txt"), "w")
        faulthandler.enable(file=fh)
        faulthandler.dump_traceback_later(60, exit=True, file=fh)   # a hung rank leaves its stack behind
        torch.cuda.set_device(0)
    dist.init_process_group(pg, rank=rank, world_size=world)
    try:
        import contextlib
        c, pod_cpu, pod_mem = _case(**(case or {}))
        dev = torch.device("cuda:0" if use_gpu else "cpu")
        sh = rdist.row_shard_for(rank, world, c.row_ptr)
        T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
        assign = T(c.assign)
        args = (T(c.use_cpu), T(c.cap_cpu), T(pod_cpu), T(pod_mem), c.N, c.S, R)
        st = torch.cuda.Stream(dev) if ordered else None
        if st is not None:
            st.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(st) if st is not None else contextlib.nullcontext():
            be = (rdist.LibrskRoundsBackend(c.row_ptr, c.col_idx, pod_cpu, device=dev, stream_ordered=ordered,
                                            fused=fused)
                  if use_gpu else OracleRoundsBackend(c.row_ptr, c.col_idx))
            res = rdist.RowShardedRounds(sh, be).run(assign, *args)
        if use_gpu:
            torch.cuda.synchronize(dev)
        out_q.put((rank, res["evict"].cpu().numpy(), res["target"].cpu().numpy(), res["cut"].cpu().numpy(),
                   assign.cpu().numpy(), res["use"].cpu().numpy()))
    except BaseException:  # noqa: BLE001 - report to the parent instead of leaving the peer in a collective
        import traceback
        out_q.put(("error", rank, traceback.format_exc()))
        out_q.close()
        out_q.join_thread()   # flush the report before the hard exit
        os._exit(1)
    finally:
        dist.destroy_process_group()


def _run(world, R, use_gpu=False, pg="gloo", ordered=False, fused=True, case=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, R, q, use_gpu, pg, ordered, fused, case))
             for r in range(world)]
    for p in procs:
        p.start()
    outs = []
    try:
        for _ in range(world):
            try:
                o = q.get(timeout=100)
            except Exception:
                raise AssertionError(f"no result; exit codes {[p.exitcode for p in procs]}") from None
            assert o[0] != "error", f"rank {o[1]} failed:\n{o[2]}"
            outs.append(o)
    finally:
        for p in procs:
            p.join(30)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    return sorted(outs, key=lambda o: o[0])


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_rounds_bit_equal_oracle_rounds(world):
    R = 5
    c, pod_cpu, _ = _case()
    ev, tg, cut, a, u = _expected(c, pod_cpu, R)
    assert (ev >= 0).sum() > R * c.S // 2 and (tg >= 0).sum() > 0      # real evictions and moves
    for rank, e, t, k, a_r, u_r in _run(world, R):
        assert np.array_equal(e, ev), f"rank {rank}: evictions differ"
        assert np.array_equal(t, tg), f"rank {rank}: targets differ"
        assert np.array_equal(k, cut), f"rank {rank}: cut costs differ"
        assert np.array_equal(a_r, a), f"rank {rank}: assign replica differs"
        assert np.array_equal(u_r, u), f"rank {rank}: usage differs"


def test_row_shards_cover_rows_once():
    from rsk import dist as rdist
    c, _, _ = _case()
    for world in (1, 2, 3, 8):
        b = [rdist.row_shard_for(r, world, c.row_ptr) for r in range(world)]
        assert b[0].r0 == 0 and b[-1].r1 == c.P
        assert all(b[k].r1 == b[k + 1].r0 for k in range(world - 1))


@pytest.mark.gpu
def test_row_sharded_rounds_on_librsk_world2():
    """Two processes on the one GPU (librsk per rank, gloo collectives) against
    oracle_rounds."""
    R = 4
    c, pod_cpu, _ = _case()
    ev, tg, cut, a, u = _expected(c, pod_cpu, R)
    for rank, e, t, k, a_r, u_r in _run(2, R, use_gpu=True):
        assert np.array_equal(e, ev) and np.array_equal(t, tg), f"rank {rank}"
        assert np.array_equal(k, cut) and np.array_equal(a_r, a) and np.array_equal(u_r, u), f"rank {rank}"


@pytest.mark.gpu
def test_row_sharded_rounds_rccl_world1():
    """One rank over the "nccl" (RCCL) process group: the collectives run on
    device tensors, as on an 8-GPU node."""
    R = 3
    c, pod_cpu, _ = _case()
    ev, tg, cut, a, u = _expected(c, pod_cpu, R)
    (rank, e, t, k, a_r, u_r), = _run(1, R, use_gpu=True, pg="nccl")
    assert np.array_equal(e, ev) and np.array_equal(t, tg) and np.array_equal(k, cut)
    assert np.array_equal(a_r, a) and np.array_equal(u_r, u)


@pytest.mark.gpu
def test_row_sharded_rounds_stream_ordered_rccl_world1():
    """The stream-ordered backend (librsk on the current torch stream, no host
    syncs between phases; bench.py's rounds rate) against oracle_rounds."""
    R = 3
    c, pod_cpu, _ = _case()
    ev, tg, cut, a, u = _expected(c, pod_cpu, R)
    (rank, e, t, k, a_r, u_r), = _run(1, R, use_gpu=True, pg="nccl", ordered=True)
    assert np.array_equal(e, ev) and np.array_equal(t, tg) and np.array_equal(k, cut)
    assert np.array_equal(a_r, a) and np.array_equal(u_r, u)


@pytest.mark.gpu
def test_row_sharded_rounds_stream_ordered_gloo_world2():
    """The stream-ordered backend with real multi-rank collectives (two ranks on
    the one GPU, gloo on device tensors): librsk kernels, torch ops and every
    all-reduce / all-gather ordered on each rank's torch stream, against
    oracle_rounds."""
    R = 4
    c, pod_cpu, _ = _case()
    ev, tg, cut, a, u = _expected(c, pod_cpu, R)
    for rank, e, t, k, a_r, u_r in _run(2, R, use_gpu=True, ordered=True):
        assert np.array_equal(e, ev) and np.array_equal(t, tg), f"rank {rank}"
        assert np.array_equal(k, cut) and np.array_equal(a_r, a) and np.array_equal(u_r, u), f"rank {rank}"


@pytest.mark.gpu
@pytest.mark.parametrize("ordered", [False, True])
def test_row_sharded_rounds_unfused_world2(ordered):
    """The per-phase librsk calls (fused=False: detect, pick, evict key / decode,
    place, cut delta, apply as separate launches) against oracle_rounds; the
    tests above run the fused round (rsk_rows_detect_setup, rsk_rows_pick / _place / _move)."""
    R = 4
    c, pod_cpu, _ = _case()
    ev, tg, cut, a, u = _expected(c, pod_cpu, R)
    for rank, e, t, k, a_r, u_r in _run(2, R, use_gpu=True, ordered=ordered, fused=False):
        assert np.array_equal(e, ev) and np.array_equal(t, tg), f"rank {rank}"
        assert np.array_equal(k, cut) and np.array_equal(a_r, a) and np.array_equal(u_r, u), f"rank {rank}"


# N = 300 nodes (five 64-node blocks): moves between blocks, so the fused move
# launch re-reduces the old node's block beside the new one's (wave 1's
# blk_update) and the scenario's maxima over several blocks (scn_reduce)
BIG = dict(seed=7, P=6000, N=300, S=64)


def _cross_block_moves(c, ev, tg):
    """Moves whose pod leaves one 64-node block for another, replayed in order."""
    a = c.assign.copy().reshape(c.P, c.S)
    n = 0
    for e_r, t_r in zip(ev, tg):
        for s in range(c.S):
            e, t = int(e_r[s]), int(t_r[s])
            if e >= 0 and t >= 0:
                n += int(a[e, s] // 64 != t // 64)
                a[e, s] = t
    return n


@pytest.mark.gpu
@pytest.mark.parametrize("world,pg", [(1, "nccl"), (2, "gloo")])
def test_row_sharded_rounds_fused_cross_block(world, pg):
    """the fused row-sharded round (rsk_rows_detect_setup / _pick /
    _place / _move with the block maxima) at N = 300 over 12 rounds, world 1
    over RCCL and world 2 over gloo, against oracle_rounds round by round;
    most moves cross 64-node blocks."""
    R = 12
    c, pod_cpu, _ = _case(**BIG)
    ev, tg, cut, a, u = _expected(c, pod_cpu, R)
    assert (tg >= 0).sum() > R * c.S // 2
    assert _cross_block_moves(c, ev, tg) > R * c.S // 4
    for rank, e, t, k, a_r, u_r in _run(world, R, use_gpu=True, pg=pg, case=BIG):
        assert np.array_equal(e, ev) and np.array_equal(t, tg), f"rank {rank}"
        assert np.array_equal(k, cut) and np.array_equal(a_r, a) and np.array_equal(u_r, u), f"rank {rank}"


@pytest.mark.gpu
def test_row_sharded_rounds_fused_equals_unfused_world2():
    """The fused round and the per-phase calls give the same rounds at N = 300."""
    R = 12
    f = _run(2, R, use_gpu=True, case=BIG)
    g = _run(2, R, use_gpu=True, fused=False, case=BIG)
    for x, y in zip(f, g):
        for a_, b_ in zip(x[1:], y[1:]):
            assert np.array_equal(a_, b_)


def test_cross_block_case_moves_between_blocks():
    """CPU: the BIG case really moves pods between 64-node blocks (oracle)."""
    R = 12
    c, pod_cpu, _ = _case(**BIG)
    ev, tg, cut, a, u = _expected(c, pod_cpu, R)
    assert (tg >= 0).sum() > R * c.S // 2
    assert _cross_block_moves(c, ev, tg) > R * c.S // 4


def test_row_sharded_rounds_cross_block_gloo_world2_cpu():
    """The BIG case through the row-sharded loop on CPU (gloo, oracle backend)."""
    R = 6
    c, pod_cpu, _ = _case(**BIG)
    ev, tg, cut, a, u = _expected(c, pod_cpu, R)
    for rank, e, t, k, a_r, u_r in _run(2, R, case=BIG):
        assert np.array_equal(e, ev) and np.array_equal(t, tg), f"rank {rank}"
        assert np.array_equal(k, cut) and np.array_equal(a_r, a) and np.array_equal(u_r, u), f"rank {rank}"
