"""Multi-GPU layouts of the placement path.

Scenario sharding (configs 3 and 5, the default):

One process per GPU (torch.distributed; backend "nccl" = RCCL over xGMI on
ROCm, "gloo" on CPU for tests).  Scenarios are independent what-if batches, so
rank r owns global scenarios [r·S_local, (r+1)·S_local) against a replicated
relation plan and per-node constants: the data path needs no collective.  The
helpers below are the only exchanges, and both are optional summaries:

* ``gather_scenarios`` — all-gather a per-scenario result vector (e.g. the
  chosen node per scenario for one pod, or per-scenario metrics) so rank 0 sees
  the global batch; payload S_local words per rank.
* ``allreduce_sum`` — sum of per-scenario scalar metrics (cut cost, counts).

Per-rank inputs are generated (or loaded) for the rank's own scenario range, so
no assignment matrix ever crosses xGMI.

Pod-row sharding (config 4, 1M pods x 50k nodes x 64 scenarios):

* ``row_shard_for`` — rank r owns a contiguous range of CSR rows balanced by
  nnz (+1 per row, so empty rows still cost a target word) and keeps the full
  ``assign[P*S]`` replica; its plan is built on that row subset.
* ``gather_rows`` — all-gather of every rank's ``target`` rows back into the
  full ``target[P*S]``: P*S/G int32 per rank over RCCL.  It is the only
  data-path exchange of a round and is timed separately from scoring.
"""
from __future__ import annotations

import os
import sys
from dataclasses import dataclass


@dataclass(frozen=True)
class ScenarioShard:
    rank: int
    world: int
    s_local: int

    @property
    def s0(self) -> int:
        """First global scenario id of this rank."""
        return self.rank * self.s_local

    @property
    def s_total(self) -> int:
        return self.world * self.s_local

    def global_ids(self):
        return range(self.s0, self.s0 + self.s_local)


def shard_for(rank: int, world: int, s_local: int) -> ScenarioShard:
    if not (0 <= rank < world) or s_local <= 0:
        raise ValueError(f"bad shard rank={rank} world={world} s_local={s_local}")
    return ScenarioShard(rank, world, s_local)


def gather_scenarios(local, group=None):
    """All-gather rank-local per-scenario tensors [..., S_local] into [..., S_total]
    (scenario-minor concatenation in rank order)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local.contiguous(), group=group)
    return torch.cat(parts, dim=-1)


def allreduce_sum(t, group=None):
    import torch.distributed as dist
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


@dataclass(frozen=True)
class RowShard:
    rank: int
    world: int
    r0: int      # first row owned
    r1: int      # one past the last row owned
    bounds: tuple  # every rank's [r0, r1) start, world + 1 entries

    @property
    def rows(self):
        import numpy as np
        return np.arange(self.r0, self.r1, dtype=np.int32)

    @property
    def q(self) -> int:
        return self.r1 - self.r0


def row_shard_for(rank: int, world: int, row_ptr) -> RowShard:
    """Contiguous row ranges with about equal (nnz + rows) per rank."""
    import numpy as np
    if not (0 <= rank < world):
        raise ValueError(f"bad shard rank={rank} world={world}")
    rp = np.asarray(row_ptr, dtype=np.int64)
    P = len(rp) - 1
    cost = rp + np.arange(P + 1, dtype=np.int64)  # prefix of (deg + 1)
    total = int(cost[-1])
    bounds = [0] + [int(np.searchsorted(cost, total * k // world, side="left")) for k in range(1, world)] + [P]
    for k in range(1, world + 1):  # monotone, so every range is well formed (possibly empty)
        bounds[k] = max(bounds[k], bounds[k - 1])
    return RowShard(rank, world, bounds[rank], bounds[rank + 1], tuple(bounds))


def gather_rows(local, shard: RowShard, S: int, group=None):
    """All-gather the row-sharded ``target`` (rank-local [q*S] tensor) into the
    full [P*S] vector, rows in order.  Ranges may differ in length: each rank
    pads to the longest and the padding is dropped after the exchange."""
    import torch
    import torch.distributed as dist
    b = shard.bounds
    qmax = max(b[k + 1] - b[k] for k in range(shard.world))
    buf = torch.zeros(qmax * S, dtype=local.dtype, device=local.device)
    buf[: local.numel()] = local.reshape(-1)
    parts = [torch.empty_like(buf) for _ in range(shard.world)]
    dist.all_gather(parts, buf, group=group)
    return torch.cat([parts[k][: (b[k + 1] - b[k]) * S] for k in range(shard.world)])


# ---------------------------------------------------------------------------
# Pod-row-sharded multi-round loop (SURVEY.md §8e pod-row sharding x §8f item 1)
# ---------------------------------------------------------------------------
# The reference's loop, per scenario (main.py:56-101): monitor -> detection ->
# pod_delete (pick_max_pod) -> edit_cluster -> communication (CAR) -> the next
# round re-monitors the live cluster.  Rank r owns pod rows [r0, r1) (balanced
# by nnz, ``row_shard_for``) and keeps the full assign[P*S] replica; per round:
#
#   monitor   per-node CPU / mem of the pods in its rows (rsk_node_reduce on
#             its row slice once, then moved with its pods in the update
#             phase) -> int64 all-reduce SUM of the N*S partials;
#             use = base + CPU sums, base = the usage no pod accounts for
#             (use0 minus the round-0 sums, fixed)
#   detect    cpu_pct -> hazard / most hazardous node, replicated (N*S, tiny)
#   evict     its rows' first max-CPU pod on most[s] (rsk_pick_max_pod on the
#             slice), packed (cpu, -pod) -> int64 all-reduce MAX over S
#   place     the CAR target of the evicted pod, by the rank owning its row
#             (rsk_rounds_place), then an all-gather of every rank's changed
#             slice (target per scenario, RSK_TARGET_NO_EVICT where not its
#             pod) -> the element-wise max is the round's move
#   update    assign[p_s, s] = t_s on every replica (the pod moves when
#             t_s >= 0); the owning rank moves the pod's CPU / mem from its
#             old node's partial to the new one (exact integer deltas)
#   cut cost  directed cut over its rows (rsk_cut_cost_rows) -> int64
#             all-reduce SUM over S (communicationcost.py:37-45, /2 there)
#
# Integer sums make the recomputed usage equal the single-process loop's
# incremental update exactly, so the result is bit-equal to rsk_rounds_run /
# oracle_rounds (tests/test_dist_rounds.py).  The per-rank compute goes through
# a backend object: ``LibrskRoundsBackend`` (librsk on the rank's GPU, device
# pointers) is the product path; tests supply a CPU backend for gloo runs on
# machines without a GPU.

NO_EVICT = -3


def _coll_tensor(t):
    """(tensor to hand to the collective, copy-back needed): gloo takes host tensors."""
    import torch.distributed as dist
    if t.is_cuda and dist.get_backend() == "gloo":
        return t.cpu(), True
    return t, False


def _multi_rank() -> bool:
    import torch.distributed as dist
    return dist.is_initialized() and dist.get_world_size() > 1


def allreduce_(t, op="sum", group=None):
    """In-place all-reduce of t (SUM or MAX) on whatever device the backend
    needs; a no-op without a process group (one rank)."""
    import torch.distributed as dist
    if not dist.is_initialized():
        return t
    red = dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX
    x, back = _coll_tensor(t)
    dist.all_reduce(x, op=red, group=group)
    if back:
        t.copy_(x)
    return t


def allgather(t, group=None):
    """[world, *t.shape] stack of every rank's t ([1, ...] without a process group)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return t.unsqueeze(0)
    x, back = _coll_tensor(t.contiguous())
    parts = [torch.empty_like(x) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, x, group=group)
    out = torch.stack(parts)
    return out.to(t.device) if back else out


class LibrskRoundsBackend:
    """Per-rank compute of the row-sharded loop on librsk (device pointers on the
    rank's GPU; every call is asynchronous on the context's stream, which is the
    current torch stream's device)."""

    def __init__(self, row_ptr, col_idx, pod_cpu, ctx=None, device=None, stream_ordered=False, fused=True):
        import numpy as np
        import torch
        from . import api
        from ._lib import RSK_F_DEVICE, Context, check, default_context
        self.dev = torch.device(device or "cuda")
        # stream_ordered: a context of its own whose stream IS the current torch
        # stream, so librsk kernels, torch ops and collectives order on one
        # stream and the host never waits between phases
        self.stream_ordered = stream_ordered
        if stream_ordered:
            cur = torch.cuda.current_stream(self.dev).cuda_stream
            if not cur:  # the legacy default stream (handle 0) would read as "the context's own"
                raise ValueError("stream_ordered needs a non-default current torch stream (torch.cuda.stream(...))")
            self.ctx = Context(self.dev.index if self.dev.index is not None else torch.cuda.current_device())
            self.ctx.set_stream(cur)
        else:
            self.ctx = ctx or default_context()
        self.rounds = api.Rounds(row_ptr, col_idx, pod_cpu, ctx=self.ctx)   # deduplicated CSR for the CAR step
        rp = np.ascontiguousarray(row_ptr, np.int32)
        ci = np.ascontiguousarray(col_idx if len(col_idx) else [0], np.int32)
        self.row_ptr = torch.from_numpy(rp).to(self.dev)
        self.col_idx = torch.from_numpy(ci).to(self.dev)
        self.P = rp.shape[0] - 1
        # the CSR's transpose (rows holding each pod), for the cut's per-move delta
        nnz = int(rp[-1])
        src = np.repeat(np.arange(self.P, dtype=np.int32), np.diff(rp))
        order = np.argsort(ci[:nnz], kind="stable")
        rvp = np.zeros(self.P + 1, np.int32)
        np.cumsum(np.bincount(ci[:nnz], minlength=self.P), out=rvp[1:])
        self.rev_ptr = torch.from_numpy(rvp).to(self.dev)
        self.rev_idx = torch.from_numpy(np.ascontiguousarray(src[order] if nnz else np.zeros(1, np.int32))).to(self.dev)
        self._F, self._check = RSK_F_DEVICE, check
        # fused: the round as rsk_rows_detect_setup once, then rsk_rows_pick / _place / _move (four
        # launches around the collectives); else the per-phase calls below
        self.fused = fused

    def _sync(self):
        import torch
        if not self.stream_ordered:
            torch.cuda.synchronize(self.dev)   # torch-stream inputs ready / librsk-stream outputs done

    def node_partials(self, assign_rows, pod_cpu_rows, pod_mem_rows, q, N, S):
        import torch
        self._sync()
        cnt = torch.empty(N * S, dtype=torch.int32, device=self.dev)
        cpu = torch.empty(N * S, dtype=torch.int64, device=self.dev)
        mem = torch.empty(N * S, dtype=torch.int64, device=self.dev)
        self._check(self.ctx.lib.rsk_node_reduce(self.ctx.handle, assign_rows.data_ptr(), q, S,
                                                 pod_cpu_rows.data_ptr(), pod_mem_rows.data_ptr(), N, cnt.data_ptr(),
                                                 cpu.data_ptr(), mem.data_ptr(), self._F))
        self._sync()
        return cpu, mem

    def detect(self, use, cap, N, S, threshold):
        import torch
        self._sync()
        pct = torch.empty(N * S, dtype=torch.int32, device=self.dev)
        haz = torch.empty(N * S, dtype=torch.uint8, device=self.dev)
        most = torch.empty(S, dtype=torch.int32, device=self.dev)
        L, h = self.ctx.lib, self.ctx.handle
        self._check(L.rsk_cpu_pct(h, use.data_ptr(), cap.data_ptr(), N, S, pct.data_ptr(), self._F))
        self._check(L.rsk_detect(h, pct.data_ptr(), N, S, threshold, haz.data_ptr(), most.data_ptr(), self._F))
        self._sync()
        return haz, most

    def pick_rows(self, assign_rows, pod_cpu_rows, q, S, most):
        import torch
        self._sync()
        out = torch.empty(S, dtype=torch.int32, device=self.dev)
        self._check(self.ctx.lib.rsk_pick_max_pod(self.ctx.handle, assign_rows.data_ptr(), pod_cpu_rows.data_ptr(), q,
                                                  S, most.data_ptr(), out.data_ptr(), self._F))
        self._sync()
        return out

    def place(self, assign, S, cap, use, haz, N, evict):
        import torch
        self._sync()
        out = torch.empty(S, dtype=torch.int32, device=self.dev)
        self.rounds.place(assign, S, cap, use, haz, N, evict, out, device=True)
        self._sync()
        return out

    def pick_rows16(self, shadow_rows, pod_cpu_rows, q, S, most):
        """pick_rows over the rank's u16 shadow (N <= 65535, S % 8 == 0)."""
        import torch
        self._sync()
        out = torch.empty(S, dtype=torch.int32, device=self.dev)
        self._check(self.ctx.lib.rsk_pick_max_pod16(self.ctx.handle, shadow_rows.data_ptr(), pod_cpu_rows.data_ptr(),
                                                    q, S, most.data_ptr(), out.data_ptr(), self._F))
        self._sync()
        return out

    def cut_delta(self, assign, S, evict, target, r0, r1, N, cut):
        """cut[s] += the change of the rank's directed cut that the round's moves make
        (called before apply: assign still holds the old nodes)."""
        self._sync()
        self._check(self.ctx.lib.rsk_rows_cut_delta(self.ctx.handle, self.row_ptr.data_ptr(), self.col_idx.data_ptr(),
                                                    self.rev_ptr.data_ptr(), self.rev_idx.data_ptr(), self.P, r0, r1,
                                                    assign.data_ptr(), S, evict.data_ptr(), target.data_ptr(), N,
                                                    cut.data_ptr(), self._F))
        self._sync()

    # the per-round glue of RowShardedRounds.run in one librsk launch each
    def evict_key(self, loc, r0, pod_cpu, S):
        import torch
        self._sync()
        key = torch.empty(S, dtype=torch.int64, device=self.dev)
        self._check(self.ctx.lib.rsk_rows_evict_key(self.ctx.handle, loc.data_ptr(), S, r0, pod_cpu.data_ptr(),
                                                    key.data_ptr(), self._F))
        self._sync()
        return key

    def evict_decode(self, key, S):
        import torch
        self._sync()
        ev = torch.empty(S, dtype=torch.int32, device=self.dev)
        self._check(self.ctx.lib.rsk_rows_evict_decode(self.ctx.handle, key.data_ptr(), S, self.P, ev.data_ptr(),
                                                       self._F))
        self._sync()
        return ev

    def apply(self, assign, S, evict, target, r0, r1, N, pod_cpu, pod_mem, cpu_part, mem_part, shadow=None):
        self._sync()
        self._check(self.ctx.lib.rsk_rows_apply(self.ctx.handle, assign.data_ptr(), S, evict.data_ptr(),
                                                target.data_ptr(), r0, r1, self.P, N, pod_cpu.data_ptr(),
                                                pod_mem.data_ptr(), cpu_part.data_ptr(), mem_part.data_ptr(),
                                                None if shadow is None else shadow.data_ptr(), self._F))
        self._sync()

    def cut_rows(self, assign, S, r0, r1):
        import torch
        self._sync()
        out = torch.empty(S, dtype=torch.int64, device=self.dev)
        self._check(self.ctx.lib.rsk_cut_cost_rows(self.ctx.handle, self.row_ptr.data_ptr(), self.col_idx.data_ptr(),
                                                   self.P, r0, r1, assign.data_ptr(), S, None, out.data_ptr(),
                                                   self._F))
        self._sync()
        return out

    # ---- the fused round (RowShardedRounds.run when self.fused) ----
    def round_buffers(self, N, S):
        """Per-run device buffers of the fused round.  The eviction key starts at
        zero and rows_place leaves it zero for the next round; the detect state
        (usage replica, hazard flags, block maxima, most-hazardous key, zero
        case) is set up once and kept in step by rows_move."""
        import torch
        z = lambda n, dt: torch.zeros(n, dtype=dt, device=self.dev)  # noqa: E731
        nb = int(self.ctx.lib.rsk_rows_blk_bytes(N, S))
        return {"use": z(N * S, torch.int32), "haz": z(N * S, torch.uint8), "most": z(S, torch.int64),
                "key": z(S, torch.int64), "zc_cnt": z(S, torch.int32), "zc_key": z(S, torch.int64),
                "blk": z(max(nb, 8), torch.uint8)}

    def rows_detect_setup(self, use, cap, N, S, threshold, b):
        """b["use"] = use (the replica), and the detect state from it."""
        self._sync()
        b["use"].copy_(use)
        self._check(self.ctx.lib.rsk_rows_detect_setup(self.ctx.handle, b["use"].data_ptr(), cap.data_ptr(), N, S,
                                                       threshold, b["haz"].data_ptr(), b["blk"].data_ptr(),
                                                       b["most"].data_ptr(), b["zc_cnt"].data_ptr(),
                                                       b["zc_key"].data_ptr(), self._F))
        self._sync()

    def rows_pick(self, rows, q, S, r0, pod_cpu, b):
        self._sync()
        self._check(self.ctx.lib.rsk_rows_pick(self.ctx.handle, rows.data_ptr() if q else None, rows.element_size(),
                                               q, S, r0, pod_cpu.data_ptr(), b["most"].data_ptr(),
                                               b["key"].data_ptr(), self._F))
        self._sync()

    def rows_place(self, assign, S, cap, N, r0, r1, b):
        import torch
        self._sync()
        ev = torch.empty(S, dtype=torch.int32, device=self.dev)
        tg = torch.empty(S, dtype=torch.int32, device=self.dev)
        self._check(self.ctx.lib.rsk_rows_place(self.rounds.handle, assign.data_ptr(), S, cap.data_ptr(),
                                                b["use"].data_ptr(), b["haz"].data_ptr(), N, r0, r1,
                                                b["most"].data_ptr(), b["key"].data_ptr(), b["zc_cnt"].data_ptr(),
                                                b["zc_key"].data_ptr(), ev.data_ptr(), tg.data_ptr(), self._F))
        self._sync()
        return ev, tg

    def rows_move(self, assign, S, evict, target, r0, r1, N, pod_cpu, pod_mem, cpu_part, mem_part, shadow, cut,
                  cap, threshold, b):
        self._sync()
        self._check(self.ctx.lib.rsk_rows_move(self.ctx.handle, self.row_ptr.data_ptr(), self.col_idx.data_ptr(),
                                               self.rev_ptr.data_ptr(), self.rev_idx.data_ptr(), self.P, r0, r1,
                                               assign.data_ptr(), S, evict.data_ptr(), target.data_ptr(), N,
                                               pod_cpu.data_ptr(), pod_mem.data_ptr(), cpu_part.data_ptr(),
                                               mem_part.data_ptr(), None if shadow is None else shadow.data_ptr(),
                                               cut.data_ptr(), b["use"].data_ptr(), cap.data_ptr(), threshold,
                                               b["haz"].data_ptr(), b["blk"].data_ptr(), b["most"].data_ptr(),
                                               b["zc_cnt"].data_ptr(), b["zc_key"].data_ptr(), self._F))
        self._sync()

    def close(self):
        self.rounds.close()
        if self.stream_ordered:
            self.ctx.close()


class RowShardedRounds:
    """R rounds of the loop above for S scenarios over this rank's pod rows.

    ``run(assign, use0, cap, pod_cpu, pod_mem, N, R)`` takes full-size tensors on
    the backend's device (the assign replica is updated in place) and returns a
    dict: evict / target / cut as [R, S] tensors (cut = directed count after the
    round's move), the final use [N*S] int32, and per-phase wall times (ms,
    summed over rounds; "place" is the scoring-only leg)."""

    def __init__(self, shard: RowShard, backend, group=None):
        self.shard, self.be, self.group = shard, backend, group

    def _local_partials(self, assign, pod_cpu, pod_mem, N, S):
        r0, r1 = self.shard.r0, self.shard.r1
        return self.be.node_partials(assign[r0 * S:r1 * S], pod_cpu[r0:r1], pod_mem[r0:r1], r1 - r0, N, S)

    def _partials(self, assign, pod_cpu, pod_mem, N, S):
        cpu, mem = self._local_partials(assign, pod_cpu, pod_mem, N, S)
        allreduce_(cpu, "sum", self.group)
        allreduce_(mem, "sum", self.group)
        return cpu, mem

    def run(self, assign, use0, cap, pod_cpu, pod_mem, N, S, R, threshold=30):
        import time
        import torch
        dev = assign.device
        r0, r1 = self.shard.r0, self.shard.r1
        t = {"setup": 0.0, "monitor": 0.0, "detect": 0.0, "evict": 0.0, "place": 0.0, "exchange": 0.0, "update": 0.0,
             "cut": 0.0}
        c = time.perf_counter()

        def tick(name, t0):
            t[name] += (time.perf_counter() - t0) * 1e3
            return time.perf_counter()

        # the rank's per-node partials over its rows, reduced once here and then
        # kept in step with the moves of its pods (exact integer deltas: the
        # same sums a full re-reduction of the rows gives, without the pass
        # over all P x S assignments per round)
        lp_cpu, lp_mem = self._local_partials(assign, pod_cpu, pod_mem, N, S)
        cpu0 = lp_cpu.clone()
        allreduce_(cpu0, "sum", self.group)
        base = use0.to(torch.int64) - cpu0            # usage no pod accounts for
        pm64 = pod_mem.to(torch.int64)
        glue = hasattr(self.be, "apply")   # the backend's fused per-round glue (librsk), else torch ops
        pc32, pm64c = pod_cpu.to(torch.int32).contiguous(), pm64.contiguous()
        # the cut kept as a running count: the full count over the rank's rows
        # once, then per round the exact delta of the round's moves (only edges
        # at the moved pod change, communicationcost.py:40-43)
        delta = hasattr(self.be, "cut_delta")
        cut_local = self.be.cut_rows(assign, S, r0, r1) if delta else None
        # the eviction scan over a u16 shadow of the rank's rows when node ids fit
        shadow = None
        if hasattr(self.be, "pick_rows16") and N <= 65535 and S % 8 == 0 and r1 > r0:
            rows = assign[r0 * S:r1 * S]
            shadow = torch.where((rows >= 0) & (rows < N), rows, torch.full_like(rows, 65535)).to(torch.int16)
        evs, tgs, cuts = [], [], []
        tick("setup", c)
        sidx = torch.arange(S, device=dev)
        pc64 = pod_cpu.to(torch.int64)
        mask32 = (1 << 32) - 1
        trace = os.environ.get("RSK_DIST_TRACE")
        if getattr(self.be, "fused", False) and delta:
            return self._run_fused(assign, base, cap, pc32, pm64c, lp_cpu, lp_mem, cut_local, shadow, N, S, R,
                                   threshold, t)
        for rnd in range(R):
            if trace:
                print(f"[rank {self.shard.rank}] round {rnd}", file=sys.stderr, flush=True)
            c = time.perf_counter()
            if _multi_rank():   # the monitor's exchange: every rank's CPU / mem partials summed
                cpu, mem = lp_cpu.clone(), lp_mem.clone()
                allreduce_(cpu, "sum", self.group)
                allreduce_(mem, "sum", self.group)
            else:               # one rank: its partials are the totals (no copies)
                cpu = lp_cpu
            use = (base + cpu).to(torch.int32)
            c = tick("monitor", c)
            haz, most = self.be.detect(use, cap, N, S, threshold)
            c = tick("detect", c)
            if shadow is not None:
                loc = self.be.pick_rows16(shadow, pc32[r0:r1], r1 - r0, S, most)
            else:
                loc = self.be.pick_rows(assign[r0 * S:r1 * S], pod_cpu[r0:r1], r1 - r0, S, most)
            if glue:
                key = self.be.evict_key(loc, r0, pc32, S)
            else:
                loc = loc.to(torch.int64)
                gp = torch.where(loc >= 0, loc + r0, torch.zeros_like(loc))
                key = torch.where(loc >= 0, (pc64[gp] << 32) | (mask32 - gp), torch.full_like(loc, -1))
            allreduce_(key, "max", self.group)
            if glue:
                evict = self.be.evict_decode(key, S)
            else:
                evict = torch.where(key >= 0, mask32 - (key & mask32), torch.full_like(key, -1)).to(torch.int32)
            c = tick("evict", c)
            mine = (evict >= r0) & (evict < r1)
            tgt_local = self.be.place(assign, S, cap, use, haz, N, torch.where(mine, evict, torch.full_like(evict, -1)))
            c = tick("place", c)
            # the changed slices of every rank (one rank: its own)
            target = allgather(tgt_local, self.group).max(dim=0).values if _multi_rank() else tgt_local
            c = tick("exchange", c)
            if glue:  # one librsk launch
                target = target.contiguous()
                if delta:
                    self.be.cut_delta(assign, S, evict, target, r0, r1, N, cut_local)
                c = tick("cut", c)
                self.be.apply(assign, S, evict, target, r0, r1, N, pc32, pm64c, lp_cpu, lp_mem, shadow)
                c = tick("update", c)
                cut = cut_local.clone() if delta else self.be.cut_rows(assign, S, r0, r1)
                allreduce_(cut, "sum", self.group)
                tick("cut", c)
                evs.append(evict)
                tgs.append(target)
                cuts.append(cut)
                continue
            # fixed-shape ops over all S scenarios (no boolean indexing, which
            # would sync the host): scenarios without a move write their own
            # value back and add zero deltas at index 0
            if delta:
                self.be.cut_delta(assign, S, evict, target, r0, r1, N, cut_local)
            # the move rule of rsk_rows_apply / rsk_rows_cut_delta: evict in [0, P), target in [0, N)
            moved = (evict >= 0) & (evict < assign.numel() // S) & (target >= 0) & (target < N)
            av = assign.view(-1, S)
            ep = evict.clamp(min=0).long()
            old = av[ep, sidx].long()
            et = target.long()
            av[ep, sidx] = torch.where(moved, target, old.to(target.dtype))
            own = moved & (ep >= r0) & (ep < r1)   # this rank's pods: move their usage in its partials
            src = own & (old >= 0) & (old < N)
            dst = own & (et < N)
            zero = torch.zeros_like(old)
            i_src = torch.where(src, old * S + sidx, zero)
            i_dst = torch.where(dst, et * S + sidx, zero)
            lp_cpu.index_add_(0, i_src, torch.where(src, -pc64[ep], zero))
            lp_mem.index_add_(0, i_src, torch.where(src, -pm64[ep], zero))
            lp_cpu.index_add_(0, i_dst, torch.where(dst, pc64[ep], zero))
            lp_mem.index_add_(0, i_dst, torch.where(dst, pm64[ep], zero))
            c = tick("update", c)
            cut = cut_local.clone() if delta else self.be.cut_rows(assign, S, r0, r1)
            allreduce_(cut, "sum", self.group)
            tick("cut", c)
            evs.append(evict)
            tgs.append(target)
            cuts.append(cut)
        return self._finish(base, lp_cpu, evs, tgs, cuts, S, dev, t)

    def _finish(self, base, lp_cpu, evs, tgs, cuts, S, dev, t):
        import torch
        # the final usage from the partials kept exact round by round (no second
        # pass over the rows)
        cpu = lp_cpu.clone()
        allreduce_(cpu, "sum", self.group)
        use_final = (base + cpu).to(torch.int32)
        empty = torch.empty(0, S, dtype=torch.int32, device=dev)
        return {"evict": torch.stack(evs) if evs else empty, "target": torch.stack(tgs) if tgs else empty,
                "cut": torch.stack(cuts) if cuts else empty.to(torch.int64), "use": use_final, "ms": t}

    def _run_fused(self, assign, base, cap, pc32, pm64, lp_cpu, lp_mem, cut_local, shadow, N, S, R, threshold, t):
        """The rounds of ``run`` with the backend's fused launches.  Round 0's
        usage (base + the all-reduced partials) seeds a usage replica on every
        rank with its hazard flags, per-(scenario, 64-node block) maxima, most
        hazardous node and zero case (``rsk_rows_detect_setup``); every round
        then: the eviction scan straight to the packed all-reduce key, CAR of
        this rank's evicted pods (the key decoded in the kernel), the target
        all-gather, and the move, which updates the replica and re-reduces the
        two changed blocks on every rank (the moves are known to all ranks), so
        no round re-reads the N x S usage or all-reduces the partials.  Same
        results as the unfused loop."""
        import time
        import torch
        be, dev = self.be, assign.device
        r0, r1 = self.shard.r0, self.shard.r1
        b = be.round_buffers(N, S)
        rows = shadow if shadow is not None else assign[r0 * S:r1 * S]
        multi = _multi_rank()
        c = time.perf_counter()
        cpu0 = lp_cpu.clone()
        allreduce_(cpu0, "sum", self.group)
        be.rows_detect_setup((base + cpu0).to(torch.int32), cap, N, S, threshold, b)
        t["setup"] += (time.perf_counter() - c) * 1e3
        evs, tgs, cuts = [], [], []
        for _ in range(R):
            c = time.perf_counter()
            be.rows_pick(rows, r1 - r0, S, r0, pc32, b)
            allreduce_(b["key"], "max", self.group)
            t["evict"] += (time.perf_counter() - c) * 1e3
            c = time.perf_counter()
            evict, target = be.rows_place(assign, S, cap, N, r0, r1, b)
            t["place"] += (time.perf_counter() - c) * 1e3
            c = time.perf_counter()
            if multi:
                target = allgather(target, self.group).max(dim=0).values.contiguous()
            t["exchange"] += (time.perf_counter() - c) * 1e3
            c = time.perf_counter()
            be.rows_move(assign, S, evict, target, r0, r1, N, pc32, pm64, lp_cpu, lp_mem, shadow, cut_local, cap,
                         threshold, b)
            t["update"] += (time.perf_counter() - c) * 1e3
            c = time.perf_counter()
            cut = cut_local.clone()
            allreduce_(cut, "sum", self.group)
            t["cut"] += (time.perf_counter() - c) * 1e3
            evs.append(evict)
            tgs.append(target)
            cuts.append(cut)
        return self._finish(base, lp_cpu, evs, tgs, cuts, S, dev, t)
