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
