"""Multi-GPU layout of the placement path: scenario sharding.

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
