"""Multi-GPU sharding for batched resolution: one process per GPU, weak scaling.

Resolution problems are independent, so ranks never exchange
data: each rank generates/lowers/solves its own shard of catalogs and
torch.distributed is used only for the barrier around the timed region and the
max-over-ranks of its duration.  RCCL ("nccl") on the GPU box, gloo on CPU.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


def shard_seed(base_seed: int, rank: int, per_rank: int) -> int:
    """Seed of a rank's shard: catalogs base+rank*per_rank .. are that rank's
    (the generator derives catalog q of a batch from seed+q, so shards are
    disjoint slices of one global catalog sequence)."""
    return base_seed + rank * per_rank


def strong_range(total: int, rank: int, world: int) -> tuple[int, int]:
    """Strong scaling: rank's contiguous share [lo, hi) of `total` catalogs
    (sizes differ by at most one)."""
    return total * rank // world, total * (rank + 1) // world


@dataclass
class Group:
    rank: int = 0
    world: int = 1
    local: int = 0
    backend: str | None = None

    def barrier(self) -> None:
        if self.world > 1:
            import torch.distributed as dist
            dist.barrier()

    def max(self, x: float) -> float:
        if self.world == 1:
            return x
        import torch
        import torch.distributed as dist
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, x: float) -> list:
        if self.world == 1:
            return [x]
        import torch
        import torch.distributed as dist
        dev = "cuda" if self.backend == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        out = [torch.zeros_like(t) for _ in range(self.world)]
        dist.all_gather(out, t)
        return [float(o.item()) for o in out]

    def close(self) -> None:
        if self.world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()


def init_from_env(backend: str = "nccl") -> Group:
    """RANK / WORLD_SIZE / LOCAL_RANK / MASTER_* as torchrun sets them."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch
        import torch.distributed as dist
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend)
    return Group(rank, world, local, backend if world > 1 else None)


def aggregate_rate(units_per_rank: int, world: int, steps: int, max_elapsed_s: float) -> float:
    """Whole-job throughput: all units all ranks processed / the slowest rank's time."""
    return world * units_per_rank * steps / max_elapsed_s
