"""Multi-GPU plumbing for the bench and multi-process drivers.

Stripes are independent: every rank owns its own shard on
its own GPU and nothing crosses GPUs on the data path -- no RCCL collective.
torch.distributed (gloo, CPU tensors) is used only for the start barrier and
for reducing the timings (max wall time, summed bytes) to rank 0.
"""
from __future__ import annotations

import os


def shard_range(total: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [begin, end) share of `total` units for `rank` (sizes differ by <= 1)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(total, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


class Dist:
    """RANK / LOCAL_RANK / WORLD_SIZE from the launcher (torchrun); gloo only."""

    def __init__(self, backend: str = "gloo"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", str(self.rank)))
        self.pg = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            if not dist.is_initialized():
                dist.init_process_group(backend, rank=self.rank, world_size=self.world)
            self.pg = dist

    def barrier(self):
        if self.pg:
            self.pg.barrier()

    def _reduce(self, x: float, op) -> float:
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.pg.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.pg.ReduceOp.MAX) if self.pg else x

    def sum(self, x: float) -> float:
        return self._reduce(x, self.pg.ReduceOp.SUM) if self.pg else x

    def gather(self, obj) -> list:
        """Every rank's obj (picklable), in rank order, on every rank."""
        if not self.pg:
            return [obj]
        out = [None] * self.world
        self.pg.all_gather_object(out, obj)
        return out

    def close(self):
        if self.pg and self.pg.is_initialized():
            self.pg.destroy_process_group()
