"""Process-group context: one process per GPU, ``torch.distributed`` over RCCL (xGMI) on MI355X
or gloo on CPU (tests).

Bucket ownership is static: bucket ``b`` lives on rank ``b % world``.  Two bucketed indexes with
equal bucket counts are therefore co-partitioned and a JoinIndexRule join moves no data between
GPUs; only index builds (and non-index shuffles) exchange rows, with all-to-all.
"""
from __future__ import annotations

import os
from typing import List, Optional


class DistContext:
    def __init__(self, rank: int, world: int, backend: str, device=None):
        self.rank = rank
        self.world = world
        self.backend = backend
        self.device = device

    @staticmethod
    def from_env(init: bool = True, backend: Optional[str] = None) -> Optional["DistContext"]:
        import torch
        import torch.distributed as dist
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world <= 1 and not dist.is_initialized():
            return None
        rank = int(os.environ.get("RANK", "0"))
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        device = None
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            device = torch.device("cuda", local)
        if init and not dist.is_initialized():
            kw = {}
            if backend == "nccl":
                kw["device_id"] = device
            dist.init_process_group(backend=backend, rank=rank, world_size=world, **kw)
        return DistContext(dist.get_rank(), dist.get_world_size(), backend, device)

    # -- collectives ------------------------------------------------------------------------------
    def barrier(self) -> None:
        import torch.distributed as dist
        if self.backend == "nccl":
            dist.barrier(device_ids=[self.device.index])
        else:
            dist.barrier()

    def all_gather_object(self, obj) -> List:
        import torch.distributed as dist
        out = [None] * self.world
        dist.all_gather_object(out, obj)
        return out

    def broadcast_object(self, obj, src: int = 0):
        import torch.distributed as dist
        box = [obj]
        dist.broadcast_object_list(box, src=src)
        return box[0]

    def all_reduce_agg(self, sums, cnts, mins, maxs):
        """Combine partial aggregates (sum, count, min, max) across ranks — 4 small RCCL calls."""
        import torch.distributed as dist
        dist.all_reduce(sums, op=dist.ReduceOp.SUM)
        dist.all_reduce(cnts, op=dist.ReduceOp.SUM)
        dist.all_reduce(mins, op=dist.ReduceOp.MIN)
        dist.all_reduce(maxs, op=dist.ReduceOp.MAX)
        return sums, cnts, mins, maxs

    def all_reduce_max_float(self, x: float) -> float:
        import torch
        import torch.distributed as dist
        dev = self.device if self.backend == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def owns(self, bucket: int) -> bool:
        return bucket % self.world == self.rank


def attach(session, ctx: Optional[DistContext]) -> None:
    session.dist = ctx
