"""Process-group context: one process per GPU, ``torch.distributed`` over RCCL (xGMI) on MI355X
or gloo on CPU (tests).

Bucket ownership follows the session's owner map for each bucket count
(``parallel/placement.py``: size-balanced LPT, ``b % world`` when bucket sizes are equal, heavy
buckets of an integer key cut into key ranges across ranks).  Every index and query-time shuffle
with that bucket count uses the same map, so two bucketed indexes with equal bucket counts are
co-partitioned and a JoinIndexRule join moves no data between GPUs; only index builds (and
non-index shuffles) exchange rows, with all-to-all.
"""
from __future__ import annotations

import os
from typing import List, Optional


class _PendingCombine:
    """Partials of one query on their way to the host (pinned, stream-ordered copy)."""

    def __init__(self, packed):
        import torch
        self.result = None
        self.error = None      # set on every entry of a flush that failed
        if packed.is_cuda:
            self.host = torch.empty(packed.numel(), dtype=torch.uint8, pin_memory=True)
            self.host.copy_(packed, non_blocking=True)
            self.event = torch.cuda.Event()
            self.event.record()
        else:
            self.host, self.event = packed.clone(), None

    def wait(self) -> None:
        if self.event is not None:
            self.event.synchronize()


def _reduce_ranks(x):
    """(sum, count, min, max) over ranks, in rank order, of ``x``: [world, 4, GA * 8] bytes."""
    s = x[:, 0].copy().view("<f8").sum(axis=0)
    c = x[:, 1].copy().view("<i8").sum(axis=0)
    mn = x[:, 2].copy().view("<f8").min(axis=0)
    mx = x[:, 3].copy().view("<f8").max(axis=0)
    return s, c, mn, mx


class DistContext:
    def __init__(self, rank: int, world: int, backend: str, device=None):
        self.rank = rank
        self.world = world
        self.backend = backend
        self.device = device
        self._pending_combines: list = []

    @staticmethod
    def from_env(init: bool = True, backend: Optional[str] = None) -> Optional["DistContext"]:
        import torch
        import torch.distributed as dist
        world = int(os.environ.get("WORLD_SIZE", "1"))
        if world <= 1 and not dist.is_initialized():
            return None
        rank = int(os.environ.get("RANK", "0"))
        if backend is None:
            backend = os.environ.get("HS_DIST_BACKEND") or (
                "nccl" if torch.cuda.is_available() else "gloo")
        device = None
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            device = torch.device("cuda", local)
        elif torch.cuda.is_available():
            # gloo + GPU: ranks may share one device (multi-rank rehearsal on a 1-GPU box);
            # collectives are staged through host memory.
            local = int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count()
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

    def _staged(self, t) -> bool:
        return self.backend != "nccl" and t is not None and t.is_cuda

    def all_reduce(self, t, op: str = "sum"):
        """In-place all-reduce (RCCL on device; host-staged for gloo + CUDA tensors)."""
        import torch.distributed as dist
        rop = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN,
               "max": dist.ReduceOp.MAX}[op]
        if self._staged(t):
            h = t.cpu()
            dist.all_reduce(h, op=rop)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=rop)
        return t

    def all_gather_tensor(self, t):
        """``[world * n]`` concatenation (rank order) of every rank's 1-D tensor ``t`` (same n
        on every rank): one RCCL all-gather on device, host-staged for gloo + CUDA tensors."""
        import torch
        import torch.distributed as dist
        if self._staged(t):
            h = t.cpu()
            parts = [torch.empty_like(h) for _ in range(self.world)]
            dist.all_gather(parts, h)
            return torch.cat(parts).to(t.device)
        if self.backend == "nccl":
            out = torch.empty(self.world * t.numel(), dtype=t.dtype, device=t.device)
            dist.all_gather_into_tensor(out, t.contiguous())
            return out
        parts = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(parts, t.contiguous())
        return torch.cat(parts)

    def all_to_all_single(self, out, inp, out_splits=None, in_splits=None):
        import torch.distributed as dist
        if self._staged(inp):
            ho = out.new_empty(out.shape, device="cpu")
            dist.all_to_all_single(ho, inp.cpu(), output_split_sizes=out_splits,
                                   input_split_sizes=in_splits)
            out.copy_(ho)
        else:
            dist.all_to_all_single(out, inp, output_split_sizes=out_splits,
                                   input_split_sizes=in_splits)
        return out

    def all_reduce_agg(self, sums, cnts, mins, maxs):
        """Combine partial aggregates (sum, count, min, max) across ranks — 4 small RCCL calls."""
        self.all_reduce(sums, "sum")
        self.all_reduce(cnts, "sum")
        self.all_reduce(mins, "min")
        self.all_reduce(maxs, "max")
        return sums, cnts, mins, maxs

    def combine_aggs_host(self, sums, cnts, mins, maxs):
        """``combine_aggs_async(...)()``: the combined partials as numpy arrays."""
        return self.combine_aggs_async(sums, cnts, mins, maxs)()

    def combine_aggs_async(self, sums, cnts, mins, maxs):
        """Cross-rank combine of partial aggregates in ONE collective: the four [GA] partials
        (already one contiguous device block when they come from the kernels' output buffer)
        are all-gathered as raw bytes and copied to pinned host memory, all stream-ordered;
        the returned ``fetch()`` waits for that copy and reduces in rank order on the host —
        deterministic sums, one small RCCL call instead of four all-reduces plus a D2H, and
        nothing blocks the host before the caller asks for the result.
        ``fetch()`` returns numpy (sum f64, count i64, min f64, max f64)."""
        import numpy as np
        import torch
        import torch.distributed as dist
        GA = int(sums.numel() if hasattr(sums, "numel") else sums.size)
        if isinstance(sums, np.ndarray):
            packed = torch.from_numpy(np.concatenate(
                [np.ascontiguousarray(x).view(np.uint8) for x in (sums, cnts, mins, maxs)]))
        else:
            buf = getattr(sums, "hs_buf", None)
            packed = buf if buf is not None and buf.numel() == 32 * GA else torch.cat(
                [x.contiguous().view(torch.uint8) for x in (sums, cnts, mins, maxs)])
        if self.backend == "nccl":
            packed = packed.to(self.device, non_blocking=True)
            out = torch.empty(self.world * packed.numel(), dtype=torch.uint8, device=self.device)
            dist.all_gather_into_tensor(out, packed)
            h = torch.empty(out.numel(), dtype=torch.uint8, pin_memory=True)
            h.copy_(out, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            # gloo (host-staged): the partials go to pinned memory stream-ordered now, and the
            # collective waits until a result is asked for; every combine pending at that point
            # travels in ONE all-gather (ranks submit and fetch in the same program order, so
            # they coalesce the same entries)
            ent = _PendingCombine(packed)
            self._pending_combines.append(ent)

            def fetch_gloo():
                if ent.result is None and ent.error is None:
                    self._flush_combines()
                if ent.error is not None:
                    raise ent.error
                return _reduce_ranks(ent.result.numpy().reshape(self.world, 4, GA * 8))
            return fetch_gloo

        def fetch():
            if ev is not None:
                ev.synchronize()
            x = h.numpy().reshape(self.world, 4, GA * 8)
            s = x[:, 0].copy().view(np.float64).sum(axis=0)
            c = x[:, 1].copy().view(np.int64).sum(axis=0)
            mn = x[:, 2].copy().view(np.float64).min(axis=0)
            mx = x[:, 3].copy().view(np.float64).max(axis=0)
            return s, c, mn, mx
        return fetch

    def _flush_combines(self) -> None:
        """One all-gather for every pending (gloo) partial-aggregate combine."""
        import torch
        import torch.distributed as dist
        pend, self._pending_combines = self._pending_combines, []
        for e in pend:
            e.wait()
        flat = torch.cat([e.host for e in pend])
        # ranks must coalesce the same entries (a rank that abandoned a query between submit
        # and fetch would shift every later result): agree on (count, total bytes, layout hash)
        # first and fail loudly on a mismatch instead of hanging or misattributing results
        lay = 0
        for e in pend:
            lay = (lay * 1000003 + int(e.host.numel())) & ((1 << 62) - 1)
        hdr = torch.tensor([len(pend), int(flat.numel()), lay], dtype=torch.int64)
        hdrs = [torch.empty_like(hdr) for _ in range(self.world)]
        dist.all_gather(hdrs, hdr)
        if any(not torch.equal(h, hdr) for h in hdrs):
            err = RuntimeError("cross-rank combine mismatch: ranks have different pending "
                               f"aggregates {[h.tolist() for h in hdrs]}")
            for e in pend:      # every coalesced entry reports the mismatch
                e.error = err
            raise err
        parts = [torch.empty_like(flat) for _ in range(self.world)]
        dist.all_gather(parts, flat)
        allr = torch.stack(parts)             # [world, total bytes]
        off = 0
        for e in pend:
            nb = e.host.numel()
            e.result = allr[:, off:off + nb].contiguous()
            off += nb

    def all_gather_rows(self, rows):
        """Concatenation over ranks (in rank order) of each rank's int64 ``[n_r, w]`` numpy
        rows: one all-gather of the counts, one of the rows padded to the largest count (RCCL
        on device tensors; gloo on host tensors) — no pickling."""
        import numpy as np
        import torch
        import torch.distributed as dist
        n, w = rows.shape
        dev = self.device if self.backend == "nccl" else "cpu"
        cnt = torch.tensor([n], dtype=torch.int64, device=dev)
        counts = [torch.zeros_like(cnt) for _ in range(self.world)]
        dist.all_gather(counts, cnt)
        # one device -> host read of all the counts (not one ``.item()`` sync per rank)
        counts = torch.cat(counts).cpu().tolist()
        mx = max(counts)
        if mx == 0:
            return np.zeros((0, w), dtype=np.int64)
        buf = torch.zeros((mx, w), dtype=torch.int64)
        if n:
            buf[:n] = torch.from_numpy(np.ascontiguousarray(rows))
        buf = buf.to(dev)
        outs = [torch.empty_like(buf) for _ in range(self.world)]
        dist.all_gather(outs, buf)
        return torch.cat([o[:c] for o, c in zip(outs, counts)]).cpu().numpy()

    def agree_any(self, flags) -> list:
        """Element-wise OR of a list of booleans over all ranks (one small max all-reduce on a
        tensor — used where every rank must take the same data-dependent decision)."""
        import torch
        dev = self.device if self.backend == "nccl" else "cpu"
        t = torch.tensor([1 if f else 0 for f in flags] or [0], dtype=torch.int64, device=dev)
        self.all_reduce(t, "max")
        return [bool(v) for v in t.cpu().tolist()][:len(flags)]

    def all_reduce_max_float(self, x: float) -> float:
        import torch
        dev = self.device if self.backend == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        self.all_reduce(t, "max")
        return float(t.item())

    def all_reduce_sum_float(self, x: float) -> float:
        import torch
        dev = self.device if self.backend == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        self.all_reduce(t, "sum")
        return float(t.item())


def attach(session, ctx: Optional[DistContext]) -> None:
    session.dist = ctx
