"""Row exchange for index builds: the Spark hash-partition shuffle (K3) as an all-to-all.

Rows are ordered by destination rank (stable, so per-source order is kept), a counts all-to-all
tells every rank how much it receives, then each column moves with one ``all_to_all_single`` with
uneven splits.  Over RCCL on an MI355X node every rank pair has its own xGMI link, so the exchange
drives all 7 links at once instead of being ring/per-link bound.
"""
from __future__ import annotations

from typing import List, Optional, Tuple


def order_by_dest(dest, world: int):
    """Stable permutation grouping rows by destination + per-destination counts."""
    import torch
    if dest.is_cuda:
        from ..exec.device_table import DeviceColumn
        from ..ops import kernels as K
        import pyarrow as pa
        perm = K.sort_permutation([DeviceColumn(dest, None, pa.int32())])
    else:
        perm = torch.argsort(dest, stable=True).to(torch.int32)
    counts = torch.bincount(dest.long(), minlength=world).to(torch.int64)
    return perm, counts


def exchange(columns: List, dest, world: int, ctx=None) -> Tuple[List, "object"]:
    """Send row i of every column to rank ``dest[i]``.  Returns (received columns, recv counts).

    ``ctx`` is the session's DistContext (RCCL, or host-staged gloo for CPU rehearsals)."""
    import torch
    import torch.distributed as dist
    a2a = ctx.all_to_all_single if ctx is not None else (
        lambda o, i, os_=None, is_=None: dist.all_to_all_single(o, i, output_split_sizes=os_,
                                                                  input_split_sizes=is_))
    perm, send_counts = order_by_dest(dest, world)
    recv_counts = torch.empty_like(send_counts)
    a2a(recv_counts, send_counts)
    send = send_counts.cpu().tolist()
    recv = recv_counts.cpu().tolist()
    total = int(sum(recv))
    out = []
    for c in columns:
        if c is None:
            out.append(None)
            continue
        if c.is_cuda:
            from ..exec.device_table import DeviceColumn
            from ..ops import kernels as K
            import pyarrow as pa
            src = K.gather_columns([DeviceColumn(c, None, pa.int64())], perm, want_valid=False)[0].data
        else:
            src = c.index_select(0, perm.long())
        dst = torch.empty((total,) + tuple(c.shape[1:]), dtype=c.dtype, device=c.device)
        a2a(dst, src.contiguous(), recv, send)
        out.append(dst)
    return out, recv_counts


def bytes_moved(columns: List, dest_counts, rank: int) -> int:
    """Bytes this rank sends to other ranks (diagnostic; excludes its own slice)."""
    per_row = sum(c.element_size() for c in columns if c is not None)
    counts = dest_counts.cpu().tolist()
    return per_row * (sum(counts) - counts[rank])
