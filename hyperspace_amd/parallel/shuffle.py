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


def exchange(columns: List, dest, world: int, group=None) -> Tuple[List, "object"]:
    """Send row i of every column to rank ``dest[i]``.  Returns (received columns, recv counts)."""
    import torch
    import torch.distributed as dist
    perm, send_counts = order_by_dest(dest, world)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
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
        dist.all_to_all_single(dst, src.contiguous(), output_split_sizes=recv,
                               input_split_sizes=send, group=group)
        out.append(dst)
    return out, recv_counts


def bytes_moved(columns: List, dest_counts, rank: int) -> int:
    """Bytes this rank sends to other ranks (diagnostic; excludes its own slice)."""
    per_row = sum(c.element_size() for c in columns if c is not None)
    counts = dest_counts.cpu().tolist()
    return per_row * (sum(counts) - counts[rank])
