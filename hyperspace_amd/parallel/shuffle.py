"""Row exchange API used by tests and callers that route rows by an explicit destination rank.

``exchange(columns, dest, world, ctx)`` sends row ``i`` of every column to rank ``dest[i]``
through the packed all-to-all of ``parallel/exchange.py`` (one payload collective for all
columns).  ``None`` entries pass through as ``None``.  Rows arrive grouped by source rank, each
source's rows in their original order.
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np


def exchange(columns: List, dest, world: int, ctx=None) -> Tuple[List, "object"]:
    """Returns (received columns, per-source receive counts)."""
    import torch
    from .exchange import RowExchange
    live = [c for c in columns if c is not None]
    ex = RowExchange(ctx, [c.dtype for c in live], dest.device)
    if ctx is not None and ex.world != world:
        raise ValueError(f"exchange: world {world} != process group size {ex.world}")
    ex.add(live, dest.to(torch.int32))
    # a device batch is deferred until its counts copy lands (RowExchange._add_device):
    # received_rows() issues it, so its receive counts exist before finish() consumes the batch
    ex.received_rows()
    counts = torch.from_numpy(np.asarray(ex.batches[0].counts, dtype=np.int64).copy())
    got = iter(ex.finish())
    return [None if c is None else next(got) for c in columns], counts


def bytes_moved(columns: List, dest_counts, rank: int) -> int:
    """Bytes this rank sends to other ranks (diagnostic; excludes its own slice)."""
    per_row = sum(c.element_size() for c in columns if c is not None)
    counts = dest_counts.cpu().tolist()
    return per_row * (sum(counts) - counts[rank])
