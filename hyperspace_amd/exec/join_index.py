"""Cached join index for co-located joins of device-resident index tables.

The JoinIndexRule join of two covering indexes (``JoinIndexRule.scala:63-69``)
runs on two bucketed tables that are sorted by the join key inside every bucket and immutable for
the life of their HBM residency (``exec/device_cache.py``).  The row-level result of matching
their keys therefore never changes between queries — only the predicates and aggregates do.

So the first join of a (left table, right table, key pair) computes a *join index*: for every
left row, the first right row with an equal key (``-1`` for none), as int32 in HBM (4 bytes per
left row: 2.4 GB for SF100 lineitem out of 288 GB).  It is built with the same span + LDS search
the merge-join kernels use (``hs_join_index_kernel`` in ``csrc/kernels/join.hip``).  Every later
join of the pair is a streaming scan of the left table that gathers the right columns at the
indexed rows (``jit.gen_join_index_agg``): no per-tile span records, no LDS staging, no binary
search, and the left key column is not even read.  This is the classic join index of relational
engines (a materialised row-id mapping), kept resident instead of recomputed per query.

Eligibility: integer join keys and a right side whose non-null keys are unique (checked once per
right table; FK joins such as lineitem -> orders), fewer than 2**31 right rows.  Anything else
keeps the merge-join kernels.  The index lives on the left table object, so it is freed with the
table when the device cache evicts it; the right table is held weakly, so its eviction
invalidates the entry.
"""
from __future__ import annotations

import ctypes as C
import weakref
from typing import Optional

from ..ops import _lib as NL
from ..ops import kernels as K
from .device_table import DeviceColumn, DeviceTable


def right_keys_unique(table: DeviceTable, col: DeviceColumn) -> bool:
    """True when the non-null values of the sorted-per-bucket key column are unique.  Equal
    keys hash to the same bucket, so duplicates are adjacent: one pass over the column."""
    cache = table.__dict__.setdefault("_unique_keys", {})
    hit = cache.get(id(col))
    if hit is not None and hit[0] is col:
        return hit[1]
    import torch
    d = col.data
    if d.numel() < 2:
        ok = True
    else:
        eq = d[1:] == d[:-1]
        if col.valid is not None:
            v = col.valid.bool()
            eq &= v[1:] & v[:-1]
        ok = not bool(torch.any(eq).item())
    cache[id(col)] = (col, ok)
    return ok


def eligible(left_table: DeviceTable, right_table: DeviceTable, lcol: DeviceColumn,
             rcol: DeviceColumn) -> bool:
    if lcol.is_float or rcol.is_float or lcol.dictionary is not None or \
            rcol.dictionary is not None:
        return False
    if right_table.num_rows >= 2 ** 31 - 1:
        return False
    return right_keys_unique(right_table, rcol)


def get_join_index(jp: NL.JoinParams, left_table: DeviceTable, right_table: DeviceTable,
                   lcol: DeviceColumn, rcol: DeviceColumn, rstart, rlen, rbucket) -> Optional[object]:
    """int32 [left rows] device tensor: first matching right row of every left row, or -1.

    ``rstart/rlen/rbucket`` must be the left table's full ranges (every row of every bucket).
    ``jp`` supplies the key column descriptors (slots ``jp.lkey`` / ``jp.rkey``)."""
    cache = left_table.__dict__.setdefault("_join_index", {})
    key = (id(lcol), id(rcol))
    hit = cache.get(key)
    if hit is not None:
        rref, lc, rc, jidx = hit
        if rref() is right_table and lc is lcol and rc is rcol:
            return jidx
    import torch
    from . import jit
    dev = rstart.device
    tile = NL.lib().hs_join_tile_rows()
    max_tiles = K.join_max_tiles(left_table.num_rows, rlen.numel())
    tp, spans = jit._join_spans(jp, rstart, rlen, rbucket, right_table.bucket_offsets, max_tiles,
                                tile, cache=False)
    jidx = torch.full((max(left_table.num_rows, 1),), -1, dtype=torch.int32, device=dev)
    grid = NL.lib().hs_scan_grid()
    NL.check(NL.lib().hs_join_index(C.byref(jp), rlen.numel(), NL.ptr(tp), NL.ptr(spans), grid,
                                    NL.ptr(jidx), NL.stream_ptr()), "hs_join_index")
    cache[key] = (weakref.ref(right_table), lcol, rcol, jidx)
    return jidx
