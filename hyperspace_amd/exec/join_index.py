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
import os
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
    if lcol.is_float or rcol.is_float:
        return False
    if (lcol.dictionary is None) != (rcol.dictionary is None) or \
            (lcol.dictionary is not None and lcol.dictionary is not rcol.dictionary):
        return False   # string keys: only codes into one shared (unified) dictionary compare
    if right_table.num_rows >= 2 ** 31 - 1:
        return False
    return right_keys_unique(right_table, rcol)


class JoinIndex:
    """A join index in HBM.  ``width`` 4: ``codes`` is int32 [left rows] (j or -1).  ``width``
    1 / 2: block-coded — ``codes`` uint8 / uint16 per row, ``base`` int32 per block of
    ``2**log_blk`` rows, ``j = base[row >> log_blk] + code`` and the all-ones code = no match.
    Right rows of a block of left rows are a short monotone span for FK joins (lineitem ->
    orders: ~32 orders per 128 lines), so one byte per row usually suffices: the join kernel
    streams 1 byte per left row instead of 4."""

    def __init__(self, codes, width: int, base=None, log_blk: int = 0):
        self.codes, self.width, self.base, self.log_blk = codes, width, base, log_blk

    def nbytes(self) -> int:
        n = self.codes.numel() * self.codes.element_size()
        return n + (self.base.numel() * 4 if self.base is not None else 0)

    def decoded(self, n: int):
        """int32 [n] j-or--1 view (tests / debugging)."""
        import torch
        if self.width == 4:
            return self.codes[:n]
        c = self.codes[:n].to(torch.int64)
        if self.width == 2:
            c = c & 0xFFFF
        sent = (1 << (8 * self.width)) - 1
        b = self.base.to(torch.int64).repeat_interleave(1 << self.log_blk)[:n]
        return torch.where(c == sent, torch.full_like(c, -1), b + c).to(torch.int32)


# block-coded join indexes (HS_JOIN_INDEX_CODED=0 keeps int32 rows)
CODED = os.environ.get("HS_JOIN_INDEX_CODED", "1") == "1"
# (code width, log2 block rows) tried in order; the first that fits every block wins
CODINGS = ((1, 7), (2, 8))


def _block_code(jidx, width: int, log_blk: int) -> Optional[JoinIndex]:
    import torch
    n = jidx.numel()
    B = 1 << log_blk
    nb = (n + B - 1) // B
    j = torch.full((nb * B,), -1, dtype=torch.int64, device=jidx.device)
    j[:n] = jidx
    j = j.view(nb, B)
    big = 1 << 62
    base = torch.where(j >= 0, j, torch.full_like(j, big)).min(dim=1).values
    base = torch.where(base == big, torch.zeros_like(base), base)
    off = j - base[:, None]
    sent = (1 << (8 * width)) - 1
    if not bool(((j < 0) | (off < sent)).all().item()):
        return None
    code = torch.where(j >= 0, off, torch.full_like(off, sent)).to(torch.int32).reshape(-1)
    if width == 1:
        codes = code.to(torch.uint8)
    else:   # low 16 bits of each int32 (little-endian), stored as int16
        codes = code.view(torch.uint8).view(-1, 4)[:, :2].contiguous().view(torch.int16).reshape(-1)
    return JoinIndex(codes, width, base.to(torch.int32), log_blk)


def get_join_index(jp: NL.JoinParams, left_table: DeviceTable, right_table: DeviceTable,
                   lcol: DeviceColumn, rcol: DeviceColumn, rstart, rlen, rbucket) -> JoinIndex:
    """The join index of the pair: first matching right row of every left row (or none).

    ``rstart/rlen/rbucket`` must be the left table's full ranges (every row of every bucket).
    ``jp`` supplies the key column descriptors (slots ``jp.lkey`` / ``jp.rkey``)."""
    cache = left_table.__dict__.setdefault("_join_index", {})
    key = (id(lcol), id(rcol))
    hit = cache.get(key)
    if hit is not None:
        rref, lc, rc, ji = hit
        if rref() is right_table and lc is lcol and rc is rcol:
            return ji
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
    ji = None
    if CODED:
        for width, log_blk in CODINGS:
            ji = _block_code(jidx[:left_table.num_rows], width, log_blk)
            if ji is not None:
                break
    if ji is None:
        ji = JoinIndex(jidx, 4)
    cache[key] = (weakref.ref(right_table), lcol, rcol, ji)
    return ji
