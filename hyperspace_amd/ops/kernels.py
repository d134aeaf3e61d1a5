"""Python entry points for the HIP kernels.  All buffers are torch tensors on the current device;
every launch goes on the current torch stream (so it composes with torch ops, RCCL collectives and
hipGraph capture).  Kernels never allocate; workspaces are torch allocations made here.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import List, Optional, Sequence

import numpy as np

from . import _lib as NL


def _torch():
    import torch
    return torch


# ------------------------------------------------------------------------------------------------
# K3: Spark Murmur3 bucketing
# ------------------------------------------------------------------------------------------------
def hash_xform(atype) -> int:
    """``HashCol.xform`` that makes a device column hash as Spark's logical value
    (``utils/murmur3.py``): decimals (float64 storage) hash their unscaled long, timestamps hash
    microseconds.  Raises for decimals too wide to round-trip exactly through float64."""
    import pyarrow as pa
    if pa.types.is_decimal(atype):
        if atype.precision > 15:
            raise ValueError(f"device hash of {atype}: precision > 15 is not exact in float64 "
                             "storage")
        return NL.XF_DECIMAL | int(atype.scale)
    if pa.types.is_timestamp(atype):
        k = {"s": 6, "ms": 3, "us": 0, "ns": -3}[atype.unit]
        if k > 0:
            return NL.XF_MUL | k
        if k < 0:
            return NL.XF_FDIV | -k
    return NL.XF_NONE


_DICT_BYTES: dict = {}


def dictionary_bytes(dictionary, device):
    """(int64 offsets [n+1], uint8 chars) of a string dictionary on the device, uploaded once
    per dictionary object (the entry keeps a reference, so its id is not reused)."""
    import numpy as np
    import pyarrow as pa
    torch = _torch()
    key = (id(dictionary), str(device))
    hit = _DICT_BYTES.get(key)
    if hit is not None and hit[0] is dictionary:
        return hit[1], hit[2]
    d = dictionary.cast(pa.large_binary()) if not pa.types.is_large_binary(dictionary.type) \
        else dictionary
    bufs = d.buffers()
    n = len(d)
    offs = np.frombuffer(bufs[1], dtype=np.int64, count=n + 1, offset=d.offset * 8) \
        if n else np.zeros(1, np.int64)
    base = int(offs[0])
    chars = np.frombuffer(bufs[2], dtype=np.uint8)[base:int(offs[-1])] \
        if n and bufs[2] is not None else np.zeros(1, np.uint8)
    o = torch.from_numpy((offs - base).copy()).to(device)
    ch = torch.from_numpy(np.ascontiguousarray(chars) if len(chars) else np.zeros(1, np.uint8)) \
        .to(device)
    if len(_DICT_BYTES) > 256:
        _DICT_BYTES.clear()
    _DICT_BYTES[key] = (dictionary, o, ch)
    return o, ch


def _hash_params(cols, num_buckets: int, seed: int = 42) -> NL.HashParams:
    if len(cols) > NL.HASH_MAX_COLS:
        raise ValueError("too many bucket columns")
    p = NL.HashParams()
    for i, c in enumerate(cols):
        vp = c.valid.data_ptr() if c.valid is not None else 0
        if c.offsets is not None:
            p.cols[i] = NL.HashCol(c.chars.data_ptr(), vp, c.offsets.data_ptr(), 0, NL.STR, 0)
        elif c.dictionary is not None:
            # dictionary codes: each row hashes its dictionary entry's bytes on the device
            doff, dchars = dictionary_bytes(c.dictionary, c.data.device)
            p.cols[i] = NL.HashCol(c.data.data_ptr(), vp, doff.data_ptr(), dchars.data_ptr(),
                                   NL.STRDICT, 0)
        else:
            p.cols[i] = NL.HashCol(c.data.data_ptr(), vp, 0, 0, c.hs_type, hash_xform(c.atype))
    p.ncols = len(cols)
    p.num_buckets = int(num_buckets)
    p.seed = seed
    return p


def murmur3_bucket(cols, num_buckets: int, with_counts: bool = True):
    """Returns (bucket int32 [n], counts int64 [num_buckets] or None)."""
    torch = _torch()
    n = len(cols[0])
    dev = cols[0].data.device
    out = torch.empty(n, dtype=torch.int32, device=dev)
    counts = torch.zeros(num_buckets, dtype=torch.int64, device=dev) if with_counts else None
    p = _hash_params(cols, num_buckets)
    NL.check(NL.lib().hs_murmur3_bucket(C.byref(p), n, NL.ptr(out), NL.ptr(counts), NL.stream_ptr()),
             "hs_murmur3_bucket")
    return out, counts


def murmur3_hash(cols):
    torch = _torch()
    n = len(cols[0])
    out = torch.empty(n, dtype=torch.int32, device=cols[0].data.device)
    p = _hash_params(cols, 1)
    NL.check(NL.lib().hs_murmur3_hash(C.byref(p), n, NL.ptr(out), NL.stream_ptr()), "hs_murmur3_hash")
    return out


# ------------------------------------------------------------------------------------------------
# K4: radix sort -> permutation
# ------------------------------------------------------------------------------------------------
def compact_probe(col, maxk: int):
    """Result block of ``hs_compact_probe`` (csrc/kernels/compact.hip) for a device column, as
    a host int64 array: one two-stage reduction launch pair and one small readback."""
    torch = _torch()
    L = NL.lib()
    dev = col.data.device
    res = torch.empty(int(L.hs_compact_result_size()), dtype=torch.int64, device=dev)
    ws = torch.empty(int(L.hs_compact_probe_ws_elems()), dtype=torch.int64, device=dev)
    d = col.data.contiguous()
    v = col.valid.contiguous() if col.valid is not None else None
    NL.check(L.hs_compact_probe(d.data_ptr(), v.data_ptr() if v is not None else None, d.numel(),
                                col.hs_type, maxk, res.data_ptr(), ws.data_ptr(),
                                NL.stream_ptr()), "hs_compact_probe")
    return res.cpu().numpy()


def _int_range(col):
    """(any valid, min, max) of an integer column over valid rows (``compact_probe``)."""
    r = compact_probe(col, 0)
    return bool(r[0]), int(r[3]), int(r[4])


def _sortable_range(col) -> tuple:
    """(kmin, bits) of the order-preserving image over valid rows (host sync: one small D2H)."""
    torch = _torch()
    d = col.data
    t = col.hs_type
    if d.numel() == 0:
        return 0, 0
    if t in (NL.F32, NL.F64):
        # full-width images; only "no valid row" needs a look at the data
        if col.valid is not None and not bool(col.valid.any()):
            return 0, 0
        return 0, 32 if t == NL.F32 else 64
    if d.is_cuda and t in (NL.I8, NL.I16, NL.I32, NL.I64, NL.BOOL, NL.U32):
        anyv, lo, hi = _int_range(col)
        if not anyv:
            return 0, 0
    else:
        if col.valid is not None:
            vm = col.valid.bool()
            if not bool(vm.any()):
                return 0, 0
            d = d[vm]
        lo, hi = torch.aminmax(d)
        lo, hi = lo.item(), hi.item()
    width = {NL.I8: 8, NL.I16: 16, NL.I32: 32, NL.I64: 64, NL.BOOL: 8, NL.U32: 32, NL.U64: 64}[t]
    if t in (NL.BOOL, NL.U32, NL.U64):
        kmin = int(lo)
    else:
        kmin = (int(lo) + (1 << (width - 1))) & ((1 << width) - 1)
    span = int(hi) - int(lo)
    bits = max(1, span.bit_length()) if span > 0 else 0
    return kmin, bits


def sort_permutation(key_cols: Sequence, init_perm=None, extra_leading=None):
    """Stable ascending (NULLS FIRST) permutation over ``key_cols`` (most significant first).

    ``extra_leading`` is an optional (int32 tensor, bits) most-significant key (e.g. bucket ids).
    """
    torch = _torch()
    from ..exec.device_table import DeviceColumn
    import pyarrow as pa
    cols = list(key_cols)
    if extra_leading is not None:
        t, _bits = extra_leading
        cols = [DeviceColumn(t, None, pa.int32())] + cols
    n = len(cols[0])
    dev = cols[0].data.device
    specs = (NL.SortKeySpec * len(cols))()
    for i, c in enumerate(cols):
        kmin, bits = _sortable_range(c)
        specs[i] = NL.SortKeySpec(c.desc(), kmin, bits, 1 if c.valid is not None else 0)
    L = NL.lib()
    ws = torch.empty(int(L.hs_sort_workspace_bytes(n)), dtype=torch.uint8, device=dev)
    if init_perm is None:
        perm = torch.empty(n, dtype=torch.int32, device=dev)
        init = 0
    else:
        perm = init_perm.clone()
        init = 1
    NL.check(L.hs_sort_columns(specs, len(cols), n, NL.ptr(perm), init, NL.ptr(ws), ws.numel(),
                               NL.stream_ptr()), "hs_sort_columns")
    return perm


def merge_plan(run_off: np.ndarray, run_group: np.ndarray) -> List[np.ndarray]:
    """Pair tables ({start, mid, end} int64 rows) of the pairwise merge rounds that turn the
    sorted runs ``[run_off[r], run_off[r + 1])`` into one sorted run per group (runs of a group
    are adjacent; groups never merge).  Each round merges runs 2i and 2i + 1 of every group; an
    odd last run is carried as a pair with an empty right half."""
    groups: List[List[int]] = []
    for r in range(len(run_off) - 1):
        if run_off[r + 1] == run_off[r]:
            continue
        if groups and groups[-1][0] == run_group[r]:
            groups[-1][1].append(int(run_off[r + 1]))
        else:
            groups.append((run_group[r], [int(run_off[r]), int(run_off[r + 1])]))
    bounds = [g[1] for g in groups]
    rounds = []
    while any(len(b) > 2 for b in bounds):
        # every round covers all rows (the keys / permutation ping-pong between two buffers):
        # a group already merged is a copy pair
        pairs, nb = [], []
        for b in bounds:
            nxt = [b[0]]
            for i in range(0, len(b) - 1, 2):
                s, m = b[i], b[i + 1]
                e = b[i + 2] if i + 2 < len(b) else m
                pairs.append((s, m, e))
                nxt.append(e)
            nb.append(nxt)
        rounds.append(np.asarray(pairs, dtype=np.int64).reshape(-1, 3))
        bounds = nb
    return rounds


def merge_runs_permutation(key_cols: Sequence, run_off: np.ndarray, run_group: np.ndarray):
    """Stable ascending (NULLS FIRST) permutation of rows made of runs already sorted by
    ``key_cols``, grouped by ``run_group`` (e.g. bucket ids; groups stay in place): the order
    ``sort_permutation([group] + key_cols)`` gives for such input, from ceil(log2(runs)) merge
    rounds instead of a radix sort (K6).  None when the composite key exceeds 64 bits."""
    torch = _torch()
    cols = list(key_cols)
    n = len(cols[0])
    dev = cols[0].data.device
    if len(cols) > NL.MERGE_MAX_KEYS:
        return None
    mk = NL.MergeKeys()
    total = 0
    for i, c in enumerate(cols):
        kmin, bits = _sortable_range(c)
        mk.col[i] = c.desc()
        mk.kmin[i] = kmin
        mk.bits[i] = bits
        mk.nullable[i] = 1 if c.valid is not None else 0
        total += bits + mk.nullable[i]
    mk.nkeys = len(cols)
    if total > 64:
        return None
    rounds = merge_plan(np.asarray(run_off, np.int64), np.asarray(run_group))
    perm = torch.arange(n, dtype=torch.int32, device=dev)
    if not rounds or n == 0:
        return perm
    L = NL.lib()
    ka = torch.empty(n, dtype=torch.int64, device=dev)
    kb = torch.empty_like(ka)
    pb = torch.empty_like(perm)
    NL.check(L.hs_merge_make_keys(C.byref(mk), n, NL.ptr(ka), NL.stream_ptr()),
             "hs_merge_make_keys")
    # the runs must really be sorted in this order (files written by another writer may order
    # floats or strings differently): otherwise the caller sorts from scratch
    if n > 1:
        starts = torch.zeros(n, dtype=torch.bool, device=dev)
        ro = torch.from_numpy(np.asarray(run_off[:-1], np.int64)).to(dev)
        starts[ro[ro < n]] = True
        ks = ka ^ torch.tensor(-(1 << 63), dtype=torch.int64, device=dev)   # unsigned order
        if bool(((ks[1:] < ks[:-1]) & ~starts[1:]).any()):
            return None
    pa_, first = perm, True
    for pairs in rounds:
        dp = torch.from_numpy(pairs.reshape(-1)).to(dev)
        NL.check(L.hs_merge_round(NL.ptr(ka), 0 if first else NL.ptr(pa_), NL.ptr(kb),
                                  NL.ptr(pb), NL.ptr(dp), len(pairs), n, NL.stream_ptr()),
                 "hs_merge_round")
        first = False
        ka, kb = kb, ka
        pa_, pb = pb, pa_
    return pa_


def exclusive_scan_i64(x):
    torch = _torch()
    n = x.numel()
    out = torch.empty_like(x)
    L = NL.lib()
    tmp = torch.empty(max(1, int(L.hs_scan_tmp_elems(n))), dtype=torch.int64, device=x.device)
    NL.check(L.hs_exclusive_scan_i64(NL.ptr(x), NL.ptr(out), n, NL.ptr(tmp), tmp.numel(),
                                     NL.stream_ptr()), "hs_exclusive_scan_i64")
    return out


# ------------------------------------------------------------------------------------------------
# Gather
# ------------------------------------------------------------------------------------------------
# packed-row gather (hs_gather_packed, opt-in: HS_GATHER_PACKED=1): tables of at least this many
# rows, records of at most PACKED_MAX_BYTES.  Off by default: at SF100 it cut the li_shipdate
# build's sort+gather 0.102 -> 0.082 s (a random permutation) but raised li_orderkey's
# 0.060 -> 0.274 s (a permutation that is nearly sequential within each bucket, where the
# per-column gather already streams, plus the record buffer's allocation):
# profiles/build_packed_gather_r3.log
PACKED_MIN_ROWS = 1 << 20
PACKED_MAX_BYTES = 64
# HS_GATHER_PACKED=auto (default): packed records only for permutations that jump around - the
# median distance between the source rows of neighbouring outputs, over an evenly spaced sample,
# at least PACKED_MIN_JUMP rows (a random permutation: ~n/3; li_orderkey's nearly sequential
# one: ~1)
PACKED_MIN_JUMP = 64
PACKED_SAMPLE = 4096


def sample_positions(n: int, k: int, device):
    """min(k, n - 1) evenly spaced int64 positions in [0, n - 2] (integer arithmetic: a float32
    linspace rounds positions of large n past the end)."""
    torch = _torch()
    k = min(k, n - 1)
    return torch.arange(k, dtype=torch.int64, device=device) * (n - 2) // max(k - 1, 1)


def _random_permutation(idx) -> bool:
    """Whether ``idx`` reads its sources scattered (one small D2H of a sample of neighbouring
    index pairs)."""
    torch = _torch()
    n = idx.numel()
    if n < 2:
        return False
    pos = sample_positions(n, PACKED_SAMPLE, idx.device)
    d = (idx.index_select(0, pos + 1).long() - idx.index_select(0, pos).long()).abs()
    return float(d.float().median().item()) >= PACKED_MIN_JUMP


def _packed_layout(cols, want_valid: bool):
    """(row_bytes, value offsets, validity base) of the packed records of ``cols`` (fields by
    descending width, so every field is naturally aligned), or None when records would exceed
    PACKED_MAX_BYTES."""
    order = sorted(range(len(cols)), key=lambda j: -cols[j].data.element_size())
    offs = [0] * len(cols)
    at = 0
    for j in order:
        offs[j] = at
        at += cols[j].data.element_size()
    vbase = at
    if any(c.valid is not None and want_valid for c in cols):
        at += len(cols)
    rb = (at + 15) // 16 * 16
    return (rb, offs, vbase) if rb <= PACKED_MAX_BYTES else None


def gather_columns(cols: list, idx, want_valid: bool = True, padded: bool = False) -> list:
    """Gather a list of DeviceColumns by ``idx`` (int32 or int64 tensor) in one launch.
    ``padded``: ``idx`` (int64) may hold -1 for outer-join padding rows, which come out NULL
    (every output column then carries a validity mask).  Scattered permutations of large
    multi-column tables (``HS_GATHER_PACKED=auto``: ``_random_permutation``; ``1``: always,
    ``0``: never) go through packed records (``hs_gather_packed``): one random sector per row
    instead of one per column."""
    torch = _torch()
    from ..exec.device_table import DeviceColumn
    n = idx.numel()
    mode = os.environ.get("HS_GATHER_PACKED", "auto")
    if (not padded and len(cols) >= 2 and len(cols) <= NL.GATHER_MAX_COLS and
            n >= PACKED_MIN_ROWS and mode in ("1", "auto") and
            len({len(c.data) for c in cols}) == 1 and
            (mode == "1" or _random_permutation(idx))):
        lay = _packed_layout(cols, want_valid)
        if lay is not None:
            rb, offs, vbase = lay
            n_src = len(cols[0].data)
            free, _ = torch.cuda.mem_get_info(cols[0].data.device)
            if n_src * rb < free // 2:
                return _gather_packed(cols, idx, want_valid, rb, offs, vbase, n_src)
    out = []
    for i in range(0, len(cols), NL.GATHER_MAX_COLS):
        chunk = cols[i:i + NL.GATHER_MAX_COLS]
        p = NL.GatherParams()
        res = []
        for j, c in enumerate(chunk):
            dst = torch.empty(n, dtype=c.data.dtype, device=c.data.device)
            dv = torch.empty(n, dtype=torch.uint8, device=c.data.device) \
                if ((c.valid is not None and want_valid) or padded) else None
            p.cols[j] = NL.GatherCol(c.data.data_ptr(), dst.data_ptr(),
                                     c.valid.data_ptr() if c.valid is not None else 0,
                                     dv.data_ptr() if dv is not None else 0,
                                     c.data.element_size(), 0)
            res.append(DeviceColumn(dst, dv, c.atype, c.dictionary))
        p.ncols = len(chunk)
        p.idx_is_u32 = 1 if idx.dtype == torch.int32 else 0
        NL.check(NL.lib().hs_gather(C.byref(p), NL.ptr(idx), n, NL.stream_ptr()), "hs_gather")
        out.extend(res)
    return out


def _gather_packed(cols, idx, want_valid, rb: int, offs, vbase: int, n_src: int) -> list:
    torch = _torch()
    from ..exec.device_table import DeviceColumn
    n = idx.numel()
    dev = cols[0].data.device
    p = NL.GatherParams()
    res = []
    for j, c in enumerate(cols):
        dst = torch.empty(n, dtype=c.data.dtype, device=dev)
        dv = torch.empty(n, dtype=torch.uint8, device=dev) \
            if (c.valid is not None and want_valid) else None
        p.cols[j] = NL.GatherCol(c.data.data_ptr(), dst.data_ptr(),
                                 c.valid.data_ptr() if c.valid is not None else 0,
                                 dv.data_ptr() if dv is not None else 0,
                                 c.data.element_size(), offs[j])
        res.append(DeviceColumn(dst, dv, c.atype, c.dictionary))
    p.ncols = len(cols)
    p.idx_is_u32 = 1 if idx.dtype == torch.int32 else 0
    rows = torch.empty(max(n_src, 1) * rb, dtype=torch.uint8, device=dev)
    NL.check(NL.lib().hs_gather_packed(C.byref(p), rb, vbase, n_src, NL.ptr(rows), NL.ptr(idx),
                                       n, NL.stream_ptr()), "hs_gather_packed")
    return res


def mark_rows(idx, n: int):
    """uint8 [n]: 1 at every row id of ``idx`` (int64; negative ids ignored)."""
    torch = _torch()
    mark = torch.zeros(max(n, 1), dtype=torch.uint8, device=idx.device)
    NL.check(NL.lib().hs_mark_rows(NL.ptr(idx), idx.numel(), NL.ptr(mark), NL.stream_ptr()),
             "hs_mark_rows")
    return mark


def select_marked(rows, mark, want: int):
    """The row ids of ``rows`` (int64, order kept) whose ``mark`` byte equals ``want``."""
    torch = _torch()
    L = NL.lib()
    n = rows.numel()
    dev = rows.device
    ws = torch.empty(max(int(L.hs_select_marked_blocks(n)), 1), dtype=torch.int64, device=dev)
    total = torch.empty(1, dtype=torch.int64, device=dev)
    out = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    NL.check(L.hs_select_marked(NL.ptr(rows), n, NL.ptr(mark), int(want), NL.ptr(ws),
                                NL.ptr(total), NL.ptr(out), NL.stream_ptr()), "hs_select_marked")
    return out[:int(total.item())]


def histogram(ids, num_bins: int):
    """int64 counts of int32 ``ids`` over ``[0, num_bins)`` (LDS-privatised HIP histogram;
    replaces ``torch.bincount`` on the build path)."""
    torch = _torch()
    out = torch.empty(num_bins, dtype=torch.int64, device=ids.device)
    if num_bins > 16384:
        return torch.bincount(ids.long(), minlength=num_bins)
    NL.check(NL.lib().hs_histogram(NL.ptr(ids), ids.numel(), num_bins, NL.ptr(out),
                                   NL.stream_ptr()), "hs_histogram")
    return out


MAX_BITMAP_BITS = 1 << 33     # 1 GiB of HBM: a key domain wider than this is not bitmapped


def key_domain(col):
    """(lo, hi, non-null count) of an integer device column, or None when it holds no non-null
    key or is not an integer column.  One host sync."""
    torch = _torch()
    if col.hs_type not in (NL.I8, NL.I16, NL.I32, NL.I64, NL.U32) or col.offsets is not None:
        return None
    d = col.data
    if d.numel() == 0:
        return None
    if col.valid is not None:
        vm = col.valid.bool()
        x = d.long()
        st = torch.stack([torch.where(vm, x, torch.iinfo(torch.int64).max).min(),
                          torch.where(vm, x, torch.iinfo(torch.int64).min).max(),
                          vm.sum()]).cpu().tolist()
        if st[2] == 0:
            return None
        return int(st[0]), int(st[1]), int(st[2])
    mm = torch.aminmax(d)
    lo, hi = (int(v) for v in torch.stack([mm.min.long(), mm.max.long()]).cpu().tolist())
    return lo, hi, int(d.numel())


def key_bitmap(col, lo: int, nbits: int, check: bool = True):
    """(int64 words, duplicate flag) of the non-null integer keys of device column ``col`` as
    bits (key - lo) of an ``nbits``-bit bitmap (csrc/kernels/key_bitmap.hip).  Every key must
    lie in [lo, lo + nbits).  ``check=False``: the caller knows the keys are unique and in the
    domain - no flag read, no host synchronization (the flag is None)."""
    torch = _torch()
    d = col.data
    words = torch.zeros(max((nbits + 63) // 64, 1), dtype=torch.int64, device=d.device)
    flags = torch.zeros(1, dtype=torch.int32, device=d.device)
    desc = col.desc()
    NL.check(NL.lib().hs_key_bitmap(C.byref(desc), d.numel(), int(lo), int(nbits), NL.ptr(words),
                                    NL.ptr(flags), NL.stream_ptr()), "hs_key_bitmap")
    if not check:
        return words, None
    f = int(flags.item())
    if f & 2:
        raise RuntimeError("hs_key_bitmap: key outside its domain")
    return words, bool(f & 1)


def bitmap_popcount(words) -> int:
    torch = _torch()
    out = torch.zeros(1, dtype=torch.int64, device=words.device)
    NL.check(NL.lib().hs_bitmap_popcount(NL.ptr(words), words.numel(), NL.ptr(out),
                                         NL.stream_ptr()), "hs_bitmap_popcount")
    return int(out.item())


def str_hash64(ptr, ln):
    """int64 hash per string value given as (device address int64, length int32) tensors
    (csrc/kernels/strings.hip)."""
    torch = _torch()
    out = torch.empty(ptr.numel(), dtype=torch.int64, device=ptr.device)
    NL.check(NL.lib().hs_str_hash64(NL.ptr(ptr), NL.ptr(ln), ptr.numel(), NL.ptr(out),
                                    NL.stream_ptr()), "hs_str_hash64")
    return out


def str_gather(ptr, ln):
    """(int32 offsets [n + 1] on the host, uint8 bytes on the device) of the values
    (address, length): Arrow string layout of the selection."""
    torch = _torch()
    l64 = ln.clamp(min=0).long()
    off = torch.zeros(ptr.numel() + 1, dtype=torch.int64, device=ptr.device)
    torch.cumsum(l64, 0, out=off[1:])
    offh = off.cpu()
    out = torch.empty(max(int(offh[-1]), 1), dtype=torch.uint8, device=ptr.device)
    NL.check(NL.lib().hs_str_gather(NL.ptr(ptr), NL.ptr(ln), NL.ptr(off), ptr.numel(),
                                    NL.ptr(out), NL.stream_ptr()), "hs_str_gather")
    return offh, out


def str_differ(a, alen, b, blen):
    """bool per value: value i of (a, alen) differs from value i of (b, blen)."""
    torch = _torch()
    out = torch.empty(a.numel(), dtype=torch.uint8, device=a.device)
    NL.check(NL.lib().hs_str_differ(NL.ptr(a), NL.ptr(alen), NL.ptr(b), NL.ptr(blen), a.numel(),
                                    NL.ptr(out), NL.stream_ptr()), "hs_str_differ")
    return out.bool()


def lookup_i32(table, codes):
    """``table[codes]`` for an int32 table and int32 codes, through the gather kernel."""
    from ..exec.device_table import DeviceColumn
    import pyarrow as pa
    return gather_columns([DeviceColumn(table, None, pa.int32())], codes, want_valid=False)[0].data


def bucket_offsets_from_sorted(sorted_bucket, num_buckets: int):
    torch = _torch()
    off = torch.empty(num_buckets + 1, dtype=torch.int64, device=sorted_bucket.device)
    NL.check(NL.lib().hs_bucket_offsets(NL.ptr(sorted_bucket), sorted_bucket.numel(), num_buckets,
                                        NL.ptr(off), NL.stream_ptr()), "hs_bucket_offsets")
    return off


# ------------------------------------------------------------------------------------------------
# Scan: ranges, filter+aggregate, filter+select
# ------------------------------------------------------------------------------------------------
def range_search(key_col, bucket_off, buckets=None, lo=None, lo_incl=True, hi=None, hi_incl=True):
    """Per-bucket [start, len) of rows whose sorted key lies in the bound interval.

    ``lo``/``hi`` are sortable uint64 images (see ``sortable_image``); None = unbounded.
    Returns (rstart, rlen, rbucket) int64/int64/int32 device tensors of length nb.
    """
    torch = _torch()
    dev = bucket_off.device
    nb = (buckets.numel() if buckets is not None else bucket_off.numel() - 1)
    rstart = torch.empty(nb, dtype=torch.int64, device=dev)
    rlen = torch.empty(nb, dtype=torch.int64, device=dev)
    rbucket = torch.empty(nb, dtype=torch.int32, device=dev)
    kd = key_col.desc()
    NL.check(NL.lib().hs_range_search(C.byref(kd), NL.ptr(bucket_off), NL.ptr(buckets), nb,
                                      1 if lo is not None else 0, int(lo or 0), 1 if lo_incl else 0,
                                      1 if hi is not None else 0, int(hi or 0), 1 if hi_incl else 0,
                                      NL.ptr(rstart), NL.ptr(rlen), NL.ptr(rbucket), NL.stream_ptr()),
             "hs_range_search")
    return rstart, rlen, rbucket


def probe_ranges(key_col, bucket_off, pbucket, pkey):
    """Per probe (bucket int32, sortable key image as int64 bits), the [start, len) run of rows
    of that bucket whose sorted key equals it.  Returns (rstart, rlen, rbucket)."""
    torch = _torch()
    n = int(pbucket.numel())
    dev = bucket_off.device
    rstart = torch.empty(n, dtype=torch.int64, device=dev)
    rlen = torch.empty(n, dtype=torch.int64, device=dev)
    rbucket = torch.empty(n, dtype=torch.int32, device=dev)
    kd = key_col.desc()
    NL.check(NL.lib().hs_probe_ranges(C.byref(kd), NL.ptr(bucket_off), NL.ptr(pbucket),
                                      NL.ptr(pkey), n, NL.ptr(rstart), NL.ptr(rlen),
                                      NL.ptr(rbucket), NL.stream_ptr()), "hs_probe_ranges")
    return rstart, rlen, rbucket


def full_ranges(bucket_off_host: np.ndarray, device, buckets: Optional[List[int]] = None):
    torch = _torch()
    off = bucket_off_host
    bs = np.arange(len(off) - 1) if buckets is None else np.asarray(buckets, dtype=np.int64)
    rstart = torch.from_numpy(off[bs].astype(np.int64)).to(device)
    rlen = torch.from_numpy((off[bs + 1] - off[bs]).astype(np.int64)).to(device)
    rbucket = torch.from_numpy(bs.astype(np.int32)).to(device)
    return rstart, rlen, rbucket


def ranges_to_tiles(rlen, tile_rows: int = None):
    """Exclusive prefix of per-range tile counts (``tp[R]`` = total).  Scan kernels use the scan
    tile; the join wrappers below compute their own prefix with the join tile."""
    torch = _torch()
    R = rlen.numel()
    tp = torch.empty(R + 1, dtype=torch.int64, device=rlen.device)
    tr = int(tile_rows or NL.lib().hs_scan_tile_rows())
    NL.check(NL.lib().hs_ranges_to_tiles(NL.ptr(rlen), R, tr, NL.ptr(tp), NL.stream_ptr()),
             "hs_ranges_to_tiles")
    return tp


def sortable_image(value, hs_type: int) -> int:
    """Host mirror of hs_sortable for a literal."""
    import struct
    if hs_type == NL.F64:
        b = struct.unpack("<Q", struct.pack("<d", float(value)))[0]
        return (~b) & 0xFFFFFFFFFFFFFFFF if b >> 63 else b | (1 << 63)
    if hs_type == NL.F32:
        b = struct.unpack("<I", struct.pack("<f", float(value)))[0]
        return ((~b) & 0xFFFFFFFF) if b >> 31 else (b | 0x80000000)
    width = {NL.I8: 8, NL.I16: 16, NL.I32: 32, NL.I64: 64}.get(hs_type)
    if width is None:
        return int(value)
    return (int(value) + (1 << (width - 1))) & ((1 << width) - 1)


def agg_outputs(GA: int, dev):
    """(sum f64, count i64, min f64, max f64) [GA] as views of ONE device buffer, so the host
    reads a query's aggregate result with a single D2H copy (``sum.hs_buf``)."""
    torch = _torch()
    buf = torch.empty(32 * max(GA, 1), dtype=torch.uint8, device=dev)
    n = 8 * GA
    s = buf[0:n].view(torch.float64)
    c = buf[n:2 * n].view(torch.int64)
    mn = buf[2 * n:3 * n].view(torch.float64)
    mx = buf[3 * n:4 * n].view(torch.float64)
    s.hs_buf = buf
    return s, c, mn, mx


def agg_to_host(sums, cnts, mins, maxs):
    """numpy views of the four aggregate outputs with one D2H copy when they share a buffer."""
    buf = getattr(sums, "hs_buf", None)
    if buf is None:
        return sums.cpu().numpy(), cnts.cpu().numpy(), mins.cpu().numpy(), maxs.cpu().numpy()
    h = buf.cpu().numpy()
    n = sums.numel() * 8
    return (h[0:n].view(np.float64), h[n:2 * n].view(np.int64), h[2 * n:3 * n].view(np.float64),
            h[3 * n:4 * n].view(np.float64))


def agg_to_host_async(sums, cnts, mins, maxs):
    """Queue the D2H of the four aggregate outputs into pinned memory and return ``fetch()``,
    which waits for that copy only (not for the whole device) and returns numpy views."""
    torch = _torch()
    buf = getattr(sums, "hs_buf", None)
    if buf is None or buf.numel() != 32 * sums.numel():
        buf = torch.cat([x.contiguous().view(torch.uint8) for x in (sums, cnts, mins, maxs)])
    h = torch.empty(buf.numel(), dtype=torch.uint8, pin_memory=True)
    h.copy_(buf, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    n = sums.numel() * 8

    def fetch():
        ev.synchronize()
        a = h.numpy()
        return (a[0:n].view(np.float64), a[n:2 * n].view(np.int64),
                a[2 * n:3 * n].view(np.float64), a[3 * n:4 * n].view(np.float64))
    return fetch


def scan_agg(params: NL.ScanParams, rstart, rlen, tile_prefix, grid: int = None):
    """Returns (sum f64 [GA], count i64 [GA], min f64 [GA], max f64 [GA]) device tensors."""
    torch = _torch()
    L = NL.lib()
    grid = grid or L.hs_scan_grid()
    GA = params.naggs * (params.num_groups if params.group_col >= 0 else 1)
    dev = rstart.device
    ps = torch.empty(grid * GA, dtype=torch.float64, device=dev)
    pc_ = torch.empty(grid * GA, dtype=torch.int64, device=dev)
    pmn = torch.empty(grid * GA, dtype=torch.float64, device=dev)
    pmx = torch.empty(grid * GA, dtype=torch.float64, device=dev)
    os_, oc, omn, omx = agg_outputs(GA, dev)
    NL.check(L.hs_scan_agg(C.byref(params), NL.ptr(rstart), NL.ptr(rlen), rstart.numel(),
                           NL.ptr(tile_prefix), grid, NL.ptr(ps), NL.ptr(pc_), NL.ptr(pmn),
                           NL.ptr(pmx), NL.ptr(os_), NL.ptr(oc), NL.ptr(omn), NL.ptr(omx),
                           NL.stream_ptr()), "hs_scan_agg")
    return os_, oc, omn, omx


def scan_bitmap(params: NL.ScanParams, rstart, rlen, tile_prefix, key_slot: int, lo: int,
                nbits: int):
    """int64 words of an ``nbits``-bit bitmap with bit (key - lo) set for the key column
    ``key_slot`` of every row passing the predicate (csrc/kernels/scan_filter.hip
    ``hs_scan_bitmap``): filter and bitmap build in one launch, no host synchronization."""
    torch = _torch()
    L = NL.lib()
    words = torch.zeros(max((nbits + 63) // 64, 1), dtype=torch.int64, device=rstart.device)
    NL.check(L.hs_scan_bitmap(C.byref(params), NL.ptr(rstart), NL.ptr(rlen), rstart.numel(),
                              NL.ptr(tile_prefix), L.hs_scan_grid(), int(key_slot), int(lo),
                              int(nbits), NL.ptr(words), NL.stream_ptr()), "hs_scan_bitmap")
    return words


def scan_select(params: NL.ScanParams, rstart, rlen, tile_prefix, max_tiles: int):
    """Row ids (int64, ascending within each range) of rows passing the predicate."""
    torch = _torch()
    L = NL.lib()
    grid = L.hs_scan_grid()
    dev = rstart.device
    counts = torch.zeros(max_tiles + 1, dtype=torch.int64, device=dev)
    NL.check(L.hs_scan_count(C.byref(params), NL.ptr(rstart), NL.ptr(rlen), rstart.numel(),
                             NL.ptr(tile_prefix), grid, NL.ptr(counts), NL.stream_ptr()),
             "hs_scan_count")
    offs = exclusive_scan_i64(counts)
    total = int(offs[-1].item())
    out = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
    NL.check(L.hs_scan_select(C.byref(params), NL.ptr(rstart), NL.ptr(rlen), rstart.numel(),
                              NL.ptr(tile_prefix), NL.ptr(offs), grid, NL.ptr(out),
                              NL.stream_ptr()), "hs_scan_select")
    return out[:total]


# ------------------------------------------------------------------------------------------------
# Join
# ------------------------------------------------------------------------------------------------
def join_max_tiles(left_rows: int, num_ranges: int) -> int:
    """Upper bound of the join tile count over ``num_ranges`` ranges of ``left_rows`` rows."""
    return left_rows // NL.lib().hs_join_tile_rows() + num_ranges + 1


def join_agg(params: NL.JoinParams, rstart, rlen, rbucket, roff, max_tiles: int,
             grid: int = None):
    """``max_tiles`` (see ``join_max_tiles``) sizes the per-tile span scratch."""
    torch = _torch()
    L = NL.lib()
    tile_prefix = ranges_to_tiles(rlen, L.hs_join_tile_rows())
    grid = grid or L.hs_scan_grid()
    GA = params.naggs * (params.num_groups if params.group_col >= 0 else 1)
    dev = rstart.device
    ps = torch.empty(grid * GA, dtype=torch.float64, device=dev)
    pc_ = torch.empty(grid * GA, dtype=torch.int64, device=dev)
    pmn = torch.empty(grid * GA, dtype=torch.float64, device=dev)
    pmx = torch.empty(grid * GA, dtype=torch.float64, device=dev)
    os_, oc, omn, omx = agg_outputs(GA, dev)
    spans = torch.empty(4 * max(max_tiles, 1), dtype=torch.int64, device=dev)
    NL.check(L.hs_join_agg(C.byref(params), NL.ptr(rstart), NL.ptr(rlen), NL.ptr(rbucket),
                           NL.ptr(roff), rstart.numel(), NL.ptr(tile_prefix), int(max_tiles),
                           NL.ptr(spans), grid, NL.ptr(ps), NL.ptr(pc_), NL.ptr(pmn), NL.ptr(pmx),
                           NL.ptr(os_), NL.ptr(oc), NL.ptr(omn), NL.ptr(omx), NL.stream_ptr()),
             "hs_join_agg")
    return os_, oc, omn, omx


def join_pairs(params: NL.JoinParams, rstart, rlen, rbucket, roff, max_tiles: int):
    torch = _torch()
    L = NL.lib()
    tile_prefix = ranges_to_tiles(rlen, L.hs_join_tile_rows())
    grid = L.hs_scan_grid()
    dev = rstart.device
    counts = torch.zeros(max_tiles + 1, dtype=torch.int64, device=dev)
    spans = torch.empty(4 * max(max_tiles, 1), dtype=torch.int64, device=dev)
    NL.check(L.hs_join_count(C.byref(params), NL.ptr(rstart), NL.ptr(rlen), NL.ptr(rbucket),
                             NL.ptr(roff), rstart.numel(), NL.ptr(tile_prefix), int(max_tiles),
                             NL.ptr(spans), grid, NL.ptr(counts), NL.stream_ptr()), "hs_join_count")
    offs = exclusive_scan_i64(counts)
    total = int(offs[-1].item())
    ol = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
    orr = torch.empty(max(total, 1), dtype=torch.int64, device=dev)
    NL.check(L.hs_join_emit(C.byref(params), rstart.numel(), NL.ptr(tile_prefix), NL.ptr(spans),
                            grid, NL.ptr(offs), NL.ptr(ol), NL.ptr(orr), NL.stream_ptr()),
             "hs_join_emit")
    return ol[:total], orr[:total]
