"""Lossless lightweight compression of HBM-resident index columns (frame-of-reference, with an
optional exact decimal scale for floating-point columns).

The fused query kernels are HBM-bandwidth bound, so the bytes per row they stream are the cost
model.  Index columns are immutable once loaded, so the executor derives a compact copy per
column once and the generated kernels (``exec/jit.py``) decode it in registers:

    value = base + code                  (integers, dates, timestamps, dictionary codes)
    value = (double)(base + code) / 10^k (floats that are exact k-digit decimals, e.g. prices)

``code`` is a signed 8/16/32-bit integer chosen from the value range.  An encoding is kept only if
decoding reproduces every valid row *bit for bit* (checked on the device), so results are exact —
e.g. TPC-H ``l_discount`` becomes 1 byte/row instead of 8, ``l_orderkey`` 4 instead of 8.  Columns
that do not qualify simply have no compact form and are read at full width.
"""
from __future__ import annotations

from typing import Optional

from ..ops import _lib as NL

_INT_TYPES = (NL.I8, NL.I16, NL.I32, NL.I64, NL.U32, NL.BOOL)
_FLOAT_TYPES = (NL.F64,)
_MAX_SCALE_DIGITS = 4


class Compact:
    __slots__ = ("codes", "width", "base", "scale", "logical_type", "lo", "hi", "g16", "runs",
                 "_g16_wide")

    def __init__(self, codes, width: int, base: int, scale: Optional[float], logical_type: int,
                 lo: Optional[int] = None, hi: Optional[int] = None):
        self.codes = codes          # torch int8/int16/int32 tensor (biased: code = v - base)
        self.width = width          # bytes per row
        self.base = int(base)
        self.scale = scale          # None for integers, 10**k for decimals
        self.logical_type = logical_type
        self.lo, self.hi = lo, hi   # range of the (integer / scaled) values of valid rows
        self.g16 = False            # grouped16(): derived 16-bit form (None: not applicable)
        self.runs = False           # key_runs(): derived run-length form (None: not applicable)

    def nbytes(self) -> int:
        n = self.codes.numel() * self.width
        n += self.g16.nbytes() if self.g16 else 0
        return n + (self.runs.extra_bytes() if self.runs else 0)

    def signature(self) -> tuple:
        """Shape-relevant part (codegen key): literals like base/scale are kernel arguments."""
        return (self.width, self.scale is not None)


GROUP_ROWS = 64


WIDE_GROUP = -(1 << 31)


class GroupedCompact(Compact):
    """16-bit codes relative to a per-64-row group base: value = base + gbase[row >> 6] +
    (uint16) code.  Derived from a sorted integer column's 32-bit compact form (an index's
    bucket-sorted key: neighbouring rows hold close keys), it halves the bytes a merge join
    streams for the left key (``exec/jit.py`` ``MJ_KEY16``).  A group spanning 2^16 codes or
    more (one straddling two buckets) is *wide*: its base is ``WIDE_GROUP`` and readers take
    its 32-bit codes from ``wide`` (the parent compact's codes)."""
    __slots__ = ("gbase", "wide")

    def __init__(self, codes, gbase, wide, base: int, logical_type: int, lo, hi):
        super().__init__(codes, 2, base, None, logical_type, lo, hi)
        self.gbase = gbase          # int32 [ceil(n / 64)]: the group's smallest 32-bit code
        self.wide = wide            # int32 codes of every row (read for wide groups only)

    def nbytes(self) -> int:
        return self.codes.numel() * 2 + self.gbase.numel() * 4

    def signature(self) -> tuple:
        return (2, False, GROUP_ROWS)


def grouped16(c: Compact, max_wide: float = 0.01) -> Optional[GroupedCompact]:
    """The 16-bit grouped form of the 32-bit integer compact ``c`` (computed once, kept on
    ``c``), or None when more than ``max_wide`` of its 64-row groups are wide (a refusal is
    re-examined for a more tolerant ``max_wide``)."""
    if c.g16 is not False and (c.g16 is not None or getattr(c, "_g16_wide", 1.0) >= max_wide):
        return c.g16
    c.g16 = None
    c._g16_wide = max_wide
    if c.scale is not None or c.lo is None or c.width != 4 or c.codes.numel() == 0:
        return None
    r = group16(c.codes, max_wide)
    if r is None:
        return None
    c.g16 = GroupedCompact(r[0], r[1], c.codes, c.base, c.logical_type, c.lo, c.hi)
    return c.g16


def group16(x, max_wide: float):
    """(codes16, gbase) of a sorted-within-groups int32 code array ``x``: per 64-element group
    its smallest code (``WIDE_GROUP`` when the group spans 2^16 codes or more) and each
    element's uint16 offset from it (0 in wide groups, whose readers take ``x``); None when more
    than ``max_wide`` of the groups are wide."""
    import torch
    n = x.numel()
    if n == 0:
        return None
    pad = (-n) % GROUP_ROWS
    xp = torch.cat([x, x[-1:].expand(pad)]) if pad else x
    g = xp.view(-1, GROUP_ROWS)
    gmin = g.amin(dim=1)
    wide = ((g.amax(dim=1).long() - gmin.long()) >= (1 << 16)) | (gmin == WIDE_GROUP)
    if float(wide.float().mean().item()) > max_wide:
        return None
    gbase = torch.where(wide, torch.full_like(gmin, WIDE_GROUP), gmin)
    d = g.long() - gmin.long().unsqueeze(1)
    d = torch.where(wide.unsqueeze(1), torch.zeros_like(d), d).reshape(-1)[:n]
    codes = torch.where(d >= (1 << 15), d - (1 << 16), d).to(torch.int16)   # uint16 bits
    return codes.contiguous(), gbase.contiguous()


class RunCompact(Compact):
    """Run-length form of a bucket-sorted 32-bit integer key (csrc/kernels/key_runs.hip): a
    covering index is sorted by its indexed columns inside each bucket, so its leading key is a
    sequence of runs of equal values (TPC-H ``l_orderkey``: 1-7 rows per key).  The run-keyed
    merge join (``exec/jit.py`` ``MJ_RUNS``) reads, per row, only which run holds it:

        gmask[g]   rows of 64-row group g that start a run (uint64 bits)
        gruns[g]   index of the run holding row 64 * g (int32)
        runkeys[r] code of run r (int32)

    ~1.2 instead of 4 bytes per row at 4 rows per run.  ``codes`` stays the parent's full 32-bit
    codes, so every other reader (spans, aggregate tails, group keys) is unchanged."""
    __slots__ = ("runkeys", "gmask", "gruns", "nruns", "k16")

    def __init__(self, parent: Compact, runkeys, gmask, gruns):
        super().__init__(parent.codes, parent.width, parent.base, parent.scale,
                         parent.logical_type, parent.lo, parent.hi)
        self.runkeys, self.gmask, self.gruns = runkeys, gmask, gruns
        self.nruns = int(runkeys.numel())
        self.k16 = False

    def keys16(self, max_wide: float = 0.1):
        """(runkeys16, group bases) of the run keys, per 64-run group (``group16``; computed
        once): the run-keyed join's phase 1 reads 2 instead of 4 bytes per run."""
        if self.k16 is False:
            self.k16 = group16(self.runkeys, max_wide)
        return self.k16

    def extra_bytes(self) -> int:
        n = self.runkeys.numel() * 4 + self.gmask.numel() * 8 + self.gruns.numel() * 4
        if self.k16:
            n += self.k16[0].numel() * 2 + self.k16[1].numel() * 4
        return n

    def nbytes(self) -> int:
        return self.codes.numel() * self.width + self.extra_bytes()

    def signature(self) -> tuple:
        return (4, False, "runs")


# the run form pays off when a run covers this many rows on average (4 bytes per run + 12 per
# 64 rows against 4 per row)
MIN_ROWS_PER_RUN = 1.5


def key_runs(c: Compact) -> Optional[RunCompact]:
    """The run-length form of the 32-bit integer compact ``c`` (computed once, kept on ``c``),
    or None when it does not apply or its runs are too short to pay off."""
    if c.runs is not False:
        return c.runs
    c.runs = None
    if c.scale is not None or c.lo is None or c.width != 4 or c.codes.numel() == 0 or \
            c.codes.numel() >= (1 << 31):
        return None
    x = c.codes
    runkeys, gmask, gruns = (_runs_device if x.is_cuda else runs_torch)(x)
    if runkeys.numel() * MIN_ROWS_PER_RUN > x.numel():
        return None
    c.runs = RunCompact(c, runkeys, gmask, gruns)
    return c.runs


def _runs_device(x):
    import torch
    L = NL.lib()
    n = x.numel()
    ng = (n + 63) // 64
    gmask = torch.empty(ng, dtype=torch.int64, device=x.device)
    gcnt = torch.empty(ng, dtype=torch.int64, device=x.device)
    NL.check(L.hs_key_runs_mask(x.data_ptr(), n, gmask.data_ptr(), gcnt.data_ptr(),
                                NL.stream_ptr()), "hs_key_runs_mask")
    incl = torch.cumsum(gcnt, 0)
    nruns = int(incl[-1].item())
    gexcl = incl - gcnt
    del incl, gcnt
    gruns = torch.empty(ng, dtype=torch.int32, device=x.device)
    runkeys = torch.empty(nruns, dtype=torch.int32, device=x.device)
    NL.check(L.hs_key_runs_fill(x.data_ptr(), n, gmask.data_ptr(), gexcl.data_ptr(),
                                gruns.data_ptr(), runkeys.data_ptr(), NL.stream_ptr()),
             "hs_key_runs_fill")
    return runkeys, gmask, gruns


def runs_torch(x):
    """PyTorch reference of ``hs_key_runs_mask`` + ``hs_key_runs_fill``: (runkeys int32,
    gmask int64 bit patterns, gruns int32)."""
    import torch
    n = x.numel()
    start = torch.ones(n, dtype=torch.bool, device=x.device)
    if n > 1:
        start[1:] = x[1:] != x[:-1]
    runkeys = x[start].to(torch.int32)
    ng = (n + 63) // 64
    sp = torch.zeros(ng * 64, dtype=torch.int64, device=x.device)
    sp[:n] = start.long()
    g = sp.view(ng, 64)
    w = torch.tensor([1 << i for i in range(63)] + [-(1 << 63)], dtype=torch.int64,
                     device=x.device)
    gmask = (g * w).sum(1)              # distinct bits: the wrapping sum is their OR
    cnt = g.sum(1)
    gexcl = torch.cumsum(cnt, 0) - cnt
    gruns = (gexcl + g[:, 0] - 1).to(torch.int32)
    return runkeys, gmask, gruns


def run_of(gmask, gruns, row: int) -> int:
    """Host reference of the kernels' run_of(row)."""
    g, i = row >> 6, row & 63
    m = int(gmask[g]) & ((1 << 64) - 1)
    below = ((2 << i) - 2) & ((1 << 64) - 1)
    return int(gruns[g]) + bin(m & below).count("1")


def _width_for(span: int):
    for w, bits in ((1, 8), (2, 16), (4, 32)):
        if span < (1 << bits):
            return w, 1 << (bits - 1)
    return None, None


def _codes(v, lo: int, w: int, bias: int):
    import torch
    dt = {1: torch.int8, 2: torch.int16, 4: torch.int32}[w]
    return (v - (lo + bias)).to(dt)


def encode(col) -> Optional[Compact]:
    """Compact form of a DeviceColumn, or None when no encoding is narrower and exact.

    Device columns: one ``hs_compact_probe`` pass decides the encoding and one
    ``hs_compact_encode`` pass writes the codes (csrc/kernels/compact.hip); host tensors use
    the PyTorch reference below (same decisions, same codes)."""
    if col.data.is_cuda and col.offsets is None and col.hs_type in _INT_TYPES + _FLOAT_TYPES:
        return _encode_device(col)
    return _encode_torch(col)


class DeviceColumnView:
    """(data, valid, hs_type) triple in the shape ``kernels.compact_probe`` reads."""
    __slots__ = ("data", "valid", "hs_type")

    def __init__(self, data, valid, hs_type):
        self.data, self.valid, self.hs_type = data, valid, hs_type


def _encode_device(col) -> Optional[Compact]:
    import torch
    L = NL.lib()
    t = col.hs_type
    d = col.data.contiguous()
    n = d.numel()
    if n == 0:
        return None
    valid = col.valid.contiguous() if col.valid is not None else None
    from ..ops import kernels as K
    r = K.compact_probe(DeviceColumnView(d, valid, t), _MAX_SCALE_DIGITS)
    if not r[0]:
        return None
    k_used, scale = 0, None
    if t in _INT_TYPES:
        lo, hi = int(r[3]), int(r[4])
    else:
        if r[1] or r[2]:          # non-finite, or -0.0 (would decode as +0.0)
            return None
        for k in range(_MAX_SCALE_DIGITS + 1):
            b = 5 + 4 * k
            if r[b + 1]:          # |round(x * 10^k)| >= 2^52
                return None
            if not r[b]:
                k_used, scale = k, float(10 ** k)
                lo, hi = int(r[b + 2]), int(r[b + 3])
                break
        else:
            return None
    w, bias = _width_for(hi - lo)
    if w is None or w >= d.element_size():
        return None
    dt = {1: torch.int8, 2: torch.int16, 4: torch.int32}[w]
    codes = torch.empty(n, dtype=dt, device=d.device)
    NL.check(L.hs_compact_encode(d.data_ptr(), valid.data_ptr() if valid is not None else None,
                                 n, t, k_used, lo + bias, lo, w, codes.data_ptr(),
                                 NL.stream_ptr()), "hs_compact_encode")
    return Compact(codes, w, lo + bias, scale, t, lo, hi)


def _encode_torch(col) -> Optional[Compact]:
    import torch
    t = col.hs_type
    d = col.data
    n = d.numel()
    if n == 0 or col.offsets is not None:
        return None
    vm = col.valid.bool() if col.valid is not None else None
    if t in _INT_TYPES:
        v = d.long()
        if vm is not None:
            if not bool(vm.any()):
                return None
            lo = int(torch.where(vm, v, torch.iinfo(torch.int64).max).min().item())
            hi = int(torch.where(vm, v, torch.iinfo(torch.int64).min).max().item())
            v = torch.where(vm, v, lo)
        else:
            lo, hi = (int(x.item()) for x in torch.aminmax(v))
        w, bias = _width_for(hi - lo)
        if w is None or w >= d.element_size():
            return None
        return Compact(_codes(v, lo, w, bias), w, lo + bias, None, t, lo, hi)
    if t in _FLOAT_TYPES:
        x = d.double()
        if vm is not None:
            if not bool(vm.any()):
                return None
            x = torch.where(vm, x, x[vm][0])
        if not bool(torch.isfinite(x).all()):
            return None
        # -0.0 would decode as +0.0 (code 0): keep such columns uncompressed
        if bool(((x == 0) & torch.signbit(x)).any()):
            return None
        for k in range(_MAX_SCALE_DIGITS + 1):
            s = float(10 ** k)
            q = torch.round(x * s)
            if float(q.abs().max().item()) >= 2.0 ** 52:
                return None
            # divide by a device tensor: torch implements division by a Python scalar as a
            # multiply by its reciprocal on the GPU (not correctly rounded), while the kernels
            # decode with an IEEE division
            back = (q / torch.full((), s, dtype=torch.float64, device=q.device)).view(torch.int64)
            same = bool((back == x.view(torch.int64)).all())  # bit-exact
            if not same:
                continue
            qi = q.long()
            lo, hi = (int(a.item()) for a in torch.aminmax(qi))
            w, bias = _width_for(hi - lo)
            if w is None or w >= d.element_size():
                return None
            return Compact(_codes(qi, lo, w, bias), w, lo + bias, s, t, lo, hi)
        return None
    return None


def compact_of(col) -> Optional[Compact]:
    """Cached compact form (computed on first use; tables are immutable)."""
    c = getattr(col, "compact", False)
    if c is False:
        c = encode(col)
        col.compact = c
    return c
