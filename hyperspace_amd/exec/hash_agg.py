"""High-cardinality and multi-column GROUP BY on the device, plus ORDER BY ... LIMIT (top-k).

The dense path in ``exec/gpu.py`` aggregates into LDS, one slot per value of a single small
integer group column.  Everything else — several group columns (TPC-H Q3 groups by
``l_orderkey, o_orderdate, o_shippriority``), millions of groups, float or string keys — runs
in *hash mode*:

1. ``KeyPlan`` packs the group columns into one 64-bit key: each integer / dictionary-code
   column contributes ``value - lo`` (+1 with a 0 code for NULL when nullable) in its own bit
   field, with ``lo`` and the widths taken from the columns' value domains (the same domains on
   every rank, so partial groups of different GPUs carry identical keys).  A single 64-bit
   integer or float column is used raw (float images normalise -0.0 and NaN).
2. The fused scan / merge-join kernels (``exec/jit.py``, ``_hash_accumulate``) insert the rows
   into a global open-addressing table (``csrc/kernels/hash_agg.hip``); a wavefront reduces
   runs of equal keys first, so sorted inputs cost about one probe per group and batch.
3. ``hs_hagg_extract`` compacts occupied slots into dense arrays (and resets them, so tables are
   reused without a memset).  With ``ORDER BY <expr> LIMIT k`` the top-k candidates are picked on
   the device (order-preserving images, LDS bitonic top-k, ties at the k-th value kept) and only
   those rows cross PCIe; the host finishes the exact multi-key sort over them.

A table that overflows its probe budget (more groups than the size guess) sets a flag, is
re-sized 4x and the query re-runs; the size that worked is remembered per query shape.
Reference: the rules only swap scans (JoinIndexRule.scala:63-69, RuleUtils.scala:264-292), Spark
runs every operator above them; ``E2EHyperspaceRulesTest.scala:1004-1019`` checks full results.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import pyarrow as pa

from ..ops import _lib as NL
from .compile import Unsupported

EMPTY = (1 << 64) - 1
# table slots per group seen on the previous run of a query shape (HS_HAGG_SLOTS_PER_GROUP)
SLOTS_PER_GROUP = float(os.environ.get("HS_HAGG_SLOTS_PER_GROUP", "2"))
MIN_SLOTS = 1 << 12
MAX_SLOTS = 1 << 29
_INT_TYPES = (NL.I8, NL.I16, NL.I32, NL.I64, NL.U32, NL.BOOL)


@dataclass
class KeyCol:
    slot: int            # kernel column slot
    attr: object         # the grouping attribute (output)
    kind: str            # "int" | "f32" | "f64"
    nullable: bool
    lo: int = 0
    bits: int = 0
    shift: int = 0
    dictionary: Optional[pa.Array] = None
    atype: Optional[pa.DataType] = None
    scale: float = 0.0   # kind "dec": value = (lo + code) / scale


class KeyPlan:
    """Packing of a query's group columns into the hash table's 64-bit key."""

    def __init__(self, cols: List[KeyCol], mode: str, own_counts: Tuple[bool, ...],
                 need_star: bool = True):
        self.cols = cols
        self.mode = mode                  # "packed" | "raw_int" | "raw_float"
        self.own_counts = own_counts      # per aggregate: its own non-null count is kept
        # the implicit COUNT(*) is accumulated only when a result reads it (COUNT / AVG);
        # otherwise every stored group counts as one row (groups exist only with rows)
        self.need_star = need_star
        self.slots = [c.slot for c in cols]

    def shape(self) -> tuple:
        return (self.mode, tuple((c.slot, c.kind, c.nullable) for c in self.cols),
                self.own_counts, self.need_star)

    def values(self) -> Dict[str, int]:
        v = {}
        if self.mode == "packed":
            for j, c in enumerate(self.cols):
                v[f"HL{j}"] = c.lo
                v[f"HS{j}"] = c.shift
                if c.kind == "dec":
                    v[f"HQ{j}"] = c.scale
        return v

    # -- host decode ---------------------------------------------------------------------------
    def unpack(self, keys: np.ndarray, nulls: np.ndarray) -> List[pa.Array]:
        out = []
        if self.mode != "packed":
            c = self.cols[0]
            mask = nulls.astype(bool) if c.nullable else None
            if self.mode == "raw_float":
                vals = keys.view(np.float64)
            else:
                vals = keys.view(np.int64)
            out.append(_to_arrow(c, vals, mask))
            return out
        for c in self.cols:
            m = np.uint64((1 << c.bits) - 1) if c.bits < 64 else np.uint64(EMPTY)
            code = (keys >> np.uint64(c.shift)) & m if c.bits else np.zeros_like(keys)
            mask = None
            if c.nullable:
                mask = code == 0
                code = code - np.uint64(1)
            if c.kind == "f32":
                vals = code.astype(np.uint32).view(np.float32).astype(np.float64)
            elif c.kind == "dec":
                # the decode the kernels and the encoder verified: (lo + code) / scale
                vals = (code.astype(np.int64) + np.int64(c.lo)).astype(np.float64) / c.scale
            else:
                vals = code.astype(np.int64) + np.int64(c.lo)
            if mask is not None:
                vals = np.where(mask, 0, vals)
            out.append(_to_arrow(c, vals, mask))
        return out


def _to_arrow(c: KeyCol, vals: np.ndarray, mask) -> pa.Array:
    t = c.atype
    if c.dictionary is not None:
        codes = pa.array(vals.astype(np.int32), mask=mask)
        return c.dictionary.take(codes)
    if c.kind in ("f32", "f64", "dec"):
        arr = pa.array(vals.astype(np.float64), mask=mask)
        return arr.cast(t) if t is not None and not pa.types.is_float64(t) else arr
    arr = pa.array(vals.astype(np.int64), mask=mask)
    if t is None or pa.types.is_int64(t):
        return arr
    if pa.types.is_date32(t):
        return pa.array(vals.astype(np.int32), mask=mask).view(pa.date32())
    if pa.types.is_timestamp(t):
        return arr.view(pa.int64()).cast(t)
    if pa.types.is_boolean(t):
        return pa.array(vals.astype(bool), mask=mask)
    try:
        return arr.cast(t)
    except (pa.ArrowInvalid, pa.ArrowNotImplementedError):
        return arr


def plan_keys(items, own_counts, need_star: bool = True) -> KeyPlan:
    """``items``: (slot, attr, DeviceColumn, (lo, span)) per group column, in GROUP BY order;
    the domain covers every part and rank (span 0 = no non-null values), so all launches of a
    query (bucket-union parts, ranks) pack keys identically."""
    cols: List[KeyCol] = []
    for slot, attr, c, _ in items:
        nullable = c.valid is not None
        if c.offsets is not None:
            raise Unsupported("raw string group key")
        if c.dictionary is not None:
            kind = "int"
        elif c.hs_type == NL.F64:
            kind = "f64"
        elif c.hs_type == NL.F32:
            kind = "f32"
        elif c.hs_type in _INT_TYPES:
            kind = "int"
        else:
            raise Unsupported(f"group key type {c.atype}")
        cols.append(KeyCol(slot, attr, kind, nullable, dictionary=c.dictionary, atype=c.atype))
    if len(cols) == 1 and cols[0].kind in ("f64", "f32"):
        return KeyPlan(cols, "raw_float", own_counts, need_star)
    shift = 0
    for k, (_, _, c, dom) in zip(cols, items):
        if k.kind == "f64":
            # exact decimal column (exec/encoding.py): packs q = rint(x * scale) - lo
            if len(dom) < 3 or not dom[2]:
                raise Unsupported("float64 column without an exact decimal form in a "
                                  "multi-column group key")
            k.kind, k.scale = "dec", float(dom[2])
            k.lo = int(dom[0])
            k.bits = max(0, int(max(dom[1], 1) - 1 + (1 if k.nullable else 0)).bit_length())
        elif k.kind == "f32":
            k.lo, k.bits = 0, 32 + (1 if k.nullable else 0)
        elif k.dictionary is not None:
            k.lo, span = 0, max(len(k.dictionary), 1)
            k.bits = max(0, int(span - 1 + (1 if k.nullable else 0)).bit_length())
        else:
            lo, span = dom[0], dom[1]
            k.lo = int(lo)
            k.bits = max(0, int(max(span, 1) - 1 + (1 if k.nullable else 0)).bit_length())
        k.shift = shift
        shift += k.bits
    if shift > 64:
        if len(cols) == 1 and cols[0].kind == "int":
            return KeyPlan(cols, "raw_int", own_counts, need_star)
        raise Unsupported("group key does not pack into 64 bits")
    return KeyPlan(cols, "packed", own_counts, need_star)


# ------------------------------------------------------------------------------------------------
# Tables
# ------------------------------------------------------------------------------------------------
class HashTable:
    """One device hash table (M probe slots + 2 direct slots, NA aggregates per group, SoA).
    Tables are pooled per (M, NA, min/max) and always left clean by ``extract`` (reset)."""

    def __init__(self, M: int, NA: int, minmax: bool, device):
        import torch
        self.M, self.NA, self.minmax, self.device = M, NA, minmax, device
        n = (M + 2) * NA
        self.keys = torch.empty(M + 2, dtype=torch.int64, device=device)
        self.sums = torch.empty(n, dtype=torch.float64, device=device)
        self.cnts = torch.empty(n, dtype=torch.int64, device=device)
        self.mins = torch.empty(n, dtype=torch.float64, device=device) if minmax else None
        self.maxs = torch.empty(n, dtype=torch.float64, device=device) if minmax else None
        self.flag = torch.zeros(4, dtype=torch.int64, device=device)
        NL.check(NL.lib().hs_hagg_init(NL.ptr(self.keys), NL.ptr(self.sums), NL.ptr(self.cnts),
                                       NL.ptr(self.mins), NL.ptr(self.maxs), M, NA,
                                       NL.stream_ptr()), "hs_hagg_init")

    def kernel_values(self) -> Dict[str, int]:
        return {"hkeys": self.keys.data_ptr(), "hsum": self.sums.data_ptr(),
                "hcnt": self.cnts.data_ptr(),
                "hmin": self.mins.data_ptr() if self.mins is not None else 0,
                "hmax": self.maxs.data_ptr() if self.maxs is not None else 0,
                "HM": self.M, "hflag": self.flag.data_ptr()}

    def extract(self, star: int) -> "Groups":
        """Stream-ordered: dense groups of this table (SoA, capacity M + 2 rows; the count ``G``
        stays on the device until ``Groups.count()``), the table reset for the next query."""
        import torch
        L = NL.lib()
        cap = self.M + 2
        g = Groups.alloc(self.NA, cap, self.minmax, self.device)
        ws = torch.empty(int(L.hs_hagg_extract_blocks(self.M)), dtype=torch.int64,
                         device=self.device)
        g.total = torch.empty(2, dtype=torch.int64, device=self.device)
        NL.check(L.hs_hagg_extract(NL.ptr(self.keys), NL.ptr(self.sums), NL.ptr(self.cnts),
                                   NL.ptr(self.mins), NL.ptr(self.maxs), self.M, self.NA, star, 1,
                                   NL.ptr(ws), NL.ptr(g.total), NL.ptr(self.flag), cap,
                                   NL.ptr(g.keys), NL.ptr(g.nulls), NL.ptr(g.sums),
                                   NL.ptr(g.cnts), NL.ptr(g.mins), NL.ptr(g.maxs),
                                   NL.stream_ptr()), "hs_hagg_extract")
        return g


class Groups:
    """Dense per-group arrays on the device (SoA, row stride ``cap``): keys (u64 bits), nulls
    (raw single-column NULL key), and NA (sum, count, min, max) partials per group."""

    def __init__(self, NA: int, cap: int, device):
        self.NA, self.cap, self.device = NA, cap, device
        self.keys = self.nulls = self.sums = self.cnts = self.mins = self.maxs = None
        self.total = None
        self._host_total = None

    @staticmethod
    def alloc(NA: int, cap: int, minmax: bool, device) -> "Groups":
        import torch
        g = Groups(NA, cap, device)
        c = max(cap, 1)
        g.keys = torch.empty(c, dtype=torch.int64, device=device)
        g.nulls = torch.empty(c, dtype=torch.uint8, device=device)
        g.sums = torch.empty(c * NA, dtype=torch.float64, device=device)
        g.cnts = torch.empty(c * NA, dtype=torch.int64, device=device)
        g.mins = torch.empty(c * NA, dtype=torch.float64, device=device) if minmax else None
        g.maxs = torch.empty(c * NA, dtype=torch.float64, device=device) if minmax else None
        return g

    def count(self) -> Tuple[int, bool]:
        if self._host_total is None:
            h = self.total.cpu().numpy()
            self._host_total = (int(h[0]), bool(h[1]))
        return self._host_total

    def set_count(self, n: int) -> None:
        self._host_total = (n, False)

    def _cols(self, t, G: int):
        """[G, NA] host array of a SoA device array (columns at stride cap)."""
        if t is None:
            return None
        return t.view(self.NA, self.cap)[:, :G].cpu().numpy().T

    def to_host(self, n: Optional[int] = None) -> dict:
        G = self.count()[0] if n is None else n
        out = {"keys": self.keys[:G].cpu().numpy().view(np.uint64),
               "nulls": self.nulls[:G].cpu().numpy(),
               "sums": self._cols(self.sums, G), "cnts": self._cols(self.cnts, G)}
        out["mins"] = self._cols(self.mins, G) if self.mins is not None else \
            np.full((G, self.NA), np.inf)
        out["maxs"] = self._cols(self.maxs, G) if self.maxs is not None else \
            np.full((G, self.NA), -np.inf)
        return out

    def take(self, rows, n: int) -> "Groups":
        """Groups ``rows[:n]`` (uint32 device indices) as a new dense set."""
        g = Groups.alloc(self.NA, max(n, 1), self.mins is not None, self.device)
        NL.check(NL.lib().hs_hagg_take(NL.ptr(rows), n, NL.ptr(self.keys), NL.ptr(self.nulls),
                                       NL.ptr(self.sums), NL.ptr(self.cnts), NL.ptr(self.mins),
                                       NL.ptr(self.maxs), self.NA, self.cap, g.cap,
                                       NL.ptr(g.keys), NL.ptr(g.nulls), NL.ptr(g.sums),
                                       NL.ptr(g.cnts), NL.ptr(g.mins), NL.ptr(g.maxs),
                                       NL.stream_ptr()), "hs_hagg_take")
        g.set_count(n)
        return g

    @staticmethod
    def from_host(host: dict, NA: int, minmax: bool, device) -> "Groups":
        """Dense groups uploaded from host arrays (keys u64, nulls u8, [G, NA] aggregates)."""
        import torch
        G = len(host["keys"])
        g = Groups(NA, max(G, 1), device)

        def soa(a, dt):
            return torch.from_numpy(np.ascontiguousarray(a.T).reshape(-1)).to(device) if G \
                else torch.zeros(NA, dtype=dt, device=device)
        g.keys = torch.from_numpy(host["keys"].view(np.int64).copy()).to(device) if G else \
            torch.zeros(1, dtype=torch.int64, device=device)
        g.nulls = torch.from_numpy(host["nulls"].astype(np.uint8)).to(device) if G else \
            torch.zeros(1, dtype=torch.uint8, device=device)
        g.sums = soa(host["sums"], torch.float64)
        g.cnts = soa(host["cnts"], torch.int64)
        g.mins = soa(host["mins"], torch.float64) if minmax else None
        g.maxs = soa(host["maxs"], torch.float64) if minmax else None
        g.set_count(G)
        return g


class TablePool:
    def __init__(self):
        self._tables: Dict[tuple, HashTable] = {}
        self.sizes: Dict[tuple, int] = {}     # query shape -> slots that held its groups

    def get(self, M: int, NA: int, minmax: bool, device) -> HashTable:
        k = (M, NA, minmax)
        t = self._tables.get(k)
        if t is None:
            # keep the pool bounded: tables of other sizes are dropped (re-created on demand)
            big = [x for x in self._tables if x[0] >= (1 << 24)]
            for x in big:
                del self._tables[x]
            t = HashTable(M, NA, minmax, device)
            self._tables[k] = t
        return t

    def slots_for(self, shape_key, estimate: int) -> int:
        M = self.sizes.get(shape_key)
        if M is None:
            M = next_pow2(max(MIN_SLOTS, min(2 * max(estimate, 1), 1 << 22)))
        return M

    def record(self, shape_key, M: int, groups: int) -> None:
        # next time: at least SLOTS_PER_GROUP x the groups seen (load <= 0.5 by default), never
        # below what worked
        want = next_pow2(max(MIN_SLOTS, int(SLOTS_PER_GROUP * groups)))
        self.sizes[shape_key] = max(want, min(M, want * 2))


def next_pow2(n: int) -> int:
    return 1 << max(0, int(n - 1).bit_length())


# ------------------------------------------------------------------------------------------------
# Top-k
# ------------------------------------------------------------------------------------------------
# image sources (csrc/kernels/hash_agg.hip topk_images_kernel)
SRC_SUM, SRC_COUNT, SRC_MIN, SRC_MAX, SRC_AVG, SRC_KEYFIELD, SRC_RAWINT, SRC_RAWFLT = range(8)


@dataclass
class OrderSource:
    src: int
    agg: int = 0
    cnt_slot: int = 0
    shift: int = 0
    mask: int = 0
    nullable: bool = False
    desc: bool = False


def topk_candidates(g: Groups, G: int, o: OrderSource, k: int) -> Tuple[Groups, int]:
    """The groups whose primary ORDER BY image is within the k smallest at 36-bit resolution (a
    superset of the top k under the full ordering: ties at the k-th image are all kept)."""
    import torch
    L = NL.lib()
    dev = g.device
    if G <= k:
        return g, G
    img = torch.empty(G, dtype=torch.int64, device=dev)
    NL.check(L.hs_topk_images(NL.ptr(g.keys), NL.ptr(g.nulls), NL.ptr(g.sums), NL.ptr(g.cnts),
                              NL.ptr(g.mins), NL.ptr(g.maxs), G, g.cap, o.src, o.agg, o.cnt_slot,
                              o.shift, C.c_uint64(o.mask), int(o.nullable), int(o.desc),
                              NL.ptr(img), NL.stream_ptr()), "hs_topk_images")
    ws = _topk_ws(dev)
    sel = torch.empty(G, dtype=torch.int32, device=dev)
    NL.check(L.hs_topk_select(NL.ptr(img), G, k, NL.ptr(ws["st"]), NL.ptr(ws["hist"]),
                              NL.ptr(sel), NL.ptr(ws["count"]), NL.stream_ptr()), "hs_topk_select")
    n = int(ws["count"].item())
    return g.take(sel, n), n


class TopKPlan:
    """ORDER BY <SUM or COUNT aggregate> LIMIT k over a key-run walk (jit_runs bits scan, hash
    mode): keys whose passing rows the walk sees whole keep their final aggregates in per-lane
    top-2 registers (jit._topk_insert: no cross-lane work and no memory traffic per key) instead
    of a hash-table slot.  At the end every wavefront writes its K best entries (key read from
    the entry's row only then) to its own K slots, its K-th best value and the largest value it
    dropped (jit._topk_flush; no atomics in the walk).  A small kernel
    (csrc/kernels/topk_runs.hip) reduces the wavefronts' K-th best and dropped values to the
    bound of every value the slots do not hold; the radix select of the table path
    (``topk_candidates``' hs_topk_select) picks the slots' top k from their images.  Values are
    compared in the "larger is better" image (negated for an ascending order).

    A lane keeps two entries and displaces a third, and a slot tie at a wavefront's K-th value
    may be left out: when that bound reaches the k-th best value overall the caller re-runs the
    exact table path (a tie, or three of the top k in one lane of one wavefront)."""
    K = 32          # slots per wavefront (16 for LIMIT <= 16: half the select's input)

    def __init__(self, agg: int, src_count: bool, desc: bool, NA: int, K: int = 32):
        assert K in (16, 32)
        self.agg, self.src_count, self.desc, self.NA = agg, src_count, desc, NA
        self.K = K
        self.nwv = 0
        self.cap = 0
        self.used = False

    def shape(self) -> tuple:
        return ("topk", self.agg, self.src_count, self.desc, self.K)

    def bind(self, nwv: int, device) -> None:
        """Slots for ``nwv`` wavefronts (the bits scan's grid)."""
        import torch
        if self.nwv == nwv and self.cap:
            return
        self.nwv, self.cap = nwv, nwv * self.K
        e = lambda n, t: torch.empty(n, dtype=t, device=device)  # noqa: E731
        self.keys, self.vimg = e(self.cap, torch.int64), e(self.cap, torch.int64)
        self.sums, self.cnts = e(self.cap * self.NA, torch.float64), e(self.cap * self.NA, torch.int64)
        self.wth, self.dmx = e(nwv, torch.int64), e(nwv, torch.int64)
        # [max K-th best, unused, max dropped value] (images of -inf, 0, -inf)
        neg_inf = int(np.array([-np.inf]).view(np.int64)[0]) ^ 0x7FFFFFFFFFFFFFFF
        self._ctl0 = torch.tensor([neg_inf, 0, neg_inf], dtype=torch.int64, device=device)
        self.ctl = e(3, torch.int64)

    def kernel_values(self) -> Dict[str, int]:
        return {"TKK": self.keys.data_ptr(), "TKV": self.vimg.data_ptr(),
                "TKS": self.sums.data_ptr(), "TKC": self.cnts.data_ptr(),
                "TKW": self.wth.data_ptr(), "TKD": self.dmx.data_ptr(), "TKCAP": self.cap}

    def finish(self, stream) -> None:
        """Queued after the walk: the bound over wavefronts."""
        self.ctl.copy_(self._ctl0, non_blocking=True)
        NL.check(NL.lib().hs_topk_runs_threshold(NL.ptr(self.wth), NL.ptr(self.dmx), self.nwv,
                                                 NL.ptr(self.ctl), stream),
                 "hs_topk_runs_threshold")

    @staticmethod
    def _unimg(v: int) -> float:
        bits = v if v >= 0 else v ^ 0x7FFFFFFFFFFFFFFF
        return float(np.array([bits], dtype=np.int64).view(np.float64)[0])

    OUT = 256       # candidates copied to the host (more: ties of the k-th value, exact path)

    def empty_image(self) -> int:
        """The slot image of an empty slot (-inf, complemented to smallest-first)."""
        neg = int(np.array([-np.inf]).view(np.int64)[0]) ^ 0x7FFFFFFFFFFFFFFF
        return (~(neg ^ (1 << 63))) & ((1 << 64) - 1)

    FD_COLS = 4     # right columns a device functional-dependency lookup returns

    def gather(self, g: "Groups", cnt_slot: int, k: int, fd: Optional[dict] = None) -> np.ndarray:
        """Queue the selection of the top ``k`` over the slots and the table's dense groups
        ``g`` (count on the device) - one image array, one radix select - and the packed copy
        of the candidates and bounds (csrc/kernels/topk_runs.hip); returns the host block (the
        query's one synchronization).  ``fd``: the functional-dependency lookup of the
        candidates' keys in the right table ({"raw", "lo", "shift", "mask", "key", "off", "nb",
        "cols"}, exec/gpu.py ``_fd_device``), queued before the copy into the same block."""
        import torch
        L = NL.lib()
        dev = self.keys.device
        n = self.cap + g.cap
        if getattr(self, "_img", None) is None or self._img.numel() < n:
            self._img = torch.empty(n, dtype=torch.int64, device=dev)
            self._sel = torch.empty(n, dtype=torch.int32, device=dev)
        if getattr(self, "_out", None) is None:
            self._out = torch.empty(self._fd_base() + self.OUT * (1 + 2 * self.FD_COLS),
                                    dtype=torch.int64, device=dev)
            self._host = torch.empty(self._out.numel(), dtype=torch.int64, pin_memory=True)
        ws = _topk_ws(dev)
        st = NL.stream_ptr()
        empty = C.c_uint64(self.empty_image())
        NL.check(L.hs_topk_runs_images(NL.ptr(self.vimg), NL.ptr(self.sums), NL.ptr(self.cnts),
                                       self.cap, empty, NL.ptr(g.sums), NL.ptr(g.cnts),
                                       NL.ptr(g.total), g.cap, self.agg, cnt_slot,
                                       int(self.src_count), int(self.desc), NL.ptr(self._img),
                                       st), "hs_topk_runs_images")
        NL.check(L.hs_topk_select(NL.ptr(self._img), n, k, NL.ptr(ws["st"]), NL.ptr(ws["hist"]),
                                  NL.ptr(self._sel), NL.ptr(ws["count"]), st), "hs_topk_select")
        NL.check(L.hs_topk_runs_gather(NL.ptr(self._sel), NL.ptr(ws["count"]), self.OUT,
                                       NL.ptr(self.keys), NL.ptr(self.vimg), NL.ptr(self.sums),
                                       NL.ptr(self.cnts), self.cap, empty, NL.ptr(g.keys),
                                       NL.ptr(g.nulls), NL.ptr(g.sums), NL.ptr(g.cnts), g.cap,
                                       NL.ptr(g.total), NL.ptr(self.ctl), self.NA,
                                       NL.ptr(self._out), st), "hs_topk_runs_gather")
        if fd is not None:
            cols = fd["cols"]
            descs = (NL.ColDesc * max(len(cols), 1))(*[c.desc() for c in cols])
            kd = fd["key"].desc()
            NL.check(L.hs_topk_runs_fd(NL.ptr(self._out), self.OUT, int(fd["raw"]), fd["lo"],
                                       fd["shift"], C.c_uint64(fd["mask"]), C.byref(kd),
                                       NL.ptr(fd["off"]), fd["nb"], descs, len(cols),
                                       self._out.data_ptr() + 8 * self._fd_base(), st),
                     "hs_topk_runs_fd")
        self._host.copy_(self._out, non_blocking=True)
        torch.cuda.current_stream(dev).synchronize()
        return self._host.numpy()

    def _fd_base(self) -> int:
        return 8 + self.OUT * (2 + 2 * self.NA)

    def unpack(self, blk: np.ndarray, nfd: int = 0) -> dict:
        """The host block of ``gather``: {"n" candidates selected, "bound" (the largest value
        the slots do not hold), "G" table groups, "over" table overflow, "host" group arrays of
        the live candidates (None when more than OUT), "empty" empty slots among them}."""
        O, NA = self.OUT, self.NA
        n = int(blk[0])
        out = {"n": n, "bound": max(self._unimg(int(blk[1])), self._unimg(int(blk[2]))),
               "G": int(blk[3]), "over": bool(blk[4]), "host": None, "empty": 0}
        if n > O:
            return out
        flag = blk[8 + O:8 + O + n]
        live = (flag & 2) == 0
        sums = np.stack([blk[8 + (2 + a) * O:8 + (2 + a) * O + n] for a in range(NA)], axis=1)
        cnts = np.stack([blk[8 + (2 + NA + a) * O:8 + (2 + NA + a) * O + n]
                         for a in range(NA)], axis=1)
        m = int(live.sum())
        out["empty"] = n - m
        out["host"] = {"keys": blk[8:8 + n][live].view(np.uint64).copy(),
                       "nulls": (flag[live] & 1).astype(np.uint8),
                       "sums": sums[live].view(np.float64).copy(),
                       "cnts": cnts[live].copy(),
                       "mins": np.full((m, NA), np.inf), "maxs": np.full((m, NA), -np.inf)}
        if nfd:
            b = self._fd_base()
            out["fd"] = (blk[b:b + n][live].copy(),
                         [blk[b + (1 + a) * O:b + (1 + a) * O + n][live].copy()
                          for a in range(nfd)],
                         [blk[b + (1 + nfd + a) * O:b + (1 + nfd + a) * O + n][live] != 0
                          for a in range(nfd)])
        return out

    def image(self, sums, cnts) -> "np.ndarray":
        """Order values of host group arrays in the kernel's image (larger is better)."""
        v = cnts[:, self.agg].astype(np.float64) if self.src_count else sums[:, self.agg]
        return v if self.desc else -v


_ZEROS: Dict[tuple, object] = {}


def _zeros_u8(n: int, dev):
    import torch
    z = _ZEROS.get((n, str(dev)))
    if z is None:
        z = _ZEROS[(n, str(dev))] = torch.zeros(n, dtype=torch.uint8, device=dev)
    return z


_TOPK_WS: Dict[object, dict] = {}


def _topk_ws(dev) -> dict:
    """Radix-select state + histogram (the kernels leave the histogram zeroed)."""
    import torch
    w = _TOPK_WS.get(dev)
    if w is None:
        w = {"st": torch.zeros(2, dtype=torch.int64, device=dev),
             "hist": torch.zeros(int(NL.lib().hs_topk_bins()), dtype=torch.int32, device=dev),
             "count": torch.zeros(1, dtype=torch.int64, device=dev)}
        _TOPK_WS[dev] = w
    return w


__all__ = ["KeyPlan", "KeyCol", "plan_keys", "HashTable", "Groups", "TablePool",
           "OrderSource", "topk_candidates", "TopKPlan", "Unsupported"]
