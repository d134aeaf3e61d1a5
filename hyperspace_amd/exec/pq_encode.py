"""Device-side Parquet encoding of index bucket files (SURVEY.md §2.3 K4 "Parquet encode
kernels"; host framing in ``csrc/runtime/hs_parquet_write.cpp``).

The sorted, bucket-major index columns are still in HBM when the build writes them, so the
encoding happens there:

* **dictionary build** — a strided sample of each fixed-width column is uniqued on the device;
  if it is small (``DICT_MAX``) every value is looked up in it by bit pattern
  (``hs_pq_dict_codes``; a miss falls back to a full device unique), giving int32 codes.
  String columns are already codes into a sorted host dictionary.
* **bit-packing** — ``hs_pq_pack`` writes one bit-packed run per data page (one page per bucket
  file row group).
* PLAIN columns (high cardinality) are their own payload.

Only the encoded bytes cross PCIe: for the TPC-H ``l_shipdate`` index (``l_discount`` 11
values, ``l_quantity`` 50, ``l_shipdate`` 2.5k) that is ~12 B/row instead of 28.  The host
writes each bucket file with ``pwritev`` straight from the pinned D2H buffers.

* **Snappy** (the default index codec, as Spark writes) — data pages are compressed on the device
  (``csrc/kernels/snappy_encode.hip``, ``snappy_pages``), so only compressed bytes cross PCIe;
  the small dictionary pages with the host build of the same match finder.

Files are Parquet v1 (data page V1, UNCOMPRESSED or SNAPPY, optional flat columns) with data
pages of at most ``PAGE_ROWS`` rows (so the device read path inflates one page per wavefront),
written by ``hs_pq_write_file2``.  Nullable columns carry their definition levels as one
bit-packed run per page (packed on the device from the validity bytes) and encode only their
non-null values.  Types: BOOLEAN (bit-packed PLAIN), INT8/INT16 (INT32 + INT logical type),
INT32, INT64, DATE, TIMESTAMP(ms/us/ns), DECIMAL up to 18 digits (INT64 + DECIMAL), FLOAT,
DOUBLE and dictionary strings.  Anything else (nested types, seconds timestamps, wider decimals,
string dictionaries over ``DICT_MAX_STRINGS``, another codec) returns ``None`` with the reason
in ``LAST_FALLBACK`` and the caller writes with pyarrow (``LAST_BUILD_STATS["writer"]``).
"""
from __future__ import annotations

import ctypes as C
import math
import os
import time
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import pyarrow as pa

from ..ops import _lib as NL
from .device_table import DeviceColumn, is_string

DICT_MAX = 4096          # fixed-width dictionaries (repeated in every row group's chunk)
DICT_MAX_STRINGS = 1 << 16
SAMPLE = 1 << 16

PAGE_DTYPE = np.dtype([("row0", "<i8"), ("n", "<i8"), ("out_off", "<i8"), ("gpre", "<i8")])


class WCol(C.Structure):
    _fields_ = [("name", C.c_char_p), ("ptype", C.c_int32), ("logical", C.c_int32),
                ("dict", C.c_int32), ("bit_width", C.c_int32), ("dict_page", C.c_void_p),
                ("dict_bytes", C.c_int64), ("dict_count", C.c_int64), ("payload", C.c_void_p),
                ("payload_bytes", C.c_int64), ("dict_raw_bytes", C.c_int64),
                ("payload_raw_bytes", C.c_int64), ("codec", C.c_int32), ("pad", C.c_int32)]


CODEC_IDS = {"none": 0, "uncompressed": 0, "snappy": 1}
# raw encoded bytes compressed per Snappy launch (slots take ~1.17x that in HBM)
SNAPPY_GROUP_BYTES = int(os.environ.get("HS_SNAPPY_GROUP_BYTES", str(2 << 30)))
SNAPPY_CHUNK_DTYPE = np.dtype([("src", "<u8"), ("len", "<i8")])


def _varint(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def snappy_stream_host(raw: np.ndarray) -> np.ndarray:
    """Whole Snappy stream (length preamble + elements) of a small host buffer, e.g. a
    dictionary page, with the host build of the device match finder."""
    L = NL.lib()
    raw = np.ascontiguousarray(raw, dtype=np.uint8)
    ch = int(L.hs_snappy_chunk_bytes())
    parts = [np.frombuffer(_varint(len(raw)), dtype=np.uint8)]
    for s in range(0, len(raw), ch):
        piece = raw[s:s + ch]
        buf = np.empty(int(L.hs_snappy_max_compressed(len(piece))), dtype=np.uint8)
        k = int(L.hs_snappy_compress_host(piece.ctypes.data, len(piece), buf.ctypes.data))
        if k < 0:
            raise RuntimeError("hs_snappy_compress_host failed")
        parts.append(buf[:k])
    return np.concatenate(parts)


class _SnappyGroup:
    """Device state of one compressed page group between ``snappy_launch`` and
    ``snappy_finish``."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def snappy_launch(plans, p_first: int, p_end: int, device) -> _SnappyGroup:
    """Queue the compression of pages [p_first, p_end) of every column on the current
    stream (no host wait): pages are cut into 64 KiB chunks, one wavefront each
    (csrc/kernels/snappy_encode.hip), into fixed-size slots."""
    import torch
    L = NL.lib()
    ch = int(L.hs_snappy_chunk_bytes())
    npg = p_end - p_first
    lo = np.stack([cp.page_off[p_first:p_end] for cp in plans]).astype(np.int64)
    hi = np.stack([cp.page_off[p_first + 1:p_end + 1] for cp in plans]).astype(np.int64)
    base = np.array([cp.payload.data_ptr() for cp in plans], dtype=np.uint64)
    plen = (hi - lo).reshape(-1)
    nchk = np.maximum(1, -(-plen // ch))
    first = np.concatenate([[0], np.cumsum(nchk)]).astype(np.int64)
    total = int(first[-1])
    page_of = np.repeat(np.arange(plen.size), nchk)
    k = np.arange(total, dtype=np.int64) - first[page_of]
    tab = np.empty(total, dtype=SNAPPY_CHUNK_DTYPE)
    src_page = (np.repeat(base, npg) + lo.reshape(-1).astype(np.uint64))
    tab["src"] = src_page[page_of] + (k * ch).astype(np.uint64)
    tab["len"] = np.minimum(ch, plen[page_of] - k * ch)
    slot = int(L.hs_snappy_max_compressed(ch))
    # pinned source: the chunk-table copy is queued, not waited for (a pageable copy would
    # block the host until the stream drains, serializing the groups)
    htab = torch.from_numpy(tab.view(np.uint8)).pin_memory()
    dtab = torch.empty(htab.numel(), dtype=torch.uint8, device=device)
    dtab.copy_(htab, non_blocking=True)
    slots = torch.empty(total * slot, dtype=torch.uint8, device=device)
    sizes = torch.empty(total, dtype=torch.int32, device=device)
    NL.check(L.hs_snappy_compress(dtab.data_ptr(), total, slots.data_ptr(), slot,
                                  sizes.data_ptr(), NL.stream_ptr()), "hs_snappy_compress")
    hsizes = torch.empty(total, dtype=torch.int32, pin_memory=True)
    hsizes.copy_(sizes, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    return _SnappyGroup(dtab=dtab, slots=slots, sizes=sizes, hsizes=hsizes, event=ev,
                        first=first, total=total, slot=slot, nplans=len(plans), npg=npg)


def snappy_finish(g: _SnappyGroup, device):
    """Wait for group ``g``'s chunk sizes, then pack the used slot bytes page by page on the
    current stream: (packed device buffer, offsets [col][page] into it, compressed sizes)."""
    import torch
    L = NL.lib()
    t_sync = time.perf_counter()
    g.event.synchronize()
    WRITE_PHASES["snappy_sync_s"] = WRITE_PHASES.get("snappy_sync_s", 0.0) + \
        time.perf_counter() - t_sync
    hsz = g.hsizes.numpy().astype(np.int64)
    dst = np.concatenate([[0], np.cumsum(hsz)]).astype(np.int64)
    zsize = np.add.reduceat(hsz, g.first[:-1]).reshape(g.nplans, g.npg)
    zoff = dst[g.first[:-1]].reshape(g.nplans, g.npg)
    out = torch.empty(max(1, int(dst[-1])), dtype=torch.uint8, device=device)
    hdst = torch.from_numpy(dst[:-1].copy()).pin_memory()
    ddst = torch.empty_like(hdst, device=device)
    ddst.copy_(hdst, non_blocking=True)
    NL.check(L.hs_snappy_pack(g.slots.data_ptr(), g.slot, g.sizes.data_ptr(), ddst.data_ptr(),
                              g.total, out.data_ptr(), NL.stream_ptr()), "hs_snappy_pack")
    return out, zoff, zsize


def snappy_pages(plans, p_first: int, p_end: int, device):
    """Compress pages [p_first, p_end) of every column on the device (current stream):
    returns (packed device buffer, offsets [col][page - p_first] into it, compressed sizes of
    the same shape).  The chunk sizes come back to the host once, then one pack launch
    concatenates the used slot bytes page by page."""
    return snappy_finish(snappy_launch(plans, p_first, p_end, device), device)


_ZSTREAMS: Dict[tuple, object] = {}
# compress streams the Snappy groups alternate over: group g is compressed AND copied out on
# stream g % Z, so one group's D2H (on the SDMA engines: a copy queued behind the kernel that
# produced it on the same stream) runs while the next group compresses on the other stream -
# with one stream the two serialize (profiles/build_timeline_r6.txt)
COMPRESS_STREAMS = max(1, int(os.environ.get("HS_PQ_ZSTREAMS", "2")))


def compress_stream(device, k: int = 0):
    """Compress stream ``k`` of the device: index pages are Snappy-compressed on it and, with
    ``D2H_ON_COMPRESS_STREAM``, copied out on it too."""
    import torch
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _ZSTREAMS.get((idx, k))
    if st is None:
        st = _ZSTREAMS[(idx, k)] = torch.cuda.Stream(device=device)
    return st


# copy streams the index pages leave HBM on (HS_PQ_D2H_STREAMS)
D2H_STREAMS = int(os.environ.get("HS_PQ_D2H_STREAMS", "2"))
# Snappy pages: copy them out on the compressor's own stream.  Issued on the copy streams the
# D2H copies ran as blit kernels on the CUs beside the compressor's waves (~18 GB/s,
# profiles/build_timeline_r5.txt); queued behind the compressor they run on the SDMA engines
# (profiles/build_copy_stats_sf100_r5_d2h_serial.csv)
D2H_ON_COMPRESS_STREAM = os.environ.get("HS_PQ_D2H_ON_COMPRESS", "1") == "1"
# seconds of the last builds' write phases (reset by device_build per build)
WRITE_PHASES: Dict[str, float] = {}
_WP_LOCK = __import__("threading").Lock()


class WPage(C.Structure):
    _fields_ = [("levels", C.c_void_p), ("levels_bytes", C.c_int64), ("levels_raw", C.c_int64),
                ("payload", C.c_void_p), ("payload_bytes", C.c_int64), ("payload_raw", C.c_int64),
                ("nvals", C.c_int64), ("nonnull", C.c_int64)]


class WCol2(C.Structure):
    _fields_ = [("name", C.c_char_p), ("ptype", C.c_int32), ("logical", C.c_int32),
                ("lp0", C.c_int32), ("lp1", C.c_int32), ("dict", C.c_int32),
                ("bit_width", C.c_int32), ("codec", C.c_int32), ("nullable", C.c_int32),
                ("dict_page", C.c_void_p), ("dict_bytes", C.c_int64), ("dict_count", C.c_int64),
                ("dict_raw_bytes", C.c_int64), ("null_count", C.c_int64),
                ("pages", C.POINTER(WPage)), ("npages", C.c_int32), ("pad", C.c_int32)]


def _writer():
    from .jit import runtime
    L = runtime()
    if not getattr(L, "_hs_pqw", False):
        L.hs_pq_write_file2.restype = C.c_int
        L.hs_pq_write_file2.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_int64),
                                        C.POINTER(WCol2), C.c_char_p]
        L._hs_pqw = True
    return L


# last reason write_buckets handed a build to the pyarrow writer (None: it wrote on the device)
LAST_FALLBACK: Dict[str, Optional[str]] = {"reason": None}
_TS_UNITS = {"ms": 0, "us": 1, "ns": 2}


class _Phys:
    """Parquet physical type, logical annotation and the device conversion of one column."""
    __slots__ = ("ptype", "logical", "lp0", "lp1", "eb", "conv")

    def __init__(self, ptype, logical=0, lp0=0, lp1=0, eb=0, conv=None):
        self.ptype, self.logical, self.lp0, self.lp1, self.eb, self.conv = \
            ptype, logical, lp0, lp1, eb, conv


def _physical(t: pa.DataType) -> Optional[_Phys]:
    """How column type ``t`` is written (physical type 0 BOOLEAN, 1 INT32, 2 INT64, 4 FLOAT,
    5 DOUBLE, 6 BYTE_ARRAY; logical 1 DATE, 2 STRING, 3 INT, 4 TIMESTAMP, 5 DECIMAL), or None
    when the device writer does not cover it."""
    if pa.types.is_boolean(t):
        return _Phys(0, eb=1, conv="bits")
    if pa.types.is_date32(t):
        return _Phys(1, 1, eb=4)
    if pa.types.is_int32(t):
        return _Phys(1, eb=4)
    if pa.types.is_int64(t):
        return _Phys(2, eb=8)
    if pa.types.is_int8(t) or pa.types.is_int16(t):
        return _Phys(1, 3, t.bit_width, 1, eb=4, conv="widen")
    if pa.types.is_float32(t):
        return _Phys(4, eb=4)
    if pa.types.is_float64(t):
        return _Phys(5, eb=8)
    if pa.types.is_timestamp(t) and t.unit in _TS_UNITS:
        return _Phys(2, 4, _TS_UNITS[t.unit], 1 if t.tz is not None else 0, eb=8)
    if pa.types.is_decimal(t) and t.precision <= 18 and t.bit_width == 128:
        return _Phys(2, 5, t.precision, t.scale, eb=8, conv="decimal")
    if is_string(t):
        return _Phys(6, 2)
    return None


class ColPlan:
    def __init__(self, name: str, ph: _Phys):
        self.name = name
        self.bname = name.encode()
        self.ph = ph
        self.ptype, self.logical, self.eb = ph.ptype, ph.logical, ph.eb
        self.dict = False
        self.bw = 0
        self.dict_page: Optional[np.ndarray] = None
        self.dict_count = 0
        self.fdict_page: List[np.ndarray] = []   # per file: its dictionary page (PLAIN values)
        self.fdict_count: List[int] = []
        self.fbw: List[int] = []                 # per file: code bit width
        self.fdict_z = None
        self.payload = None          # device uint8: the value segment of every page
        self.page_off: Optional[np.ndarray] = None   # byte offset of every page (+ end)
        self.nullable = False
        self.levels: Optional["_Seg"] = None          # definition-level bits of every page
        self.nonnull: Optional[np.ndarray] = None    # non-null rows of every page

    @property
    def encoded_bytes(self) -> int:
        return int(self.page_off[-1]) + (self.levels.encoded_bytes if self.levels else 0)


class _Seg:
    """A device byte buffer cut into per-page segments (the shape snappy_launch compresses)."""

    def __init__(self, payload, page_off: np.ndarray):
        self.payload, self.page_off = payload, page_off

    @property
    def encoded_bytes(self) -> int:
        return int(self.page_off[-1])


def _bit_width(n: int) -> int:
    return max(1, math.ceil(math.log2(max(n, 2))))


def _string_dict_page(d: pa.Array) -> np.ndarray:
    """PLAIN BYTE_ARRAY encoding of a string dictionary: (u32 length, bytes) per entry."""
    a = d.cast(pa.large_string()).combine_chunks() if isinstance(d, pa.ChunkedArray) else \
        d.cast(pa.large_string())
    bufs = a.buffers()
    offs = np.frombuffer(bufs[1], dtype=np.int64)[a.offset:a.offset + len(a) + 1]
    data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
    lens = np.diff(offs).astype(np.uint32)
    out = np.empty(int(lens.sum()) + 4 * len(a), dtype=np.uint8)
    # (u32 len, bytes) records: record i starts at its bytes offset plus 4 * i
    starts = (offs[:-1] - offs[0]) + 4 * np.arange(len(a), dtype=np.int64)
    hdr = lens.view(np.uint8).reshape(-1, 4)
    for k in range(4):
        out[starts + k] = hdr[:, k]
    body = np.repeat(starts + 4 - (offs[:-1] - offs[0]), lens.astype(np.int64))
    out[body + np.arange(int(lens.sum()), dtype=np.int64)] = data[offs[0]:offs[-1]]
    return out


def _dict_codes(v, eb: int, dbits, device):
    import torch
    codes = torch.empty(v.numel(), dtype=torch.int32, device=device)
    miss = torch.zeros(1, dtype=torch.int32, device=device)
    NL.check(NL.lib().hs_pq_dict_codes(v.data_ptr(), v.numel(), eb, dbits.data_ptr(),
                                       dbits.numel(), codes.data_ptr(), miss.data_ptr(),
                                       NL.stream_ptr()), "hs_pq_dict_codes")
    return codes, bool(miss.item())


def _pack(codes, rows0: np.ndarray, n: np.ndarray, bw, device):
    """Bit-pack int32 ``codes`` page by page (``hs_pq_pack``): page p packs codes
    [rows0[p], rows0[p] + n[p]) into ceil(n[p] / 8) * bw bytes (``bw`` an int, or an array of
    per-page widths); returns (device bytes, page byte offsets + end)."""
    import torch
    groups = (n + 7) // 8
    per_page = not np.isscalar(bw)
    sizes = groups * (np.asarray(bw, dtype=np.int64) if per_page else bw)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    gpre = np.concatenate([[0], np.cumsum(groups)]).astype(np.int64)
    tab = np.empty(len(n), dtype=PAGE_DTYPE)
    tab["row0"], tab["n"], tab["out_off"], tab["gpre"] = rows0, n, off[:-1], gpre[:-1]
    dtab = torch.from_numpy(tab.view(np.uint8).copy()).to(device)
    out = torch.empty(int(off[-1]) + 16, dtype=torch.uint8, device=device)
    dbw = None
    if per_page:
        bwa = np.asarray(bw, dtype=np.int32)
        if len(bwa) and (bwa.min() < 1 or bwa.max() > 16):
            raise ValueError("bit widths must be in 1..16")
        dbw = torch.from_numpy(bwa.copy()).to(device)
    if int(gpre[-1]):
        NL.check(NL.lib().hs_pq_pack(codes.data_ptr(), dtab.data_ptr(), len(tab), int(gpre[-1]),
                                     0 if per_page else bw,
                                     dbw.data_ptr() if dbw is not None else None,
                                     out.data_ptr(), NL.stream_ptr()), "hs_pq_pack")
    return out, off


def _file_dicts(codes, n_dict: int, fo: np.ndarray, device):
    """Per-file dictionaries (``hs_pq_dict_mark`` / ``hs_pq_dict_remap``): ``codes`` (int32,
    into a sorted job-wide dictionary of ``n_dict`` entries, rows of file f at [fo[f],
    fo[f + 1])) are rewritten in place as codes into the sorted subset file f uses; returns that
    subset per file (job-dictionary indices).  A file's encoded bytes then depend only on its
    own rows: one-pass, bucket-range-streamed and multi-rank builds write identical files, as
    Spark writes a dictionary per column chunk."""
    import torch
    L = NL.lib()
    nf = len(fo) - 1
    dw = (n_dict + 31) // 32
    n = int(fo[-1])
    present = torch.zeros(nf * dw, dtype=torch.int32, device=device)
    fo_d = torch.from_numpy(np.ascontiguousarray(fo, dtype=np.int64)).to(device)
    NL.check(L.hs_pq_dict_mark(codes.data_ptr(), fo_d.data_ptr(), nf, n, dw, present.data_ptr(),
                               NL.stream_ptr()), "hs_pq_dict_mark")
    bits = np.unpackbits(present.cpu().numpy().view(np.uint8), bitorder="little") \
        .reshape(nf, dw * 32)
    cnt = bits.reshape(nf, dw, 32).sum(2, dtype=np.int64)
    wpre = (np.cumsum(cnt, 1) - cnt).astype(np.int32)
    wpre_d = torch.from_numpy(wpre.reshape(-1).copy()).to(device)
    NL.check(L.hs_pq_dict_remap(codes.data_ptr(), fo_d.data_ptr(), nf, n, dw, present.data_ptr(),
                                wpre_d.data_ptr(), NL.stream_ptr()), "hs_pq_dict_remap")
    return [np.nonzero(bits[f])[0] for f in range(nf)]


def _values(dc: DeviceColumn, ph: _Phys):
    """The column's stored values as written: int8/int16 widened to int32, decimals (float64
    storage) as scaled int64 (exact for the precisions written: <= 18 digits), booleans as
    int32 0/1 for the bit packer."""
    import torch
    v = dc.data
    if ph.conv == "widen" or ph.conv == "bits":
        return v.to(torch.int32)
    if ph.conv == "decimal":
        return torch.round(v.double() * float(10 ** ph.lp1)).to(torch.int64)
    if ph.ptype == 6:
        return v
    return v.view(torch.int32 if ph.eb == 4 else torch.int64)


def plan_columns(cols: Dict[str, DeviceColumn], names: Sequence[str], schema: pa.Schema,
                 pages: np.ndarray, device, files=None) -> Optional[List[ColPlan]]:
    """Encode every column's pages on the device; None (reason in ``LAST_FALLBACK``) if some
    column needs the pyarrow writer.  Nullable columns get definition-level bits per page and
    only their non-null values encoded (RLE_DICTIONARY codes, PLAIN values or BOOLEAN bits).
    Dictionary columns get one dictionary per file of ``files`` (``page_table``; all pages one
    file when None): ``ColPlan.fdict_page`` / ``fdict_count`` / ``fbw`` per file index."""
    import torch
    plans = []
    n_pg = pages["n"].astype(np.int64)
    r0_pg = pages["row0"].astype(np.int64)
    if files is None:
        files = [(0, [(0, len(pages), int(n_pg.sum()))])]
    fpg = [_file_pages(f) for f in files]
    page_file = np.empty(len(pages), dtype=np.int64)
    for fi, (p0, p1) in enumerate(fpg):
        page_file[p0:p1] = fi
    for name in names:
        dc = cols[name]
        t = schema.field(name).type
        ph = _physical(t)
        if ph is None:
            LAST_FALLBACK["reason"] = f"column {name}: type {t}"
            return None
        cp = ColPlan(name, ph)
        v = _values(dc, ph)
        # definition levels: compact the non-null values, page bounds in compacted positions
        c0, m = r0_pg, n_pg
        if dc.valid is not None:
            vb = dc.valid != 0
            cnt = torch.cumsum(vb.to(torch.int64), 0)
            bounds = torch.from_numpy(np.concatenate([r0_pg, [r0_pg[-1] + n_pg[-1]]])).to(device)
            at = torch.where(bounds > 0, cnt.index_select(0, (bounds - 1).clamp(min=0)),
                             torch.zeros_like(bounds)).cpu().numpy()
            c0 = at[:-1]
            m = np.diff(at)
            if int(m.sum()) < int(n_pg.sum()):
                cp.nullable = True
                lev, loff = _pack(vb.to(torch.int32), r0_pg, n_pg, 1, device)
                cp.levels = _Seg(lev, loff)
                v = v.index_select(0, torch.nonzero(vb).squeeze(1))
        cp.nonnull = m
        codes = None
        if ph.ptype == 6:
            d = dc.dictionary
            if d is None or len(d) > DICT_MAX_STRINGS:
                LAST_FALLBACK["reason"] = f"column {name}: string dictionary over " \
                                          f"{DICT_MAX_STRINGS} entries"
                return None
            codes = v.to(torch.int32) if v.dtype != torch.int32 else v.clone()
            cp.dict_page = d
            cp.dict_count = len(d)
        elif ph.ptype == 0:
            out, off = _pack(v, c0, m, 1, device)
            cp.payload, cp.page_off = out, off
        elif v.numel():
            step = max(1, v.numel() // SAMPLE)
            u = torch.unique(v[::step])
            if 0 < u.numel() <= DICT_MAX // 2:
                codes, missed = _dict_codes(v, ph.eb, u, device)
                if missed:
                    u = torch.unique(v)
                    codes = None
                    if u.numel() <= DICT_MAX:
                        codes, _ = _dict_codes(v, ph.eb, u, device)
            if codes is not None:
                cp.dict_page = u.cpu().numpy()
                cp.dict_count = int(u.numel())
        if codes is not None:
            cp.dict = True
            codes = codes.to(torch.int32) if codes.dtype != torch.int32 else codes
            # file row ranges in this column's (non-null) value positions
            fo = np.array([c0[p0] for p0, _ in fpg] + [c0[fpg[-1][1] - 1] + m[fpg[-1][1] - 1]],
                          dtype=np.int64)
            subsets = _file_dicts(codes, cp.dict_count, fo, device) if cp.dict_count else \
                [np.zeros(0, np.int64)] * len(files)
            cp.fdict_page, cp.fdict_count, cp.fbw = [], [], []
            for idx in subsets:
                if ph.ptype == 6:
                    page = _string_dict_page(cp.dict_page.take(pa.array(idx, pa.int64()))) \
                        if len(idx) else _string_dict_page(pa.array([""], pa.string()))
                else:
                    # a file whose values are all null still gets a one-entry dictionary
                    page = cp.dict_page[idx].view(np.uint8) if len(idx) else \
                        np.zeros(ph.eb, np.uint8)
                cp.fdict_page.append(np.ascontiguousarray(page))
                cp.fdict_count.append(max(1, len(idx)))
                cp.fbw.append(_bit_width(max(1, len(idx))))
            cp.dict_page = None
            cp.bw = max(cp.fbw)
            cp.payload, cp.page_off = _pack(codes, c0, m, np.asarray(cp.fbw)[page_file], device)
        elif ph.ptype != 0:
            cp.payload = v.contiguous().view(torch.uint8) if v.numel() else \
                torch.zeros(16, dtype=torch.uint8, device=device)
            cp.page_off = np.concatenate([c0, [c0[-1] + m[-1]]]).astype(np.int64) * ph.eb
        plans.append(cp)
    LAST_FALLBACK["reason"] = None
    return plans


# footer ``created_by`` of the paged writer: readers take the device page decode for such files
CREATED_BY = "hyperspace_amd 2 (MI355X device-encoded, paged)"
# rows per data page: ~0.5 MiB of 8-byte PLAIN values, so a compressed page is one
# wavefront's inflate on the device read path (io/native_parquet.py upload_file_device)
PAGE_ROWS = int(os.environ.get("HS_PQ_PAGE_ROWS", str(1 << 16)))


def page_table(bucket_off: np.ndarray, rg_rows: int, page_rows: Optional[int] = None):
    """Data pages of every non-empty bucket: (pages, files) with ``files`` = per bucket
    (bucket, [(first page, page count, rows) per row group]).  Row groups hold ``rg_rows``
    rows, pages at most ``page_rows``."""
    rows, files = [], []
    page_rows = max(1, min(page_rows or PAGE_ROWS, rg_rows))
    for b in range(len(bucket_off) - 1):
        lo, hi = int(bucket_off[b]), int(bucket_off[b + 1])
        if hi <= lo:
            continue
        rgs = []
        for g0 in range(lo, hi, rg_rows):
            g1 = min(g0 + rg_rows, hi)
            first = len(rows)
            for r0 in range(g0, g1, page_rows):
                rows.append((r0, min(page_rows, g1 - r0), 0, 0))
            rgs.append((first, len(rows) - first, g1 - g0))
        files.append((b, rgs))
    return np.array(rows, dtype=PAGE_DTYPE), files


def _file_pages(f) -> Tuple[int, int]:
    """(first page, end page) of a file entry of ``page_table``."""
    rgs = f[1]
    return rgs[0][0], rgs[-1][0] + rgs[-1][1]


DMA_ALIGN = 256


def _dma_span(lo: int, hi: int, n: int) -> Tuple[int, int]:
    """[lo, hi) widened to DMA_ALIGN boundaries inside a device buffer of ``n`` bytes: a copy
    with an unaligned device offset goes through a blit kernel on the compute units (which
    then queues behind the compressor's waves) instead of an SDMA engine; the extra bytes are
    never read on the host (page addresses are taken relative to the returned ``lo``)."""
    if hi <= lo:
        return lo, hi
    return lo - lo % DMA_ALIGN, min(n, -(-hi // DMA_ALIGN) * DMA_ALIGN)


def write_buckets(cols: Dict[str, DeviceColumn], names: Sequence[str], schema: pa.Schema,
                  bucket_off: np.ndarray, path_of: Callable[[int], str], rg_rows: int, device,
                  chunk_bytes: int = 96 << 20, codec: str = "none") -> Optional[List[str]]:
    """Encode on the device and write one Parquet file per non-empty bucket; None when the
    columns need the pyarrow writer (reason in ``LAST_FALLBACK``).  ``codec`` "snappy"
    compresses every page segment on the device (``snappy_pages``) and dictionary pages on the
    host."""
    import torch
    from .staging import io_pool, pinned_pool
    if codec not in CODEC_IDS:
        LAST_FALLBACK["reason"] = f"codec {codec}"
        return None
    cid = CODEC_IDS[codec]
    pages, files = page_table(bucket_off, rg_rows)
    if not files:
        return []
    t_plan = time.perf_counter()
    plans = plan_columns(cols, names, schema, pages, device, files)
    WRITE_PHASES["plan_columns_s"] = WRITE_PHASES.get("plan_columns_s", 0.0) + \
        time.perf_counter() - t_plan
    if plans is None:
        return None
    for cp in plans:
        cp.fdict_z = [snappy_stream_host(dp) for dp in cp.fdict_page] \
            if cid == 1 and cp.dict else None
    file_index = {f[0]: fi for fi, f in enumerate(files)}
    # every device segment: each column's values, then the level bits of nullable columns
    segs = [cp for cp in plans] + [cp.levels for cp in plans if cp.levels is not None]
    lev_index = {}
    k = len(plans)
    for ci, cp in enumerate(plans):
        if cp.levels is not None:
            lev_index[ci] = k
            k += 1
    L = _writer()
    from .staging import copy_streams
    # batches alternate over D2H_STREAMS copy streams: their page copies run on separate DMA
    # queues instead of queueing behind one another
    d2h = copy_streams(device)[:max(1, D2H_STREAMS)]
    zsl = [compress_stream(device, k) for k in range(COMPRESS_STREAMS)] if cid == 1 else []
    if cid == 1 and D2H_ON_COMPRESS_STREAM:
        d2h = zsl
    for st in d2h + zsl:
        st.wait_stream(torch.cuda.current_stream(device))
    batches, cur, cur_bytes = [], [], 0
    for f in files:
        p0, p1 = _file_pages(f)
        nb = sum(int(sg.page_off[p1] - sg.page_off[p0]) for sg in segs)
        if cur and cur_bytes + nb > chunk_bytes:
            batches.append(cur)
            cur, cur_bytes = [], 0
        cur.append(f)
        cur_bytes += nb
    if cur:
        batches.append(cur)
    futs = []
    max_inflight = 2 * min(16, os.cpu_count() or 4)
    created_by = CREATED_BY.encode()
    groups = []
    if cid == 1:
        g, gb = [], 0
        for bi, batch in enumerate(batches):
            p0, p1 = _file_pages(batch[0])[0], _file_pages(batch[-1])[1]
            nb = sum(int(sg.page_off[p1] - sg.page_off[p0]) for sg in segs)
            if g and gb + nb > SNAPPY_GROUP_BYTES:
                groups.append(g)
                g, gb = [], 0
            g.append(bi)
            gb += nb
        if g:
            groups.append(g)
    group_of = {bi: gi for gi, g in enumerate(groups) for bi in g}
    zgroup = (-1, None, None)
    launched: Dict[int, _SnappyGroup] = {}

    def zs_of(g: int):
        return zsl[g % len(zsl)]

    def group_range(gi: int) -> Tuple[int, int]:
        return _file_pages(batches[groups[gi][0]][0])[0], \
            _file_pages(batches[groups[gi][-1]][-1])[1]
    for bi, batch in enumerate(batches):
        if len(futs) >= max_inflight:
            t_bp = time.perf_counter()
            futs[len(futs) - max_inflight].result()
            WRITE_PHASES["backpressure_s"] = WRITE_PHASES.get("backpressure_s", 0.0) + \
                time.perf_counter() - t_bp
        p_first = _file_pages(batch[0])[0]
        p_end = _file_pages(batch[-1])[1]
        host = []
        zoff = zsize = None
        gfirst = 0
        stream = d2h[bi % len(d2h)]
        if cid == 1 and D2H_ON_COMPRESS_STREAM:
            stream = zs_of(group_of[bi])     # the group's own compress stream (SDMA copies)
        with torch.cuda.stream(stream):
            if cid == 1:
                gi = group_of[bi]
                gfirst = group_range(gi)[0]
                if zgroup[0] != gi:
                    for gg in (gi, gi + 1):
                        if gg < len(groups) and gg not in launched:
                            with torch.cuda.stream(zs_of(gg)):
                                launched[gg] = snappy_launch(segs, *group_range(gg), device)
                    zs = zs_of(gi)
                    with torch.cuda.stream(zs):
                        res = snappy_finish(launched.pop(gi), device)
                        zev = torch.cuda.Event()
                        zev.record(zs)
                    for st in d2h:
                        res[0].record_stream(st)
                    zgroup = (gi, res, zev)
                stream.wait_event(zgroup[2])
                packed, zoff, zsize = zgroup[1]
                for c in range(len(segs)):
                    lo = int(zoff[c][p_first - gfirst])
                    hi = int(zoff[c][p_end - 1 - gfirst] + zsize[c][p_end - 1 - gfirst])
                    lo, hi = _dma_span(lo, hi, packed.numel())
                    h = pinned_pool().acquire(hi - lo)
                    if hi > lo:
                        h[:hi - lo].copy_(packed[lo:hi], non_blocking=True)
                    host.append((h, lo))
            else:
                for sg in segs:
                    lo, hi = int(sg.page_off[p_first]), int(sg.page_off[p_end])
                    lo, hi = _dma_span(lo, hi, sg.payload.numel())
                    h = pinned_pool().acquire(hi - lo)
                    if hi > lo:
                        h[:hi - lo].copy_(sg.payload[lo:hi], non_blocking=True)
                    host.append((h, lo))
            ev = torch.cuda.Event()
            ev.record(stream)

        def seg_page(si: int, q: int, host=None, zoff=None, zsize=None, gfirst=0):
            """(host address, bytes, raw bytes) of segment ``si`` of global page ``q``."""
            sg = segs[si]
            raw = int(sg.page_off[q + 1] - sg.page_off[q])
            h, base = host[si]
            if cid == 1:
                j = q - gfirst
                return h.data_ptr() + int(zoff[si][j]) - base, int(zsize[si][j]), raw
            return h.data_ptr() + int(sg.page_off[q]) - base, raw, raw

        def write_batch(batch=batch, host=host, ev=ev, zoff=zoff, zsize=zsize, gfirst=gfirst):
            t_w = time.perf_counter()
            ev.synchronize()
            t_s = time.perf_counter()
            out = []
            for b, rgs in batch:
                ncols, nrg = len(plans), len(rgs)
                arr = (WCol2 * (nrg * ncols))()
                rg = (C.c_int64 * nrg)()
                keep = []
                for g, (p0, pn, rows) in enumerate(rgs):
                    rg[g] = rows
                    for c, cp in enumerate(plans):
                        w = arr[g * ncols + c]
                        w.name = cp.bname
                        ph = cp.ph
                        w.ptype, w.logical, w.lp0, w.lp1 = ph.ptype, ph.logical, ph.lp0, ph.lp1
                        fi = file_index[b]
                        w.dict, w.bit_width = int(cp.dict), cp.fbw[fi] if cp.dict else cp.bw
                        w.codec, w.nullable = cid, int(cp.nullable)
                        if cp.dict:
                            dp = cp.fdict_z[fi] if cid == 1 else cp.fdict_page[fi]
                            w.dict_page = dp.ctypes.data
                            w.dict_bytes = dp.nbytes
                            w.dict_raw_bytes = cp.fdict_page[fi].nbytes
                            w.dict_count = cp.fdict_count[fi]
                        pgs = (WPage * pn)()
                        nulls = 0
                        for q in range(pn):
                            pg = pgs[q]
                            gq = p0 + q
                            pg.nvals = int(pages["n"][gq])
                            pg.nonnull = int(cp.nonnull[gq])
                            nulls += pg.nvals - pg.nonnull
                            pg.payload, pg.payload_bytes, pg.payload_raw = seg_page(
                                c, gq, host, zoff, zsize, gfirst)
                            if cp.levels is not None:
                                pg.levels, pg.levels_bytes, pg.levels_raw = seg_page(
                                    lev_index[c], gq, host, zoff, zsize, gfirst)
                        keep.append(pgs)
                        w.pages = C.cast(pgs, C.POINTER(WPage))
                        w.npages = pn
                        w.null_count = nulls
                path = path_of(b)
                rc = L.hs_pq_write_file2(path.encode(), ncols, nrg, rg, arr, created_by)
                if rc != 0:
                    raise OSError(-rc, f"native Parquet write failed: {path}")
                out.append(path)
            for h, _ in host:
                pinned_pool().release(h, torch.cuda.current_stream(device))
            with _WP_LOCK:
                WRITE_PHASES["writer_wait_d2h_s"] = WRITE_PHASES.get("writer_wait_d2h_s", 0.0) + \
                    t_s - t_w
                WRITE_PHASES["writer_write_s"] = WRITE_PHASES.get("writer_write_s", 0.0) + \
                    time.perf_counter() - t_s
            return out
        futs.append(io_pool().submit(write_batch))
    paths = []
    t_wait = time.perf_counter()
    for fu in futs:
        paths.extend(fu.result())
    WRITE_PHASES["write_tail_s"] = WRITE_PHASES.get("write_tail_s", 0.0) + \
        time.perf_counter() - t_wait
    return paths
