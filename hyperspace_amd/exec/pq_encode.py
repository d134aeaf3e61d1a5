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

Files are Parquet v1 (data page V1, UNCOMPRESSED or SNAPPY, optional flat columns); anything
outside that (nulls, booleans, decimals, timestamps, another codec) returns ``None`` so the
caller writes with pyarrow instead.
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


_ZSTREAMS: Dict[int, object] = {}


def compress_stream(device):
    """The stream index pages are Snappy-compressed on (one per device), next to the D2H copy
    stream that drains them."""
    import torch
    idx = device.index if device.index is not None else torch.cuda.current_device()
    st = _ZSTREAMS.get(idx)
    if st is None:
        st = _ZSTREAMS[idx] = torch.cuda.Stream(device=device)
    return st


# seconds of the last builds' write phases (reset by device_build per build)
WRITE_PHASES: Dict[str, float] = {}
_WP_LOCK = __import__("threading").Lock()


def _writer():
    from .jit import runtime
    L = runtime()
    if not getattr(L, "_hs_pqw", False):
        L.hs_pq_write_file.restype = C.c_int
        L.hs_pq_write_file.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_int64),
                                       C.POINTER(WCol), C.c_char_p]
        L._hs_pqw = True
    return L


def _physical(t: pa.DataType):
    """(Parquet physical type, logical 0/1 DATE/2 STRING, element bytes) or None."""
    if pa.types.is_date32(t):
        return 1, 1, 4
    if pa.types.is_int32(t):
        return 1, 0, 4
    if pa.types.is_int64(t):
        return 2, 0, 8
    if pa.types.is_float32(t):
        return 4, 0, 4
    if pa.types.is_float64(t):
        return 5, 0, 8
    if is_string(t):
        return 6, 2, 0
    return None


class ColPlan:
    def __init__(self, name: str, ptype: int, logical: int, eb: int):
        self.name = name
        self.bname = name.encode()
        self.ptype, self.logical, self.eb = ptype, logical, eb
        self.dict = False
        self.bw = 0
        self.dict_page: Optional[np.ndarray] = None
        self.dict_count = 0
        self.payload = None          # device uint8
        self.page_off: Optional[np.ndarray] = None   # byte offset of every page (+ end)

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
    lens = np.diff(offs)
    out = np.empty(int(lens.sum()) + 4 * len(a), dtype=np.uint8)
    pos = 0
    for i in range(len(a)):   # dictionaries are small (<= DICT_MAX_STRINGS)
        ln = int(lens[i])
        out[pos:pos + 4] = np.frombuffer(np.uint32(ln).tobytes(), dtype=np.uint8)
        out[pos + 4:pos + 4 + ln] = data[offs[i]:offs[i] + ln]
        pos += 4 + ln
    return out


def _dict_codes(v, eb: int, dbits, device):
    import torch
    codes = torch.empty(v.numel(), dtype=torch.int32, device=device)
    miss = torch.zeros(1, dtype=torch.int32, device=device)
    NL.check(NL.lib().hs_pq_dict_codes(v.data_ptr(), v.numel(), eb, dbits.data_ptr(),
                                       dbits.numel(), codes.data_ptr(), miss.data_ptr(),
                                       NL.stream_ptr()), "hs_pq_dict_codes")
    return codes, bool(miss.item())


def plan_columns(cols: Dict[str, DeviceColumn], names: Sequence[str], schema: pa.Schema,
                 pages: np.ndarray, device) -> Optional[List[ColPlan]]:
    """Encode every column on the device; None if some column needs the pyarrow writer."""
    import torch
    plans = []
    np_pages = pages
    gpre = np.concatenate([[0], np.cumsum((np_pages["n"] + 7) // 8)]).astype(np.int64)
    for name in names:
        dc = cols[name]
        phys = _physical(schema.field(name).type)
        if phys is None:
            return None
        if dc.valid is not None and bool((dc.valid == 0).any().item()):
            return None
        ptype, logical, eb = phys
        cp = ColPlan(name, ptype, logical, eb)
        codes = None
        if ptype == 6:
            d = dc.dictionary
            if d is None or len(d) == 0 or len(d) > DICT_MAX_STRINGS:
                return None
            codes = dc.data
            cp.dict_page = _string_dict_page(d)
            cp.dict_count = len(d)
        else:
            v = dc.data.view(torch.int32 if eb == 4 else torch.int64)
            n = v.numel()
            step = max(1, n // SAMPLE)
            u = torch.unique(v[::step])
            if 0 < u.numel() <= DICT_MAX // 2:
                codes, missed = _dict_codes(v, eb, u, device)
                if missed:
                    u = torch.unique(v)
                    codes = None
                    if u.numel() <= DICT_MAX:
                        codes, _ = _dict_codes(v, eb, u, device)
            if codes is not None:
                cp.dict_page = u.cpu().numpy().view(np.uint8)
                cp.dict_count = int(u.numel())
        if codes is not None:
            cp.dict = True
            cp.bw = _bit_width(cp.dict_count)
            sizes = ((np_pages["n"] + 7) // 8) * cp.bw
            cp.page_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
            tab = np_pages.copy()
            tab["out_off"] = cp.page_off[:-1]
            tab["gpre"] = gpre[:-1]
            dtab = torch.from_numpy(tab.view(np.uint8).copy()).to(device)
            cp.payload = torch.empty(int(cp.page_off[-1]) + 16, dtype=torch.uint8, device=device)
            NL.check(NL.lib().hs_pq_pack(codes.data_ptr(), dtab.data_ptr(), len(tab),
                                         int(gpre[-1]), cp.bw, cp.payload.data_ptr(),
                                         NL.stream_ptr()), "hs_pq_pack")
        else:
            cp.payload = dc.data.view(torch.uint8)
            cp.page_off = np.concatenate([np_pages["row0"], [np_pages["row0"][-1] +
                                                              np_pages["n"][-1]]]) * eb
        plans.append(cp)
    return plans


def page_table(bucket_off: np.ndarray, rg_rows: int) -> Tuple[np.ndarray, List[Tuple[int, int, int]]]:
    """Pages (= row groups) of every non-empty bucket and, per bucket, (bucket, first page,
    page count)."""
    rows, files = [], []
    for b in range(len(bucket_off) - 1):
        lo, hi = int(bucket_off[b]), int(bucket_off[b + 1])
        if hi <= lo:
            continue
        first = len(rows)
        for r0 in range(lo, hi, rg_rows):
            rows.append((r0, min(rg_rows, hi - r0), 0, 0))
        files.append((b, first, len(rows) - first))
    return np.array(rows, dtype=PAGE_DTYPE), files


def write_buckets(cols: Dict[str, DeviceColumn], names: Sequence[str], schema: pa.Schema,
                  bucket_off: np.ndarray, path_of: Callable[[int], str], rg_rows: int, device,
                  chunk_bytes: int = 96 << 20, codec: str = "none") -> Optional[List[str]]:
    """Encode on the device and write one Parquet file per non-empty bucket; None when the
    columns need the pyarrow writer.  ``codec`` "snappy" compresses every data page on the
    device (``snappy_pages``) and dictionary pages on the host."""
    import torch
    from .staging import copy_stream, io_pool, pinned_pool
    if codec not in CODEC_IDS:
        return None
    cid = CODEC_IDS[codec]
    pages, files = page_table(bucket_off, rg_rows)
    if not files:
        return []
    t_plan = time.perf_counter()
    plans = plan_columns(cols, names, schema, pages, device)
    WRITE_PHASES["plan_columns_s"] = WRITE_PHASES.get("plan_columns_s", 0.0) + \
        time.perf_counter() - t_plan
    if plans is None:
        return None
    for cp in plans:
        cp.dict_z = snappy_stream_host(cp.dict_page) if cid == 1 and cp.dict else None
    L = _writer()
    stream = copy_stream(device)
    stream.wait_stream(torch.cuda.current_stream(device))
    # group files into ~chunk_bytes of encoded data per D2H batch
    batches, cur, cur_bytes = [], [], 0
    for f in files:
        _, p0, pn = f
        nb = sum(int(cp.page_off[p0 + pn] - cp.page_off[p0]) for cp in plans)
        if cur and cur_bytes + nb > chunk_bytes:
            batches.append(cur)
            cur, cur_bytes = [], 0
        cur.append(f)
        cur_bytes += nb
    if cur:
        batches.append(cur)
    futs = []
    max_inflight = 2 * min(16, os.cpu_count() or 4)
    created_by = b"hyperspace_amd (MI355X device-encoded)"
    # Snappy: batches are compressed in groups of ~SNAPPY_GROUP_BYTES raw bytes, one launch each
    # (tens of thousands of 64 KiB chunks keep every CU busy); each batch then copies its slice
    # of the group's packed output
    groups = []
    if cid == 1:
        g, gb = [], 0
        for bi, batch in enumerate(batches):
            nb = sum(int(cp.page_off[batch[-1][1] + batch[-1][2]] - cp.page_off[batch[0][1]])
                     for cp in plans)
            if g and gb + nb > SNAPPY_GROUP_BYTES:
                groups.append(g)
                g, gb = [], 0
            g.append(bi)
            gb += nb
        if g:
            groups.append(g)
    group_of = {bi: gi for gi, g in enumerate(groups) for bi in g}
    zgroup = (-1, None)
    launched: Dict[int, _SnappyGroup] = {}
    zs = compress_stream(device) if cid == 1 else None

    def group_range(gi: int) -> Tuple[int, int]:
        gb0, gb1 = batches[groups[gi][0]], batches[groups[gi][-1]]
        return gb0[0][1], gb1[-1][1] + gb1[-1][2]
    for bi, batch in enumerate(batches):
        if len(futs) >= max_inflight:
            t_bp = time.perf_counter()
            futs[len(futs) - max_inflight].result()
            WRITE_PHASES["backpressure_s"] = WRITE_PHASES.get("backpressure_s", 0.0) + \
                time.perf_counter() - t_bp
        p_first = batch[0][1]
        p_end = batch[-1][1] + batch[-1][2]
        host = []
        zoff = zsize = None
        gfirst = 0
        with torch.cuda.stream(stream):
            if cid == 1:
                gi = group_of[bi]
                gfirst = group_range(gi)[0]
                if zgroup[0] != gi:
                    # compress this group (if not yet queued) and the next one on the
                    # compression stream: group g+1 compresses while g's pages are copied out
                    # and written
                    for gg in (gi, gi + 1):
                        if gg < len(groups) and gg not in launched:
                            zs.wait_stream(torch.cuda.current_stream(device))
                            with torch.cuda.stream(zs):
                                launched[gg] = snappy_launch(plans, *group_range(gg), device)
                    with torch.cuda.stream(zs):
                        res = snappy_finish(launched.pop(gi), device)
                        zev = torch.cuda.Event()
                        zev.record(zs)
                    stream.wait_event(zev)
                    res[0].record_stream(stream)
                    zgroup = (gi, res)
                packed, zoff, zsize = zgroup[1]
                for c in range(len(plans)):
                    lo = int(zoff[c][p_first - gfirst])
                    hi = int(zoff[c][p_end - 1 - gfirst] + zsize[c][p_end - 1 - gfirst])
                    h = pinned_pool().acquire(hi - lo)
                    if hi > lo:
                        h[:hi - lo].copy_(packed[lo:hi], non_blocking=True)
                    host.append((h, lo))
            else:
                for cp in plans:
                    lo, hi = int(cp.page_off[p_first]), int(cp.page_off[p_end])
                    h = pinned_pool().acquire(hi - lo)
                    if hi > lo:
                        h[:hi - lo].copy_(cp.payload[lo:hi], non_blocking=True)
                    host.append((h, lo))
            ev = torch.cuda.Event()
            ev.record(stream)

        def write_batch(batch=batch, host=host, ev=ev, zoff=zoff, zsize=zsize, gfirst=gfirst):
            t_w = time.perf_counter()
            ev.synchronize()
            t_s = time.perf_counter()
            out = []
            for b, p0, pn in batch:
                arr = (WCol * (pn * len(plans)))()
                rg = (C.c_int64 * pn)()
                for g in range(pn):
                    rg[g] = int(pages["n"][p0 + g])
                    for c, cp in enumerate(plans):
                        w = arr[g * len(plans) + c]
                        raw = int(cp.page_off[p0 + g + 1] - cp.page_off[p0 + g])
                        w.name = cp.bname
                        w.ptype, w.logical = cp.ptype, cp.logical
                        w.dict, w.bit_width = int(cp.dict), cp.bw
                        w.codec = cid
                        if cp.dict:
                            dp = cp.dict_z if cid == 1 else cp.dict_page
                            w.dict_page = dp.ctypes.data
                            w.dict_bytes = dp.nbytes
                            w.dict_raw_bytes = cp.dict_page.nbytes
                            w.dict_count = cp.dict_count
                        if cid == 1:
                            j = p0 + g - gfirst
                            h, base = host[c]
                            w.payload = h.data_ptr() + int(zoff[c][j]) - base
                            w.payload_bytes = int(zsize[c][j])
                        else:
                            h, base = host[c]
                            w.payload = h.data_ptr() + int(cp.page_off[p0 + g]) - base
                            w.payload_bytes = raw
                        w.payload_raw_bytes = raw
                path = path_of(b)
                rc = L.hs_pq_write_file(path.encode(), len(plans), pn, rg, arr, created_by)
                if rc != 0:
                    raise OSError(-rc, f"native Parquet write failed: {path}")
                out.append(path)
            for h, _ in host:   # written: the blocks can serve the next batch
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
