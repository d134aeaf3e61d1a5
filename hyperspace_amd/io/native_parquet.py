"""Native Parquet decode into HBM: host page layer in C++
(``csrc/runtime/hs_parquet.cpp``: footer/page-header Thrift parsing, Snappy, run tables) and
HIP kernels (``csrc/kernels/parquet_decode.hip``).

Device path (``upload_file_device``, default for source files; definition levels of chunks
with nulls decode on the device as well): the
host only preads the raw column chunks into one pinned block and walks the page headers; the
compressed bytes cross PCIe and two launches per batch of files decode them -
``hs_pq_inflate_kernel`` (Snappy, one wavefront per page, data-parallel tag parsing over
128-byte windows) and ``hs_pq_expand_kernel`` (RLE / bit-packed hybrid parsing, dictionary
gather or PLAIN copy, one workgroup per page).  Launches cover ~4 GB of files at once
(``decode_batch``): a page is one wavefront's serial work, so only many files' pages fill the
chip.  Large dictionary pages (and string dictionaries) are inflated on the host.

Index bucket files written by the device writer (``exec/pq_encode.py``: pages of at most
``PAGE_ROWS`` rows, ``created_by`` = ``pq_encode.CREATED_BY``) take the device path too
(``exec/device_cache.py`` checks the writer).  Host-page-layer path (``upload_file``: index
files of other writers, whose row-group-sized pages are too long for one wavefront's inflate,
and ``HS_PQ_DEVICE_NULLS=0`` for chunks with nulls):
per file every natively decodable column chunk is decompressed straight into one pinned
buffer, its RLE/bit-packed streams are cut into run tables, buffer and run tables cross PCIe
in two copies on the HIP copy stream, and the expansion kernels write the values into the
destination columns at the file's row offset.  Dictionary-encoded data crosses PCIe at its
encoded width (TPC-H ``l_quantity``: 6 bits/row instead of 64) and the host never
materialises decoded values.  Columns the page layer does not cover (strings, booleans,
decimals, timestamps, nested, non-Snappy codecs, DELTA encodings) are reported back so the
caller reads just those with pyarrow.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from typing import Dict, List, Optional, Sequence, Set

import numpy as np
import pyarrow as pa

OK, IO, CORRUPT, UNSUPPORTED, CAPACITY = 0, -1, -2, -3, -4

RUN_DTYPE = np.dtype([("dst", "<i8"), ("count", "<i8"), ("src", "<i8"), ("kind", "<i4"),
                      ("bit_width", "<i4")])
# HsPqPage (hs_parquet.cpp / parquet_decode.hip): one page of a device-decoded chunk
PAGE_DTYPE = np.dtype([("src", "<i8"), ("dst", "<i8"), ("out", "<i8"), ("dict", "<i8"),
                       ("row", "<i8"), ("csize", "<i4"), ("usize", "<i4"), ("nvals", "<i4"),
                       ("codec", "<i4"), ("kind", "<i4"), ("enc", "<i4"), ("levels", "<i4"),
                       ("eb", "<i4"), ("dict_page", "<i4"), ("nulls", "<i4"), ("valid", "<i8")])


class ChunkInfo(C.Structure):
    _fields_ = [("num_values", C.c_int64), ("num_nonnull", C.c_int64), ("dict_off", C.c_int64),
                ("dict_count", C.c_int64), ("bytes_used", C.c_int64),
                ("nvalue_runs", C.c_int64), ("nlevel_runs", C.c_int64),
                ("dict_encoded", C.c_int32), ("plain_pages", C.c_int32)]


# arrow type -> (Parquet physical type, element bytes) decodable as raw bits into our storage
def _native_kind(t: pa.DataType):
    if pa.types.is_string(t) or pa.types.is_large_string(t):
        return 6, 4                     # BYTE_ARRAY -> int32 dictionary codes (device path only)
    if pa.types.is_boolean(t):
        return 0, 1                     # BOOLEAN -> one byte per value (device path only)
    if pa.types.is_int32(t) or pa.types.is_date32(t):
        return 1, 4
    if pa.types.is_int64(t) or pa.types.is_timestamp(t) or pa.types.is_duration(t):
        # timestamps: INT64 in the unit the arrow type carries (the schema was read from the
        # file); INT96 timestamps have another physical type and stay on the host path
        return 2, 8
    if pa.types.is_float32(t):
        return 4, 4
    if pa.types.is_float64(t):
        return 5, 8
    return None


_L = None
_lock = threading.Lock()


def lib():
    global _L
    if _L is None:
        with _lock:
            if _L is None:
                from ..exec.jit import runtime
                L = runtime()
                P, I, I64 = C.c_void_p, C.c_int, C.c_int64
                for name, res, args in (
                        ("hs_pq_open", P, [C.c_char_p]), ("hs_pq_ok", I, [P]),
                        ("hs_pq_error", C.c_char_p, [P]), ("hs_pq_close", None, [P]),
                        ("hs_pq_num_rows", I64, [P]), ("hs_pq_num_row_groups", I, [P]),
                        ("hs_pq_row_group_rows", I64, [P, I]), ("hs_pq_num_columns", I, [P]),
                        ("hs_pq_find_column", I, [P, C.c_char_p]),
                        ("hs_pq_column_info", I, [P, I, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                                  C.POINTER(C.c_int)]),
                        ("hs_pq_chunk_bound", I64, [P, I, I]),
                        ("hs_pq_read_chunk", I, [P, I, I, P, I64, C.POINTER(ChunkInfo)]),
                        ("hs_pq_copy_runs", I, [P, P, P, I64, I64]),
                        ("hs_pq_run_size", I, []), ("hs_pq_info_size", I, []),
                        ("hs_pq_chunk_raw_bytes", I64, [P, I, I]),
                        ("hs_pq_chunk_max_pages", I64, [P, I, I]),
                        ("hs_pq_plan_chunk", I, [P, I, I, P, I64, I64, I64, P, I,
                                                 C.POINTER(C.c_int), C.POINTER(C.c_int64),
                                                 C.POINTER(C.c_int64), P, I64, I64,
                                                 C.POINTER(C.c_int64)]),
                        ("hs_pq_chunk_host_bound", I64, [P, I, I]),
                        ("hs_pq_page_size", I, []),
                        ("hs_pq_snappy_decompress", I64, [P, I64, P, I64]),
                        ("hs_pq_plain_strings", I64, [P, I64, I64, P, P, I64]),
                        ("hs_pq_set_host_inflate", None, [I]),
                        ("hs_pq_set_device_nulls", None, [I]),
                        ("hs_pq_set_plain_strings", None, [I])):
                    fn = getattr(L, name)
                    fn.restype = res
                    fn.argtypes = args
                # HS_PQ_HOST_INFLATE: which Snappy pages the planner inflates on the host
                # (0 none, 1 large dictionaries, 2 + tag-dense data pages, 3 two thirds of
                # those).  With batched launches and 128-byte windows the device inflates
                # tag-dense pages faster than 16 host threads (SF100 lineitem read + H2D
                # 0.34 s vs 0.42 s: profiles/build_sweep_inflate_r3_win128.jsonl)
                L.hs_pq_set_host_inflate(int(os.environ.get("HS_PQ_HOST_INFLATE", "1")))
                # HS_PQ_DEVICE_NULLS=0: chunks with nulls go through the host page layer
                # (strings: pyarrow) instead of decoding their definition levels on the device
                L.hs_pq_set_device_nulls(int(os.environ.get("HS_PQ_DEVICE_NULLS", "1")))
                # HS_PQ_PLAIN_STRINGS=0: PLAIN BYTE_ARRAY pages are read by pyarrow instead of
                # decoding to (address, length) pairs on the device
                L.hs_pq_set_plain_strings(int(os.environ.get("HS_PQ_PLAIN_STRINGS", "1")))
                if L.hs_pq_run_size() != RUN_DTYPE.itemsize or \
                        L.hs_pq_info_size() != C.sizeof(ChunkInfo) or \
                        L.hs_pq_page_size() != PAGE_DTYPE.itemsize:
                    raise RuntimeError("hs_parquet ABI mismatch: rebuild the native runtime")
                _L = L
    return _L


class PqFile:
    """Footer-level view of one Parquet file through the native page layer."""

    def __init__(self, path: str):
        self.L = lib()
        self.h = self.L.hs_pq_open(path.encode())
        self.path = path

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def close(self):
        if self.h:
            self.L.hs_pq_close(self.h)
            self.h = None

    @property
    def ok(self) -> bool:
        return bool(self.L.hs_pq_ok(self.h))

    @property
    def error(self) -> str:
        return self.L.hs_pq_error(self.h).decode()

    @property
    def num_rows(self) -> int:
        return int(self.L.hs_pq_num_rows(self.h))

    @property
    def num_row_groups(self) -> int:
        return int(self.L.hs_pq_num_row_groups(self.h))

    def row_group_rows(self, rg: int) -> int:
        return int(self.L.hs_pq_row_group_rows(self.h, rg))

    def column(self, name: str) -> int:
        return int(self.L.hs_pq_find_column(self.h, name.encode()))

    def column_info(self, col: int):
        t, d, e = C.c_int(), C.c_int(), C.c_int()
        self.L.hs_pq_column_info(self.h, col, C.byref(t), C.byref(d), C.byref(e))
        return t.value, d.value, e.value

    def read_chunk_host(self, rg: int, col: int):
        """Host-only read of one chunk (tests / debugging): (buffer, info, value runs, level
        runs)."""
        bound = int(self.L.hs_pq_chunk_bound(self.h, rg, col))
        buf = np.zeros(bound + 64, dtype=np.uint8)
        info = ChunkInfo()
        rc = self.L.hs_pq_read_chunk(self.h, rg, col, buf.ctypes.data, bound, C.byref(info))
        if rc != OK:
            return rc, None, None, None, None
        v = np.empty(info.nvalue_runs, dtype=RUN_DTYPE)
        lv = np.empty(info.nlevel_runs, dtype=RUN_DTYPE)
        self.L.hs_pq_copy_runs(self.h, v.ctypes.data, lv.ctypes.data, 0, 0)
        return rc, buf, info, v, lv


def expand_host(buf: np.ndarray, info: ChunkInfo, vruns: np.ndarray, lruns: np.ndarray,
                dtype: np.dtype):
    """Reference (numpy) expansion of a chunk's run tables — the oracle for the HIP kernels."""
    eb = dtype.itemsize
    dense = np.zeros(info.num_nonnull, dtype=dtype)
    dict_vals = None
    if info.dict_off >= 0:
        dict_vals = buf[info.dict_off:info.dict_off + info.dict_count * eb].view(dtype)
    for r in vruns:
        dst, cnt, src, kind, bw = (int(r["dst"]), int(r["count"]), int(r["src"]),
                                   int(r["kind"]), int(r["bit_width"]))
        if kind == 2:
            dense[dst:dst + cnt] = buf[src:src + cnt * eb].view(dtype)
        elif kind == 0:
            dense[dst:dst + cnt] = dict_vals[src]
        else:
            idx = _unpack(buf, src, cnt, bw)
            dense[dst:dst + cnt] = dict_vals[idx]
    valid = None
    if info.nlevel_runs:
        valid = np.zeros(info.num_values, dtype=np.uint8)
        for r in lruns:
            dst, cnt, src, kind, bw = (int(r["dst"]), int(r["count"]), int(r["src"]),
                                       int(r["kind"]), int(r["bit_width"]))
            valid[dst:dst + cnt] = (src != 0) if kind == 0 else (_unpack(buf, src, cnt, bw) != 0)
    return dense, valid


def _unpack(buf: np.ndarray, src: int, cnt: int, bw: int) -> np.ndarray:
    nbytes = (cnt * bw + 7) // 8
    bits = np.unpackbits(buf[src:src + nbytes], bitorder="little")[:cnt * bw]
    bits = bits.reshape(cnt, bw).astype(np.uint64)
    return (bits << np.arange(bw, dtype=np.uint64)).sum(axis=1).astype(np.int64)


# ------------------------------------------------------------------------------------------------
def upload_file(path: str, fields: Sequence[pa.Field], cols: Dict[str, object], lo: int, n_all: int,
                stream, device, valid_lock: threading.Lock) -> Set[str]:
    """Decode the natively supported ``fields`` of ``path`` into ``cols[name].data[lo:...]``.

    Returns the names decoded; the caller reads the others.  All device work is enqueued on
    ``stream`` (the staging copy stream)."""
    import torch
    from ..ops import _lib as NL
    f = PqFile(path)
    try:
        if not f.ok:
            return set()
        L = f.L
        plan = []
        for fld in fields:
            kind = _native_kind(fld.type)
            if kind is None or kind[0] in (0, 6):
                continue
            c = f.column(fld.name)
            if c < 0:
                continue
            ptype, _, eb = f.column_info(c)
            if eb == 0 or ptype != kind[0]:
                continue
            plan.append((fld, c, eb))
        if not plan:
            return set()
        nrg = f.num_row_groups
        rg_off = np.concatenate([[0], np.cumsum([f.row_group_rows(g) for g in range(nrg)])])
        bounds = [[int(L.hs_pq_chunk_bound(f.h, g, c)) for g in range(nrg)] for _, c, _ in plan]
        total = sum(sum((b + 15) // 16 * 16 for b in bl) for bl in bounds) + 64
        from ..exec.staging import pinned_pool
        pool = pinned_pool()
        pinned = pool.acquire(total)
        base = pinned.data_ptr()
        off = 0
        chunks = []
        vparts: List[np.ndarray] = []
        lparts: List[np.ndarray] = []
        nv = nl = 0
        done: Set[str] = set()
        for (fld, c, eb), bl in zip(plan, bounds):
            mine = []
            ok = True
            for g in range(nrg):
                info = ChunkInfo()
                rc = L.hs_pq_read_chunk(f.h, g, c, base + off, bl[g], C.byref(info))
                if rc == UNSUPPORTED:
                    ok = False
                    break
                if rc != OK:
                    raise IOError(f"{path}: native Parquet read failed ({rc}) on column "
                                  f"{fld.name}, row group {g}")
                v = np.empty(info.nvalue_runs, dtype=RUN_DTYPE)
                lv = np.empty(info.nlevel_runs, dtype=RUN_DTYPE)
                L.hs_pq_copy_runs(f.h, v.ctypes.data, lv.ctypes.data, off, 0)
                mine.append((g, info, off, v, lv))
                off += (info.bytes_used + 15) // 16 * 16
            if not ok:
                continue
            for g, info, boff, v, lv in mine:
                if info.num_values != rg_off[g + 1] - rg_off[g]:
                    raise IOError(f"{path}: column {fld.name} row group {g} has "
                                  f"{info.num_values} values, footer says "
                                  f"{rg_off[g + 1] - rg_off[g]}")
                chunks.append((fld, eb, g, info, boff, nv, len(v), nl, len(lv)))
                vparts.append(v)
                lparts.append(lv)
                nv += len(v)
                nl += len(lv)
            done.add(fld.name)
        if not done:
            pool.release(pinned, stream)
            return set()
        runs = np.concatenate(vparts + lparts) if (nv + nl) else np.empty(0, RUN_DTYPE)
        pruns = pool.acquire(max(runs.nbytes, 8))
        pruns.numpy()[:runs.nbytes] = runs.view(np.uint8)
        sp = stream.cuda_stream
        with torch.cuda.stream(stream):
            dbuf = torch.empty(off + 64, dtype=torch.uint8, device=device)
            dbuf[:off].copy_(pinned[:off], non_blocking=True)
            druns = torch.empty(max(runs.nbytes, 8), dtype=torch.uint8, device=device)
            druns.copy_(pruns[:druns.numel()], non_blocking=True)
            pool.release(pinned, stream)
            pool.release(pruns, stream)
            rsz = RUN_DTYPE.itemsize
            for fld, eb, g, info, boff, v0, vn, l0, ln in chunks:
                dc = cols[fld.name]
                row0 = lo + int(rg_off[g])
                rows = int(info.num_values)
                dst = dc.data[row0:row0 + rows]
                dict_off = info.dict_off + boff if info.dict_off >= 0 else -1
                if info.num_nonnull == rows:
                    NL.check(NL.lib().hs_pq_decode_values(
                        dbuf.data_ptr(), druns.data_ptr() + v0 * rsz, vn, dict_off,
                        info.dict_count, eb, dst.data_ptr(), sp), "hs_pq_decode_values")
                    continue
                dense = torch.empty(int(info.num_nonnull), dtype=dc.data.dtype, device=device)
                NL.check(NL.lib().hs_pq_decode_values(
                    dbuf.data_ptr(), druns.data_ptr() + v0 * rsz, vn, dict_off, info.dict_count,
                    eb, dense.data_ptr(), sp), "hs_pq_decode_values")
                from ..exec.staging import ensure_valid
                vslice = ensure_valid(dc, n_all, device, valid_lock)[row0:row0 + rows]
                NL.check(NL.lib().hs_pq_decode_levels(
                    dbuf.data_ptr(), druns.data_ptr() + (nv + l0) * rsz, ln,
                    vslice.data_ptr(), sp), "hs_pq_decode_levels")
                dst.zero_()
                dst.masked_scatter_(vslice.bool(), dense)
            # the device staging buffers must outlive the kernels queued on this stream
            dbuf.record_stream(stream)
            druns.record_stream(stream)
        return done
    finally:
        f.close()


NULLS = -5
# per-phase seconds summed over the staging threads (device decode path), reset per build
PHASES: Dict[str, float] = {}
_PH_LOCK = threading.Lock()


DMA_ALIGN = 256


def _dma_up(n: int) -> int:
    """``n`` rounded up to a DMA_ALIGN multiple: an H2D copy whose length or offsets are not
    256-byte aligned runs as a blit kernel on the compute queue instead of on an SDMA engine
    (``pq_encode._dma_span`` does the same for the encoded pages' D2H)."""
    return -(-int(n) // DMA_ALIGN) * DMA_ALIGN


def _phase(name: str, t0: float) -> float:
    import time
    t1 = time.perf_counter()
    with _PH_LOCK:
        PHASES[name] = PHASES.get(name, 0.0) + (t1 - t0)
    return t1


def plan_file(f: "PqFile", plan, raw_cap: int, raw_buf_ptr: int, host_cap: int = 0,
              host_buf_ptr: int = 0):
    """Plan every (field, column) of ``plan`` over all row groups of ``f``: pread raw chunks into
    the buffer at ``raw_buf_ptr``, inflate tag-dense pages into the one at ``host_buf_ptr`` (0:
    none, every page inflates on the device) and collect the page table.

    Returns (pages, chunks, raw_used, scratch_used, host_used, skipped): ``chunks`` = (field,
    row group, first page, npages); ``skipped`` = fields the device path cannot decode (possible
    nulls, unsupported encodings), to be decoded another way."""
    L = f.L
    nrg = f.num_row_groups
    maxp = sum(int(L.hs_pq_chunk_max_pages(f.h, g, c)) for _, c, _ in plan for g in range(nrg))
    pages = np.zeros(max(maxp, 1), dtype=PAGE_DTYPE)
    pbase = pages.ctypes.data
    chunks, skipped = [], set()
    raw_at = dst_at = h_at = npg = 0
    n = C.c_int()
    ru, du, hu = C.c_int64(), C.c_int64(), C.c_int64()
    for fld, c, eb in plan:
        mine, ok = [], True
        raw0, dst0, h0, npg0 = raw_at, dst_at, h_at, npg
        for g in range(nrg):
            rc = L.hs_pq_plan_chunk(f.h, g, c, raw_buf_ptr, raw_cap, raw_at, dst_at,
                                    pbase + npg * PAGE_DTYPE.itemsize, len(pages) - npg,
                                    C.byref(n), C.byref(ru), C.byref(du), host_buf_ptr or None,
                                    host_cap, h_at, C.byref(hu))
            if rc in (UNSUPPORTED, NULLS):
                ok = False
                break
            if rc != OK:
                raise IOError(f"{f.path}: device page plan failed ({rc}) on column {fld.name}, "
                              f"row group {g}")
            seg = pages[npg:npg + n.value]
            seg["dict_page"] = np.where(seg["dict_page"] >= 0, seg["dict_page"] + npg, -1)
            mine.append((fld, g, npg, n.value))
            npg += n.value
            raw_at += (ru.value + 15) // 16 * 16
            dst_at += (du.value + 15) // 16 * 16
            h_at += (hu.value + 15) // 16 * 16
        if ok:
            chunks += mine
        else:                                   # roll this column back
            skipped.add(fld.name)
            raw_at, dst_at, h_at, npg = raw0, dst0, h0, npg0
    return pages[:npg], chunks, raw_at, dst_at, h_at, skipped


_VALID_LOCK = threading.Lock()


class StringCodes:
    """One string column decoded on the device across the files of an upload.

    Every row-group chunk's dictionary page is parsed on the host (``hs_pq_plain_strings``) and
    given a range of codes ``[base, base + len)`` in one upload-wide code space (``add``, any
    thread); the data pages decode on the device to those codes.  ``concat`` is the dictionary
    of that code space; the caller maps it onto the job-global sorted dictionary with one device
    gather (``staging.finish_strings``).  ``host`` holds the arrow chunks of files whose pages the
    device path could not take, by file index.

    PLAIN-encoded data pages decode on the device to each value's address and length
    (``sptr`` / ``slen``, rows ``plain_rows``; the page buffers they point into are held in
    ``keep``); ``finish_plain`` hashes them into codes of a dictionary of their distinct values,
    read back from the device."""

    def __init__(self, main=None):
        self._lock = threading.Lock()
        self.size = 0
        self.parts: List[tuple] = []
        self.host: Dict[int, object] = {}
        self.main = main                  # the upload's consumer stream (allocations)
        self.sptr = self.slen = None
        self.plain_rows: List[tuple] = []
        self.keep: list = []

    def plain_arrays(self, n: int, device):
        """The column's (address int64, length int32) arrays, allocated on first need."""
        import torch
        with self._lock:
            if self.sptr is None:
                st = self.main if self.main is not None else torch.cuda.current_stream(device)
                with torch.cuda.stream(st):
                    self.sptr = torch.empty(n, dtype=torch.int64, device=device)
                    self.slen = torch.empty(n, dtype=torch.int32, device=device)
            return self.sptr, self.slen

    def add_plain(self, ranges, keep) -> None:
        with self._lock:
            self.plain_rows += ranges
            self.keep += keep

    def finish_plain(self, dc) -> None:
        """Codes of the PLAIN-page rows into ``dc.data`` (on the current stream, after the
        decode): a 64-bit hash per value (csrc/kernels/strings.hip), the distinct hashes, one
        representative value per hash copied to the host as a dictionary part, and a byte
        compare of every value with its representative - values whose hash collides with a
        different value's are resolved on the host (their bytes only)."""
        import torch
        import pyarrow.compute as pc
        from ..ops import kernels as K
        if not self.plain_rows:
            return
        dev = dc.data.device
        rr = np.array(sorted(self.plain_rows), dtype=np.int64).reshape(-1, 2)
        lens = rr[:, 1] - rr[:, 0]
        starts = torch.from_numpy(np.repeat(rr[:, 0] - np.concatenate([[0], np.cumsum(lens)[:-1]]),
                                            lens)).to(dev)
        idx = torch.arange(int(lens.sum()), dtype=torch.int64, device=dev) + starts
        if dc.valid is not None:
            idx = idx[dc.valid.index_select(0, idx) != 0]
        if idx.numel():
            ptr, ln = self.sptr.index_select(0, idx), self.slen.index_select(0, idx)
            h = K.str_hash64(ptr, ln)
            uh, inv = torch.unique(h, return_inverse=True)
            first = torch.full((uh.numel(),), idx.numel(), dtype=torch.int64, device=dev)
            first.scatter_reduce_(0, inv, torch.arange(idx.numel(), device=dev), "amin")
            rptr, rlen = ptr.index_select(0, first), ln.index_select(0, first)
            offh, chars = K.str_gather(rptr, rlen)
            arr = pa.Array.from_buffers(pa.string(), uh.numel(), [
                None, pa.py_buffer(offh.to(torch.int32).numpy()),
                pa.py_buffer(chars.cpu().numpy())])
            codes = inv + self.add(arr)
            bad = K.str_differ(ptr, ln, rptr.index_select(0, inv), rlen.index_select(0, inv))
            nb = int(bad.sum().item())
            if nb:
                # 64-bit hash collisions: these values get codes of their own
                sel = torch.nonzero(bad).squeeze(1)
                boff, bchars = K.str_gather(ptr.index_select(0, sel), ln.index_select(0, sel))
                vals = pa.Array.from_buffers(pa.string(), nb, [
                    None, pa.py_buffer(boff.to(torch.int32).numpy()),
                    pa.py_buffer(bchars.cpu().numpy())])
                d = pc.unique(vals)
                base = self.add(d)
                pos = pc.index_in(vals, value_set=d).to_numpy(zero_copy_only=False)
                codes[sel] = torch.from_numpy(pos.astype(np.int64) + base).to(dev)
            dc.data.index_copy_(0, idx, codes.to(torch.int32))
        self.sptr = self.slen = None
        self.keep = []
        self.plain_rows = []

    def add(self, arr: pa.Array) -> int:
        with self._lock:
            base = self.size
            self.size += len(arr)
            self.parts.append((base, arr))
            return base

    def concat(self) -> pa.Array:
        parts = [a for _, a in sorted(self.parts, key=lambda x: x[0])]
        return pa.concat_arrays(parts) if parts else pa.array([], pa.string())


def plain_strings(buf_ptr: int, nbytes: int, n: int) -> pa.Array:
    """Arrow string array of a PLAIN BYTE_ARRAY stream of ``n`` values at host ``buf_ptr``."""
    offs = np.empty(n + 1, dtype=np.int32)
    chars = np.empty(max(nbytes, 1), dtype=np.uint8)
    got = lib().hs_pq_plain_strings(buf_ptr, nbytes, n, offs.ctypes.data, chars.ctypes.data,
                                    len(chars))
    if got < 0:
        raise IOError("corrupt BYTE_ARRAY dictionary page")
    return pa.Array.from_buffers(pa.string(), n, [None, pa.py_buffer(offs),
                                                  pa.py_buffer(chars[:max(got, 1)])])


class PendingDecode:
    """One file's planned pages whose device decode is deferred into a batched launch
    (``decode_batch``): the page table (absolute device addresses), the device buffers the
    pages live in, and the event after their H2D copies."""

    def __init__(self, pages: np.ndarray, keep: list, event, nbytes: int):
        self.pages, self.keep, self.event, self.nbytes = pages, keep, event, nbytes


def decode_batch(pend: List["PendingDecode"], device, status, stream):
    """ONE launch pair decoding the pages of every file in ``pend`` on ``stream`` (after their
    H2D copies): a per-file launch covers a few hundred pages, too few wavefronts for 256 CUs
    when the pages are Snappy tag chains; a batch of files fills the chip.  Returns the event
    marking the decode done."""
    import torch
    from ..ops import _lib as NL
    from ..exec.staging import pinned_pool
    tables, base = [], 0
    for p in pend:
        t = p.pages.copy()
        t["dict_page"] = np.where(t["dict_page"] >= 0, t["dict_page"] + base, -1)
        tables.append(t)
        base += len(t)
        stream.wait_event(p.event)
    allp = np.concatenate(tables) if tables else np.zeros(0, PAGE_DTYPE)
    pool = pinned_pool()
    with torch.cuda.stream(stream):
        if len(allp):
            ppin = pool.acquire(allp.nbytes)
            ppin.numpy()[:allp.nbytes] = allp.view(np.uint8)
            dpages = torch.empty(allp.nbytes, dtype=torch.uint8, device=device)
            dpages.copy_(ppin[:allp.nbytes], non_blocking=True)
            pool.release(ppin, stream)
            NL.check(NL.lib().hs_pq_decode_pages(None, None, dpages.data_ptr(), len(allp),
                                                 status.data_ptr(), stream.cuda_stream),
                     "hs_pq_decode_pages")
            dpages.record_stream(stream)
        for p in pend:
            for x in p.keep:
                x.record_stream(stream)
        ev = torch.cuda.Event()
        ev.record(stream)
    return ev


def upload_file_device(path: str, fields: Sequence[pa.Field], cols: Dict[str, object], lo: int,
                       stream, device, status, strings: Optional[Dict[str, StringCodes]] = None,
                       defer: Optional[list] = None, lock=None) -> Set[str]:
    """Decode the natively supported ``fields`` of ``path`` entirely on the GPU into
    ``cols[name].data[lo:...]``: the host preads the raw column chunks into pinned memory and
    lists their pages; one H2D copy moves the compressed bytes and the page table, and two
    launches (``hs_pq_decode_pages``: Snappy inflate, then RLE / bit-packed / PLAIN expansion
    with the dictionary gather) write the values.  Errors accumulate in the device int
    ``status`` (checked once per build).  Returns the names decoded.

    String columns named in ``strings`` decode when every chunk is dictionary-encoded: the host
    parses only the (small) dictionary pages, the device expands the index pages through a
    per-chunk code table (``StringCodes``) into ``cols[name].data`` (int32).

    Chunks that may hold nulls decode their definition levels on the device too
    (``hs_pq_expand_kernel``: levels -> validity bytes, dense values spread to their rows, 0 at
    nulls); the column's validity mask is created on first need (``staging.ensure_valid`` under
    ``lock``)."""
    import time
    import torch
    from ..ops import _lib as NL
    from ..exec.staging import ensure_valid, pinned_pool
    t = time.perf_counter()
    f = PqFile(path)
    try:
        if not f.ok:
            return set()
        t = _phase("open", t)
        L = f.L
        plan = []
        for fld in fields:
            kind = _native_kind(fld.type)
            if kind is None:
                continue
            if kind[0] == 6 and (strings is None or fld.name not in strings):
                continue
            c = f.column(fld.name)
            if c < 0:
                continue
            ptype, _, eb = f.column_info(c)
            if kind[0] == 6 and ptype == 6:
                eb = 4
            elif kind[0] == 0 and ptype == 0:
                eb = 1
            if eb == 0 or ptype != kind[0]:
                continue
            plan.append((fld, c, eb))
        if not plan:
            return set()
        nrg = f.num_row_groups
        raw_cap = _dma_up(sum((int(L.hs_pq_chunk_raw_bytes(f.h, g, c)) + 15) // 16 * 16
                              for _, c, _ in plan for g in range(nrg)) + 64)
        host_cap = sum(int(L.hs_pq_chunk_host_bound(f.h, g, c)) + 16
                       for _, c, _ in plan for g in range(nrg))
        pool = pinned_pool()
        # one pinned block: [raw chunks | pages the planner inflates]
        pinned = pool.acquire(raw_cap + host_cap)
        t = _phase("pinned", t)
        pages, chunks, raw_used, scratch_bytes, host_used, skipped = plan_file(
            f, plan, raw_cap, pinned.data_ptr(), host_cap, pinned.data_ptr() + raw_cap)
        t = _phase("plan", t)
        if not chunks:
            pool.release(pinned, stream)
            return set()
        rg_off = np.concatenate([[0], np.cumsum([f.row_group_rows(g) for g in range(nrg)])])
        with torch.cuda.stream(stream):
            scratch = torch.empty(scratch_bytes + 64, dtype=torch.uint8, device=device)
            sbase = scratch.data_ptr()
            # device copy of the pinned block's used parts: raw chunks at 0, host-inflated
            # pages (tag-dense pages, large dictionaries) at raw_cap
            # both copies start and end on DMA_ALIGN boundaries (SDMA, not a blit kernel that
            # would queue behind the decode waves); the padding bytes are never read
            raw_n = min(_dma_up(raw_used), raw_cap)
            host_n = min(_dma_up(host_used), pinned.numel() - raw_cap)
            draw = torch.empty(raw_cap + _dma_up(host_used) + 64, dtype=torch.uint8,
                               device=device)
            draw[:raw_n].copy_(pinned[:raw_n], non_blocking=True)
            if host_used:
                draw[raw_cap:raw_cap + host_n].copy_(pinned[raw_cap:raw_cap + host_n],
                                                     non_blocking=True)
            for fld, g, p0, np_ in chunks:
                seg = pages[p0:p0 + np_]
                dc = cols[fld.name]
                eb = dc.data.element_size()
                row0 = lo + int(rg_off[g])
                seg["out"] = dc.data.data_ptr() + (row0 + seg["row"]) * eb
                if seg["nulls"].any():
                    v = ensure_valid(dc, dc.data.shape[0], device, lock or _VALID_LOCK)
                    seg["valid"] = np.where(seg["nulls"] != 0, v.data_ptr() + row0 + seg["row"], 0)
            # device address of every decompressed page (scratch, or the host-inflated copy)
            hbase = draw.data_ptr() + raw_cap
            pages["dst"] = np.where(pages["codec"] == 2, hbase + pages["src"],
                                    sbase + pages["dst"])
            dp = pages["dict_page"]
            pages["dict"] = np.where(dp >= 0, pages["dst"][np.maximum(dp, 0)], 0)
            plain = _plain_string_pages(chunks, pages, cols, strings, lo, rg_off, device)
            tabs = _string_code_tables(chunks, pages, pinned.data_ptr() + raw_cap, strings)
            if tabs is not None:
                tab_host, fix = tabs
                tpin = pool.acquire(tab_host.nbytes)
                tpin.numpy()[:tab_host.nbytes] = tab_host.view(np.uint8)
                dtab = torch.empty(tab_host.nbytes, dtype=torch.uint8, device=device)
                dtab.copy_(tpin[:tab_host.nbytes], non_blocking=True)
                pool.release(tpin, stream)
                dtab.record_stream(stream)
                for p0, np_, toff in fix:
                    seg = pages[p0:p0 + np_]
                    seg["dict"] = np.where(seg["kind"] == 2, 0, np.where(
                        seg["eb"] == 16, seg["dict"], dtab.data_ptr() + 4 * toff))
            if defer is not None:
                # batched decode (decode_batch): absolute source addresses, buffers kept alive
                # by the pending record until the batched launch is queued
                pages["src"] = np.where(pages["codec"] == 2, pages["src"],
                                        draw.data_ptr() + pages["src"])
                keep = [draw, scratch] + ([dtab] if tabs is not None else [])
                for sc in plain:                # the (address, length) pairs point into these
                    sc.add_plain([], [draw, scratch])
                ev = torch.cuda.Event()
                ev.record(stream)
                defer.append(PendingDecode(pages, keep, ev, draw.numel() + scratch.numel()))
                pool.release(pinned, stream)
                _phase("h2d_enqueue", t)
                return {fld.name for fld, _, _, _ in chunks}
            ppin = pool.acquire(pages.nbytes)
            ppin.numpy()[:pages.nbytes] = pages.view(np.uint8)
            dpages = torch.empty(pages.nbytes, dtype=torch.uint8, device=device)
            dpages.copy_(ppin[:pages.nbytes], non_blocking=True)
            pool.release(pinned, stream)
            pool.release(ppin, stream)
            t = _phase("h2d_enqueue", t)
            NL.check(NL.lib().hs_pq_decode_pages(draw.data_ptr(), sbase, dpages.data_ptr(),
                                                 len(pages), status.data_ptr(),
                                                 stream.cuda_stream), "hs_pq_decode_pages")
            for x in (draw, dpages, scratch):
                x.record_stream(stream)
            for sc in plain:
                sc.add_plain([], [draw, scratch])
            _phase("launch", t)
        return {fld.name for fld, _, _, _ in chunks}
    finally:
        f.close()


def _plain_string_pages(chunks, pages, cols, strings, lo: int, rg_off, device) -> list:
    """Point the PLAIN string pages (eb 16) of a file plan at their rows of the column's
    (address, length) arrays; returns the StringCodes that received such pages."""
    out = []
    if not strings:
        return out
    for fld, g, p0, np_ in chunks:
        sc = strings.get(fld.name)
        if sc is None:
            continue
        seg = pages[p0:p0 + np_]
        pl = seg["eb"] == 16
        if not pl.any():
            continue
        sptr, slen = sc.plain_arrays(cols[fld.name].data.shape[0], device)
        rows = lo + int(rg_off[g]) + seg["row"]
        seg["out"] = np.where(pl, sptr.data_ptr() + rows * 8, seg["out"])
        seg["dict"] = np.where(pl, slen.data_ptr() + rows * 4, seg["dict"])
        sc.add_plain([(int(r), int(r) + int(nv)) for r, nv in zip(rows[pl], seg["nvals"][pl])], [])
        if sc not in out:
            out.append(sc)
    return out


def _string_code_tables(chunks, pages, host_base: int, strings):
    """For the string chunks of a file plan: parse each dictionary page (inflated on the host by
    the planner, at ``host_base + src``), register it with the column's ``StringCodes`` and lay
    out the chunk's code table ``[base, base + len)``.  Returns (int32 tables, [(first page,
    pages, table offset)]) or None when the plan has no string chunk."""
    if not strings:
        return None
    tabs, fix, at = [], [], 0
    for fld, g, p0, np_ in chunks:
        sc = strings.get(fld.name)
        if sc is None:
            continue
        seg = pages[p0:p0 + np_]
        dpg = np.nonzero(seg["kind"] == 2)[0]
        if not len(dpg) and (seg["eb"] == 16).all():
            continue                            # PLAIN pages only: StringCodes.finish_plain
        if len(dpg) != 1 or seg["codec"][dpg[0]] != 2:
            raise IOError(f"string chunk of {fld.name} without a host-parsed dictionary page")
        d = seg[dpg[0]]
        arr = plain_strings(host_base + int(d["src"]), int(d["usize"]), int(d["nvals"]))
        base = sc.add(arr)
        tabs.append(np.arange(base, base + len(arr), dtype=np.int32))
        fix.append((p0, np_, at))
        at += len(arr)
    if not fix:
        return None
    return (np.concatenate(tabs) if at else np.zeros(1, np.int32)), fix


def _hybrid_host(s: np.ndarray, bw: int, nv: int) -> np.ndarray:
    """The ``nv`` values of an RLE / bit-packed hybrid stream ``s`` at bit width ``bw``."""
    out = np.zeros(nv, dtype=np.int64)
    q, done = 0, 0
    while done < nv:
        h, shift = 0, 0
        while True:
            b = int(s[q]); q += 1
            h |= (b & 0x7F) << shift
            if not b & 0x80:
                break
            shift += 7
        if h & 1:
            groups = h >> 1
            take = min(groups * 8, nv - done)
            out[done:done + take] = _unpack(s, q, take, bw) if bw else 0
            q += groups * bw
        else:
            vb = (bw + 7) // 8
            take = min(h >> 1, nv - done)
            out[done:done + take] = int.from_bytes(bytes(s[q:q + vb]), "little")
            q += vb
        done += take
    return out


def decode_plan_host(raw: np.ndarray, pages: np.ndarray, outputs: Dict[int, np.ndarray],
                     host_dicts: Optional[np.ndarray] = None,
                     valid_outputs: Optional[Dict[int, np.ndarray]] = None) -> None:
    """Reference (host) consumer of a device page plan — the oracle for hs_pq_decode_pages.
    ``outputs`` maps a page's ``out`` value to a numpy array slice receiving its values (the
    plan is built with ``out`` = synthetic keys here instead of device addresses);
    ``valid_outputs`` likewise maps ``valid`` to the validity slice of pages with nulls, whose
    values are spread to their rows with 0 at nulls (as ``hs_pq_expand_kernel`` does)."""
    L = lib()
    scratch = {}
    for i, p in enumerate(pages):
        if p["codec"] == 2:
            scratch[i] = host_dicts[p["src"]:p["src"] + p["usize"]]
            continue
        src = raw[p["src"]:p["src"] + p["csize"]]
        lv = int(p["levels"]) if p["kind"] == 1 else 0
        if p["codec"] == 0:
            data = bytes(src)
        else:
            body = np.ascontiguousarray(src[lv:])
            out = np.zeros(int(p["usize"]) - lv + 64, dtype=np.uint8)
            got = L.hs_pq_snappy_decompress(body.ctypes.data, len(body), out.ctypes.data,
                                            len(out))
            assert got == p["usize"] - lv, (got, p["usize"])
            data = bytes(src[:lv]) + out[:got].tobytes()
        scratch[i] = np.frombuffer(data, dtype=np.uint8)
    for i, p in enumerate(pages):
        if p["kind"] == 2:
            continue
        pg = scratch[i]
        voff = 0
        if p["kind"] == 0 and p["levels"]:
            voff = 4 + int(pg[:4].view(np.uint32)[0])
        elif p["kind"] == 1:
            voff = int(p["levels"])
        nv = int(p["nvals"])
        dst = outputs[int(p["out"])]
        if p["nulls"]:
            lstream = pg[4:voff] if p["kind"] == 0 else pg[:voff]
            valid = _hybrid_host(lstream, 1, nv).astype(np.uint8)
            valid_outputs[int(p["valid"])][:nv] = valid
            dense = np.zeros(nv, dtype=dst.dtype)
            nn = int(valid.sum())
            _decode_values_host(p, pg, voff, nn, dense, scratch, pages)
            dst[:nv] = 0
            dst[:nv][valid.astype(bool)] = dense[:nn]
            continue
        _decode_values_host(p, pg, voff, nv, dst, scratch, pages)


def _decode_values_host(p, pg: np.ndarray, voff: int, nv: int, dst: np.ndarray, scratch,
                        pages) -> None:
    """The ``nv`` values of data page ``p`` (bytes ``pg``, values at ``voff``) into ``dst``."""
    dt = np.dtype({1: np.uint8, 4: np.uint32}.get(int(p["eb"]), np.uint64))
    if nv == 0:
        return
    if p["eb"] == 1:                 # BOOLEAN: PLAIN bits or length-prefixed RLE, width 1
        if p["enc"] == 0:
            dst[:nv] = np.unpackbits(pg[voff:voff + (nv + 7) // 8], bitorder="little")[:nv]
        else:
            dst[:nv] = _hybrid_host(pg[voff + 4:voff + 4 + int(pg[voff:voff + 4].view(
                np.uint32)[0])], 1, nv)
        return
    if p["enc"] == 0:
        dst[:nv] = pg[voff:voff + nv * dt.itemsize].view(dt)
        return
    d = scratch[int(p["dict_page"])]
    dvals = d[:int(pages[int(p["dict_page"])]["nvals"]) * dt.itemsize].view(dt)
    bw = int(pg[voff])
    s = pg[voff + 1:]
    q, done = 0, 0
    while done < nv:
        h, shift = 0, 0
        while True:
            b = int(s[q]); q += 1
            h |= (b & 0x7F) << shift
            if not b & 0x80:
                break
            shift += 7
        if h & 1:
            groups = h >> 1
            take = min(groups * 8, nv - done)
            idx = _unpack(s, q, take, bw) if bw else np.zeros(take, np.int64)
            dst[done:done + take] = dvals[idx]
            q += groups * bw
            done += take
        else:
            cnt = h >> 1
            vb = (bw + 7) // 8
            v = int.from_bytes(bytes(s[q:q + vb]), "little")
            q += vb
            take = min(cnt, nv - done)
            dst[done:done + take] = dvals[v]
            done += take
