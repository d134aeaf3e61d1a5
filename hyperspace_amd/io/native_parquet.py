"""Native Parquet decode into HBM: host page layer in C++
(``csrc/runtime/hs_parquet.cpp``: footer/page-header Thrift parsing, Snappy, run tables) and
HIP expansion kernels (``csrc/kernels/parquet_decode.hip``).

Per file: every natively decodable column chunk is decompressed straight into one pinned
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
import threading
from typing import Dict, List, Optional, Sequence, Set

import numpy as np
import pyarrow as pa

OK, IO, CORRUPT, UNSUPPORTED, CAPACITY = 0, -1, -2, -3, -4

RUN_DTYPE = np.dtype([("dst", "<i8"), ("count", "<i8"), ("src", "<i8"), ("kind", "<i4"),
                      ("bit_width", "<i4")])


class ChunkInfo(C.Structure):
    _fields_ = [("num_values", C.c_int64), ("num_nonnull", C.c_int64), ("dict_off", C.c_int64),
                ("dict_count", C.c_int64), ("bytes_used", C.c_int64),
                ("nvalue_runs", C.c_int64), ("nlevel_runs", C.c_int64),
                ("dict_encoded", C.c_int32), ("plain_pages", C.c_int32)]


# arrow type -> (Parquet physical type, element bytes) decodable as raw bits into our storage
def _native_kind(t: pa.DataType):
    if pa.types.is_int32(t) or pa.types.is_date32(t):
        return 1, 4
    if pa.types.is_int64(t):
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
                        ("hs_pq_snappy_decompress", I64, [P, I64, P, I64])):
                    fn = getattr(L, name)
                    fn.restype = res
                    fn.argtypes = args
                if L.hs_pq_run_size() != RUN_DTYPE.itemsize or \
                        L.hs_pq_info_size() != C.sizeof(ChunkInfo):
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
            if kind is None:
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
