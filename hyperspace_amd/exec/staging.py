"""Pipelined host <-> HBM staging for index builds (SURVEY §2.3 K1/K4 I/O, §2.4 "pipeline").

Upload (``upload_files``): a thread pool decodes source files (pyarrow, one file per task) and
each worker immediately copies its fixed-width columns into pinned host memory and issues the
H2D copy on a dedicated HIP copy stream into a pre-sized device column, at the file's row
offset.  Decode of file i+1 overlaps the PCIe transfer of file i, and no concatenated host copy
of the whole table is ever built.  Row offsets come from the Parquet footers, so every file's
destination slice is known before any data is read.  Lineage ids (K2) are a per-file constant
written with a device fill — no host array at all.

Download (``download_buckets``): buckets are grouped into ~``chunk_bytes`` chunks; each chunk's
columns are copied D2H into pinned memory asynchronously, and a writer task waits on that
chunk's event and encodes/writes its Parquet files while the next chunk is still in flight.

Pinned buffers come from torch's caching host allocator, which keeps a block alive until the
copies recorded on it have completed, so buffer reuse is race-free by construction.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import threading
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from .device_table import DeviceColumn, is_string, storage_numpy_dtype

_POOL = None
UPLOAD_TIMES: Dict[str, float] = {}   # wall split of the last upload_files (build stats)
_COPY_STREAMS: Dict[int, object] = {}


def io_pool() -> cf.ThreadPoolExecutor:
    global _POOL
    if _POOL is None:
        _POOL = cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4),
                                      thread_name_prefix="hs-stage")
    return _POOL


def copy_stream(device):
    return copy_streams(device)[0]


# streams the H2D copies of a batched device-decode upload go through (0 = one per file, round
# robin over copy_streams)
UPLOAD_H2D_STREAMS = 1


def copy_streams(device, k: int = 4) -> list:
    """``k`` staging streams per device (the box exposes 4 hardware queues per process):
    uploads of different files run their H2D copies and decode kernels concurrently."""
    import torch
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _COPY_STREAMS.get(idx)
    if s is None:
        s = [torch.cuda.Stream(device=device) for _ in range(k)]
        _COPY_STREAMS[idx] = s
    return s


def ensure_valid(dc: DeviceColumn, n: int, device, lock: threading.Lock):
    """The column's validity mask, created all-valid on first use.  The fill completes before
    any thread can see the mask, so concurrent streams writing their own slices never race it."""
    import torch
    with lock:
        if dc.valid is None:
            v = torch.ones(n, dtype=torch.uint8, device=device)
            torch.cuda.current_stream(device).synchronize()
            dc.valid = v
    return dc.valid


RESERVE_BLOCK = 128 << 20


class PinnedPool:
    """Reusable pinned host blocks for staging (decode buffers, D2H encode buffers).

    Pinning is the slow part of a cold build (hipHostMalloc of GBs), so blocks are kept and
    handed out best-fit; a released block returns to the free list only after the copy recorded
    on its stream has completed.  ``reserve`` pre-pins blocks at engine start (the GPU backend
    does this), like any engine sizing its staging pool up front."""

    def __init__(self, limit_bytes: int = 8 << 30):
        self.limit = limit_bytes
        self._free: list = []
        self._pending: list = []
        self._held = 0
        self._lock = threading.Lock()

    def _reclaim(self) -> None:
        keep = []
        for t, ev in self._pending:
            if ev.query():
                self._free.append(t)
            else:
                keep.append((t, ev))
        self._pending = keep

    def _best_fit(self, nbytes: int):
        best, best_n = None, 0
        cap = max(4 * nbytes, RESERVE_BLOCK)
        for i, t in enumerate(self._free):
            n = t.hs_nbytes
            if nbytes <= n <= cap and (best is None or n < best_n):
                best, best_n = i, n
        return best

    def acquire(self, nbytes: int):
        import torch
        nbytes = max(int(nbytes), 1)
        with self._lock:
            # free blocks first; the event queries of the pending ones (one HIP call each,
            # under the lock every reader thread takes) only when nothing free fits
            best = self._best_fit(nbytes)
            if best is None:
                self._reclaim()
                best = self._best_fit(nbytes)
            if best is not None:
                return self._free.pop(best)
            size = (nbytes + (8 << 20) - 1) // (8 << 20) * (8 << 20)
            pooled = self._held + size <= self.limit
            if pooled:
                self._held += size
        t = torch.empty(size if pooled else nbytes, dtype=torch.uint8, pin_memory=True)
        t.hs_pooled = pooled
        t.hs_nbytes = t.numel()
        return t

    def release(self, t, stream) -> None:
        """Return ``t`` once the work queued on ``stream`` (its copies) has finished."""
        import torch
        if not getattr(t, "hs_pooled", False):
            return
        ev = torch.cuda.Event()
        ev.record(stream)
        with self._lock:
            self._pending.append((t, ev))

    def reserve(self, count: int = 32, nbytes: int = None) -> None:
        """Pre-pin ``count`` blocks once per process (idempotent)."""
        import torch
        nbytes = nbytes or RESERVE_BLOCK
        with self._lock:
            if self._held:
                return
        blocks = [self.acquire(nbytes) for _ in range(count)]
        with self._lock:
            self._free.extend(b for b in blocks if getattr(b, "hs_pooled", False))
        del blocks
        torch.cuda.synchronize()


_PINNED: Optional[PinnedPool] = None


def pinned_pool() -> PinnedPool:
    global _PINNED
    if _PINNED is None:
        _PINNED = PinnedPool()
    return _PINNED


_TORCH_OF_NP = None


def _torch_dtype(nd: np.dtype):
    global _TORCH_OF_NP
    import torch
    if _TORCH_OF_NP is None:
        _TORCH_OF_NP = {np.dtype(np.int8): torch.int8, np.dtype(np.int16): torch.int16,
                        np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64,
                        np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
                        np.dtype(np.uint8): torch.uint8}
    if nd == np.dtype(np.uint32):
        return torch.int32
    if nd == np.dtype(np.uint64):
        return torch.int64
    return _TORCH_OF_NP[nd]


def fixed_width_numpy(arr) -> Tuple[np.ndarray, Optional[np.ndarray]]:
    """(values in storage dtype, validity uint8 or None) of a non-string arrow column."""
    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
    t = arr.type
    nd = storage_numpy_dtype(t)
    valid = None
    if arr.null_count:
        valid = np.asarray(arr.is_valid().to_numpy(zero_copy_only=False), dtype=np.uint8)
    if pa.types.is_boolean(t):
        vals = np.asarray(arr.fill_null(False).to_numpy(zero_copy_only=False), dtype=np.uint8)
    elif pa.types.is_decimal(t):
        vals = np.asarray(arr.cast(pa.float64()).fill_null(0).to_numpy(), dtype=np.float64)
    elif pa.types.is_date32(t) or pa.types.is_timestamp(t) or pa.types.is_date64(t) or \
            pa.types.is_duration(t):
        st = pa.int32() if pa.types.is_date32(t) else pa.int64()
        a = arr.view(st)
        vals = np.asarray((a.fill_null(0) if arr.null_count else a).to_numpy(zero_copy_only=False),
                          dtype=nd)
    else:
        a = arr.fill_null(0) if arr.null_count else arr
        vals = np.asarray(a.to_numpy(zero_copy_only=False), dtype=nd)
    return vals, valid


_WARM = False
# columns the last uploads had to decode on the host (pyarrow) instead of the native page layer
HOST_DECODED: set = set()
# columns the last uploads decoded entirely on the device (raw pages -> HIP inflate + expand)
DEVICE_DECODED: set = set()


def _warm_decode_kernels() -> None:
    """Load the page-decode kernels from this (main) thread before workers launch them."""
    global _WARM
    if not _WARM:
        from ..ops import _lib as NL
        NL.check(NL.lib().hs_pq_warmup(NL.stream_ptr()), "hs_pq_warmup")
        _WARM = True


def native_decode_enabled() -> bool:
    """Native Parquet page decode (HIP) for staging; ``HS_NATIVE_PARQUET=0`` forces pyarrow."""
    return os.environ.get("HS_NATIVE_PARQUET", "1") == "1"


def device_decode_enabled() -> bool:
    """Device-only page decode (Snappy + hybrid RLE on the GPU, io/native_parquet
    ``upload_file_device``); ``HS_DEVICE_PARQUET=0`` keeps decompression and run parsing on the
    host page layer."""
    return os.environ.get("HS_DEVICE_PARQUET", "1") == "1"


def batch_decode_bytes() -> int:
    """Device bytes (compressed + inflated pages) of files whose page decode is batched into
    one launch (``HS_PQ_BATCH_BYTES``; 0 = one launch per file)."""
    return int(os.environ.get("HS_PQ_BATCH_BYTES", str(4 << 30)))


_DECODE_STREAMS: Dict[int, object] = {}


def decode_stream(device):
    """The stream batched page decodes run on (one per device)."""
    import torch
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _DECODE_STREAMS.get(idx)
    if s is None:
        s = _DECODE_STREAMS[idx] = torch.cuda.Stream(device=device)
    return s


def device_strings_enabled() -> bool:
    """Dictionary-encoded string pages decode on the device (``HS_DEVICE_STRINGS=0``: pyarrow)."""
    return os.environ.get("HS_DEVICE_STRINGS", "1") == "1"


def _h2d_async(dst, src: np.ndarray, stream) -> None:
    """Copy ``src`` into device tensor slice ``dst`` via a pinned bounce buffer on ``stream``."""
    import torch
    n = src.shape[0]
    if n == 0:
        return
    pinned = torch.empty(n, dtype=dst.dtype, pin_memory=True)
    np.copyto(pinned.numpy().view(src.dtype), src, casting="no")
    with torch.cuda.stream(stream):
        # torch's caching host allocator records an event for this copy and will not hand the
        # pinned block out again before it completes
        dst.copy_(pinned, non_blocking=True)


class UploadResult:
    def __init__(self, columns: Dict[str, DeviceColumn], num_rows: int, host_strings: dict,
                 device_strings: Optional[dict] = None, offsets: Optional[np.ndarray] = None):
        self.columns = columns
        self.num_rows = num_rows
        # name -> list of per-file arrow chunks (file order; None where the device decoded the
        # file's pages): only string columns some file had to decode on the host
        self.host_strings = host_strings
        # name -> io.native_parquet.StringCodes: string columns whose codes the device wrote
        self.device_strings = device_strings or {}
        self.offsets = offsets              # first row of every file (+ total)


def finish_strings(up: "UploadResult", cols: Dict[str, DeviceColumn], device, dist,
                   raw: Sequence[str] = (), names: Optional[Sequence[str]] = None) -> None:
    """Turn every string column of an upload into int32 codes over one job-global sorted
    dictionary (``parallel/dictionary.union_sorted``; ``dist`` None: this process only).

    Device-decoded columns (``up.device_strings``) hold upload-local codes: the dictionary is
    the union of the parsed dictionary pages plus the values of host-decoded files, and the
    codes are remapped with one gather on the device; host-decoded files' codes are computed
    on the host and copied into their row ranges.  Columns named in ``raw`` also keep their
    bytes (offsets/chars) when they were host-decoded."""
    import torch
    from ..ops import kernels as K
    from ..parallel.dictionary import union_sorted
    if names is None:
        names = list(dict.fromkeys(list(up.device_strings) + list(up.host_strings)))
    for name in names:
        sc = up.device_strings.get(name)
        chunks = up.host_strings.get(name) or []
        if sc is None:
            chunks = [c for c in chunks if c is not None]
            arr = pa.chunked_array(chunks, type=chunks[0].type) if chunks else \
                pa.chunked_array([], pa.string())
            if pa.types.is_dictionary(arr.type):
                arr = arr.cast(arr.type.value_type)
            arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
            d = union_sorted(arr, dist)
            cols[name] = DeviceColumn.from_arrow(arr, device, d, raw_strings=name in raw)
            continue
        dc = cols[name]
        sc.finish_plain(dc)          # PLAIN pages' values -> codes (a dictionary part each)
        local = sc.concat()
        host = {i: (c.cast(c.type.value_type) if pa.types.is_dictionary(c.type) else c)
                for i, c in enumerate(chunks) if c is not None}
        host = {i: (c.combine_chunks() if isinstance(c, pa.ChunkedArray) else c)
                for i, c in host.items()}
        vals = [local] + [c.cast(pa.string()) for c in host.values()]
        gd = union_sorted(pa.concat_arrays(vals) if vals else local, dist)
        if len(local):
            remap = pc.index_in(local.cast(pa.string()), value_set=gd)
            tab = torch.from_numpy(np.asarray(remap.to_numpy(zero_copy_only=False),
                                              dtype=np.int32)).to(device)
            dc.data = K.lookup_i32(tab, dc.data)
        for i, c in host.items():
            lo, hi = int(up.offsets[i]), int(up.offsets[i + 1])
            codes = pc.index_in(c.cast(pa.string()), value_set=gd).fill_null(0)
            dc.data[lo:hi].copy_(torch.from_numpy(
                np.asarray(codes.to_numpy(zero_copy_only=False), dtype=np.int32)).to(device))
            if c.null_count:
                if dc.valid is None:
                    dc.valid = torch.ones(up.num_rows, dtype=torch.uint8, device=device)
                dc.valid[lo:hi].copy_(torch.from_numpy(np.asarray(
                    c.is_valid().to_numpy(zero_copy_only=False), dtype=np.uint8)).to(device))
        cols[name] = DeviceColumn(dc.data, dc.valid, pa.string(), gd)


def upload_files(read_file: Callable[..., pa.Table], files: Sequence[str],
                 row_counts: Sequence[int], schema: pa.Schema, device,
                 lineage_ids: Optional[Sequence[int]] = None,
                 lineage_name: Optional[str] = None,
                 parquet_local: Optional[Sequence[str]] = None,
                 nullable: Optional[set] = None,
                 on_batch: Optional[Callable[[Dict[str, DeviceColumn], int, int], None]] = None,
                 file_batches: Optional[Sequence[Tuple[int, int]]] = None,
                 device_pages: Optional[bool] = None) -> UploadResult:
    """Decode ``files`` in parallel and stream their fixed-width columns into HBM.

    ``row_counts[i]`` must equal the row count ``read_file(files[i])`` returns (Parquet footer);
    string columns are returned as host arrow chunks for dictionary encoding by the caller.

    ``nullable`` names fixed-width columns that get an all-valid mask up front (so every batch
    has one).  ``on_batch(columns, lo, hi)`` is called on this thread, in order, for every
    ``file_batches`` entry ``(first file, end file)`` — empty ones included — once the rows
    ``[lo, hi)`` of those files are on the device and ordered before the current stream's next
    work, while the pool keeps decoding later files (the multi-GPU build exchanges each batch as
    it lands).

    With ``parquet_local`` (local paths of Parquet ``files``) fixed-width columns go through the
    native page layer + HIP decode (``io/native_parquet.py``); ``read_file(path, columns)`` then
    reads only the columns that path does not cover.  ``device_pages`` picks the device-only page
    decode (default: ``device_decode_enabled()``) over the host page layer + device value
    expansion; index bucket files pass False (profiles/cold_load_r2.jsonl: their row-group-sized
    Snappy pages load 0.39 s via the host page layer vs 2.2 s device-only at SF100).
    """
    import time as _t
    import torch
    t_in = _t.perf_counter()
    offs = np.concatenate([[0], np.cumsum(np.asarray(row_counts, dtype=np.int64))])
    n = int(offs[-1])
    streams = copy_streams(device)
    batched = parquet_local is not None and native_decode_enabled() and \
        (device_decode_enabled() if device_pages is None else device_pages) and \
        batch_decode_bytes() > 0
    # batched device decode: the per-file streams carry only H2D copies, so they share
    # UPLOAD_H2D_STREAMS streams (two SDMA copies at once move 35 GB/s in total, one alone 56:
    # profiles/d2h_probe_r5.jsonl); the batched decode runs on decode_stream
    up_streams = [streams[k % len(streams)] for k in range(UPLOAD_H2D_STREAMS)] \
        if batched and UPLOAD_H2D_STREAMS > 0 else streams
    cols: Dict[str, DeviceColumn] = {}
    strings: Dict[str, list] = {}
    native = parquet_local is not None and native_decode_enabled()
    use_device_pages = device_decode_enabled() if device_pages is None else device_pages
    dev_strings: Dict[str, object] = {}
    for f in schema:
        if is_string(f.type):
            strings[f.name] = [None] * len(files)
            if native and use_device_pages and device_strings_enabled():
                from ..io.native_parquet import StringCodes
                dev_strings[f.name] = StringCodes()
                # zeroed: rows of host-decoded files are remapped along with the device ones
                cols[f.name] = DeviceColumn(torch.zeros(n, dtype=torch.int32, device=device),
                                            None, pa.string())
            continue
        nd = storage_numpy_dtype(f.type)
        cols[f.name] = DeviceColumn(torch.empty(n, dtype=_torch_dtype(nd), device=device), None,
                                    f.type)
    if lineage_ids is not None:
        cols[lineage_name] = DeviceColumn(torch.empty(n, dtype=torch.int64, device=device), None,
                                          pa.int64())
    for name in (nullable or ()):
        if name in cols:
            cols[name].valid = torch.ones(n, dtype=torch.uint8, device=device)
    lock = threading.Lock()
    main = torch.cuda.current_stream(device)
    for sc in dev_strings.values():
        sc.main = main
    for st in streams:
        st.wait_stream(main)  # allocations above happen-before the copies

    t_alloc = _t.perf_counter()
    status = None
    if native:
        _warm_decode_kernels()
        status = torch.zeros(1, dtype=torch.int32, device=device)

    def work(i: int):
        torch.cuda.set_device(device)
        stream = up_streams[i % len(up_streams)]
        lo, hi = int(offs[i]), int(offs[i + 1])
        done = set()
        defer = [] if batched else None
        if native:
            from ..io import native_parquet
            flds = [f for f in schema if f.name in cols]
            if use_device_pages:
                done = native_parquet.upload_file_device(parquet_local[i], flds, cols, lo,
                                                         stream, device, status, dev_strings,
                                                         defer, lock)
                DEVICE_DECODED.update(done)
            rest_native = [f for f in flds if f.name not in done and f.name not in strings]
            if rest_native:
                done = done | native_parquet.upload_file(parquet_local[i], rest_native, cols, lo,
                                                         n, stream, device, lock)
        rest = [f for f in schema if f.name not in done]
        for f in rest:
            HOST_DECODED.add(f.name)
        if not rest:
            if lineage_ids is not None:
                with torch.cuda.stream(stream):
                    cols[lineage_name].data[lo:hi].fill_(int(lineage_ids[i]))
            return _done_event(stream), (defer[0] if defer else None)
        t = read_file(files[i], [f.name for f in rest]) if native else read_file(files[i])
        if t.num_rows != hi - lo:
            raise RuntimeError(f"row count mismatch for {files[i]}: footer {hi - lo}, read "
                               f"{t.num_rows}")
        for f in rest:
            c = t.column(f.name)
            if f.name in strings:
                strings[f.name][i] = c
                continue
            vals, valid = fixed_width_numpy(c)
            dc = cols[f.name]
            _h2d_async(dc.data[lo:hi], vals, stream)
            if valid is not None:
                _h2d_async(ensure_valid(dc, n, device, lock)[lo:hi], valid, stream)
        if lineage_ids is not None:
            with torch.cuda.stream(stream):
                cols[lineage_name].data[lo:hi].fill_(int(lineage_ids[i]))
        return _done_event(stream), (defer[0] if defer else None)

    def _done_event(stream):
        ev = torch.cuda.Event()
        ev.record(stream)
        return ev

    t_sub = _t.perf_counter()
    UPLOAD_TIMES.clear()
    UPLOAD_TIMES.update({"alloc_s": round(t_alloc - t_in, 4), "warm_s": round(t_sub - t_alloc, 4)})
    futs = [io_pool().submit(work, i) for i in range(len(files))]
    if file_batches is None:
        file_batches = [(0, len(files))]
    dec_stream = decode_stream(device) if batched else None
    if dec_stream is not None:
        dec_stream.wait_stream(main)   # the destination columns exist before any decode
    pending: list = []
    pend_bytes = [0]
    limit = batch_decode_bytes()

    def flush():
        if pending:
            from ..io import native_parquet
            main.wait_event(native_parquet.decode_batch(pending, device, status, dec_stream))
            pending.clear()
            pend_bytes[0] = 0
    for b0, b1 in file_batches:
        for fu in futs[b0:b1]:
            ev, pend = fu.result()
            main.wait_event(ev)
            if pend is not None:
                pending.append(pend)
                pend_bytes[0] += pend.nbytes
                if pend_bytes[0] >= limit:
                    flush()
        flush()   # the batch's pages are decoded before on_batch reads its rows
        if on_batch is not None:
            on_batch(cols, int(offs[b0]), int(offs[b1]))
    for fu in futs:
        fu.result()
    t_host = _t.perf_counter()
    for st in streams + ([dec_stream] if dec_stream is not None else []):
        main.wait_stream(st)
    if status is not None:
        code = int(status.item())
        UPLOAD_TIMES.update({"files_s": round(t_host - t_sub, 4),
                             "device_drain_s": round(_t.perf_counter() - t_host, 4)})
        if code:
            raise IOError(f"device Parquet decode failed (status {code}: 1 corrupt page, "
                          f"2 dictionary index out of range) in {len(files)} files")
    host_strings = {k: v for k, v in strings.items()
                    if k not in dev_strings or any(c is not None for c in v)}
    return UploadResult(cols, n, host_strings, dev_strings, offs)


def download_buckets(columns: List[DeviceColumn], names: List[str], schema: pa.Schema,
                     bucket_off: np.ndarray, write_bucket: Callable[[pa.Table, int], str],
                     device, chunk_bytes: int = 512 << 20) -> List[str]:
    """D2H the bucket-major ``columns`` chunk by chunk and write each bucket as it lands."""
    import torch
    B = len(bucket_off) - 1
    row_bytes = sum(c.data.element_size() + (1 if c.valid is not None else 0) for c in columns)
    stream = copy_stream(device)
    stream.wait_stream(torch.cuda.current_stream(device))
    chunks: List[Tuple[int, int]] = []
    b = 0
    while b < B:
        e = b
        rows = 0
        while e < B and (e == b or (rows + int(bucket_off[e + 1] - bucket_off[e])) * row_bytes
                         <= chunk_bytes):
            rows += int(bucket_off[e + 1] - bucket_off[e])
            e += 1
        chunks.append((b, e))
        b = e
    futs = []
    max_inflight = 2 * min(16, os.cpu_count() or 4)
    for b0, b1 in chunks:
        lo, hi = int(bucket_off[b0]), int(bucket_off[b1])
        if hi <= lo:
            continue
        if len(futs) >= max_inflight:
            futs[len(futs) - max_inflight].result()  # bound pinned memory in flight
        host = []
        with torch.cuda.stream(stream):
            for c in columns:
                hv = torch.empty(hi - lo, dtype=c.data.dtype, pin_memory=True)
                hv.copy_(c.data[lo:hi], non_blocking=True)
                hm = None
                if c.valid is not None:
                    hm = torch.empty(hi - lo, dtype=torch.uint8, pin_memory=True)
                    hm.copy_(c.valid[lo:hi], non_blocking=True)
                host.append((hv, hm))
            ev = torch.cuda.Event()
            ev.record(stream)

        def write_chunk(b0=b0, b1=b1, lo=lo, host=host, ev=ev):
            ev.synchronize()
            arrays = []
            for c, (hv, hm) in zip(columns, host):
                arrays.append(host_to_arrow(c, hv.numpy(), None if hm is None else hm.numpy()))
            full = pa.Table.from_arrays(arrays, names=names)
            if not full.schema.equals(schema):
                full = full.cast(schema)
            out = []
            for bb in range(b0, b1):
                s, e = int(bucket_off[bb]) - lo, int(bucket_off[bb + 1]) - lo
                if e > s:
                    out.append(write_bucket(full.slice(s, e - s), bb))
            return out
        futs.append(io_pool().submit(write_chunk))
    paths = []
    for fu in futs:
        paths.extend(fu.result())
    return paths


def host_to_arrow(c: DeviceColumn, vals: np.ndarray, valid: Optional[np.ndarray]) -> pa.Array:
    """Arrow array over host numpy values (zero-copy for plain fixed-width columns)."""
    mask = None if valid is None else (valid == 0)
    t = c.atype
    if c.dictionary is not None:
        idx = pa.array(vals.view(np.int32), pa.int32(), mask=mask)
        return c.dictionary.take(idx).cast(t) if len(c.dictionary) else pa.nulls(len(vals), t)
    if pa.types.is_boolean(t):
        return pa.array(vals.astype(bool), pa.bool_(), mask=mask)
    if pa.types.is_date32(t):
        return pa.array(vals.view(np.int32), pa.int32(), mask=mask).view(pa.date32())
    if pa.types.is_timestamp(t) or pa.types.is_date64(t) or pa.types.is_duration(t):
        return pa.array(vals.view(np.int64), pa.int64(), mask=mask).view(t)
    if pa.types.is_decimal(t):
        return pa.array(vals, pa.float64(), mask=mask).cast(t)
    return pa.array(vals, t, mask=mask)
