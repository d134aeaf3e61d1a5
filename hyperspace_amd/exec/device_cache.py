"""HBM-resident table cache for the MI355X executor.

Index data is immutable per log version, so the executor keeps decoded index columns resident in
HBM (288 GB per MI355X) and re-reads files only when the index content changes — the "keep
tensors resident instead of re-reading them" rule.  Entries are keyed by the exact file set
(path, size, mtime), the projected columns and the rank's bucket ownership (the session's owner
map, parallel/placement.py); eviction is LRU by
bytes under ``spark.hyperspace.mi.deviceCacheBytes``.

Index tables are laid out bucket-major with a ``B+1`` offset table; every bucket is sorted by the
index's indexed columns (the writer guarantees it for one-file buckets; buckets that accumulated
several files through incremental refresh are re-sorted on the device at load time).
"""
from __future__ import annotations

import threading
from collections import OrderedDict
from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

from ..io.writer import get_bucket_id
from ..utils import path_utils as P
from .device_table import DeviceColumn, DeviceTable


_FILES_KEYS: Dict[int, tuple] = {}


def _files_key(files) -> tuple:
    """Identity of a file list (path, size, mtime); memoized per list object."""
    hit = _FILES_KEYS.get(id(files))
    if hit is not None and hit[0] is files:
        return hit[1]
    k = tuple((f.path, f.length, f.modification_time) for f in files)
    if len(_FILES_KEYS) > 4096:
        _FILES_KEYS.clear()
    _FILES_KEYS[id(files)] = (files, k)
    return k


HOLDS_REACCOUNT = 16

# Device buffers that lowered queries derive and keep outside any table (the recorded run matches
# of exec/jit_runs.py, ...): live bytes, released by each buffer's finalizer.  Every cache's
# budget shrinks by them, so tables plus derived buffers stay within the planned HBM share.
_DERIVED = [0]


def track_derived(t) -> None:
    """Count device tensor ``t`` against every table cache's budget while it lives."""
    import weakref
    nb = int(t.numel()) * int(t.element_size())
    _DERIVED[0] += nb
    weakref.finalize(t, _untrack, nb)


def _untrack(nb: int) -> None:
    _DERIVED[0] -= nb


def derived_bytes() -> int:
    return _DERIVED[0]


class DeviceTableCache:
    """LRU of resident tables under an HBM byte budget.  A table's footprint includes what
    queries derive from it and keep on it (compacted column copies, join indexes, packed /
    remapped key tables — ``DeviceTable.resident_bytes``), re-measured on every hit, so the
    budget bounds what is really resident, not just the columns as loaded."""

    def __init__(self, budget_bytes: int):
        self.budget = int(budget_bytes)
        self._lru: "OrderedDict[tuple, DeviceTable]" = OrderedDict()
        self._size: Dict[tuple, int] = {}
        self._bytes = 0
        self._lock = threading.Lock()
        self.hits = 0
        self.misses = 0
        # bumped whenever a table leaves the cache: a prepared submission (exec/gpu.py
        # _AggProgram) that saw its tables resident at epoch e still holds them while the epoch
        # is e, without re-checking each table
        self.epoch = 0

    def _key(self, files, columns, extra):
        fk = _files_key(files)
        return (fk, tuple(columns), extra)

    def _evict(self, keep) -> None:
        while self._bytes > self.budget - _DERIVED[0] and len(self._lru) > 1:
            k, _ = next(iter(self._lru.items()))
            if k == keep:
                self._lru.move_to_end(k)
                k, _ = next(iter(self._lru.items()))
                if k == keep:
                    break
            self._lru.pop(k)
            self._bytes -= self._size.pop(k, 0)
            self.epoch += 1

    def get(self, files, columns, extra, loader) -> DeviceTable:
        key = self._key(files, columns, extra)
        with self._lock:
            t = self._lru.get(key)
            if t is not None:
                self._lru.move_to_end(key)
                self.hits += 1
                nb = t.resident_bytes()
                self._bytes += nb - self._size.get(key, nb)
                self._size[key] = nb
                self._evict(key)
                return t
        self.misses += 1
        t = loader()
        nb = t.resident_bytes()
        with self._lock:
            if self.budget > 0 and nb <= self.budget:
                if key in self._lru:         # replaces a concurrently loaded copy
                    self.epoch += 1
                self._lru[key] = t
                self._size[key] = nb
                self._bytes += nb
                t._hs_cache_key = key
                self._evict(key)
        return t

    def holds(self, t) -> bool:
        """Whether ``t`` is still the resident table of its key (then counted as a hit, like
        ``get``): lets the executor reuse a relation it lowered earlier without rebuilding the
        key from the file list."""
        key = getattr(t, "_hs_cache_key", None)
        if key is None:
            return False
        with self._lock:
            if self._lru.get(key) is not t:
                return False
            self._lru.move_to_end(key)
            self.hits += 1
            # re-account the structures queries derived from the table (compact codes, join
            # indexes, ...) every HOLDS_REACCOUNT hits, not on every query's check
            seen = getattr(t, "_hs_holds", 0)
            t._hs_holds = seen + 1
            if seen % HOLDS_REACCOUNT == 0:
                nb = t.resident_bytes()
                self._bytes += nb - self._size.get(key, nb)
                self._size[key] = nb
                self._evict(key)
            return True

    @property
    def resident_bytes(self) -> int:
        return self._bytes

    def clear(self):
        with self._lock:
            self.epoch += 1
            self._lru.clear()
            self._size.clear()
            self._bytes = 0


# ------------------------------------------------------------------------------------------------
# Build seeds: a device build ends with every index column sorted bucket-major in HBM — exactly
# what load_bucketed_index would read back from the files it just wrote.  The build registers
# those columns here and the first query of the new index takes them instead of re-reading,
# re-decoding and re-sorting the files (cold-query latency).  A seed matches a query's file list
# only if the owned files are the very files written, unchanged (path and size).
# ------------------------------------------------------------------------------------------------
_SEEDS: "OrderedDict[tuple, dict]" = OrderedDict()
_SEED_LOCK = threading.Lock()
SEED_STATS = {"registered": 0, "hits": 0}


def _seed_budget(session) -> int:
    from .hbm_budget import rank_budget
    return rank_budget(session.conf).cache // 2


def register_seed(session, paths, cols: Dict[str, DeviceColumn], off, rank: int, world: int,
                  num_buckets: int) -> None:
    import os
    import torch
    keep = {}
    for n, c in cols.items():
        if c.offsets is not None:       # raw string bytes: queries read dictionary codes
            continue
        keep[n] = c
    if not keep:
        return
    files = tuple(sorted((P.to_local(p), os.path.getsize(P.to_local(p))) for p in paths))
    nbytes = sum(c.nbytes() for c in keep.values())
    budget = _seed_budget(session)
    if nbytes > budget:
        return
    dev = next(iter(keep.values())).data.device
    off = np.asarray(off, dtype=np.int64)
    entry = {"cols": keep, "off": off, "off_dev": torch.from_numpy(off).to(dev),
             "bytes": nbytes, "num_buckets": num_buckets}
    with _SEED_LOCK:
        _SEEDS[(files, rank, world)] = entry
        SEED_STATS["registered"] += 1
        total = sum(e["bytes"] for e in _SEEDS.values())
        while total > budget and len(_SEEDS) > 1:
            _, old = _SEEDS.popitem(last=False)
            total -= old["bytes"]


def seeded_index(files, columns: List[str], num_buckets: int, rank: int,
                 world: int, owned_buckets=None) -> Optional[DeviceTable]:
    """The build seed of exactly this rank's share of ``files`` (buckets ``owned_buckets``,
    default ``b % world == rank``) holding ``columns``, as a table view (shared tensors), or
    None.  A build writes bucket b from rank b % world, so only a query placement that gives
    this rank those same buckets can take the seed."""
    if not _SEEDS:
        return None
    mine = set(owned_buckets) if owned_buckets is not None else \
        {b for b in range(num_buckets) if b % world == rank}
    owned = []
    for f in files:
        b = get_bucket_id(P.get_name(f.path))
        if b is None or b >= num_buckets:
            return None
        if b in mine:
            owned.append((P.to_local(f.path), int(f.length)))
    key = (tuple(sorted(owned)), rank, world)
    with _SEED_LOCK:
        e = _SEEDS.get(key)
        if e is None or e["num_buckets"] != num_buckets or \
                any(c not in e["cols"] for c in columns):
            return None
        # consumed on its first hit: the device cache owns the table from here on, so the
        # seed pins no HBM outside the cache budget
        _SEEDS.pop(key)
        SEED_STATS["hits"] += 1
    off = e["off"]
    cols = {c: e["cols"][c] for c in columns}
    return DeviceTable(cols, int(off[-1]), e["off_dev"], off)


def clear_seeds() -> None:
    with _SEED_LOCK:
        _SEEDS.clear()


def load_bucketed_index(files, columns: List[str], num_buckets: int, sort_cols: List[str], device,
                        rank: int = 0, world: int = 1, owned_buckets=None,
                        cuts=None) -> DeviceTable:
    """Load index files bucket-major for the buckets this rank owns (``owned_buckets``, default
    b % world == rank); every other bucket is an empty range of the offset table.  ``cuts``:
    {bucket: (lo, hi)} - of those buckets this rank keeps only the rows whose leading sort key
    lies in ``[lo, hi)`` (None: open; a heavy bucket cut across ranks, parallel/placement.py)."""
    import torch
    from ..ops import kernels as K
    by_bucket: Dict[int, list] = {}
    for f in files:
        b = get_bucket_id(P.get_name(f.path))
        if b is None or b >= num_buckets:
            raise ValueError(f"not an index bucket file: {f.path}")
        by_bucket.setdefault(b, []).append(f.path)
    mine = set(owned_buckets) if owned_buckets is not None else \
        {b for b in range(num_buckets) if b % world == rank}
    owned = [b for b in range(num_buckets) if b in mine and b in by_bucket]
    ordered = [(b, p) for b in owned for p in sorted(by_bucket[b])]
    paths = [p for _, p in ordered]
    counts = np.zeros(num_buckets, dtype=np.int64)
    multi = False
    if paths:
        # footers give every file's row count up front, so files stream straight into their
        # slice of presized HBM columns (staging.upload_files) with no host-side concatenation
        from . import staging
        from .pq_encode import CREATED_BY
        metas = list(staging.io_pool().map(
            lambda p: pq.ParquetFile(P.to_local(p)).metadata, paths))
        rows = [m.num_rows for m in metas]
        # files of the paged device writer (pages of at most pq_encode.PAGE_ROWS rows) decode
        # on the device, pages and all; older row-group-sized pages take the host page layer
        # (one wavefront inflates one page: profiles/cold_load_r2.jsonl)
        paged = all((m.created_by or "") == CREATED_BY for m in metas)
        for (b, _), r in zip(ordered, rows):
            multi = multi or counts[b] > 0
            counts[b] += r
        schema = pq.read_schema(P.to_local(paths[0]))
        schema = pa.schema([schema.field(c) for c in columns])

        def read_file(p, cols=None):
            return pq.read_table(P.to_local(p), columns=columns if cols is None else cols,
                                 use_threads=False)
        up = staging.upload_files(read_file, paths, rows, schema, device,
                                  parquet_local=[P.to_local(p) for p in paths],
                                  device_pages=paged)
        cols = dict(up.columns)
        # string columns -> int32 codes over one sorted dictionary: device-decoded files'
        # upload-local codes are remapped on the device, host-decoded files' are looked up
        staging.finish_strings(up, cols, device, None)
        cols = {c: cols[c] for c in columns}
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    n = int(off[-1])
    if not n:
        cols = {c: DeviceColumn(torch.empty(0, dtype=torch.int64, device=device), None, pa.int64())
                for c in columns}
    table = DeviceTable(cols, n, torch.from_numpy(off).to(device), off)
    if multi and n:
        # re-establish (bucket, sort cols) order on the device
        bucket = torch.repeat_interleave(torch.arange(num_buckets, dtype=torch.int32, device=device),
                                         torch.from_numpy(counts).to(device))
        perm = K.sort_permutation([table.columns[c] for c in sort_cols],
                                  extra_leading=(bucket, 16))
        names = list(table.columns)
        gathered = K.gather_columns([table.columns[c] for c in names], perm)
        table = DeviceTable(dict(zip(names, gathered)), n, table.bucket_offsets, off)
    if cuts and n:
        table = _cut_buckets(table, sort_cols[0], cuts, device)
    return table


def _cut_buckets(table: DeviceTable, key: str, cuts, device) -> DeviceTable:
    """The table without the rows of cut buckets outside this rank's key range (each bucket's
    rows are sorted by ``key``, so a range is one slice, found by binary search)."""
    import torch
    from ..ops import kernels as K
    off = np.asarray(table.bucket_offsets_host, dtype=np.int64)
    kc = table.columns[key]
    if kc.is_float or kc.dictionary is not None:
        # the loader passes cuts for integer keys only (placement.routes_by_key)
        raise ValueError(f"heavy-bucket cut on a non-integer key {key}")
    keep_lo, keep_hi = off[:-1].copy(), off[1:].copy()
    for b, (lo, hi) in cuts.items():
        a0, a1 = int(off[b]), int(off[b + 1])
        if a1 <= a0:
            continue
        # a bucket's null keys sort first: they belong to its first piece (lo None), like a
        # shuffled row with a null key (OwnerMap.dest); the cut searches the non-null keys
        nn = 0 if kc.valid is None else int((kc.valid[a0:a1] == 0).sum().item())
        seg = kc.data[a0 + nn:a1].long()
        s = a0 + nn + int(torch.searchsorted(seg, torch.tensor([lo], device=seg.device))[0]) \
            if lo is not None else a0
        e = a0 + nn + (int(torch.searchsorted(seg, torch.tensor([hi], device=seg.device))[0])
                       if hi is not None else a1 - a0 - nn)
        keep_lo[b], keep_hi[b] = s, max(s, e)
    counts = keep_hi - keep_lo
    idx = torch.cat([torch.arange(int(a), int(c), dtype=torch.int64, device=device)
                     for a, c in zip(keep_lo, keep_hi) if c > a] or
                    [torch.empty(0, dtype=torch.int64, device=device)])
    names = list(table.columns)
    cols = K.gather_columns([table.columns[c] for c in names], idx) if idx.numel() else \
        [DeviceColumn(table.columns[c].data[:0], None, table.columns[c].atype,
                      table.columns[c].dictionary) for c in names]
    noff = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return DeviceTable(dict(zip(names, cols)), int(noff[-1]), torch.from_numpy(noff).to(device),
                       noff)


def load_flat(files, fmt: str, columns: List[str], data_schema, options, partition_spec,
              device) -> DeviceTable:
    """Load arbitrary source files (no bucketing) as one table."""
    import torch
    from ..io.reader import read_files
    t = read_files(fmt, [f.path for f in files], data_schema, options, partition_spec, columns)
    cols = {c: DeviceColumn.from_arrow(t.column(c), device) for c in columns}
    n = t.num_rows
    off = np.array([0, n], dtype=np.int64)
    return DeviceTable(cols, n, torch.from_numpy(off).to(device), off)
