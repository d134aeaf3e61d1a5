"""Index build on MI355X (SURVEY §3.1 hot loop, kernels K1-K4; §7.2 steps 3-4).

1. scan (K1, ``staging.upload_files``): this rank's share of the source files is decoded by a
   thread pool.  Parquet goes through the native page layer: the host preads raw column chunks
   and plans their pages (``csrc/runtime/hs_parquet.cpp``), the compressed bytes cross PCIe and
   HIP kernels inflate Snappy and expand RLE / bit-packed / PLAIN / dictionary pages
   (``csrc/kernels/parquet_decode.hip``).  Dictionary-encoded string chunks decode on the device
   to codes (the host parses only their dictionary pages).  Chunks the device path does not
   take (nulls, PLAIN strings, booleans, decimals, other formats) are decoded by pyarrow;
   lineage ids (K2) are a per-file constant fill;
2. ``hs_murmur3_bucket``: Spark-compatible bucket id per row (K3; strings hash their dictionary
   entry's bytes);
3. multi-GPU: rows move to their owner rank (bucket % world) in one packed all-to-all per batch
   of files (``_BatchedExchange`` / ``parallel/exchange.RowExchange``: counts, then one payload
   collective over RCCL), overlapping the decode of the next batch;
4. ``hs_sort_columns``: one stable LSD radix sort by (bucket, indexed columns...) (K4);
5. ``hs_gather``: all columns permuted in one launch; bucket offsets from the histogram;
6. one Parquet file per owned bucket, encoded on the device (``pq_encode``: dictionary codes,
   bit packing, Snappy) and written by a host thread pool as each chunk lands.
String columns use a job-global sorted dictionary so their codes sort and exchange consistently.
Builds larger than the HBM budget run in bucket-range passes (``_streaming_build``), and the
sorted bucket columns seed the device index cache (``device_cache.register_seed``).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import time
import uuid
from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from ..index import constants as C
from ..index.builder import group_by_bucket, read_index_input, source_format
from ..io.writer import write_bucket_file
from ..ops import kernels as K
from ..utils import path_utils as P
from ..utils.conf import HyperspaceConf
from .device_table import DeviceColumn, DeviceTable, is_string

LAST_BUILD_STATS: Dict[str, float] = {}
_T0 = [0.0]
# source files per exchange batch of a multi-GPU build (decode of batch k+1 overlaps the
# all-to-all of batch k)
FILES_PER_BATCH = 8


def _global_dicts(t: pa.Table, dist) -> Dict[str, pa.Array]:
    """Job-global sorted dictionary of every string column (``parallel/dictionary.py``)."""
    from ..parallel.dictionary import union_sorted
    out = {}
    for name in t.column_names:
        if is_string(t.schema.field(name).type):
            c = t.column(name).combine_chunks()
            if pa.types.is_dictionary(c.type):
                c = c.cast(c.type.value_type)
            out[name] = union_sorted(c, dist)
    return out


def _prepare_out_dir(out_path: str, mode: str, dist) -> None:
    import shutil
    local = P.to_local(out_path)
    if dist is None or dist.rank == 0:
        if mode == "overwrite" and os.path.exists(local):
            shutil.rmtree(local)
        os.makedirs(local, exist_ok=True)
    if dist is not None:
        dist.barrier()


def _sort_and_write(session, table: Dict[str, DeviceColumn], names: List[str], bucket,
                    indexed: List[str], num_buckets: int, out_path: str, schema: pa.Schema,
                    task_id: int, presorted: bool = False, seed=None, perm=None) -> List[str]:
    """Sort rows by (bucket, indexed columns) and write one file per bucket.  ``presorted``:
    the rows already are in that order (a rewrite of single sorted files per bucket), so no
    sort or gather runs; ``perm``: that order as a row permutation (merged runs, K6)."""
    import torch
    n = int(bucket.numel())
    if n == 0:
        return []
    t0 = time.perf_counter()
    if presorted:
        gathered = [table[c] for c in names]
    else:
        if perm is None:
            perm = K.sort_permutation([table[c] for c in indexed], extra_leading=(bucket, 16))
        gathered = K.gather_columns([table[c] for c in names], perm)
    counts = K.histogram(bucket, num_buckets)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    off = np.concatenate([[0], np.cumsum(counts.cpu().numpy())]).astype(np.int64)
    codec = HyperspaceConf.index_file_codec(session.conf)
    rg = HyperspaceConf.index_row_group_rows(session.conf)
    job = str(uuid.uuid4())
    from . import staging
    paths = None
    if codec in ("none", "uncompressed", "snappy") and \
            os.environ.get("HS_NATIVE_PQ_WRITE", "1") == "1":
        # K4 on the device: dictionary build + bit-packing in HIP, host only frames pages
        from . import pq_encode
        from ..io.writer import bucket_file_name
        local = P.to_local(out_path)
        os.makedirs(local, exist_ok=True)
        paths = pq_encode.write_buckets(
            dict(zip(names, gathered)), names, schema, off,
            lambda b: os.path.join(local, bucket_file_name(task_id, job, b, codec)), rg,
            bucket.device, codec="none" if codec == "uncompressed" else codec)
    LAST_BUILD_STATS["writer"] = "device" if paths is not None else "host"
    if paths is None:
        from . import pq_encode
        LAST_BUILD_STATS["writer_fallback"] = pq_encode.LAST_FALLBACK.get("reason") or \
            ("codec " + codec if codec not in ("none", "uncompressed", "snappy") else "disabled")
        paths = staging.download_buckets(
            gathered, names, schema, off,
            lambda t, b: write_bucket_file(t, out_path, task_id, job, b, codec, rg),
            bucket.device)
    LAST_BUILD_STATS.update({"sort_gather_s": t1 - t0,
                             "d2h_write_s": time.perf_counter() - t1})
    if paths is not None:
        from . import pq_encode
        LAST_BUILD_STATS["write_phases_s"] = {k: round(v, 4) for k, v in
                                              pq_encode.WRITE_PHASES.items()}
        pq_encode.WRITE_PHASES.clear()
    if seed is not None and paths:
        # the sorted bucket-major columns are exactly what a query would load back from these
        # files: hand them to the device table cache instead of freeing them
        from .device_cache import register_seed
        register_seed(session, paths, dict(zip(names, gathered)), off, *seed)
    return paths


# decoded source bytes x this = HBM a one-pass build peaks at: source columns, bucket ids, sort
# keys and permutation (radix_sort.hip), and the gathered bucket-major copy
BUILD_SORT_FACTOR = 3.0


def plan_passes(est_bytes: int, budget: int, num_buckets: int) -> List[tuple]:
    """Bucket ranges [lo, hi) of a streaming build: one range when ``est_bytes`` fits the
    budget, else ceil(est / budget) contiguous ranges of (near) equal bucket counts (Murmur3
    spreads rows evenly over buckets), at most one bucket each."""
    passes = 1 if budget <= 0 or est_bytes <= budget else -(-int(est_bytes) // int(budget))
    passes = max(1, min(int(num_buckets), passes))
    edges = np.linspace(0, num_buckets, passes + 1).round().astype(int)
    return [(int(a), int(b)) for a, b in zip(edges[:-1], edges[1:]) if b > a]


def plan_file_groups(rows: List[int], row_bytes: int, group_budget: int) -> List[tuple]:
    """Consecutive file ranges [a, b) whose decoded bytes stay within ``group_budget`` (a
    single file larger than that is a group of its own)."""
    groups, a, acc = [], 0, 0
    for i, r in enumerate(rows):
        b = int(r) * int(row_bytes)
        if i > a and acc + b > group_budget:
            groups.append((a, i))
            a, acc = i, 0
        acc += b
    if a < len(rows):
        groups.append((a, len(rows)))
    return groups


def _build_budget(session, device) -> int:
    """The build's HBM budget: ``build.hbmBudgetBytes`` (0 = 60% of the free HBM now), capped
    by this rank's share of the device when ranks share it (exec/hbm_budget.py)."""
    import torch
    from .hbm_budget import rank_budget
    b = HyperspaceConf.build_hbm_budget_bytes(session.conf)
    free = 0
    if b <= 0:
        free, _ = torch.cuda.mem_get_info(device)
    return rank_budget(session.conf, device).build(b, free)


def _streaming_plan(session, rel, my_files, columns, lineage_ids, num_buckets, device, world):
    """(passes, file groups, row bytes, nullable columns, string dictionaries) when this rank's
    build does not fit the HBM budget (``spark.hyperspace.mi.build.hbmBudgetBytes``), else
    None.  Covers Parquet builds on any number of ranks.  String columns get their job-global
    sorted dictionary up front (``_string_dictionaries``), so every file group's codes map onto
    one code space before they are kept, exchanged and sorted."""
    dist = getattr(session, "dist", None) if world > 1 else None
    from ..io.reader import output_schema
    from .device_table import storage_numpy_dtype
    schema = output_schema(rel.data_schema, rel.location.partition_spec, columns)
    eligible = source_format(rel) == "parquet"
    if dist is None and (not eligible or not my_files):
        return None
    if dist is not None and dist.agree_any([not eligible])[0]:
        return None                  # unanimous: every rank takes the same build path
    from . import staging
    tf = time.perf_counter()
    infos = list(staging.io_pool().map(lambda f: _footer_info(f, list(schema.names)), my_files))
    LAST_BUILD_STATS["plan_footers_s"] = round(time.perf_counter() - tf, 4)
    rows = [r for r, _ in infos]
    row_bytes = sum(storage_numpy_dtype(f.type).itemsize + 1 for f in schema) + \
        (8 if lineage_ids is not None else 0) + 4
    # a rank holds its own decoded rows plus, after the exchange, its buckets' rows
    est = int(sum(rows) * row_bytes * BUILD_SORT_FACTOR)
    tb = time.perf_counter()
    budget = _build_budget(session, device)
    LAST_BUILD_STATS["plan_budget_s"] = round(time.perf_counter() - tb, 4)
    passes = plan_passes(est, budget, num_buckets)
    if dist is not None:
        # every rank runs the same passes and exchange batches (each batch is a collective)
        npass = int(dist.all_reduce_max_float(float(len(passes))))
        if npass <= 1:
            return None
        edges = np.linspace(0, num_buckets, min(npass, num_buckets) + 1).round().astype(int)
        passes = [(int(a), int(b)) for a, b in zip(edges[:-1], edges[1:]) if b > a]
        # the one-pass build's file batches (_upload_parquet), so rows of a bucket reach the
        # stable sort in the same (batch, source rank, row) order: byte-identical files
        k = int(dist.all_reduce_max_float(float(-(-len(my_files) // FILES_PER_BATCH))))
        fe = np.linspace(0, len(my_files), max(k, 1) + 1).round().astype(int)
        groups = [(int(a), int(b)) for a, b in zip(fe[:-1], fe[1:])]
        fixed = list(schema.names)
        may = set().union(*[m for _, m in infos]) if infos else set()
        part_names = {f.name for f in rel.location.partition_spec.columns} \
            if rel.location.partition_spec is not None else set()
        may |= {n for n in fixed if n in part_names or n not in rel.data_schema.names}
        agreed = dist.agree_any([n in may for n in fixed])
        nullable = {n for n, a in zip(fixed, agreed) if a}
        return passes, groups, row_bytes, nullable, _string_dictionaries(rel, my_files, schema,
                                                                         dist, device, groups)
    if len(passes) <= 1:
        return None
    groups = plan_file_groups(rows, row_bytes, max(budget // 4, 1))
    return (passes, groups, row_bytes, None,
            _string_dictionaries(rel, my_files, schema, None, device, groups))


def _string_dictionaries(rel, my_files, schema, dist, device=None,
                         groups=None) -> Dict[str, pa.Array]:
    """Job-global sorted dictionary of every string column of a streaming build, over all
    ranks.  Parquet columns decode on the device, file group by file group (``groups``), and
    contribute the dictionaries ``staging.finish_strings`` gives them - dictionary pages parsed,
    PLAIN pages hashed on the device (io/native_parquet.StringCodes) - so no string is decoded
    on the host; without the device page path the files' dictionary pages are read as
    dictionary arrays (plain-encoded pages contribute their values)."""
    import pyarrow.parquet as pq
    from ..parallel.dictionary import union_sorted
    from . import staging
    names = [f.name for f in schema if is_string(f.type)]
    if not names:
        return {}
    part_names = {f.name for f in rel.location.partition_spec.columns} \
        if rel.location.partition_spec is not None else set()
    file_cols = [n for n in names if n not in part_names and n in rel.data_schema.names]
    dev_parts: Dict[str, list] = {}
    if device is not None and file_cols and staging.native_decode_enabled() and \
            staging.device_strings_enabled() and my_files:
        sch = pa.schema([rel.data_schema.field(c) for c in file_cols])
        for a, b in (groups or [(0, len(my_files))]):
            fs = my_files[a:b]
            if not fs:
                continue
            rows = list(staging.io_pool().map(
                lambda f: pq.ParquetFile(P.to_local(f)).metadata.num_rows, fs))
            up = staging.upload_files(
                lambda f, cols=None: pq.read_table(P.to_local(f), columns=cols or file_cols),
                fs, rows, sch, device, parquet_local=[P.to_local(f) for f in fs],
                device_pages=True)
            cols = dict(up.columns)
            staging.finish_strings(up, cols, device, None)
            for n in file_cols:
                dev_parts.setdefault(n, []).append(cols[n].dictionary)
            del up, cols
        file_cols = []

    def values(f):
        out = {}
        if file_cols:
            t = pq.read_table(P.to_local(f), columns=file_cols, read_dictionary=file_cols)
            for n in file_cols:
                vals = []
                for ch in t.column(n).chunks:
                    vals.append(ch.dictionary if pa.types.is_dictionary(ch.type)
                                else pc.unique(ch))
                out[n] = vals
        rest = [n for n in names if n not in file_cols and n not in dev_parts]
        if rest:
            from ..io.reader import read_files
            t = read_files("parquet", [f], rel.data_schema, rel.options,
                           rel.location.partition_spec, rest)
            for n in rest:
                out[n] = [pc.unique(t.column(n).combine_chunks())]
        return out
    per_file = list(staging.io_pool().map(values, my_files)) \
        if len(names) > len(dev_parts) else []
    dicts = {}
    for n in names:
        parts = [a.cast(pa.string()) for v in per_file for a in v.get(n, [])] + \
            [a.cast(pa.string()) for a in dev_parts.get(n, [])]
        local = pa.concat_arrays(parts) if parts else pa.array([], pa.string())
        dicts[n] = union_sorted(local, dist)
    return dicts


def _to_dictionary(c: DeviceColumn, gd: pa.Array) -> DeviceColumn:
    """``c``'s codes re-expressed over ``gd`` (a superset of its dictionary), on the device."""
    import torch
    from ..parallel.dictionary import remap_table
    if c.dictionary is None or c.dictionary.equals(gd):
        return DeviceColumn(c.data, c.valid, c.atype, gd)
    data = c.data
    if len(c.dictionary) and len(data):
        tab = torch.from_numpy(remap_table(c.dictionary, gd)).to(data.device)
        data = K.lookup_i32(tab, data)
    return DeviceColumn(data, c.valid, c.atype, gd)


def _streaming_build(session, rel, my_files, columns, indexed, num_buckets, out_path,
                     lineage_ids, device, plan, rank) -> List[str]:
    """Build in bucket-range passes: each pass re-decodes the source file group by group,
    hashes every row and keeps only its buckets' rows (in source order), then sorts and writes
    those buckets.  Rows of a bucket meet the stable sort in the one-pass build's order, so the
    bucket files are byte-identical to a one-pass build's; HBM holds one decoded file group plus
    one pass's rows instead of the whole input."""
    import torch
    passes, groups, _, nullable, sdicts = plan
    dist = getattr(session, "dist", None)
    multi = dist is not None and dist.world > 1
    paths: List[str] = []
    t0 = time.perf_counter()
    decode_s = sort_s = 0.0
    sent_total = 0
    source_bytes = 0
    schema = names = None
    for pi, (lo, hi) in enumerate(passes):
        parts: Dict[str, list] = {}
        buckets = []
        ex = None
        for a, b in groups:
            td = time.perf_counter()
            cols, names, schema = _upload_parquet(rel, my_files[a:b], columns, indexed,
                                                  lineage_ids, device, None,
                                                  nullable_override=nullable)
            for n, gd in sdicts.items():
                cols[n] = _to_dictionary(cols[n], gd)
            if pi == 0:
                source_bytes += sum(c.nbytes() for c in cols.values())
            n_rows = len(cols[names[0]]) if names else 0
            if n_rows:
                bucket, _ = K.murmur3_bucket([cols[c] for c in indexed], num_buckets,
                                             with_counts=False)
            else:
                bucket = torch.empty(0, dtype=torch.int32, device=device)
            keep = torch.nonzero((bucket >= lo) & (bucket < hi)).squeeze(1)
            got = K.gather_columns([cols[n] for n in names], keep)
            kb = bucket.index_select(0, keep)
            if multi:
                # rows of this pass's buckets go to their owner rank (b % world): one packed
                # all-to-all per file batch, every rank the same number of batches
                from ..parallel.exchange import RowExchange
                vnames = [n for n in names if n in (nullable or set())]
                send = [c.data for c in got] + \
                    [(c.valid if c.valid is not None else
                      torch.ones(c.data.shape[0], dtype=torch.uint8, device=device))
                     for n, c in zip(names, got) if n in vnames] + [kb]
                if ex is None:
                    ex = RowExchange(dist, [t.dtype for t in send], device)
                ex.add(send, kb)
            else:
                for n, c in zip(names, got):
                    parts.setdefault(n, []).append(c)
                buckets.append(kb)
            del cols, bucket, keep, got, kb
            torch.cuda.synchronize()
            decode_s += time.perf_counter() - td
        ts = time.perf_counter()
        if multi:
            recv = ex.finish() if ex is not None else None
            if ex is not None:
                sent_total += ex.sent_bytes
            vnames = [n for n in names if n in (nullable or set())]
            table = {}
            vi = len(names)
            for j, n in enumerate(names):
                valid = None
                if n in vnames:
                    valid = recv[vi]
                    vi += 1
                atype = schema.field(n).type if n in schema.names else pa.int64()
                table[n] = DeviceColumn(recv[j], valid, atype, sdicts.get(n))
            paths += _sort_and_write(session, table, names, recv[-1], indexed, num_buckets,
                                     out_path, schema, rank)
            del table, recv
            sort_s += time.perf_counter() - ts
            continue
        table = {}
        for n in names:
            cs = parts[n]
            data = torch.cat([c.data for c in cs])
            valid = None
            if any(c.valid is not None for c in cs):
                valid = torch.cat([c.valid if c.valid is not None else
                                   torch.ones(c.data.shape[0], dtype=torch.uint8, device=device)
                                   for c in cs])
            table[n] = DeviceColumn(data, valid, cs[0].atype, cs[0].dictionary)
        del parts
        paths += _sort_and_write(session, table, names, torch.cat(buckets), indexed,
                                 num_buckets, out_path, schema, rank)
        del table, buckets
        sort_s += time.perf_counter() - ts
    if multi:
        dist.barrier()
    from . import staging
    LAST_BUILD_STATS.update({"passes": len(passes), "file_groups": len(groups),
                             "source_bytes": source_bytes, "exchange_sent_bytes": sent_total,
                             "pass_decode_s": decode_s, "pass_sort_write_s": sort_s,
                             "total_s": time.perf_counter() - t0,
                             "host_decoded": sorted(staging.HOST_DECODED),
                             "device_decoded": sorted(staging.DEVICE_DECODED)})
    return paths


def device_build_from_source(session, rel, files: List[str], columns: List[str], indexed: List[str],
                             num_buckets: int, out_path: str, lineage_ids: Optional[Dict[str, int]],
                             mode: str = "overwrite") -> List[str]:
    import torch
    dist = getattr(session, "dist", None)
    rank, world = (dist.rank, dist.world) if dist is not None else (0, 1)
    device = torch.device("cuda", torch.cuda.current_device())
    _prepare_out_dir(out_path, mode, dist)
    t0 = time.perf_counter()
    _T0[0] = t0
    my_files = files[rank::world]
    fmt = source_format(rel)
    from . import staging
    staging.HOST_DECODED.clear()
    staging.DEVICE_DECODED.clear()
    from ..io import native_parquet
    native_parquet.PHASES.clear()
    xs = _BatchedExchange(dist, num_buckets, indexed) if world > 1 else None
    LAST_BUILD_STATS.clear()
    tp = time.perf_counter()
    splan = _streaming_plan(session, rel, my_files, columns, lineage_ids, num_buckets, device,
                            world)
    LAST_BUILD_STATS["pass_plan_s"] = round(time.perf_counter() - tp, 4)
    if splan is not None:
        return _streaming_build(session, rel, my_files, columns, indexed, num_buckets, out_path,
                                lineage_ids, device, splan, rank)
    if fmt == "parquet":
        cols, names, schema = _upload_parquet(rel, my_files, columns, indexed, lineage_ids,
                                              device, dist, xs)
    else:
        cols, names, schema = _upload_generic(rel, files, my_files, columns, indexed, lineage_ids,
                                              device, dist)
    t1 = time.perf_counter()
    source_bytes = sum(c.nbytes() for c in cols.values())
    if xs is None:
        bucket, _ = K.murmur3_bucket([cols[c] for c in indexed], num_buckets, with_counts=False)
    else:
        if not xs.started:     # string columns: one batch once the global dictionaries exist
            xs.batch_all(cols, names)
        cols, bucket = xs.finish(cols, names)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    paths = _sort_and_write(session, cols, names, bucket, indexed, num_buckets, out_path, schema,
                            rank, seed=(rank, world, num_buckets))
    if dist is not None:
        dist.barrier()
    LAST_BUILD_STATS.update({"read_h2d_s": t1 - t0, "hash_exchange_s": t2 - t1,
                             "total_s": time.perf_counter() - t0, "source_bytes": source_bytes,
                             "host_decoded": sorted(staging.HOST_DECODED),
                             "device_decoded": sorted(staging.DEVICE_DECODED),
                             "upload_wall_s": dict(staging.UPLOAD_TIMES),
                             "decode_phases_s": {k: round(v, 4) for k, v in
                                                 native_parquet.PHASES.items()}})
    if xs is not None:
        LAST_BUILD_STATS.update({"exchange_batches": xs.nbatches,
                                 "exchange_sent_bytes": xs.sent_bytes})
    return paths


class _BatchedExchange:
    """Multi-GPU build shuffle: every batch of decoded source rows is hashed (Spark Murmur3 on
    the indexed columns) and sent to its owner ranks (bucket % world) with one packed
    all-to-all while the staging pool decodes the next files (``parallel/exchange.py``).
    Which columns carry a validity mask is agreed before the first batch, so every rank sends
    the same column list."""

    def __init__(self, dist, num_buckets: int, indexed: List[str]):
        self.dist, self.num_buckets, self.indexed = dist, num_buckets, indexed
        self.ex = None
        self.started = False
        self.nbatches = 0
        self.sent_bytes = 0

    def batch(self, cols: Dict[str, DeviceColumn], names: List[str], lo: int, hi: int) -> None:
        from ..parallel.exchange import RowExchange
        sl = {n: cols[n] for n in names}
        part = [DeviceColumn(c.data[lo:hi], None if c.valid is None else c.valid[lo:hi],
                             c.atype, c.dictionary, c.offsets, c.chars)
                for c in (sl[n] for n in self.indexed)]
        if any(c.offsets is not None for c in part):
            raise ValueError("batched exchange over raw-string keys: hash the whole upload")
        bucket, _ = K.murmur3_bucket(part, self.num_buckets, with_counts=False)
        send = [sl[n].data[lo:hi] for n in names] + \
            [sl[n].valid[lo:hi] for n in names if sl[n].valid is not None] + [bucket]
        if self.ex is None:
            self.ex = RowExchange(self.dist, [t.dtype for t in send], bucket.device)
        self.ex.add(send, bucket)
        self.started = True
        self.nbatches += 1

    def batch_all(self, cols, names) -> None:
        """One whole-upload batch (string columns: their codes exist only once the job-global
        dictionaries are built; indexed strings hash from raw bytes)."""
        import torch
        from ..parallel.exchange import RowExchange
        need = self.dist.agree_any([cols[n].valid is not None for n in names])
        for n, nv in zip(names, need):
            if nv and cols[n].valid is None:
                cols[n].valid = torch.ones(len(cols[n]), dtype=torch.uint8,
                                           device=cols[n].data.device)
        bucket, _ = K.murmur3_bucket([cols[c] for c in self.indexed], self.num_buckets,
                                     with_counts=False)
        send = [cols[n].data for n in names] + \
            [cols[n].valid for n in names if cols[n].valid is not None] + [bucket]
        self.ex = RowExchange(self.dist, [t.dtype for t in send], bucket.device)
        self.ex.add(send, bucket)
        self.started = True
        self.nbatches += 1

    def finish(self, cols: Dict[str, DeviceColumn], names: List[str]):
        if not self.started:
            raise RuntimeError("exchange finished before any batch")
        got = self.ex.finish()
        self.sent_bytes = self.ex.sent_bytes
        out = {}
        vi = len(names)
        for j, n in enumerate(names):
            c = cols[n]
            v = None
            if c.valid is not None:
                v = got[vi]
                vi += 1
            out[n] = DeviceColumn(got[j], v, c.atype, c.dictionary)
        return out, got[-1]


def _finish_strings(up, cols: Dict[str, DeviceColumn], indexed, device, dist) -> None:
    """Dictionary-encode string columns with a job-global sorted dictionary and upload codes.
    Columns whose dictionary pages the device decoded are remapped on the device
    (``staging.finish_strings``); the rest come from the host chunks."""
    from . import staging
    staging.finish_strings(up, cols, device, dist, names=list(up.device_strings))
    for name, chunks in up.host_strings.items():
        if name in up.device_strings:
            continue
        chunks = [c for c in chunks if c is not None]
        if name not in indexed and chunks and \
                all(pa.types.is_dictionary(c.type) for c in chunks):
            cols[name] = _dictionary_codes(chunks, device, dist)
            continue
        arr = pa.chunked_array(chunks, type=chunks[0].type) if chunks else pa.chunked_array([], pa.string())
        if pa.types.is_dictionary(arr.type):
            arr = arr.cast(pa.string())
        d = _global_dicts(pa.table({name: arr}), dist)[name]
        cols[name] = DeviceColumn.from_arrow(arr, device, d, raw_strings=name in indexed)


def _dictionary_codes(chunks, device, dist) -> DeviceColumn:
    """String column read as Parquet dictionary pages + indices (never materialised as strings
    on the host): the job-global sorted dictionary is the union of the (small) per-chunk
    dictionaries; each chunk's indices cross PCIe as int32 and are remapped to global codes
    on the device with one gather through that chunk's local -> global table."""
    import torch
    parts = [ch for c in chunks for ch in c.chunks]
    from ..parallel.dictionary import union_sorted
    local = [ch.dictionary.cast(pa.string()) for ch in parts]
    u = pa.concat_arrays(local) if local else pa.array([], pa.string())
    gdict = union_sorted(u, dist)
    n = sum(len(ch) for ch in parts)
    codes = torch.empty(n, dtype=torch.int32, device=device)
    valid = None
    if any(ch.null_count for ch in parts):
        valid = torch.ones(n, dtype=torch.uint8, device=device)
    off = 0
    for ch, d in zip(parts, local):
        m = len(ch)
        if m:
            remap = pc.index_in(d, value_set=gdict).to_numpy(zero_copy_only=False)
            remap_d = torch.from_numpy(np.array(remap, dtype=np.int32)).to(device)
            idx = np.asarray(ch.indices.fill_null(0).to_numpy(zero_copy_only=False),
                             dtype=np.int64)
            idx_d = torch.from_numpy(idx).to(device, non_blocking=False)
            codes[off:off + m] = remap_d[idx_d] if len(d) else 0
            if ch.null_count:
                vm = np.asarray(ch.is_valid().to_numpy(zero_copy_only=False), dtype=np.uint8)
                valid[off:off + m] = torch.from_numpy(vm).to(device)
        off += m
    return DeviceColumn(codes, valid, pa.string(), gdict)


def _footer_info(path: str, names: List[str]):
    """(rows, columns that may hold nulls) from one Parquet footer: a column counts as
    nullable unless every row group's statistics say null_count == 0."""
    import pyarrow.parquet as pq
    md = pq.ParquetFile(P.to_local(path)).metadata
    want = set(names)
    maybe = set()
    seen = set()
    for g in range(md.num_row_groups):
        rg = md.row_group(g)
        for c in range(rg.num_columns):
            cc = rg.column(c)
            nm = cc.path_in_schema
            if nm in want:
                seen.add(nm)
                st = cc.statistics
                if st is None or not st.has_null_count or st.null_count > 0:
                    maybe.add(nm)
    # not covered by this footer (partition columns, columns missing from the file): unknown
    maybe |= want - seen
    return md.num_rows, maybe


def _upload_parquet(rel, my_files, columns, indexed, lineage_ids, device, dist, xs=None,
                    nullable_override=None):
    """Pipelined decode -> pinned -> HBM upload of this rank's Parquet files (staging.py).
    With a multi-GPU exchange ``xs`` and no string columns, every batch of files is hashed and
    exchanged as soon as it is on the device, overlapping the decode of the next batch."""
    import pyarrow.parquet as pq
    from ..io.reader import output_schema, read_files
    from . import staging
    schema = output_schema(rel.data_schema, rel.location.partition_spec, columns)
    LAST_BUILD_STATS["pre_upload_s"] = round(time.perf_counter() - _T0[0], 4)
    tf = time.perf_counter()
    infos = list(staging.io_pool().map(lambda f: _footer_info(f, list(schema.names)), my_files))
    counts = [r for r, _ in infos]
    LAST_BUILD_STATS["footers_s"] = round(time.perf_counter() - tf, 4)

    want = columns
    part_names = {f.name for f in rel.location.partition_spec.columns} \
        if rel.location.partition_spec is not None else set()
    # included string columns are read as dictionary pages + indices (_dictionary_codes)
    dict_cols = [c for c in want if c not in indexed and c not in part_names and
                 c in rel.data_schema.names and is_string(rel.data_schema.field(c).type)]

    def read_file(f, cols=None):
        cols = want if cols is None else cols
        dcols = [c for c in cols if c in dict_cols]
        rest = [c for c in cols if c not in dcols]
        t = read_files("parquet", [f], rel.data_schema, rel.options,
                       rel.location.partition_spec, rest)
        if dcols:
            d = pq.read_table(P.to_local(f), columns=dcols, read_dictionary=dcols)
            for c in dcols:
                t = t.append_column(c, d.column(c))
            t = t.select(cols)
        return t
    lin = [lineage_ids[f] for f in my_files] if lineage_ids is not None else None
    names = list(schema.names)
    fields = list(schema)
    if lineage_ids is not None:
        names.append(C.DATA_FILE_NAME_ID)
        fields.append(pa.field(C.DATA_FILE_NAME_ID, pa.int64(), False))
    on_batch, nullable, batches = None, None, None
    if xs is not None and not any(is_string(f.type) for f in schema):
        fixed = [f.name for f in schema]
        may = set().union(*[m for _, m in infos]) if infos else set()
        # partition columns are not in the Parquet footers and may be null
        # (__HIVE_DEFAULT_PARTITION__): a mask that appeared mid-upload on one rank would send
        # one column more than its peers in the next collective batch
        may |= {n for n in fixed if n in part_names or n not in rel.data_schema.names}
        agreed = dist.agree_any([n in may for n in fixed])
        nullable = {n for n, a in zip(fixed, agreed) if a}
        on_batch = (lambda cols, lo, hi: xs.batch(cols, names, lo, hi))
        # every rank runs the same number of batches (each is a collective); ranks with fewer
        # files send empty batches
        k = int(dist.all_reduce_max_float(float(-(-len(my_files) // FILES_PER_BATCH))))
        edges = np.linspace(0, len(my_files), max(k, 1) + 1).round().astype(int)
        batches = [(int(a), int(b)) for a, b in zip(edges[:-1], edges[1:])]
    if nullable_override is not None:
        nullable = set(nullable_override)
    tu = time.perf_counter()
    up = staging.upload_files(read_file, my_files, counts, schema, device, lin,
                              C.DATA_FILE_NAME_ID,
                              parquet_local=[P.to_local(f) for f in my_files],
                              nullable=nullable, on_batch=on_batch, file_batches=batches)
    LAST_BUILD_STATS["upload_files_s"] = round(time.perf_counter() - tu, 4)
    cols = dict(up.columns)
    _finish_strings(up, cols, indexed, device, dist)
    return {n: cols[n] for n in names}, names, pa.schema(fields)


def _upload_generic(rel, files, my_files, columns, indexed, lineage_ids, device, dist):
    """Non-Parquet sources (CSV/JSON/ORC/text): host decode of the whole share, then upload."""
    from ..io.reader import read_files
    t = read_index_input(rel, my_files, columns, lineage_ids) if my_files else None
    if t is None:
        t = read_files(source_format(rel), files[:1], rel.data_schema, rel.options,
                       rel.location.partition_spec, columns).slice(0, 0)
        if lineage_ids is not None:
            t = t.append_column(pa.field(C.DATA_FILE_NAME_ID, pa.int64(), False),
                                pa.array([], pa.int64()))
    dicts = _global_dicts(t, dist)
    cols = {n: DeviceColumn.from_arrow(t.column(n), device, dicts.get(n),
                                       raw_strings=(n in indexed and n in dicts))
            for n in t.column_names}
    return cols, list(t.column_names), t.schema


def device_rewrite_buckets(session, files: List[str], indexed: List[str], out_path: str,
                           deleted_ids: Optional[List[int]], num_buckets: Optional[int]) -> List[str]:
    """K5/K6 on the device: rewrite this rank's buckets (``bucket % world == rank``) of existing
    index files, dropping rows whose lineage id is deleted.

    The files go through the same native page decode as a build (``staging.upload_files``); the
    bucket id of every row is a per-file constant written by the lineage fill.  Rows arrive
    bucket-major in file order.  When every bucket holds a single (sorted) file, a stable
    compaction keeps that order, so the rows are written without any sort
    (``RefreshIncrementalAction.scala:73-95``: deleted-file rows are filtered out of the old index
    data); buckets with several files (``OptimizeAction.scala:85-99``) are merged by the stable
    (bucket, indexed columns) radix sort."""
    import pyarrow.parquet as pq
    import torch
    dist = getattr(session, "dist", None)
    rank, world = (dist.rank, dist.world) if dist is not None else (0, 1)
    device = torch.device("cuda", torch.cuda.current_device())
    groups = group_by_bucket(files)
    if -1 in groups:
        raise ValueError("index files without bucket ids")
    mine = sorted(b for b in groups if b >= 0 and b % world == rank)
    paths_in = [f for b in mine for f in groups[b]]
    if not paths_in:
        return []
    t0 = time.perf_counter()
    file_bucket = [b for b in mine for _ in groups[b]]
    schema = pq.read_schema(P.to_local(paths_in[0]))
    schema = pa.schema([pa.field(f.name, f.type.value_type if pa.types.is_dictionary(f.type)
                                 else f.type, f.nullable) for f in schema])
    names = list(schema.names)
    from . import staging
    infos = list(staging.io_pool().map(lambda f: _footer_info(f, names), paths_in))
    counts = [r for r, _ in infos]
    nullable = set().union(*[m for _, m in infos]) if infos else set()

    def read_file(f, cols=None):
        return pq.read_table(P.to_local(f), columns=names if cols is None else cols)
    bname = "__hs_bucket"
    up = staging.upload_files(read_file, paths_in, counts, schema, device, file_bucket, bname,
                              parquet_local=[P.to_local(f) for f in paths_in],
                              nullable={n for n in nullable if not is_string(schema.field(n).type)},
                              device_pages=False)
    cols = dict(up.columns)
    bucket = cols.pop(bname).data.to(torch.int32)
    _finish_strings(up, cols, indexed, device, None)
    n = up.num_rows
    if deleted_ids:
        # K5: lineage NOT IN deleted -> bitmap probe + stable compaction, fused in one scan kernel
        from ..ops import _lib as NL
        ids = sorted(set(int(i) for i in deleted_ids))
        words = np.zeros(ids[-1] // 64 + 1, dtype=np.uint64)
        for i in ids:
            words[i >> 6] |= np.uint64(1) << np.uint64(i & 63)
        wt = torch.from_numpy(words.view(np.int64)).to(device)
        lin = cols[C.DATA_FILE_NAME_ID]
        p = NL.ScanParams()
        p.cols[0] = lin.desc()
        p.preds[0] = NL.Pred(NL.PK_BITMAP, NL.OP_NE, 0, 0, 0, len(words), 0, 0.0, wt.data_ptr())
        p.npreds, p.naggs, p.group_col = 1, 0, -1
        rstart, rlen, _ = K.full_ranges(np.array([0, n], np.int64), device)
        tp = K.ranges_to_tiles(rlen)
        rows = K.scan_select(p, rstart, rlen, tp, n // NL.lib().hs_scan_tile_rows() + 2)
        kept = K.gather_columns([cols[c] for c in names] +
                                [DeviceColumn(bucket, None, pa.int32())], rows)
        cols = dict(zip(names, kept[:-1]))
        bucket = kept[-1].data
    presorted = all(len(groups[b]) == 1 for b in mine)
    perm, how = None, "none" if presorted else "radix"
    if not presorted and os.environ.get("HS_MERGE_PATH", "1") == "1":
        # K6: every file is a sorted run; merge the runs of each bucket instead of re-sorting
        run_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        if deleted_ids:
            # runs after the stable compaction: kept rows below each file's first row
            b_at = torch.from_numpy(run_off).to(device=device, dtype=rows.dtype)
            run_off = torch.searchsorted(rows.contiguous(), b_at).cpu().numpy().astype(np.int64)
        perm = K.merge_runs_permutation([cols[c] for c in indexed], run_off,
                                        np.asarray(file_bucket))
        if perm is not None:
            how = "merge-path"
    t1 = time.perf_counter()
    out = _sort_and_write(session, cols, names, bucket, indexed,
                          num_buckets or (max(mine) + 1), out_path, schema, rank,
                          presorted=presorted, perm=perm)
    LAST_BUILD_STATS.update({"rewrite_read_h2d_s": t1 - t0, "rewrite_presorted": presorted,
                             "rewrite_sort": how,
                             "rewrite_files": len(paths_in),
                             "rewrite_total_s": time.perf_counter() - t0})
    return out
