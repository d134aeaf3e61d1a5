"""Index data builder: the build hot path (SURVEY §3.1 "HOT LOOP", kernels K1-K6).

``build_from_source``  scan source files (K1) -> attach lineage ids (K2, a per-file constant —
                       no broadcast join needed) -> Murmur3 bucket + partition (K3) ->
                       sort within bucket (K4) -> one Parquet file per bucket.
``rewrite_buckets``    per-bucket merge of existing index files, optionally dropping rows whose
                       ``_data_file_id`` was deleted (K5, incremental refresh) — used by optimize
                       (K6) as well.  The bucket is known from the file name, so no re-hash.

Each function dispatches to the MI355X device pipeline (``exec.device_build``) when the session
executes on GPU, or to the host oracle below.  Under ``torch.distributed`` the device pipeline
shuffles rows with RCCL all-to-all so that bucket ``b`` is written by rank ``b % world``.
"""
from __future__ import annotations

import uuid
from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from ..io.reader import read_files
from ..io.writer import get_bucket_id, sort_indices_by, write_bucket_file, write_bucketed_table
from ..utils import path_utils as P
from ..utils.conf import HyperspaceConf
from . import constants as C


def source_format(rel) -> str:
    return "parquet" if rel.file_format == "delta" or rel.is_index() else rel.file_format


def read_index_input(rel, files: List[str], columns: List[str], lineage_ids: Optional[Dict[str, int]]):
    """Read the index columns of ``files`` (+ ``_data_file_id`` when lineage is on)."""
    t, fidx = read_files(source_format(rel), files, rel.data_schema, rel.options,
                         rel.location.partition_spec, columns, with_file_index=True)
    if lineage_ids is not None:
        ids = np.array([lineage_ids[f] for f in files], dtype=np.int64)
        fi = fidx.to_numpy() if hasattr(fidx, "to_numpy") else np.asarray(fidx)
        t = t.append_column(pa.field(C.DATA_FILE_NAME_ID, pa.int64(), False),
                            pa.array(ids[np.asarray(fi, dtype=np.int64)] if len(fi) else
                                     np.zeros(0, np.int64)))
    return t


def build_from_source(session, rel, files: List[str], columns: List[str], indexed: List[str],
                      num_buckets: int, out_path: str, lineage_ids: Optional[Dict[str, int]],
                      mode: str = "overwrite") -> List[str]:
    if session.device_kind() == "gpu" and _device_hashable(rel, indexed):
        from ..exec.device_build import device_build_from_source
        return device_build_from_source(session, rel, files, columns, indexed, num_buckets,
                                        out_path, lineage_ids, mode)
    dist = getattr(session, "dist", None)
    if dist is not None and dist.world > 1:
        t = _spmd_host_exchange(dist, rel, files, columns, indexed, num_buckets, lineage_ids)
        return _spmd_host_write(session, dist, t, out_path, num_buckets, indexed, mode)
    t = read_index_input(rel, files, columns, lineage_ids)
    return write_bucketed_table(t, out_path, num_buckets, indexed, mode,
                                HyperspaceConf.index_file_codec(session.conf),
                                HyperspaceConf.index_row_group_rows(session.conf),
                                job_uuid=str(uuid.uuid4()))


def _device_hashable(rel, indexed: List[str]) -> bool:
    """The device Murmur3 kernel hashes decimals from float64 storage, exact only up to
    precision 15 (``ops.kernels.hash_xform``); wider decimal keys use the host build."""
    names = set(rel.data_schema.names)
    for c in indexed:
        if c in names:
            t = rel.data_schema.field(c).type
            if pa.types.is_decimal(t) and t.precision > 15:
                return False
    return True


def _columns_for_exchange(t: pa.Table, dicts: Dict[str, pa.Array], need_valid: List[bool]):
    """numpy columns of ``t`` in exchange form: fixed-width storage values (strings as codes
    into the job-global dictionary; decimal128 as two int64 words), then validity bytes."""
    from ..exec.staging import fixed_width_numpy
    vals, valids = [], []
    for name, nv in zip(t.column_names, need_valid):
        a = t.column(name).combine_chunks()
        if pa.types.is_dictionary(a.type):
            a = a.cast(a.type.value_type)
        valid = np.asarray(a.is_valid().to_numpy(zero_copy_only=False), dtype=np.uint8) \
            if a.null_count else None
        if name in dicts:
            codes = pc.index_in(a, value_set=dicts[name]).fill_null(0)
            vals.append([np.asarray(codes.to_numpy(zero_copy_only=False), dtype=np.int32)])
        elif pa.types.is_decimal(a.type):
            words = np.frombuffer(a.buffers()[1], dtype=np.int64)[2 * a.offset:2 * (a.offset + len(a))]
            words = words.reshape(-1, 2)
            vals.append([np.ascontiguousarray(words[:, 0]), np.ascontiguousarray(words[:, 1])])
        else:
            v, _ = fixed_width_numpy(a)
            vals.append([v])
        if nv:
            valids.append(valid if valid is not None else np.ones(len(a), np.uint8))
    return vals, valids


def _table_from_exchange(schema: pa.Schema, dicts, got, need_valid) -> pa.Table:
    from ..exec.device_table import DeviceColumn
    from ..exec.staging import host_to_arrow
    it = iter(got)
    parts = []
    for f in schema:
        k = 2 if pa.types.is_decimal(f.type) else 1
        parts.append([next(it).numpy() for _ in range(k)])
    arrays = []
    for f, p, nv in zip(schema, parts, need_valid):
        valid = next(it).numpy() if nv else None
        if pa.types.is_decimal(f.type):
            words = np.stack([p[0], p[1]], axis=1).reshape(-1)
            vb = None if valid is None else pa.array(valid.astype(bool)).buffers()[1]
            arr = pa.Array.from_buffers(f.type, len(p[0]), [vb, pa.py_buffer(words.tobytes())],
                                        null_count=-1 if vb is not None else 0)
        else:
            fake = DeviceColumn(None, None, f.type, dicts.get(f.name))
            arr = host_to_arrow(fake, p[0], valid)
            if not arr.type.equals(f.type):
                arr = arr.cast(f.type)
        arrays.append(arr)
    return pa.Table.from_arrays(arrays, schema=schema)


def _spmd_host_exchange(dist, rel, files: List[str], columns: List[str], indexed: List[str],
                        num_buckets: int, lineage_ids) -> pa.Table:
    """Host build under ``torch.distributed``: each rank reads its share of the source files
    (``files[rank::world]``), hashes with the Spark Murmur3 oracle, and sends every row to its
    bucket's owner with the packed all-to-all (``parallel/exchange.py``; string columns cross
    as codes into a job-global dictionary, ``parallel/dictionary.py``) — the same exchange the
    device pipeline runs over RCCL, here over gloo."""
    import torch
    from ..io.reader import output_schema
    from ..parallel.dictionary import union_sorted
    from ..parallel.exchange import RowExchange
    from ..utils import murmur3
    mine = files[dist.rank::dist.world]
    if mine:
        t = read_index_input(rel, mine, columns, lineage_ids)
    else:
        sch = output_schema(rel.data_schema, rel.location.partition_spec, columns)
        if lineage_ids is not None:
            sch = sch.append(pa.field(C.DATA_FILE_NAME_ID, pa.int64(), False))
        t = sch.empty_table()
    from ..exec.device_table import is_string
    dicts = {}
    for name in t.column_names:
        if is_string(t.schema.field(name).type):
            a = t.column(name).combine_chunks()
            if pa.types.is_dictionary(a.type):
                a = a.cast(a.type.value_type)
            dicts[name] = union_sorted(a, dist)
    need_valid = dist.agree_any([t.column(n).null_count > 0 for n in t.column_names])
    vals, valids = _columns_for_exchange(t, dicts, need_valid)
    bucket = murmur3.bucket_ids([t.column(c) for c in indexed], num_buckets) if t.num_rows \
        else np.zeros(0, np.int32)
    send = [torch.from_numpy(np.ascontiguousarray(v)) for vs in vals for v in vs] + \
        [torch.from_numpy(v) for v in valids] + [torch.from_numpy(bucket.astype(np.int32))]
    ex = RowExchange(dist, [x.dtype for x in send])
    ex.add(send, send[-1])
    got = ex.finish()
    return _table_from_exchange(t.schema, dicts, got[:-1], need_valid)


def _spmd_host_write(session, dist, t: pa.Table, out_path: str, num_buckets: int,
                     indexed: List[str], mode: str) -> List[str]:
    """Host build under ``torch.distributed``: after the exchange every rank holds exactly the
    rows of the buckets it owns (``b % world == rank``) and writes them as task ``rank`` of one
    job — one file per bucket overall, the layout the device pipeline produces."""
    import os
    err = None
    if dist.rank == 0:
        local = P.to_local(out_path)
        if mode == "overwrite" and os.path.exists(local):
            import shutil
            shutil.rmtree(local)
        elif mode == "errorifexists" and os.path.exists(local):
            err = f"path {out_path} already exists"
        os.makedirs(local, exist_ok=True)
    # one collective carries the job id and the coordinator's verdict, so no rank is left
    # waiting in a barrier the others never reach
    job, err = dist.broadcast_object((str(uuid.uuid4()), err) if dist.rank == 0 else None)
    if err is not None:
        from ..exceptions import HyperspaceException
        raise HyperspaceException(err)
    owned = {b for b in range(num_buckets) if b % dist.world == dist.rank}
    out = write_bucketed_table(t, out_path, num_buckets, indexed, "append",
                               HyperspaceConf.index_file_codec(session.conf),
                               HyperspaceConf.index_row_group_rows(session.conf),
                               task_id=dist.rank, job_uuid=job, buckets_to_write=owned)
    dist.barrier()
    return out


def group_by_bucket(files: List[str]) -> Dict[int, List[str]]:
    out: Dict[int, List[str]] = {}
    for f in files:
        b = get_bucket_id(P.get_name(f))
        out.setdefault(-1 if b is None else b, []).append(f)
    return out


def rewrite_buckets(session, files: List[str], indexed: List[str], out_path: str,
                    deleted_ids: Optional[List[int]] = None, num_buckets: int = None) -> List[str]:
    """Merge every bucket's files into one sorted file, optionally dropping deleted lineage ids."""
    if session.device_kind() == "gpu":
        from ..exec.device_build import device_rewrite_buckets
        return device_rewrite_buckets(session, files, indexed, out_path, deleted_ids, num_buckets)
    import pyarrow.parquet as pq
    codec = HyperspaceConf.index_file_codec(session.conf)
    rg = HyperspaceConf.index_row_group_rows(session.conf)
    job = str(uuid.uuid4())
    out = []
    dist = getattr(session, "dist", None)
    for b, fs in sorted(group_by_bucket(files).items()):
        if dist is not None and b % dist.world != dist.rank:
            continue
        t = pa.concat_tables([pq.read_table(P.to_local(f)) for f in fs])
        if deleted_ids:
            mask = pc.invert(pc.is_in(t.column(C.DATA_FILE_NAME_ID),
                                      value_set=pa.array(deleted_ids, pa.int64())))
            t = t.filter(mask)
        if t.num_rows == 0:
            continue
        if len(fs) > 1:
            t = t.take(pa.array(sort_indices_by(t, indexed)))
        if b < 0:
            out += write_bucketed_table(t, out_path, num_buckets, indexed, "append", codec, rg,
                                        job_uuid=job)
        else:
            out.append(write_bucket_file(t, out_path, 0, job, b, codec, rg))
    return out
