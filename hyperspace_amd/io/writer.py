"""Writers: ``df.write`` and the bucketed index writer (``saveWithBuckets``).

Reference: ``index/DataFrameWriterExtensions.scala:39-81`` — rows are hash-bucketed by the indexed
columns (Spark Murmur3, seed 42, ``pmod`` numBuckets) and sorted by the same columns inside each
bucket; one file per (task, bucket) named ``part-<task:05d>-<uuid>_<bucket:05d>.c000.<codec>.parquet``
so ``BucketingUtils.getBucketId`` (``OptimizeAction.scala:129``) can parse the bucket back.

The host path below is the oracle; the device path (``exec.device_build``) runs hash / partition /
sort on the MI355X and hands each bucket's already-sorted columns to ``write_bucket_file``.
"""
from __future__ import annotations

import os
import re
import uuid
from typing import List, Optional, Sequence

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pyarrow.parquet as pq

from ..exceptions import HyperspaceException
from ..utils import murmur3
from ..utils import path_utils as P

_BUCKET_RE = re.compile(r".*_(\d+)(?:\..*)?$")


def get_bucket_id(file_name: str) -> Optional[int]:
    """Spark ``BucketingUtils.getBucketId``."""
    m = _BUCKET_RE.match(file_name)
    return int(m.group(1)) if m else None


def bucket_file_name(task_id: int, job_uuid: str, bucket: int, codec: str) -> str:
    ext = "" if codec in ("none", "uncompressed") else f".{codec}"
    return f"part-{task_id:05d}-{job_uuid}_{bucket:05d}.c000{ext}.parquet"


def _codec(codec: str) -> str:
    return "none" if codec in ("none", "uncompressed", "plain") else codec


def write_bucket_file(table: pa.Table, directory: str, task_id: int, job_uuid: str, bucket: int,
                      codec: str = "none", row_group_rows: int = 1 << 20) -> str:
    local_dir = P.to_local(directory)
    os.makedirs(local_dir, exist_ok=True)
    name = bucket_file_name(task_id, job_uuid, bucket, _codec(codec))
    path = os.path.join(local_dir, name)
    pq.write_table(table, path, compression=_codec(codec), row_group_size=row_group_rows,
                   use_dictionary=False, write_statistics=True)
    return path


def sort_indices_by(table: pa.Table, cols: Sequence[str]) -> np.ndarray:
    if table.num_rows == 0:
        return np.zeros(0, dtype=np.int64)
    idx = pc.sort_indices(table, sort_keys=[(c, "ascending", "at_start") for c in cols])
    return np.asarray(idx)


def write_bucketed_table(table: pa.Table, path: str, num_buckets: int, bucket_cols: List[str],
                         mode: str = "overwrite", codec: str = "none",
                         row_group_rows: int = 1 << 20, task_id: int = 0,
                         job_uuid: str = None, buckets_to_write=None) -> List[str]:
    """Host reference implementation of the bucketed write (K3+K4 on the CPU)."""
    local = P.to_local(path)
    if mode == "overwrite" and os.path.exists(local) and task_id == 0:
        import shutil
        shutil.rmtree(local)
    if mode == "errorifexists" and os.path.exists(local):
        raise HyperspaceException(f"path {path} already exists")
    os.makedirs(local, exist_ok=True)
    job_uuid = job_uuid or str(uuid.uuid4())
    if table.num_rows == 0:
        return []
    bids = murmur3.bucket_ids([table.column(c) for c in bucket_cols], num_buckets)
    # sort by (bucket, cols...) — stable sort by cols first, then by bucket id
    idx = sort_indices_by(table, bucket_cols)
    b_sorted = bids[idx]
    perm = idx[np.argsort(b_sorted, kind="stable")]
    t = table.take(pa.array(perm))
    b = bids[perm]
    bounds = np.searchsorted(b, np.arange(num_buckets + 1))
    out = []
    for bucket in range(num_buckets):
        lo, hi = int(bounds[bucket]), int(bounds[bucket + 1])
        if hi <= lo:
            continue
        if buckets_to_write is not None and bucket not in buckets_to_write:
            continue
        out.append(write_bucket_file(t.slice(lo, hi - lo), path, task_id, job_uuid, bucket,
                                     codec, row_group_rows))
    return out


class DataFrameWriter:
    def __init__(self, df):
        self.df = df
        self._mode = "errorifexists"
        self._format = "parquet"
        self._partition_by: List[str] = []
        self._options: dict = {}

    def mode(self, m: str) -> "DataFrameWriter":
        self._mode = m.lower()
        return self

    def format(self, f: str) -> "DataFrameWriter":
        self._format = f.lower()
        return self

    def option(self, k, v) -> "DataFrameWriter":
        self._options[k] = str(v)
        return self

    def partitionBy(self, *cols) -> "DataFrameWriter":
        self._partition_by = list(cols)
        return self

    def saveAsTable(self, name: str) -> None:
        """Write the data and record table ``name`` in the session catalog (managed under the
        warehouse directory, or external at ``option("path", ...)``)."""
        self.df.session.catalog.save_table(name, self, self._mode)

    def reads_from(self, path: str) -> bool:
        """Whether the DataFrame being written reads files at or under ``path``: the data is
        only computed inside ``save``, so overwriting such a path would delete the input first."""
        from ..plan import logical as L
        root = os.path.abspath(P.to_local(path)).rstrip(os.sep) + os.sep
        plan = self.df.queryExecution.analyzed
        for lr in plan.collect(lambda n: isinstance(n, L.LogicalRelation)):
            loc = getattr(lr.relation, "location", None)
            paths = list(getattr(loc, "root_paths", []) or [])
            for f in (loc.all_files() if loc is not None else []):
                paths.append(f.path)
            for q in paths:
                if (os.path.abspath(P.to_local(q)).rstrip(os.sep) + os.sep).startswith(root):
                    return True
        return False

    def save(self, path: str) -> None:
        local = P.to_local(path)
        if os.path.exists(local):
            if self._mode in ("errorifexists", "error"):
                raise HyperspaceException(f"path {path} already exists.")
            if self._mode == "ignore":
                return
            if self._mode == "overwrite":
                if self.reads_from(local):
                    # Spark refuses this too (the input would be deleted before it is read)
                    raise HyperspaceException(
                        f"Cannot overwrite a path that is also being read from: {path}")
                import shutil
                shutil.rmtree(local)
        os.makedirs(local, exist_ok=True)
        t = self.df.to_arrow()
        job = str(uuid.uuid4())
        if self._partition_by:
            keys = t.select(self._partition_by).to_pylist()
            groups = {}
            for i, k in enumerate(keys):
                groups.setdefault(tuple(k[c] for c in self._partition_by), []).append(i)
            data_cols = [c for c in t.column_names if c not in self._partition_by]
            for n, (key, rows) in enumerate(sorted(groups.items(), key=lambda kv: repr(kv[0]))):
                sub = os.path.join(local, *[f"{c}={'__HIVE_DEFAULT_PARTITION__' if v is None else v}"
                                            for c, v in zip(self._partition_by, key)])
                os.makedirs(sub, exist_ok=True)
                self._write_one(t.take(pa.array(rows)).select(data_cols), sub, n, job)
        else:
            self._write_one(t, local, 0, job)

    def _write_one(self, t: pa.Table, directory: str, part: int, job: str) -> None:
        fmt = self._format
        if fmt == "parquet":
            pq.write_table(t, os.path.join(directory, f"part-{part:05d}-{job}.c000.snappy.parquet"),
                           compression="snappy")
        elif fmt == "csv":
            import pyarrow.csv as pcsv
            header = self._options.get("header", "false").lower() == "true"
            pcsv.write_csv(t, os.path.join(directory, f"part-{part:05d}-{job}.c000.csv"),
                           write_options=pcsv.WriteOptions(include_header=header))
        elif fmt == "json":
            import json
            with open(os.path.join(directory, f"part-{part:05d}-{job}.c000.json"), "w") as f:
                for row in t.to_pylist():
                    f.write(json.dumps(row, default=str) + "\n")
        elif fmt == "orc":
            import pyarrow.orc as po
            po.write_table(t, os.path.join(directory, f"part-{part:05d}-{job}.c000.orc"))
        else:
            raise HyperspaceException(f"unsupported write format {fmt}")

    def parquet(self, path: str) -> None:
        self._format = "parquet"
        self.save(path)

    def csv(self, path: str, header=None) -> None:
        self._format = "csv"
        if header is not None:
            self._options["header"] = str(header).lower()
        self.save(path)

    def json(self, path: str) -> None:
        self._format = "json"
        self.save(path)

    def orc(self, path: str) -> None:
        self._format = "orc"
        self.save(path)
