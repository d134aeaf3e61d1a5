"""Delta Lake source (reference ``index/sources/delta/DeltaLakeFileBasedSource.scala:35-226``).

No Delta library exists in this environment, so the transaction log is read natively:
``_delta_log/<version:020d>.json`` commits (``add`` / ``remove`` / ``metaData`` actions) plus
optional Parquet checkpoints (``_last_checkpoint``).  ``versionAsOf`` time travel is supported.
A tiny writer (``write_delta``) exists so tests and benchmarks can produce Delta tables.

Signature = ``tableVersion + path`` and the internal file format is ``parquet``, as in the
reference.
"""
from __future__ import annotations

import json
import os
import time
import uuid
from typing import Dict, List, Optional

import pyarrow as pa
import pyarrow.parquet as pq

from ..exceptions import HyperspaceException
from ..index.log_entry import Content, Hdfs, Relation
from ..plan import logical as L
from ..plan.types import schema_from_json, schema_to_json
from ..utils import path_utils as P
from ..utils.file_utils import FileStatus
from .interfaces import FileBasedSourceProvider, SourceProviderBuilder

LOG_DIR = "_delta_log"


class DeltaSnapshot:
    def __init__(self, table_path: str, version: int, files: Dict[str, dict], schema: pa.Schema,
                 partition_columns: List[str]):
        self.table_path = table_path
        self.version = version
        self.files = files  # relative path -> add action
        self.schema = schema
        self.partition_columns = partition_columns


def _log_versions(local_table: str) -> List[int]:
    d = os.path.join(local_table, LOG_DIR)
    if not os.path.isdir(d):
        raise HyperspaceException(f"{local_table} is not a Delta table")
    return sorted(int(n[:-5]) for n in os.listdir(d) if n.endswith(".json") and n[:-5].isdigit())


def read_snapshot(table_path: str, version: Optional[int] = None) -> DeltaSnapshot:
    local = P.to_local(table_path)
    versions = _log_versions(local)
    if not versions:
        raise HyperspaceException(f"empty Delta log at {table_path}")
    target = versions[-1] if version is None else int(version)
    if target not in versions and not any(v <= target for v in versions):
        raise HyperspaceException(f"version {target} not found in {table_path}")
    files: Dict[str, dict] = {}
    meta = None
    start = 0
    cp_path = os.path.join(local, LOG_DIR, "_last_checkpoint")
    if os.path.exists(cp_path):
        cp = json.load(open(cp_path))
        cpv = int(cp["version"])
        if cpv <= target:
            t = pq.read_table(os.path.join(local, LOG_DIR, f"{cpv:020d}.checkpoint.parquet"))
            for row in t.to_pylist():
                if row.get("add"):
                    files[row["add"]["path"]] = row["add"]
                if row.get("metaData"):
                    meta = row["metaData"]
            start = cpv + 1
    for v in versions:
        if v < start or v > target:
            continue
        with open(os.path.join(local, LOG_DIR, f"{v:020d}.json")) as f:
            for line in f:
                if not line.strip():
                    continue
                a = json.loads(line)
                if "add" in a:
                    files[a["add"]["path"]] = a["add"]
                elif "remove" in a:
                    files.pop(a["remove"]["path"], None)
                elif "metaData" in a:
                    meta = a["metaData"]
    if meta is None:
        raise HyperspaceException(f"no metaData action in Delta log {table_path}")
    schema = schema_from_json(meta["schemaString"])
    return DeltaSnapshot(P.make_absolute(local), target, files, schema,
                         list(meta.get("partitionColumns") or []))


class DeltaFileIndex(L.FileIndex):
    """``TahoeLogFileIndex`` analog: files of one snapshot version."""

    kind = "TahoeLogFileIndex"

    def __init__(self, snapshot: DeltaSnapshot):
        self.snapshot = snapshot
        self.path = snapshot.table_path
        self.table_version = snapshot.version
        files = []
        parts = {}
        for rel, add in sorted(snapshot.files.items()):
            q = P.join(self.path, rel)
            files.append(FileStatus(q, int(add.get("size", 0)), int(add.get("modificationTime", 0))))
            if add.get("partitionValues"):
                parts[P.get_parent(q)] = dict(add["partitionValues"])
        pcols = pa.schema([f for f in snapshot.schema if f.name in snapshot.partition_columns])
        for d, vals in parts.items():
            for f in pcols:
                v = vals.get(f.name)
                if v is not None and pa.types.is_integer(f.type):
                    vals[f.name] = int(v)
        spec = L.PartitionSpec(pcols, parts, self.path if len(pcols) else None)
        super().__init__([self.path], files, spec)


def load_delta_relation(session, path: str, options: dict, schema=None) -> L.HadoopFsRelation:
    version = options.get("versionAsOf")
    snap = read_snapshot(path, int(version) if version is not None else None)
    loc = DeltaFileIndex(snap)
    data_schema = pa.schema([f for f in snap.schema if f.name not in snap.partition_columns])
    return L.HadoopFsRelation(loc, loc.partition_schema, data_schema, None, "delta", dict(options))


def write_delta(table: pa.Table, path: str, mode: str = "append",
                partition_by: Optional[List[str]] = None) -> int:
    """Minimal Delta writer: one parquet file per call (per partition), one commit JSON."""
    local = P.to_local(path)
    log_dir = os.path.join(local, LOG_DIR)
    os.makedirs(log_dir, exist_ok=True)
    versions = _log_versions(local) if os.listdir(log_dir) else []
    version = versions[-1] + 1 if versions else 0
    actions = []
    now = int(time.time() * 1000)
    if version == 0:
        actions.append({"protocol": {"minReaderVersion": 1, "minWriterVersion": 2}})
        actions.append({"metaData": {"id": str(uuid.uuid4()), "format": {"provider": "parquet",
                                                                           "options": {}},
                                     "schemaString": schema_to_json(table.schema),
                                     "partitionColumns": list(partition_by or []),
                                     "configuration": {}, "createdTime": now}})
    if mode == "overwrite" and versions:
        for rel in read_snapshot(path).files:
            actions.append({"remove": {"path": rel, "deletionTimestamp": now, "dataChange": True}})
    groups = {(): table}
    if partition_by:
        groups = {}
        keys = table.select(partition_by).to_pylist()
        idx: Dict[tuple, list] = {}
        for i, k in enumerate(keys):
            idx.setdefault(tuple(k[c] for c in partition_by), []).append(i)
        for k, rows in idx.items():
            groups[k] = table.take(pa.array(rows)).drop(partition_by)
    for k, t in groups.items():
        sub = "/".join(f"{c}={v}" for c, v in zip(partition_by or [], k))
        name = f"part-00000-{uuid.uuid4()}-c000.snappy.parquet"
        rel = f"{sub}/{name}" if sub else name
        os.makedirs(os.path.dirname(os.path.join(local, rel)), exist_ok=True)
        pq.write_table(t, os.path.join(local, rel), compression="snappy")
        st = os.stat(os.path.join(local, rel))
        actions.append({"add": {"path": rel, "size": st.st_size,
                                "partitionValues": {c: str(v) for c, v in zip(partition_by or [], k)},
                                "modificationTime": st.st_mtime_ns // 1_000_000,
                                "dataChange": True}})
    with open(os.path.join(log_dir, f"{version:020d}.json"), "w") as f:
        for a in actions:
            f.write(json.dumps(a) + "\n")
    return version


def delete_delta_files(path: str, rel_paths: List[str]) -> int:
    local = P.to_local(path)
    version = _log_versions(local)[-1] + 1
    now = int(time.time() * 1000)
    with open(os.path.join(local, LOG_DIR, f"{version:020d}.json"), "w") as f:
        for r in rel_paths:
            f.write(json.dumps({"remove": {"path": r, "deletionTimestamp": now,
                                           "dataChange": True}}) + "\n")
    return version


class DeltaLakeFileBasedSource(FileBasedSourceProvider):
    def __init__(self, session):
        self.session = session

    @staticmethod
    def _loc(lr):
        if isinstance(lr, L.LogicalRelation) and isinstance(lr.relation.location, DeltaFileIndex):
            return lr.relation.location
        return None

    def create_relation(self, lr, tracker):
        loc = self._loc(lr)
        if loc is None:
            return None
        content = Content.from_leaf_files(loc.all_files(), tracker)
        opts = {k: v for k, v in lr.relation.options.items() if k != "path"}
        opts["versionAsOf"] = str(loc.table_version)
        bp = self.partition_base_path(loc)
        if bp[0] is not None:
            opts["basePath"] = bp[0]
        return Relation([loc.path], Hdfs(content), schema_to_json(lr.relation.data_schema),
                        "delta", opts)

    def refresh_relation(self, relation):
        if relation.file_format != "delta":
            return None
        opts = {k: v for k, v in relation.options.items() if k not in ("versionAsOf", "timestampAsOf")}
        return Relation(relation.root_paths, relation.data, relation.data_schema_json, "delta", opts)

    def internal_file_format_name(self, relation):
        return "parquet" if relation.file_format == "delta" else None

    def signature(self, lr):
        loc = self._loc(lr)
        return None if loc is None else f"{loc.table_version}{loc.path}"

    def all_files(self, lr):
        loc = self._loc(lr)
        return None if loc is None else list(loc.all_files())

    def partition_base_path(self, location):
        if not isinstance(location, DeltaFileIndex):
            return None
        return (location.path,) if len(location.partition_schema) else (None,)

    def lineage_pairs(self, lr, tracker):
        if self._loc(lr) is None:
            return None
        return [(k[0], v) for k, v in tracker.get_file_to_id_map().items()]

    def has_parquet_as_source_format(self, lr):
        return True if self._loc(lr) is not None else None


class DeltaLakeFileBasedSourceBuilder(SourceProviderBuilder):
    def build(self, session):
        return DeltaLakeFileBasedSource(session)
