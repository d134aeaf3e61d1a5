"""Rows returned by ``indexes()`` / ``index(name)`` (reference ``index/IndexStatistics.scala:43-196``)."""
from __future__ import annotations

import pyarrow as pa

from ..utils import path_utils as P
from . import constants as C

INDEX_SUMMARY_COLUMNS = ["name", "indexedColumns", "includedColumns", "numBuckets", "schema",
                         "indexLocation", "state"]
EXTENDED_COLUMNS = INDEX_SUMMARY_COLUMNS + [
    "kind", "hasLineage", "numIndexFiles", "sizeIndexFiles", "numSourceFiles", "sizeSourceFiles",
    "numAppendedFiles", "sizeAppendedFiles", "numDeletedFiles", "sizeDeletedFiles",
    "indexContentPaths"]

SCHEMA = pa.schema([
    ("name", pa.string()), ("indexedColumns", pa.list_(pa.string())),
    ("includedColumns", pa.list_(pa.string())), ("numBuckets", pa.int32()),
    ("schema", pa.string()), ("indexLocation", pa.string()), ("state", pa.string()),
    ("kind", pa.string()), ("hasLineage", pa.bool_()), ("numIndexFiles", pa.int32()),
    ("sizeIndexFiles", pa.int64()), ("numSourceFiles", pa.int32()), ("sizeSourceFiles", pa.int64()),
    ("numAppendedFiles", pa.int32()), ("sizeAppendedFiles", pa.int64()),
    ("numDeletedFiles", pa.int32()), ("sizeDeletedFiles", pa.int64()),
    ("indexContentPaths", pa.list_(pa.string()))])


def index_dir_path(entry) -> str:
    root = entry.content.root
    path = root.name
    while not root.files and len(root.sub_dirs) == 1:
        root = root.sub_dirs[0]
        path = P.join(path, root.name)
    return path


def index_content_directory_paths(entry) -> list:
    root = entry.content.root
    prefix = root.name
    while len(root.sub_dirs) == 1 and not root.sub_dirs[0].name.startswith(
            C.INDEX_VERSION_DIRECTORY_PREFIX):
        prefix += f"{root.sub_dirs[0].name}/"
        root = root.sub_dirs[0]
    return [f"{prefix}{d.name}" for d in root.sub_dirs]


def statistics(entry, extended: bool = False) -> dict:
    d = {"name": entry.name, "indexedColumns": list(entry.indexed_columns),
         "includedColumns": list(entry.included_columns), "numBuckets": entry.num_buckets,
         "schema": entry.derived_dataset.schema_string, "indexLocation": index_dir_path(entry),
         "state": entry.state}
    if extended:
        ci = entry.content.file_infos
        src = entry.source_file_info_set
        app, dele = entry.appended_files, entry.deleted_files
        d.update({"kind": entry.derived_dataset.kind, "hasLineage": entry.has_lineage_column,
                  "numIndexFiles": len(ci), "sizeIndexFiles": sum(f.size for f in ci),
                  "numSourceFiles": len(src), "sizeSourceFiles": sum(f.size for f in src),
                  "numAppendedFiles": len(app), "sizeAppendedFiles": sum(f.size for f in app),
                  "numDeletedFiles": len(dele), "sizeDeletedFiles": sum(f.size for f in dele),
                  "indexContentPaths": index_content_directory_paths(entry)})
    return d


def to_table(rows: list, extended: bool = False) -> pa.Table:
    cols = EXTENDED_COLUMNS if extended else INDEX_SUMMARY_COLUMNS
    schema = pa.schema([SCHEMA.field(c) for c in cols])
    return pa.Table.from_pylist([{c: r[c] for c in cols} for r in rows], schema=schema)
