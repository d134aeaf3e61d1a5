"""File-based sources: ``session.read.parquet/csv/json/orc/text/format(...).load(...)``.

Builds a ``LogicalRelation`` over an ``InMemoryFileIndex`` (leaf-file listing + hive partition
discovery), mirroring what Spark's ``DataSource.resolveRelation`` gives the reference's
``DefaultFileBasedSource`` (``DefaultFileBasedSource.scala:58-124``).  Reading the bytes is done
by ``read_files`` (pyarrow on the host; the device executor has its own native Parquet path).
"""
from __future__ import annotations

import glob as _glob
import os
from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa

from ..exceptions import HyperspaceException
from ..index import constants as C
from ..plan import logical as L
from ..utils import file_utils as FU
from ..utils import path_utils as P

SUPPORTED_FORMATS = ("parquet", "csv", "json", "orc", "text", "avro", "delta")

_POOL = None


def _io_pool():
    """Shared host decode pool (files are decoded concurrently; pyarrow releases the GIL)."""
    global _POOL
    if _POOL is None:
        import concurrent.futures as cf
        _POOL = cf.ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4))
    return _POOL


def _infer_partition_value(v: str):
    if v == "__HIVE_DEFAULT_PARTITION__":
        return None, None
    try:
        iv = int(v)
        return iv, (pa.int32() if -2 ** 31 <= iv < 2 ** 31 else pa.int64())
    except ValueError:
        pass
    try:
        return float(v), pa.float64()
    except ValueError:
        return v, pa.string()


def discover_partitions(files: List[FU.FileStatus], roots: List[str],
                        base_path: Optional[str]) -> L.PartitionSpec:
    """Hive-style ``k=v`` directory discovery below ``basePath`` (or the roots)."""
    bases = [P.to_local(base_path)] if base_path else [P.to_local(r) for r in roots]
    parts: Dict[str, dict] = {}
    col_types: Dict[str, pa.DataType] = {}
    col_order: List[str] = []
    for f in files:
        d = os.path.dirname(P.to_local(f.path))
        base = next((b for b in bases if d == b or d.startswith(b.rstrip("/") + "/")), None)
        if base is None:
            continue
        rel = os.path.relpath(d, base)
        if rel == ".":
            continue
        values = {}
        for seg in rel.split("/"):
            if "=" not in seg:
                values = None
                break
            k, v = seg.split("=", 1)
            pv, pt = _infer_partition_value(v)
            values[k] = pv
            if k not in col_types:
                col_order.append(k)
                col_types[k] = pt or pa.string()
            elif pt is not None and not col_types[k].equals(pt):
                col_types[k] = pa.string() if pa.types.is_string(pt) or \
                    pa.types.is_string(col_types[k]) else pa.float64()
        if values:
            parts[P.qualify(d)] = values
    if not parts:
        return L.PartitionSpec()
    schema = pa.schema([pa.field(k, col_types[k], True) for k in col_order])
    bp = base_path or (roots[0] if len(roots) == 1 else None)
    return L.PartitionSpec(schema, parts, P.make_absolute(bp) if bp else None)


def list_files(paths: List[str]) -> tuple:
    roots, files = [], []
    for p in paths:
        local = P.to_local(p)
        matches = sorted(_glob.glob(local)) if any(ch in local for ch in "*?[") else [local]
        if not matches:
            raise HyperspaceException(f"Path does not exist: {p}")
        for m in matches:
            if not os.path.exists(m):
                raise HyperspaceException(f"Path does not exist: {p}")
            q = P.make_absolute(m)
            roots.append(q)
            if os.path.isdir(m):
                files.extend(FU.list_leaf_files(q))
            else:
                files.append(FU.get_fs().get_file_status(q))
    return roots, files


def infer_schema(fmt: str, files: List[FU.FileStatus], options: dict) -> pa.Schema:
    if not files:
        raise HyperspaceException("Unable to infer schema: no files found")
    first = P.to_local(files[0].path)
    if fmt == "parquet":
        import pyarrow.parquet as pq
        return pq.read_schema(first)
    if fmt == "orc":
        import pyarrow.orc as po
        return po.ORCFile(first).schema
    t = read_one(fmt, first, None, options)
    return t.schema


def _csv_opts(options: dict, schema: Optional[pa.Schema]):
    import pyarrow.csv as pcsv
    header = str(options.get("header", "false")).lower() == "true"
    sep = options.get("sep", options.get("delimiter", ","))
    ropts = pcsv.ReadOptions(autogenerate_column_names=not header)
    if schema is not None and not header:
        ropts = pcsv.ReadOptions(column_names=schema.names)
    popts = pcsv.ParseOptions(delimiter=sep)
    infer = str(options.get("inferSchema", "false")).lower() == "true"
    copts = pcsv.ConvertOptions()
    if schema is not None:
        copts = pcsv.ConvertOptions(column_types={f.name: f.type for f in schema})
    elif not infer:
        copts = None  # handled by caller: cast everything to string
    return ropts, popts, copts, infer


def read_one(fmt: str, local_path: str, schema: Optional[pa.Schema], options: dict) -> pa.Table:
    if fmt == "parquet":
        import pyarrow.parquet as pq
        t = pq.read_table(local_path, columns=schema.names if schema is not None else None)
    elif fmt == "orc":
        import pyarrow.orc as po
        t = po.ORCFile(local_path).read(columns=schema.names if schema is not None else None)
    elif fmt == "csv":
        import pyarrow.csv as pcsv
        ropts, popts, copts, infer = _csv_opts(options, schema)
        if copts is None:
            t = pcsv.read_csv(local_path, read_options=ropts, parse_options=popts)
            if not infer:
                t = pa.table({n: c.cast(pa.string()) for n, c in zip(t.column_names, t.columns)})
        else:
            t = pcsv.read_csv(local_path, read_options=ropts, parse_options=popts,
                              convert_options=copts)
        if not str(options.get("header", "false")).lower() == "true" and schema is None:
            t = t.rename_columns([f"_c{i}" for i in range(t.num_columns)])
    elif fmt == "json":
        import pyarrow.json as pjson
        kw = {}
        if schema is not None:
            kw["parse_options"] = pjson.ParseOptions(explicit_schema=schema)
        t = pjson.read_json(local_path, **kw)
    elif fmt == "text":
        with open(local_path, "r", encoding="utf-8") as f:
            lines = f.read().splitlines()
        t = pa.table({"value": pa.array(lines, pa.string())})
    elif fmt == "avro":
        from .avro import read_avro
        t = read_avro(local_path)
    else:
        raise HyperspaceException(f"unsupported format {fmt}")
    if schema is not None:
        cols = []
        for f in schema:
            if f.name in t.column_names:
                c = t.column(f.name)
                if not c.type.equals(f.type):
                    c = c.cast(f.type)
                cols.append(c)
            else:
                cols.append(pa.nulls(t.num_rows, f.type))
        t = pa.Table.from_arrays(cols, schema=schema)
    return t


def output_schema(data_schema: pa.Schema, partition_spec: Optional[L.PartitionSpec] = None,
                  columns: Optional[List[str]] = None) -> pa.Schema:
    """Schema ``read_files`` returns: requested data columns, then partition columns."""
    pspec = partition_spec or L.PartitionSpec()
    data_cols = [f for f in data_schema if columns is None or f.name in columns]
    part_cols = [f for f in pspec.columns if (columns is None or f.name in columns)
                 and f.name not in data_schema.names]
    return pa.schema(data_cols + part_cols)


def read_files(fmt: str, files: List[str], data_schema: pa.Schema, options: dict,
               partition_spec: Optional[L.PartitionSpec] = None,
               columns: Optional[List[str]] = None, with_file_index: bool = False) -> pa.Table:
    """Read & concatenate files, appending partition columns; optional per-row file index."""
    pspec = partition_spec or L.PartitionSpec()
    need = columns
    data_cols = [f for f in data_schema if need is None or f.name in need]
    part_cols = [f for f in pspec.columns if (need is None or f.name in need)
                 and f.name not in data_schema.names]
    out_schema = pa.schema(data_cols + part_cols)
    file_idx = []
    read_schema = pa.schema(data_cols)

    def one(fq):
        local = P.to_local(fq)
        if fmt == "parquet" and not data_cols:
            import pyarrow.parquet as pq
            t = pq.read_table(local, columns=[])
        else:
            t = read_one(fmt, local, read_schema, options)
        if part_cols:
            nrows = t.num_rows
            pdir = P.qualify(os.path.dirname(local))
            vals = pspec.partitions.get(pdir, {})
            for f in part_cols:
                t = t.append_column(f, pa.array([vals.get(f.name)] * nrows, f.type))
        return t

    if len(files) > 1:
        tables = list(_io_pool().map(one, files))
    else:
        tables = [one(f) for f in files]
    if with_file_index:
        for i, t in enumerate(tables):
            file_idx.append(pa.array(np.full(t.num_rows, i, dtype=np.int32)))
    if not tables:
        t = out_schema.empty_table()
    elif len(tables) == 1:
        t = tables[0].select(out_schema.names)
        t = t if t.schema.equals(out_schema) else t.cast(out_schema)
    else:
        t = pa.concat_tables([x.select(out_schema.names).cast(out_schema) for x in tables])
    if with_file_index:
        idx = pa.chunked_array(file_idx, pa.int32()) if file_idx else pa.array([], pa.int32())
        return t, idx
    return t


class DataFrameReader:
    def __init__(self, session):
        self.session = session
        self._format = "parquet"
        self._options: Dict[str, str] = {}
        self._schema: Optional[pa.Schema] = None

    def format(self, fmt: str) -> "DataFrameReader":
        self._format = fmt.lower()
        return self

    def option(self, key: str, value) -> "DataFrameReader":
        self._options[key] = str(value).lower() if isinstance(value, bool) else str(value)
        return self

    def options(self, opts: dict = None, **kw) -> "DataFrameReader":
        for k, v in dict(opts or {}, **kw).items():
            self.option(k, v)
        return self

    def schema(self, schema) -> "DataFrameReader":
        if isinstance(schema, str):
            from ..plan.types import schema_from_json
            schema = schema_from_json(schema)
        self._schema = schema
        return self

    def load(self, *paths):
        from ..plan.dataframe import DataFrame
        if len(paths) == 1 and isinstance(paths[0], (list, tuple)):
            paths = tuple(paths[0])
        if not paths and "path" in self._options:
            paths = (self._options["path"],)
        fmt = self._format
        if fmt == "delta":
            from ..sources.delta import load_delta_relation
            rel = load_delta_relation(self.session, paths[0], self._options, self._schema)
            return DataFrame(self.session, L.LogicalRelation(rel))
        if fmt not in SUPPORTED_FORMATS:
            raise HyperspaceException(f"unsupported format {fmt}")
        roots, files = list_files(list(paths))
        base = self._options.get("basePath")
        pspec = discover_partitions(files, roots, base)
        data_schema = self._schema
        if data_schema is None:
            data_schema = infer_schema(fmt, files, self._options)
        data_schema = pa.schema([f for f in data_schema if f.name not in pspec.columns.names])
        opts = dict(self._options)
        location = L.FileIndex(roots, files, pspec)
        rel = L.HadoopFsRelation(location, pspec.columns, data_schema, None, fmt, opts)
        return DataFrame(self.session, L.LogicalRelation(rel))

    def parquet(self, *paths):
        return self.format("parquet").load(*paths)

    def csv(self, *paths, header=None, inferSchema=None):
        if header is not None:
            self.option("header", header)
        if inferSchema is not None:
            self.option("inferSchema", inferSchema)
        return self.format("csv").load(*paths)

    def json(self, *paths):
        return self.format("json").load(*paths)

    def orc(self, *paths):
        return self.format("orc").load(*paths)

    def avro(self, *paths):
        return self.format("avro").load(*paths)

    def text(self, *paths):
        return self.format("text").load(*paths)


def relation_files(rel: L.HadoopFsRelation) -> List[str]:
    return [f.path for f in rel.location.all_files()]


GLOBBING_PATTERN_KEY = C.GLOBBING_PATTERN_KEY
