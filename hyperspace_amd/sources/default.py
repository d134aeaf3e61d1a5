"""Default file-based source (reference ``index/sources/default/DefaultFileBasedSource.scala:42-325``).

Handles relations over an ``InMemoryFileIndex`` in the conf-driven format list
(avro, csv, json, orc, parquet, text).  The signature is the reference's md5 fold of
``len + mtime + path`` over files sorted by path, so signatures computed here match indexes built
by the reference on the same files.
"""
from __future__ import annotations

import glob
import os

from ..exceptions import HyperspaceException
from ..index import constants as C
from ..index.log_entry import Content, Hdfs, Relation
from ..plan import logical as L
from ..plan.types import schema_to_json
from ..utils import path_utils as P
from ..utils.cache import CacheWithTransform
from ..utils.conf import HyperspaceConf
from ..utils.hashing import md5_hex
from .interfaces import FileBasedSourceProvider, SourceProviderBuilder


def file_fingerprint(f) -> str:
    return f"{f.length}{f.modification_time}{f.path}"


class DefaultFileBasedSource(FileBasedSourceProvider):
    def __init__(self, session):
        self.session = session
        self._formats = CacheWithTransform(
            lambda: HyperspaceConf.supported_file_formats_for_default_file_based_source(session.conf),
            lambda s: {x.strip().lower() for x in s.split(",")})

    def _supported(self, fmt: str) -> bool:
        return fmt is not None and fmt.lower() in self._formats.load()

    def _handles(self, lr) -> bool:
        if not isinstance(lr, L.LogicalRelation):
            return False
        rel = lr.relation
        return type(rel.location) is L.FileIndex and self._supported(rel.file_format)

    def create_relation(self, lr, tracker):
        if not self._handles(lr):
            return None
        rel = lr.relation
        files = rel.location.all_files()
        content = Content.from_leaf_files(files, tracker)
        if content is None:
            raise HyperspaceException("Cannot create an index on a relation without files.")
        opts = {k: v for k, v in rel.options.items() if k != "path"}
        bp = self.partition_base_path(rel.location)
        if bp is not None and bp[0] is not None:
            opts["basePath"] = bp[0]
        pattern = opts.get(C.GLOBBING_PATTERN_KEY)
        if pattern:
            glob_paths = {}
            for p in [x.strip() for x in pattern.split(",")]:
                q = P.make_absolute(p)
                glob_paths[q] = {P.make_absolute(m) for m in glob.glob(P.to_local(q))}
            values = set().union(*glob_paths.values()) if glob_paths else set()
            if not all(r in values for r in rel.location.root_paths):
                raise HyperspaceException(
                    "Some glob patterns do not match with available root paths of the source data. "
                    f"Please check if {pattern} matches all of {','.join(rel.location.root_paths)}.")
            roots = list(glob_paths.keys())
        else:
            roots = list(rel.location.root_paths)
        return Relation(roots, Hdfs(content), schema_to_json(rel.data_schema), rel.file_format, opts)

    def refresh_relation(self, relation):
        return relation if self._supported(relation.file_format) else None

    def internal_file_format_name(self, relation):
        return relation.file_format if self._supported(relation.file_format) else None

    def signature(self, lr):
        if not self._handles(lr):
            return None
        acc = ""
        for f in sorted(lr.relation.location.all_files(), key=lambda s: s.path):
            acc = md5_hex(acc + file_fingerprint(f))
        return acc

    def all_files(self, lr):
        if not isinstance(lr, L.LogicalRelation) or type(lr.relation.location) is not L.FileIndex:
            return None
        return list(lr.relation.location.all_files())

    def partition_base_path(self, location):
        if type(location) is not L.FileIndex:
            return None
        spec = location.partition_spec
        if spec.partitions:
            first = sorted(spec.partitions.keys())[0]
            path = first
            for _ in spec.columns:
                path = P.get_parent(path)
            return (path,)
        return (None,)

    def lineage_pairs(self, lr, tracker):
        if not self._handles(lr):
            return None
        return [(k[0].replace("file:/", "file:///"), v)
                for k, v in tracker.get_file_to_id_map().items()]

    def has_parquet_as_source_format(self, lr):
        if not self._handles(lr):
            return None
        return lr.relation.file_format == "parquet"


class DefaultFileBasedSourceBuilder(SourceProviderBuilder):
    def build(self, session):
        return DefaultFileBasedSource(session)


__all__ = ["DefaultFileBasedSource", "DefaultFileBasedSourceBuilder", "os"]
