"""Pluggable source provider manager (reference
``index/sources/FileBasedSourceProviderManager.scala:39-201``).

Builders come from ``spark.hyperspace.index.sources.fileBasedBuilders`` (comma-separated dotted
Python class paths) and are rebuilt only when the conf value changes.
"""
from __future__ import annotations

import importlib

from ..exceptions import HyperspaceException
from ..utils.cache import CacheWithTransform
from ..utils.conf import HyperspaceConf
from .interfaces import FileBasedSourceProvider, SourceProviderBuilder

# Reference class names map onto the native providers so reference-written confs keep working.
_ALIASES = {
    "com.microsoft.hyperspace.index.sources.default.DefaultFileBasedSourceBuilder":
        "hyperspace_amd.sources.default.DefaultFileBasedSourceBuilder",
    "com.microsoft.hyperspace.index.sources.delta.DeltaLakeFileBasedSourceBuilder":
        "hyperspace_amd.sources.delta.DeltaLakeFileBasedSourceBuilder",
}


def _load_class(name: str):
    name = _ALIASES.get(name, name)
    mod, _, cls = name.rpartition(".")
    return getattr(importlib.import_module(mod), cls)


class FileBasedSourceProviderManager:
    def __init__(self, session):
        self.session = session
        self._providers = CacheWithTransform(
            lambda: HyperspaceConf.file_based_source_builders(session.conf), self._build)

    def _build(self, names: str):
        out = []
        for name in [n.strip() for n in names.split(",") if n.strip()]:
            try:
                builder = _load_class(name)()
            except Exception as e:  # noqa: BLE001
                raise HyperspaceException(f"Cannot load SourceProviderBuilder: '{name}'") from e
            if not isinstance(builder, SourceProviderBuilder):
                raise HyperspaceException(f"Cannot load SourceProviderBuilder: '{name}'")
            p = builder.build(self.session)
            if not isinstance(p, FileBasedSourceProvider):
                raise HyperspaceException(f"'{builder}' did not build FileBasedSourceProvider: '{p}')")
            out.append(p)
        return out

    def _run(self, fn):
        result, owner = None, None
        for p in self._providers.load():
            cur = fn(p)
            if cur is not None:
                if owner is not None:
                    raise HyperspaceException(
                        "Multiple source providers returned valid results: "
                        f"'{type(p).__name__}' and '{type(owner).__name__}'")
                result, owner = cur, p
        if owner is None:
            raise HyperspaceException("No source provider returned valid results.")
        return result

    def create_relation(self, logical_relation, tracker):
        return self._run(lambda p: p.create_relation(logical_relation, tracker))

    def refresh_relation(self, relation):
        return self._run(lambda p: p.refresh_relation(relation))

    def internal_file_format_name(self, relation) -> str:
        return self._run(lambda p: p.internal_file_format_name(relation))

    def signature(self, logical_relation) -> str:
        return self._run(lambda p: p.signature(logical_relation))

    def all_files(self, logical_relation) -> list:
        return self._run(lambda p: p.all_files(logical_relation))

    def partition_base_path(self, location):
        return self._run(lambda p: p.partition_base_path(location))[0]

    def lineage_pairs(self, logical_relation, tracker):
        return self._run(lambda p: p.lineage_pairs(logical_relation, tracker))

    def has_parquet_as_source_format(self, logical_relation) -> bool:
        return self._run(lambda p: p.has_parquet_as_source_format(logical_relation))
