"""Source provider SPI (reference ``index/sources/interfaces.scala:32-154``).

Each method returns ``None`` when the provider does not handle the relation; the manager requires
exactly one provider to answer (``FileBasedSourceProviderManager.scala:153-173``).
"""
from __future__ import annotations

from typing import List, Optional, Tuple


class SourceProvider:
    pass


class SourceProviderBuilder:
    def build(self, session) -> SourceProvider:
        raise NotImplementedError


class FileBasedSourceProvider(SourceProvider):
    def create_relation(self, logical_relation, file_id_tracker):
        return None

    def refresh_relation(self, relation):
        return None

    def internal_file_format_name(self, relation) -> Optional[str]:
        return None

    def signature(self, logical_relation) -> Optional[str]:
        return None

    def all_files(self, logical_relation) -> Optional[list]:
        return None

    def partition_base_path(self, location) -> Optional[Tuple[Optional[str]]]:
        """``Some(Some(path))`` -> ``(path,)``; ``Some(None)`` -> ``(None,)``; ``None`` -> None."""
        return None

    def lineage_pairs(self, logical_relation, file_id_tracker) -> Optional[List[tuple]]:
        return None

    def has_parquet_as_source_format(self, logical_relation) -> Optional[bool]:
        return None
