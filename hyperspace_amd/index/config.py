"""Covering-index specification (reference ``index/IndexConfig.scala:28-166``,
``python/hyperspace/indexconfig.py:1-14``)."""
from __future__ import annotations

from typing import Sequence


class IndexConfig:
    def __init__(self, indexName: str, indexedColumns: Sequence[str],
                 includedColumns: Sequence[str] = ()):
        if not indexName or not indexedColumns:
            raise ValueError("Empty index name or indexed columns are not allowed.")
        self.indexName = indexName
        self.indexedColumns = list(indexedColumns)
        self.includedColumns = list(includedColumns or [])
        lower_idx = [c.lower() for c in self.indexedColumns]
        lower_inc = [c.lower() for c in self.includedColumns]
        if len(set(lower_idx)) < len(lower_idx):
            raise ValueError("Duplicate indexed column names are not allowed.")
        if len(set(lower_inc)) < len(lower_inc):
            raise ValueError("Duplicate included column names are not allowed.")
        if any(c in lower_inc for c in lower_idx):
            raise ValueError("Duplicate column names in indexed/included columns are not allowed.")
        self._lower_idx = lower_idx
        self._lower_inc = lower_inc

    # snake_case aliases used internally
    @property
    def index_name(self):
        return self.indexName

    @property
    def indexed_columns(self):
        return self.indexedColumns

    @property
    def included_columns(self):
        return self.includedColumns

    def __eq__(self, o):
        return isinstance(o, IndexConfig) and self.indexName.lower() == o.indexName.lower() and \
            self._lower_idx == o._lower_idx and set(self._lower_inc) == set(o._lower_inc)

    def __hash__(self):
        return hash((tuple(self._lower_idx), frozenset(self._lower_inc)))

    def __repr__(self):
        return (f"[indexName: {self.indexName}; indexedColumns: {', '.join(self._lower_idx)}; "
                f"includedColumns: {', '.join(self._lower_inc)}]")

    @staticmethod
    def builder() -> "IndexConfigBuilder":
        return IndexConfigBuilder()


class IndexConfigBuilder:
    """Builder with single-set guards (``IndexConfig.scala:88-158``)."""

    def __init__(self):
        self._name = ""
        self._indexed: list = []
        self._included: list = []

    def indexName(self, name: str) -> "IndexConfigBuilder":
        if self._name:
            raise RuntimeError("Index name is already set.")
        if not name:
            raise ValueError("Empty index name is not allowed.")
        self._name = name
        return self

    def indexBy(self, col: str, *cols: str) -> "IndexConfigBuilder":
        if self._indexed:
            raise RuntimeError("Indexed columns are already set.")
        self._indexed = [col, *cols]
        return self

    def include(self, col: str, *cols: str) -> "IndexConfigBuilder":
        if self._included:
            raise RuntimeError("Included columns are already set.")
        self._included = [col, *cols]
        return self

    def create(self) -> IndexConfig:
        return IndexConfig(self._name, self._indexed, self._included)
