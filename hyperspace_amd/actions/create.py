"""Index creation (reference ``actions/CreateActionBase.scala:32-220``, ``CreateAction.scala:30-82``)."""
from __future__ import annotations

from typing import List, Optional, Tuple

import pyarrow as pa

from ..exceptions import HyperspaceException
from ..index import constants as C
from ..index import signatures as S
from ..index.builder import build_from_source
from ..index.config import IndexConfig
from ..index.log_entry import (Content, CoveringIndex, FileIdTracker, IndexLogEntry,
                               LogicalPlanFingerprint, Signature, Source, SparkPlan)
from ..plan import logical as L
from ..plan.types import schema_to_json
from ..telemetry.events import CreateActionEvent
from ..utils import path_utils as P
from ..utils.conf import HyperspaceConf
from ..utils.resolver import resolve, resolve_one
from . import states
from .base import Action


class CreateActionBase:
    """Shared index-building logic for create / refresh / optimize."""

    def __init__(self, session, data_manager):
        self.session = session
        self.data_manager = data_manager
        self.file_id_tracker = FileIdTracker()
        self._index_data_path = None
        # Pin the target version now: under SPMD every rank must agree on it before any rank
        # creates the directory.
        _ = self.index_data_path

    @property
    def index_data_path(self) -> str:
        if self._index_data_path is None:
            latest = self.data_manager.get_latest_version_id()
            self._index_data_path = self.data_manager.get_path(0 if latest is None else latest + 1)
        return self._index_data_path

    def num_buckets_for_index(self) -> int:
        return HyperspaceConf.num_buckets_for_index(self.session.conf)

    def has_lineage(self) -> bool:
        return HyperspaceConf.index_lineage_enabled(self.session.conf)

    # -- column resolution ------------------------------------------------------------------------
    def resolve_config(self, df, config: IndexConfig) -> Tuple[List[str], List[str]]:
        names = df.columns
        cs = self.session.case_sensitive
        idx = resolve(config.indexedColumns, names, cs)
        inc = resolve(config.includedColumns, names, cs)
        if idx is None or inc is None:
            unresolved = [c for c in config.indexedColumns + config.includedColumns
                          if resolve_one(c, names, cs) is None]
            raise HyperspaceException(
                f"Columns '{','.join(unresolved)}' could not be resolved from available source "
                f"columns '{','.join(names)}'")
        return idx, inc

    def _relation(self, df) -> L.LogicalRelation:
        plan = df.queryExecution.optimized_plan
        if not isinstance(plan, L.LogicalRelation):
            raise HyperspaceException("Only creating index over HDFS file based scan nodes is supported.")
        return plan

    def index_columns(self, df, config) -> Tuple[List[str], List[str], List[str]]:
        idx, inc = self.resolve_config(df, config)
        cols = idx + inc
        extra: List[str] = []
        if self.has_lineage():
            rel = self._relation(df).relation
            cs = self.session.case_sensitive
            extra = [p for p in rel.partition_schema.names if resolve_one(p, cols, cs) is None]
        return idx, inc, extra

    def index_schema(self, df, idx, inc, extra) -> pa.Schema:
        by_name = {f.name: f for f in df.schema}
        fields = [by_name[c] for c in idx + inc + extra]
        if self.has_lineage():
            fields.append(pa.field(C.DATA_FILE_NAME_ID, pa.int64(), False))
        return pa.schema(fields)

    def source_relations(self, df):
        from ..hyperspace import get_context
        mgr = get_context(self.session).source_provider_manager
        return [mgr.create_relation(p, self.file_id_tracker)
                for p in df.queryExecution.optimized_plan.collect(
                    lambda x: isinstance(x, L.LogicalRelation))]

    def get_index_log_entry(self, df, config: IndexConfig, path: str) -> IndexLogEntry:
        from ..hyperspace import get_context
        provider = S.create()
        idx, inc, extra = self.index_columns(df, config)
        plan = df.queryExecution.optimized_plan
        sig = provider.signature(plan, self.session)
        if sig is None:
            raise HyperspaceException("Invalid plan for creating an index.")
        relations = self.source_relations(df)
        assert len(relations) == 1
        props = {}
        if self.has_lineage():
            props[C.LINEAGE_PROPERTY] = "true"
        mgr = get_context(self.session).source_provider_manager
        if isinstance(plan, L.LogicalRelation) and mgr.has_parquet_as_source_format(plan):
            props[C.HAS_PARQUET_AS_SOURCE_FORMAT_PROPERTY] = "true"
        abs_path = path if P.is_qualified(path) else P.make_absolute(path)
        return IndexLogEntry(
            config.indexName,
            CoveringIndex(idx, inc, schema_to_json(self.index_schema(df, idx, inc, extra)),
                          self.num_buckets_for_index(), props),
            Content.from_directory(abs_path, self.file_id_tracker),
            Source(SparkPlan(relations, None, None,
                             LogicalPlanFingerprint([Signature(provider.name, sig)]))),
            {})

    def lineage_ids(self, files: List[str]) -> Optional[dict]:
        if not self.has_lineage():
            return None
        by_path = {p: v for (p, _, _), v in self.file_id_tracker.get_file_to_id_map().items()}
        out = {}
        for path in files:
            if path not in by_path:
                raise HyperspaceException(f"no file id for {path}")
            out[path] = by_path[path]
        return out

    def write(self, df, config: IndexConfig, files: Optional[List[str]] = None,
              mode: str = "overwrite") -> List[str]:
        """``repartition(numBuckets, indexed) + saveWithBuckets`` (``CreateActionBase.scala:122-140``)."""
        lr = self._relation(df)
        idx, inc, extra = self.index_columns(df, config)
        if files is None:
            files = [f.path for f in lr.relation.location.all_files()]
        # make sure every file has an id before lineage is attached
        for f in lr.relation.location.all_files():
            self.file_id_tracker.add_file(f)
        return build_from_source(self.session, lr.relation, files, idx + inc + extra, idx,
                                 self.num_buckets_for_index(), self.index_data_path,
                                 self.lineage_ids(files), mode)


class CreateAction(CreateActionBase, Action):
    transient_state = states.CREATING
    final_state = states.ACTIVE

    def __init__(self, session, df, config: IndexConfig, log_manager, data_manager):
        CreateActionBase.__init__(self, session, data_manager)
        Action.__init__(self, log_manager, session)
        self.df = df
        self.config = config

    def log_entry(self):
        return self.get_index_log_entry(self.df, self.config, self.index_data_path)

    def validate(self) -> None:
        if not L.is_logical_relation(self.df.queryExecution.optimized_plan):
            raise HyperspaceException("Only creating index over HDFS file based scan nodes is supported.")
        if resolve(self.config.indexedColumns + self.config.includedColumns, self.df.columns,
                   self.session.case_sensitive) is None:
            raise HyperspaceException("Index config is not applicable to dataframe schema.")
        latest = self.log_manager.get_latest_log()
        if latest is not None and latest.state != states.DOESNOTEXIST:
            raise HyperspaceException(f"Another Index with name {self.config.indexName} already exists")

    def op(self) -> None:
        self.write(self.df, self.config)

    def event(self, app_info, message):
        try:
            index = self.log_entry()
        except Exception:  # noqa: BLE001
            index = None
        return CreateActionEvent(app_info, self.config, index, self.df.plan.tree_string(), message)
