"""Refresh actions (reference ``RefreshActionBase.scala:37-148``, ``RefreshAction.scala:33-58``,
``RefreshIncrementalAction.scala:47-145``, ``RefreshQuickAction.scala:32-80``)."""
from __future__ import annotations

from typing import List

from ..exceptions import HyperspaceException, NoChangesException
from ..index import signatures as S
from ..index.builder import rewrite_buckets
from ..index.config import IndexConfig
from ..index.log_entry import Content, FileInfo, LogicalPlanFingerprint, Signature
from ..plan import logical as L
from ..telemetry.events import (RefreshActionEvent, RefreshIncrementalActionEvent,
                                RefreshQuickActionEvent)
from . import states
from .base import Action
from .create import CreateActionBase


class RefreshActionBase(CreateActionBase, Action):
    transient_state = states.REFRESHING
    final_state = states.ACTIVE

    def __init__(self, session, log_manager, data_manager):
        CreateActionBase.__init__(self, session, data_manager)
        Action.__init__(self, log_manager, session)
        self._previous = None
        self._df = None
        self._current_files = None
        self.file_id_tracker = self.previous_entry.file_id_tracker

    @property
    def previous_entry(self):
        if self._previous is None:
            e = self.log_manager.get_log(self.base_id)
            if e is None:
                raise HyperspaceException("LogEntry must exist for refresh operation")
            self._previous = e
        return self._previous

    def num_buckets_for_index(self) -> int:
        return self.previous_entry.num_buckets

    def has_lineage(self) -> bool:
        return self.previous_entry.has_lineage_column

    @property
    def df(self):
        """Rebuild the source DataFrame from the stored Relation (``:68-86``)."""
        if self._df is None:
            from ..hyperspace import get_context
            rel = get_context(self.session).source_provider_manager.refresh_relation(
                self.previous_entry.relations[0])
            from ..plan.types import schema_from_json
            reader = self.session.read.schema(schema_from_json(rel.data_schema_json)) \
                .format(rel.file_format).options(rel.options)
            self._df = reader.load(*rel.root_paths)
        return self._df

    @property
    def index_config(self) -> IndexConfig:
        p = self.previous_entry
        return IndexConfig(p.name, p.indexed_columns, p.included_columns)

    def validate(self) -> None:
        if self.previous_entry.state.upper() != states.ACTIVE:
            raise HyperspaceException(
                f"Refresh is only supported in {states.ACTIVE} state. "
                f"Current index state is {self.previous_entry.state}")

    @property
    def current_files(self) -> set:
        if self._current_files is None:
            from ..hyperspace import get_context
            mgr = get_context(self.session).source_provider_manager
            rels = self.df.queryExecution.optimized_plan.collect(
                lambda x: isinstance(x, L.LogicalRelation))
            self._current_files = {FileInfo.from_status(f, self.file_id_tracker.add_file(f), True)
                                   for f in mgr.all_files(rels[0])}
        return self._current_files

    @property
    def deleted_files(self) -> List[FileInfo]:
        orig = self.previous_entry.relations[0].data.content.file_infos
        return sorted(orig - self.current_files, key=lambda f: f.name)

    @property
    def appended_files(self) -> List[FileInfo]:
        orig = self.previous_entry.relations[0].data.content.file_infos
        return sorted(self.current_files - orig, key=lambda f: f.name)


class RefreshAction(RefreshActionBase):
    """Full rebuild into a new ``v__=N``."""

    def log_entry(self):
        return self.get_index_log_entry(self.df, self.index_config, self.index_data_path)

    def op(self) -> None:
        self.write(self.df, self.index_config)

    def validate(self) -> None:
        super().validate()
        if self.current_files == self.previous_entry.source_file_info_set:
            raise NoChangesException("Refresh full aborted as no source data changed.")

    def event(self, app_info, message):
        return RefreshActionEvent(app_info, self.log_entry(), message)


class RefreshIncrementalAction(RefreshActionBase):
    """Index appended files into a new version; drop deleted files' rows via lineage."""

    def op(self) -> None:
        appended = self.appended_files
        deleted = self.deleted_files
        if appended:
            self.write(self.df, self.index_config, files=[f.name for f in appended])
        if deleted:
            # K5: bitmap/set filter over the previous index's files, per bucket (no re-hash).
            rewrite_buckets(self.session, list(self.previous_entry.content.files),
                            self.index_config.indexedColumns, self.index_data_path,
                            [f.id for f in deleted], self.previous_entry.num_buckets)

    def validate(self) -> None:
        super().validate()
        if not self.appended_files and not self.deleted_files:
            raise NoChangesException("Refresh incremental aborted as no source data change found.")
        if self.deleted_files and not self.has_lineage():
            raise HyperspaceException(
                "Index refresh (to handle deleted source data) is only supported on an index with "
                "lineage.")

    def log_entry(self):
        entry = self.get_index_log_entry(self.df, self.index_config, self.index_data_path)
        if not self.deleted_files:
            merged = Content(self.previous_entry.content.root.merge(entry.content.root))
            return entry.copy(content=merged)
        return entry

    def event(self, app_info, message):
        return RefreshIncrementalActionEvent(app_info, self.log_entry(), message)


class RefreshQuickAction(RefreshActionBase):
    """Metadata-only refresh: record appended/deleted files for Hybrid Scan."""

    def op(self) -> None:
        pass

    def validate(self) -> None:
        super().validate()
        if not self.appended_files and not self.deleted_files:
            raise NoChangesException("Refresh quick aborted as no source data change found.")
        if self.deleted_files and not self.previous_entry.has_lineage_column:
            raise HyperspaceException(
                "Index refresh to handle deleted source data is only supported on an index with "
                "lineage.")

    def log_entry(self):
        provider = S.create()
        sig = provider.signature(self.df.queryExecution.optimized_plan, self.session)
        fp = LogicalPlanFingerprint([Signature(provider.name, sig)])
        return self.previous_entry.copy_with_update(fp, self.appended_files, self.deleted_files)

    def event(self, app_info, message):
        return RefreshQuickActionEvent(app_info, self.log_entry(), message)
