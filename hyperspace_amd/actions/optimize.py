"""Index compaction (reference ``actions/OptimizeAction.scala:59-160``).

Quick mode compacts files below ``spark.hyperspace.index.optimize.fileSizeThreshold``; full mode
compacts everything; only buckets holding more than one candidate file are rewritten.  The state
is deliberately not validated (Appendix B quirk 6).
"""
from __future__ import annotations

from ..exceptions import HyperspaceException, NoChangesException
from ..index import constants as C
from ..index.builder import rewrite_buckets
from ..index.log_entry import Content, Directory
from ..io.writer import get_bucket_id
from ..telemetry.events import OptimizeActionEvent
from ..utils import file_utils as FU
from ..utils import path_utils as P
from ..utils.conf import HyperspaceConf
from . import states
from .base import Action
from .create import CreateActionBase


class OptimizeAction(CreateActionBase, Action):
    transient_state = states.OPTIMIZING
    final_state = states.ACTIVE

    def __init__(self, session, log_manager, data_manager, mode: str):
        CreateActionBase.__init__(self, session, data_manager)
        Action.__init__(self, log_manager, session)
        self.mode = mode
        self._prev = None
        self._split = None
        self.file_id_tracker = self.previous_entry.file_id_tracker

    @property
    def previous_entry(self):
        if self._prev is None:
            e = self.log_manager.get_log(self.base_id)
            if e is None:
                raise HyperspaceException("LogEntry must exist for optimize operation")
            self._prev = e
        return self._prev

    def _files(self):
        if self._split is None:
            infos = sorted(self.previous_entry.content.file_infos, key=lambda f: f.name)
            if self.mode.lower() == C.OPTIMIZE_MODE_QUICK:
                thr = HyperspaceConf.optimize_file_size_threshold(self.session.conf)
                cands = [f for f in infos if f.size < thr]
                large = [f for f in infos if f.size >= thr]
            else:
                cands, large = infos, []
            per_bucket = {}
            for f in cands:
                per_bucket.setdefault(get_bucket_id(P.get_name(f.name)), []).append(f)
            to_opt = [f for fs in per_bucket.values() if len(fs) > 1 for f in fs]
            single = [f for fs in per_bucket.values() if len(fs) <= 1 for f in fs]
            self._split = (to_opt, single + large)
        return self._split

    def validate(self) -> None:
        if self.mode.lower() not in C.OPTIMIZE_MODES:
            raise HyperspaceException(f"Unsupported optimize mode '{self.mode}' found.")
        if not self._files()[0]:
            raise NoChangesException(
                "Optimize aborted as no optimizable index files smaller than "
                f"{HyperspaceConf.optimize_file_size_threshold(self.session.conf)} found.")

    def op(self) -> None:
        rewrite_buckets(self.session, [f.name for f in self._files()[0]],
                        self.previous_entry.indexed_columns, self.index_data_path, None,
                        self.previous_entry.num_buckets)

    def log_entry(self):
        new_content = Content.from_directory(self.index_data_path, self.file_id_tracker)
        ignore = self._files()[1]
        if ignore:
            fs = FU.get_fs()
            d = Directory.from_leaf_files([fs.get_file_status(f.name) for f in ignore],
                                          self.file_id_tracker)
            return self.previous_entry.copy(content=Content(new_content.root.merge(d)))
        return self.previous_entry.copy(content=new_content)

    def event(self, app_info, message):
        return OptimizeActionEvent(app_info, self.log_entry(), message)
