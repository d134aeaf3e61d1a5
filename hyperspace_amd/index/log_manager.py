"""Operation log of an index (reference ``index/IndexLogManager.scala:33-166``).

Layout: ``<index>/_hyperspace_log/<int id>`` plus a ``latestStable`` copy.  ``write_log`` is an
optimistic-concurrency commit: the JSON is written to ``temp<uuid>`` and published with a hard
link, which fails atomically with EEXIST when another writer already owns ``id`` — a true
create-if-absent, unlike the reference's exists-check + rename.
"""
from __future__ import annotations

import logging
from typing import Optional

from ..actions.states import STABLE_STATES
from ..utils import file_utils as FU
from ..utils import path_utils as P
from . import constants as C
from .log_entry import LogEntry

log = logging.getLogger(__name__)


class IndexLogManager:
    def get_log(self, id: int) -> Optional[LogEntry]:
        raise NotImplementedError

    def get_latest_id(self) -> Optional[int]:
        raise NotImplementedError

    def get_latest_log(self) -> Optional[LogEntry]:
        i = self.get_latest_id()
        return self.get_log(i) if i is not None else None

    def get_latest_stable_log(self) -> Optional[LogEntry]:
        raise NotImplementedError

    def create_latest_stable_log(self, id: int) -> bool:
        raise NotImplementedError

    def delete_latest_stable_log(self) -> bool:
        raise NotImplementedError

    def write_log(self, id: int, entry: LogEntry) -> bool:
        raise NotImplementedError


class IndexLogManagerImpl(IndexLogManager):
    def __init__(self, index_path: str, fs=None):
        self.index_path = index_path if P.is_qualified(index_path) else P.make_absolute(index_path)
        self.fs = fs or FU.get_fs(self.index_path)
        self.log_path = P.join(self.index_path, C.HYPERSPACE_LOG)
        self.latest_stable_path = P.join(self.log_path, C.LATEST_STABLE_LOG_NAME)

    def _path(self, id: int) -> str:
        return P.join(self.log_path, str(id))

    def _read(self, path: str) -> Optional[LogEntry]:
        if not self.fs.exists(path):
            return None
        return LogEntry.from_json(FU.read_contents(self.fs, path))

    def get_log(self, id: int) -> Optional[LogEntry]:
        return self._read(self._path(id))

    def get_latest_id(self) -> Optional[int]:
        if not self.fs.exists(self.log_path):
            return None
        ids = []
        for s in self.fs.list_status(self.log_path):
            try:
                ids.append(int(s.name))
            except ValueError:
                pass
        return max(ids) if ids else None

    def get_latest_stable_log(self) -> Optional[LogEntry]:
        entry = self._read(self.latest_stable_path)
        if entry is None:
            latest = self.get_latest_id()
            if latest is not None:
                for i in range(latest, -1, -1):
                    e = self.get_log(i)
                    if e is not None and e.state in STABLE_STATES:
                        return e
            return None
        assert entry.state in STABLE_STATES
        return entry

    def create_latest_stable_log(self, id: int) -> bool:
        entry = self.get_log(id)
        if entry is None:
            log.error("Unable to get LogEntry for id = '%s'", id)
            return False
        if entry.state not in STABLE_STATES:
            log.error("Found LogEntry with non stable state = %s for id = '%s'", entry.state, id)
            return False
        try:
            return self.fs.copy(self._path(id), self.latest_stable_path)
        except Exception as e:  # noqa: BLE001 — mirrors the reference's Try(...)
            log.error("Failed to create the latest stable log with id = '%s': %s", id, e)
            return False

    def delete_latest_stable_log(self) -> bool:
        try:
            if not self.fs.exists(self.latest_stable_path):
                return True
            return self.fs.delete(self.latest_stable_path, True)
        except Exception as e:  # noqa: BLE001
            log.error("Failed to delete the latest stable log: %s", e)
            return False

    def write_log(self, id: int, entry: LogEntry) -> bool:
        target = self._path(id)
        if self.fs.exists(target):
            return False
        temp = P.join(self.log_path, FU.temp_name())
        try:
            self.fs.mkdirs(self.log_path)
            FU.create_file(self.fs, temp, entry.to_json())
            return self.fs.link_if_absent(temp, target)
        except Exception as e:  # noqa: BLE001
            log.error("Failed to write log with id = '%s': %s", id, e)
            return False
        finally:
            try:
                self.fs.delete(temp, False)
            except Exception:  # noqa: BLE001
                pass
