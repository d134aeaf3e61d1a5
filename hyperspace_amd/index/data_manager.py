"""Versioned index data directories ``v__=<n>`` (reference ``index/IndexDataManager.scala:38-74``)."""
from __future__ import annotations

from typing import Optional

from ..utils import file_utils as FU
from ..utils import path_utils as P
from . import constants as C


class IndexDataManager:
    def get_latest_version_id(self) -> Optional[int]:
        raise NotImplementedError

    def get_path(self, id: int) -> str:
        raise NotImplementedError

    def delete(self, id: int) -> None:
        raise NotImplementedError


class IndexDataManagerImpl(IndexDataManager):
    def __init__(self, index_path: str, fs=None):
        self.index_path = index_path if P.is_qualified(index_path) else P.make_absolute(index_path)
        self.fs = fs or FU.get_fs(self.index_path)

    def get_latest_version_id(self) -> Optional[int]:
        if not self.fs.exists(self.index_path):
            return None
        prefix = C.INDEX_VERSION_DIRECTORY_PREFIX + "="
        ids = [int(s.name[len(prefix):]) for s in self.fs.list_status(self.index_path)
               if s.name.startswith(C.INDEX_VERSION_DIRECTORY_PREFIX)]
        return max(ids) if ids else None

    def get_path(self, id: int) -> str:
        return P.join(self.index_path, f"{C.INDEX_VERSION_DIRECTORY_PREFIX}={id}")

    def delete(self, id: int) -> None:
        self.fs.delete(self.get_path(id), True)
