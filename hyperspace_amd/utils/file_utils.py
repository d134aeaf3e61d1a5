"""Filesystem helpers (reference: ``util/FileUtils.scala:28-124``, ``index/factories.scala``).

``LocalFileSystem`` is the single FS implementation; it is reached through
``FileSystemFactory`` so tests can substitute fakes exactly like the reference's Mockito seams.
All paths crossing this API are Hadoop-qualified strings (``file:/...``).

Commits use ``os.link`` (atomic create-if-absent on POSIX) instead of the reference's
exists-check + rename, which is racy.
"""
from __future__ import annotations

import os
import shutil
import uuid
from dataclasses import dataclass

from . import path_utils as P


@dataclass(frozen=True)
class FileStatus:
    path: str            # qualified path, e.g. file:/tmp/data/part-0.parquet
    length: int          # bytes
    modification_time: int  # epoch milliseconds
    is_dir: bool = False

    @property
    def name(self) -> str:
        return P.get_name(self.path)


def _stat(local: str) -> FileStatus:
    st = os.stat(local)
    return FileStatus(P.qualify(os.path.abspath(local)), st.st_size,
                      st.st_mtime_ns // 1_000_000, os.path.isdir(local))


class LocalFileSystem:
    def exists(self, path: str) -> bool:
        return os.path.exists(P.to_local(path))

    def is_dir(self, path: str) -> bool:
        return os.path.isdir(P.to_local(path))

    def get_file_status(self, path: str) -> FileStatus:
        return _stat(P.to_local(path))

    def list_status(self, path: str) -> list:
        local = P.to_local(path)
        if not os.path.isdir(local):
            if os.path.exists(local):
                return [_stat(local)]
            raise FileNotFoundError(path)
        out = []
        with os.scandir(local) as it:
            for e in it:
                st = e.stat()
                out.append(FileStatus(P.qualify(os.path.abspath(e.path)), st.st_size,
                                      st.st_mtime_ns // 1_000_000, e.is_dir()))
        out.sort(key=lambda s: s.path)
        return out

    def mkdirs(self, path: str) -> None:
        os.makedirs(P.to_local(path), exist_ok=True)

    def delete(self, path: str, recursive: bool = True) -> bool:
        local = P.to_local(path)
        if not os.path.exists(local):
            return False
        if os.path.isdir(local):
            if recursive:
                shutil.rmtree(local)
            else:
                os.rmdir(local)
        else:
            os.remove(local)
        return True

    def read_text(self, path: str) -> str:
        with open(P.to_local(path), "r", encoding="utf-8") as f:
            return f.read()

    def write_text(self, path: str, content: str) -> None:
        local = P.to_local(path)
        os.makedirs(os.path.dirname(local), exist_ok=True)
        with open(local, "w", encoding="utf-8") as f:
            f.write(content)
            f.flush()
            os.fsync(f.fileno())

    def rename(self, src: str, dst: str) -> bool:
        os.replace(P.to_local(src), P.to_local(dst))
        return True

    def link_if_absent(self, src: str, dst: str) -> bool:
        """Atomically publish ``src`` at ``dst``; False if ``dst`` already exists."""
        try:
            os.link(P.to_local(src), P.to_local(dst))
            return True
        except FileExistsError:
            return False

    def copy(self, src: str, dst: str) -> bool:
        shutil.copyfile(P.to_local(src), P.to_local(dst))
        return True


_FS = LocalFileSystem()


def get_fs(path: str = None) -> LocalFileSystem:
    return _FS


def create_file(fs, path: str, contents: str) -> None:
    """``FileUtils.createFile``: contents must be non-empty (``FileUtils.scala:37-42``)."""
    if not contents:
        raise ValueError("Empty contents are not allowed for createFile.")
    fs.write_text(path, contents)


def read_contents(fs, path: str) -> str:
    return fs.read_text(path)


def delete(path: str) -> None:
    get_fs(path).delete(path, True)


def get_directory_size(path: str) -> int:
    total = 0
    for root, _, files in os.walk(P.to_local(path)):
        for f in files:
            total += os.path.getsize(os.path.join(root, f))
    return total


def list_leaf_files(path: str, fs=None, path_filter=P.data_path_filter,
                    throw_if_not_exists: bool = False) -> list:
    """Recursive listing of data files under ``path`` (``IndexLogEntry.scala:301-315``)."""
    fs = fs or get_fs(path)
    try:
        statuses = fs.list_status(path)
    except FileNotFoundError:
        if throw_if_not_exists:
            raise
        return []
    files = [s for s in statuses if not s.is_dir and path_filter(s.name)]
    for d in statuses:
        if d.is_dir and path_filter(d.name):
            files.extend(list_leaf_files(d.path, fs, path_filter, throw_if_not_exists))
    return files


def temp_name(prefix: str = "temp") -> str:
    return prefix + str(uuid.uuid4())
