"""Hadoop-style path helpers for the local filesystem.

The reference stores fully qualified Hadoop paths (``file:/tmp/a/b``) in its metadata
(``util/PathUtils.scala:22-40``, ``IndexLogEntry.scala:235-316``).  This module converts between
local OS paths and that qualified string form, and exposes the ``DataPathFilter`` used when
listing data files (hidden ``_``/``.`` files are skipped unless the name contains ``=``).
"""
from __future__ import annotations

import os
import posixpath

SCHEME = "file:"


def is_qualified(path: str) -> bool:
    return path.startswith("file:")


def to_local(path: str) -> str:
    """``file:/a/b`` / ``file:///a/b`` / ``/a/b`` -> ``/a/b``."""
    if path.startswith("file:"):
        rest = path[5:]
        while rest.startswith("//"):
            rest = rest[1:]
        return rest if rest else "/"
    return path


def make_absolute(path: str) -> str:
    """Qualify a path the way ``PathUtils.makeAbsolute`` does: ``file:/abs/path``."""
    local = os.path.abspath(to_local(str(path)))
    return qualify(local)


def qualify(local_abs: str) -> str:
    local_abs = posixpath.normpath(local_abs) if local_abs != "/" else "/"
    if local_abs == "/":
        return "file:/"
    return "file:" + local_abs


def get_name(qpath: str) -> str:
    p = to_local(qpath).rstrip("/")
    return posixpath.basename(p)


def get_parent(qpath: str):
    local = to_local(qpath)
    if local in ("/", ""):
        return None
    parent = posixpath.dirname(local.rstrip("/")) or "/"
    return qualify(parent)


def is_root(qpath: str) -> bool:
    return to_local(qpath) in ("/", "")


def join(parent: str, child: str) -> str:
    """Hadoop ``new Path(parent, child)`` for the qualified local scheme."""
    if is_qualified(parent):
        base = to_local(parent)
        return qualify(posixpath.join(base, child))
    return posixpath.join(parent, child)


def data_path_filter(name: str) -> bool:
    """``PathUtils.DataPathFilter``: accept unless hidden (``_x`` without ``=``, or ``.x``)."""
    return not ((name.startswith("_") and "=" not in name) or name.startswith("."))
