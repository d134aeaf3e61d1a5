"""On-disk index metadata model (reference ``index/IndexLogEntry.scala:36-686``, ``LogEntry.scala``).

Every class serializes to exactly the JSON field set and order of the reference (the canonical
example is ``IndexLogEntryTest.scala:83-185``) so log directories written by either engine are
interchangeable.  ``to_json_obj`` produces ordered dicts for ``utils.json_utils.to_json``;
``from_json_obj`` is tolerant of missing optional fields.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..exceptions import HyperspaceException
from ..utils import json_utils
from ..utils import path_utils as P
from ..utils.file_utils import FileStatus, get_fs, list_leaf_files
from . import constants as C

VERSION = "0.1"


# ------------------------------------------------------------------------------------------------
# Content / Directory / FileInfo
# ------------------------------------------------------------------------------------------------
class FileInfo:
    """(name, size, modifiedTime, id); equality and hash ignore ``id`` (``:321-344``)."""
    __slots__ = ("name", "size", "modified_time", "id")

    def __init__(self, name: str, size: int, modified_time: int, id: int = C.UNKNOWN_FILE_ID):
        self.name = name
        self.size = int(size)
        self.modified_time = int(modified_time)
        self.id = int(id)

    @staticmethod
    def from_status(s: FileStatus, id: int, as_full_path: bool) -> "FileInfo":
        if s.is_dir:
            raise ValueError("FileInfo is applicable for files, not directories.")
        return FileInfo(s.path if as_full_path else s.name, s.length, s.modification_time, id)

    def __eq__(self, o):
        return isinstance(o, FileInfo) and self.name == o.name and self.size == o.size \
            and self.modified_time == o.modified_time

    def __hash__(self):
        return hash((self.name, self.size, self.modified_time))

    def __repr__(self):
        return f"FileInfo({self.name!r}, {self.size}, {self.modified_time}, {self.id})"

    def to_json_obj(self):
        return {"name": self.name, "size": self.size, "modifiedTime": self.modified_time,
                "id": self.id}

    @staticmethod
    def from_json_obj(o) -> "FileInfo":
        return FileInfo(o["name"], o["size"], o["modifiedTime"], o.get("id", C.UNKNOWN_FILE_ID))


class Directory:
    def __init__(self, name: str, files: Optional[List[FileInfo]] = None,
                 sub_dirs: Optional[List["Directory"]] = None):
        self.name = name
        self.files = list(files or [])
        self.sub_dirs = list(sub_dirs or [])

    def __eq__(self, o):
        return isinstance(o, Directory) and self.name == o.name and \
            self.files == o.files and self.sub_dirs == o.sub_dirs

    def __hash__(self):
        return hash((self.name, len(self.files), len(self.sub_dirs)))

    def __repr__(self):
        return f"Directory({self.name!r}, {self.files!r}, {self.sub_dirs!r})"

    def merge(self, that: "Directory") -> "Directory":
        """Union of two trees with the same root name (``IndexLogEntry.scala:123-172``)."""
        if self.name != that.name:
            raise HyperspaceException(
                f"Merging directories with names {self.name} and {that.name} failed. "
                "Directory names must be same for merging directories.")
        mine = {d.name: d for d in self.sub_dirs}
        theirs = {d.name: d for d in that.sub_dirs}
        merged = []
        for name in list(mine.keys()) + [n for n in theirs.keys() if n not in mine]:
            if name in mine and name in theirs:
                merged.append(mine[name].merge(theirs[name]))
            else:
                merged.append(mine.get(name) or theirs[name])
        return Directory(self.name, self.files + that.files, merged)

    def to_json_obj(self):
        return {"name": self.name, "files": [f.to_json_obj() for f in self.files],
                "subDirs": [d.to_json_obj() for d in self.sub_dirs]}

    @staticmethod
    def from_json_obj(o) -> "Directory":
        return Directory(o["name"], [FileInfo.from_json_obj(f) for f in o.get("files") or []],
                         [Directory.from_json_obj(d) for d in o.get("subDirs") or []])

    # -- builders --------------------------------------------------------------------------------
    @staticmethod
    def from_directory(path: str, tracker: "FileIdTracker", path_filter=P.data_path_filter,
                       throw_if_not_exists: bool = False, fs=None) -> "Directory":
        leaf = list_leaf_files(path, fs, path_filter, throw_if_not_exists)
        if leaf:
            return Directory.from_leaf_files(leaf, tracker)
        return Directory._create_empty(P.make_absolute(path) if not P.is_qualified(path) else path)

    @staticmethod
    def _create_empty(qpath: str, sub_dirs=None) -> "Directory":
        while True:
            if P.is_root(qpath):
                return Directory(qpath, sub_dirs=sub_dirs or [])
            sub_dirs = [Directory(P.get_name(qpath), sub_dirs=sub_dirs or [])]
            qpath = P.get_parent(qpath)

    @staticmethod
    def from_leaf_files(files: List[FileStatus], tracker: "FileIdTracker") -> "Directory":
        if not files:
            raise ValueError("Empty files list found while creating a Directory.")
        if any(f.is_dir for f in files):
            raise ValueError("All files must be leaf files for creation of Directory.")
        by_parent: Dict[str, List[FileStatus]] = {}
        for f in files:
            by_parent.setdefault(P.get_parent(f.path), []).append(f)
        path_to_dir: Dict[str, Directory] = {}
        for dir_path in sorted(by_parent):
            infos = [FileInfo.from_status(f, tracker.add_file(f), as_full_path=False)
                     for f in by_parent[dir_path]]
            if dir_path in path_to_dir:
                path_to_dir[dir_path].files.extend(infos)
                continue
            cur = dir_path
            directory = Directory(cur if P.is_root(cur) else P.get_name(cur), infos, [])
            path_to_dir[cur] = directory
            while P.get_parent(cur) is not None and P.get_parent(cur) not in path_to_dir:
                cur = P.get_parent(cur)
                directory = Directory(cur if P.is_root(cur) else P.get_name(cur), [], [directory])
                path_to_dir[cur] = directory
            if P.get_parent(cur) is not None:
                path_to_dir[P.get_parent(cur)].sub_dirs.append(directory)
        root = files[0].path
        while not P.is_root(root):
            root = P.get_parent(root)
        return path_to_dir[root]


class Content:
    def __init__(self, root: Directory):
        self.root = root
        self._files = None
        self._file_infos = None

    def __eq__(self, o):
        return isinstance(o, Content) and self.root == o.root

    def __hash__(self):
        return hash(self.root)

    def __repr__(self):
        return f"Content({self.root!r})"

    def _rec(self, prefix: str, d: Directory, fn, out):
        for f in d.files:
            out.append(fn(f, prefix))
        for sd in d.sub_dirs:
            self._rec(P.join(prefix, sd.name), sd, fn, out)

    @property
    def files(self) -> List[str]:
        """Fully qualified paths of all files in the tree."""
        if self._files is None:
            out: list = []
            self._rec(self.root.name, self.root, lambda f, pre: P.join(pre, f.name), out)
            self._files = out
        return self._files

    @property
    def file_infos(self) -> set:
        if self._file_infos is None:
            out: list = []
            self._rec(self.root.name, self.root,
                      lambda f, pre: FileInfo(P.join(pre, f.name), f.size, f.modified_time, f.id),
                      out)
            self._file_infos = set(out)
        return self._file_infos

    def to_json_obj(self):
        return {"root": self.root.to_json_obj(),
                "fingerprint": {"kind": "NoOp", "properties": {}}}

    @staticmethod
    def from_json_obj(o) -> "Content":
        return Content(Directory.from_json_obj(o["root"]))

    @staticmethod
    def from_directory(path: str, tracker: "FileIdTracker", path_filter=P.data_path_filter,
                       throw_if_not_exists: bool = False) -> "Content":
        return Content(Directory.from_directory(path, tracker, path_filter, throw_if_not_exists))

    @staticmethod
    def from_leaf_files(files: List[FileStatus], tracker: "FileIdTracker") -> Optional["Content"]:
        return Content(Directory.from_leaf_files(files, tracker)) if files else None


# ------------------------------------------------------------------------------------------------
# Derived dataset / source description
# ------------------------------------------------------------------------------------------------
@dataclass
class CoveringIndex:
    indexed: List[str]
    included: List[str]
    schema_string: str
    num_buckets: int
    properties: Dict[str, str] = field(default_factory=dict)
    kind: str = "CoveringIndex"
    kind_abbr: str = "CI"

    def to_json_obj(self):
        return {"properties": {"columns": {"indexed": list(self.indexed),
                                           "included": list(self.included)},
                               "schemaString": self.schema_string,
                               "numBuckets": self.num_buckets,
                               "properties": dict(self.properties)},
                "kind": self.kind, "kindAbbr": self.kind_abbr}

    @staticmethod
    def from_json_obj(o) -> "CoveringIndex":
        p = o["properties"]
        return CoveringIndex(list(p["columns"]["indexed"]), list(p["columns"]["included"]),
                             p["schemaString"], int(p["numBuckets"]), dict(p.get("properties") or {}),
                             o.get("kind", "CoveringIndex"), o.get("kindAbbr", "CI"))


@dataclass(frozen=True)
class Signature:
    provider: str
    value: str

    def to_json_obj(self):
        return {"provider": self.provider, "value": self.value}


@dataclass
class LogicalPlanFingerprint:
    signatures: List[Signature]

    def to_json_obj(self):
        return {"properties": {"signatures": [s.to_json_obj() for s in self.signatures]},
                "kind": "LogicalPlan"}

    @staticmethod
    def from_json_obj(o):
        return LogicalPlanFingerprint([Signature(s["provider"], s["value"])
                                       for s in o["properties"]["signatures"]])


@dataclass
class Update:
    appended_files: Optional[Content] = None
    deleted_files: Optional[Content] = None

    def to_json_obj(self):
        return {"deletedFiles": self.deleted_files.to_json_obj() if self.deleted_files else None,
                "appendedFiles": self.appended_files.to_json_obj() if self.appended_files else None}

    @staticmethod
    def from_json_obj(o):
        if o is None:
            return None
        a, d = o.get("appendedFiles"), o.get("deletedFiles")
        return Update(Content.from_json_obj(a) if a else None, Content.from_json_obj(d) if d else None)


@dataclass
class Hdfs:
    content: Content
    update: Optional[Update] = None
    kind: str = "HDFS"

    def to_json_obj(self):
        props = {"content": self.content.to_json_obj()}
        props["update"] = self.update.to_json_obj() if self.update is not None else None
        return {"properties": props, "kind": self.kind}

    @staticmethod
    def from_json_obj(o):
        p = o["properties"]
        return Hdfs(Content.from_json_obj(p["content"]), Update.from_json_obj(p.get("update")),
                    o.get("kind", "HDFS"))


@dataclass
class Relation:
    root_paths: List[str]
    data: Hdfs
    data_schema_json: str
    file_format: str
    options: Dict[str, str]

    def to_json_obj(self):
        return {"rootPaths": list(self.root_paths), "data": self.data.to_json_obj(),
                "dataSchemaJson": self.data_schema_json, "fileFormat": self.file_format,
                "options": dict(self.options)}

    @staticmethod
    def from_json_obj(o):
        return Relation(list(o["rootPaths"]), Hdfs.from_json_obj(o["data"]), o["dataSchemaJson"],
                        o["fileFormat"], dict(o.get("options") or {}))


@dataclass
class SparkPlan:
    relations: List[Relation]
    raw_plan: Optional[str]
    sql: Optional[str]
    fingerprint: LogicalPlanFingerprint
    kind: str = "Spark"

    def to_json_obj(self):
        return {"properties": {"relations": [r.to_json_obj() for r in self.relations],
                               "rawPlan": self.raw_plan, "sql": self.sql,
                               "fingerprint": self.fingerprint.to_json_obj()},
                "kind": self.kind}

    @staticmethod
    def from_json_obj(o):
        p = o["properties"]
        return SparkPlan([Relation.from_json_obj(r) for r in p["relations"]], p.get("rawPlan"),
                         p.get("sql"), LogicalPlanFingerprint.from_json_obj(p["fingerprint"]),
                         o.get("kind", "Spark"))


@dataclass
class Source:
    plan: SparkPlan

    def to_json_obj(self):
        return {"plan": self.plan.to_json_obj()}


# ------------------------------------------------------------------------------------------------
# Log entries
# ------------------------------------------------------------------------------------------------
class LogEntry:
    """Base entry with mutable ``id/state/timestamp/enabled`` (``LogEntry.scala:22-30``)."""

    def __init__(self, version: str):
        self.version = version
        self.id = 0
        self.state = ""
        self.timestamp = int(time.time() * 1000)
        self.enabled = True

    @staticmethod
    def from_json(text: str) -> "LogEntry":
        m = json_utils.json_to_map(text)
        if m.get("version") == VERSION:
            return IndexLogEntry.from_json_obj(m)
        raise HyperspaceException(f"Unsupported log entry found: version = {m.get('version')}")


class IndexLogEntry(LogEntry):
    def __init__(self, name: str, derived_dataset: CoveringIndex, content: Content,
                 source: Source, properties: Optional[Dict[str, str]] = None):
        super().__init__(VERSION)
        self.name = name
        self.derived_dataset = derived_dataset
        self.content = content
        self.source = source
        self.properties = dict(properties or {})
        self._tags: Dict = {}
        self._file_id_tracker = None

    # -- serialization -----------------------------------------------------------------------------
    def to_json_obj(self):
        return {"name": self.name, "derivedDataset": self.derived_dataset.to_json_obj(),
                "content": self.content.to_json_obj(), "source": self.source.to_json_obj(),
                "properties": dict(self.properties), "version": self.version, "id": self.id,
                "state": self.state, "timestamp": self.timestamp, "enabled": self.enabled}

    def to_json(self) -> str:
        return json_utils.to_json(self.to_json_obj())

    @staticmethod
    def from_json_obj(o) -> "IndexLogEntry":
        e = IndexLogEntry(o["name"], CoveringIndex.from_json_obj(o["derivedDataset"]),
                          Content.from_json_obj(o["content"]),
                          Source(SparkPlan.from_json_obj(o["source"]["plan"])),
                          dict(o.get("properties") or {}))
        e.id = int(o.get("id", 0))
        e.state = o.get("state", "")
        e.timestamp = int(o.get("timestamp", 0))
        e.enabled = bool(o.get("enabled", True))
        return e

    def copy(self, **changes) -> "IndexLogEntry":
        e = IndexLogEntry(changes.get("name", self.name),
                          changes.get("derived_dataset", self.derived_dataset),
                          changes.get("content", self.content),
                          changes.get("source", self.source),
                          changes.get("properties", self.properties))
        e.id, e.state, e.timestamp, e.enabled = self.id, self.state, self.timestamp, self.enabled
        return e

    # -- accessors -------------------------------------------------------------------------------
    @property
    def schema(self):
        """The index data schema (parsed once per schema string: rules ask on every query)."""
        from ..plan.types import schema_from_json
        ss = self.derived_dataset.schema_string
        hit = self.__dict__.get("_schema_cache")
        if hit is None or hit[0] != ss:
            hit = (ss, schema_from_json(ss))
            self.__dict__["_schema_cache"] = hit
        return hit[1]

    @property
    def created(self) -> bool:
        return self.state == "ACTIVE"

    @property
    def relations(self) -> List[Relation]:
        assert len(self.source.plan.relations) == 1
        return self.source.plan.relations

    @property
    def source_file_info_set(self) -> set:
        return self.relations[0].data.content.file_infos

    @property
    def source_files_size_in_bytes(self) -> int:
        return sum(f.size for f in self.source_file_info_set)

    @property
    def source_update(self) -> Optional[Update]:
        return self.relations[0].data.update

    @property
    def appended_files(self) -> set:
        u = self.source_update
        return u.appended_files.file_infos if u is not None and u.appended_files else set()

    @property
    def deleted_files(self) -> set:
        u = self.source_update
        return u.deleted_files.file_infos if u is not None and u.deleted_files else set()

    @property
    def has_source_update(self) -> bool:
        return self.source_update is not None and (bool(self.appended_files) or
                                                   bool(self.deleted_files))

    def copy_with_update(self, latest_fingerprint: LogicalPlanFingerprint,
                         appended: List[FileInfo], deleted: List[FileInfo]) -> "IndexLogEntry":
        """Quick-refresh metadata update (``IndexLogEntry.scala:483-505``)."""
        tracker = self.file_id_tracker

        def to_status(f: FileInfo):
            return FileStatus(f.name, f.size, f.modified_time, False)
        rel = self.relations[0]
        new_rel = Relation(rel.root_paths,
                           Hdfs(rel.data.content,
                                Update(Content.from_leaf_files([to_status(f) for f in appended], tracker),
                                       Content.from_leaf_files([to_status(f) for f in deleted], tracker))),
                           rel.data_schema_json, rel.file_format, rel.options)
        plan = SparkPlan([new_rel], self.source.plan.raw_plan, self.source.plan.sql,
                         latest_fingerprint)
        return self.copy(source=Source(plan))

    @property
    def num_buckets(self) -> int:
        return self.derived_dataset.num_buckets

    @property
    def indexed_columns(self) -> List[str]:
        return self.derived_dataset.indexed

    @property
    def included_columns(self) -> List[str]:
        return self.derived_dataset.included

    @property
    def bucket_spec(self):
        from ..plan.logical import BucketSpec
        return BucketSpec(self.num_buckets, list(self.indexed_columns), list(self.indexed_columns))

    @property
    def config(self):
        from .config import IndexConfig
        return IndexConfig(self.name, self.indexed_columns, self.included_columns)

    @property
    def signature(self) -> Signature:
        sigs = self.source.plan.fingerprint.signatures
        assert len(sigs) == 1
        return sigs[0]

    @property
    def has_lineage_column(self) -> bool:
        return str(self.derived_dataset.properties.get(
            C.LINEAGE_PROPERTY, C.INDEX_LINEAGE_ENABLED_DEFAULT)).lower() == "true"

    @property
    def has_parquet_as_source_format(self) -> bool:
        return self.relations[0].file_format == "parquet" or str(
            self.derived_dataset.properties.get(C.HAS_PARQUET_AS_SOURCE_FORMAT_PROPERTY,
                                                "false")).lower() == "true"

    @property
    def file_id_tracker(self) -> "FileIdTracker":
        if self._file_id_tracker is None:
            t = FileIdTracker()
            t.add_file_info(self.source_file_info_set | self.content.file_infos)
            self._file_id_tracker = t
        return self._file_id_tracker

    def __eq__(self, o):
        return isinstance(o, IndexLogEntry) and self.config == o.config and \
            self.signature == o.signature and self.num_buckets == o.num_buckets and \
            self.content.root == o.content.root and \
            self.source.plan.relations == o.source.plan.relations and self.state == o.state

    def __hash__(self):
        return hash((self.name.lower(), self.signature, self.num_buckets))

    def __repr__(self):
        return f"IndexLogEntry({self.name}, id={self.id}, state={self.state})"

    # -- rule-time tag cache (``:564-602``) ----------------------------------------------------------
    def set_tag_value(self, plan, tag, value):
        self._tags[(id(plan) if plan is not None else None, tag)] = value

    def get_tag_value(self, plan, tag):
        return self._tags.get((id(plan) if plan is not None else None, tag))

    def unset_tag_value(self, plan, tag):
        self._tags.pop((id(plan) if plan is not None else None, tag), None)

    def with_cached_tag(self, plan, tag, fn):
        key = (id(plan) if plan is not None else None, tag)
        if key in self._tags:
            return self._tags[key]
        v = fn()
        self._tags[key] = v
        return v


class FileIdTracker:
    """Dense monotonically increasing file ids = lineage values (``IndexLogEntry.scala:617-686``)."""

    def __init__(self):
        self._max_id = -1
        self._map: Dict[tuple, int] = {}

    @property
    def max_file_id(self) -> int:
        return self._max_id

    def get_file_to_id_map(self) -> Dict[tuple, int]:
        return self._map

    def get_file_id(self, path: str, size: int, mtime: int) -> Optional[int]:
        return self._map.get((path, size, mtime))

    def add_file_info(self, files) -> None:
        for f in files:
            if f.id == C.UNKNOWN_FILE_ID:
                raise HyperspaceException(f"Cannot add file info with unknown id. (file: {f.name}).")
            key = (f.name, f.size, f.modified_time)
            existing = self._map.get(key)
            if existing is not None:
                if existing != f.id:
                    raise HyperspaceException(
                        "Adding file info with a conflicting id. "
                        f"(existing id: {existing}, new id: {f.id}, file: {f.name}).")
            else:
                self._map[key] = f.id
                self._max_id = max(self._max_id, f.id)

    def add_file(self, status: FileStatus) -> int:
        key = (status.path, status.length, status.modification_time)
        v = self._map.get(key)
        if v is None:
            self._max_id += 1
            v = self._max_id
            self._map[key] = v
        return v
