"""Metadata model: the JSON spec example, Content/Directory building and merging on real temp
dirs, FileIdTracker, quick-refresh ``copy_with_update`` (reference ``IndexLogEntryTest.scala``)."""
import json
import os

import pytest

from hyperspace_amd.exceptions import HyperspaceException
from hyperspace_amd.index.log_entry import (Content, CoveringIndex, Directory, FileIdTracker,
                                            FileInfo, Hdfs, IndexLogEntry, LogEntry,
                                            LogicalPlanFingerprint, Relation, Signature, Source,
                                            SparkPlan, Update)
from hyperspace_amd.utils import path_utils as P
from hyperspace_amd.utils.file_utils import FileStatus

SCHEMA = ('{"type":"struct","fields":[{"name":"RGUID","type":"string","nullable":true,'
          '"metadata":{}},{"name":"Date","type":"string","nullable":true,"metadata":{}}]}')

# Spec-shaped entry (same field set/order as the canonical example, our own values).
SPEC = """
{
  "name" : "specIndex",
  "derivedDataset" : {
    "properties" : {
      "columns" : {
        "indexed" : [ "c1" ],
        "included" : [ "c2", "c3" ]
      },
      "schemaString" : %s,
      "numBuckets" : 200,
      "properties" : { }
    },
    "kind" : "CoveringIndex"
  },
  "content" : {
    "root" : { "name" : "indexRoot", "files" : [ ], "subDirs" : [ ] },
    "fingerprint" : { "kind" : "NoOp", "properties" : { } }
  },
  "source" : {
    "plan" : {
      "properties" : {
        "relations" : [ {
          "rootPaths" : [ "srcRoot" ],
          "data" : {
            "properties" : {
              "content" : {
                "root" : {
                  "name" : "src",
                  "files" : [ { "name" : "a", "size" : 120, "modifiedTime" : 5, "id" : 0 },
                              { "name" : "b", "size" : 80, "modifiedTime" : 6, "id" : 1 } ],
                  "subDirs" : [ ]
                },
                "fingerprint" : { "kind" : "NoOp", "properties" : { } }
              },
              "update" : {
                "deletedFiles" : {
                  "root" : { "name" : "", "files" : [ { "name" : "a", "size" : 7,
                             "modifiedTime" : 7, "id" : 2 } ], "subDirs" : [ ] },
                  "fingerprint" : { "kind" : "NoOp", "properties" : { } }
                },
                "appendedFiles" : null
              }
            },
            "kind" : "HDFS"
          },
          "dataSchemaJson" : "schemaJson",
          "fileFormat" : "fmt",
          "options" : { }
        } ],
        "rawPlan" : null,
        "sql" : null,
        "fingerprint" : {
          "properties" : { "signatures" : [ { "provider" : "prov", "value" : "sigValue" } ] },
          "kind" : "LogicalPlan"
        }
      },
      "kind" : "Spark"
    }
  },
  "properties" : { },
  "version" : "0.1",
  "id" : 0,
  "state" : "ACTIVE",
  "timestamp" : 1600000000000,
  "enabled" : true
}""" % json.dumps(SCHEMA)


def _expected():
    rel = Relation(["srcRoot"],
                   Hdfs(Content(Directory("src", [FileInfo("a", 120, 5, 0), FileInfo("b", 80, 6, 1)])),
                        Update(None, Content(Directory("", [FileInfo("a", 7, 7, 2)])))),
                   "schemaJson", "fmt", {})
    plan = SparkPlan([rel], None, None, LogicalPlanFingerprint([Signature("prov", "sigValue")]))
    e = IndexLogEntry("specIndex", CoveringIndex(["c1"], ["c2", "c3"], SCHEMA, 200, {}),
                      Content(Directory("indexRoot")), Source(plan), {})
    e.state = "ACTIVE"
    e.timestamp = 1600000000000
    return e


def test_spec_example_parses():
    actual = LogEntry.from_json(SPEC)
    assert actual == _expected()
    assert actual.source_files_size_in_bytes == 200
    assert actual.timestamp == 1600000000000 and actual.enabled and actual.version == "0.1"
    assert [f.name for f in actual.schema] == ["RGUID", "Date"]
    assert actual.deleted_files == {FileInfo("a", 7, 7)}
    assert actual.appended_files == set()


def test_round_trip_and_field_order():
    e = _expected()
    text = e.to_json()
    back = LogEntry.from_json(text)
    assert back == e and back.to_json() == text
    top = list(json.loads(text).keys())
    assert top == ["name", "derivedDataset", "content", "source", "properties", "version", "id",
                   "state", "timestamp", "enabled"]
    rel = json.loads(text)["source"]["plan"]["properties"]["relations"][0]
    assert list(rel.keys()) == ["rootPaths", "data", "dataSchemaJson", "fileFormat", "options"]
    assert text.startswith('{\n  "name" : "specIndex"')


def test_unsupported_version_rejected():
    bad = SPEC.replace('"version" : "0.1"', '"version" : "0.2"')
    with pytest.raises(HyperspaceException):
        LogEntry.from_json(bad)


def test_file_info_equality_ignores_id():
    assert FileInfo("f", 1, 2, 3) == FileInfo("f", 1, 2, 9)
    assert len({FileInfo("f", 1, 2, 3), FileInfo("f", 1, 2, 4)}) == 1
    assert FileInfo("f", 1, 2) != FileInfo("f", 1, 3)


def _touch(path, n=10):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as f:
        f.write(b"x" * n)


def test_content_from_directory_lists_all_files(tmp_path):
    _touch(str(tmp_path / "d" / "f1.parquet"))
    _touch(str(tmp_path / "d" / "sub" / "f2.parquet"), 20)
    _touch(str(tmp_path / "d" / "_SUCCESS"))
    _touch(str(tmp_path / "d" / ".crc"))
    tracker = FileIdTracker()
    c = Content.from_directory(str(tmp_path / "d"), tracker)
    assert c.root.name == "file:/"
    files = sorted(c.files)
    q = P.make_absolute(str(tmp_path / "d"))
    assert files == sorted([P.join(q, "f1.parquet"), P.join(P.join(q, "sub"), "f2.parquet")])
    assert tracker.max_file_id == 1
    assert {f.size for f in c.file_infos} == {10, 20}


def test_content_from_empty_directory(tmp_path):
    os.makedirs(tmp_path / "empty")
    c = Content.from_directory(str(tmp_path / "empty"), FileIdTracker())
    assert c.files == []
    # root is the file system root with one Directory per path segment
    d = c.root
    names = []
    while d.sub_dirs:
        d = d.sub_dirs[0]
        names.append(d.name)
    assert names[-1] == "empty"


def test_from_leaf_files_and_merge(tmp_path):
    _touch(str(tmp_path / "a" / "x1"))
    _touch(str(tmp_path / "a" / "x2"))
    _touch(str(tmp_path / "b" / "y1"))
    tr = FileIdTracker()

    def st(p):
        s = os.stat(p)
        return FileStatus(P.make_absolute(p), s.st_size, int(s.st_mtime * 1000), False)
    d1 = Directory.from_leaf_files([st(str(tmp_path / "a" / "x1"))], tr)
    d2 = Directory.from_leaf_files([st(str(tmp_path / "a" / "x2")),
                                    st(str(tmp_path / "b" / "y1"))], tr)
    merged = Content(d1.merge(d2))
    assert sorted(P.get_name(f) for f in merged.files) == ["x1", "x2", "y1"]
    with pytest.raises(HyperspaceException):
        Directory("a").merge(Directory("b"))
    with pytest.raises(ValueError):
        Directory.from_leaf_files([], tr)


def test_file_id_tracker():
    t = FileIdTracker()
    a = t.add_file(FileStatus("file:/a", 1, 1, False))
    b = t.add_file(FileStatus("file:/b", 1, 1, False))
    assert (a, b) == (0, 1)
    assert t.add_file(FileStatus("file:/a", 1, 1, False)) == 0
    assert t.get_file_id("file:/b", 1, 1) == 1 and t.max_file_id == 1
    t.add_file_info([FileInfo("file:/c", 1, 1, 7)])
    assert t.max_file_id == 7
    with pytest.raises(HyperspaceException):
        t.add_file_info([FileInfo("file:/c", 1, 1, 8)])
    with pytest.raises(HyperspaceException):
        t.add_file_info([FileInfo("file:/d", 1, 1)])


def test_copy_with_update_quick_refresh():
    e = _expected()
    e2 = e.copy_with_update(LogicalPlanFingerprint([Signature("prov", "new")]),
                            [FileInfo("file:/src/new1", 5, 5, 10)],
                            [FileInfo("file:/src/a", 120, 5, 0)])
    assert e2.signature.value == "new"
    assert {f.name for f in e2.appended_files} == {"file:/src/new1"}
    assert {f.name for f in e2.deleted_files} == {"file:/src/a"}
    assert e.signature.value == "sigValue"  # original untouched
    assert e2.has_source_update


def test_tags_are_per_plan():
    e = _expected()
    p1, p2 = object(), object()
    e.set_tag_value(p1, "T", 1)
    assert e.get_tag_value(p1, "T") == 1 and e.get_tag_value(p2, "T") is None
    calls = []
    assert e.with_cached_tag(p2, "T", lambda: calls.append(1) or 5) == 5
    assert e.with_cached_tag(p2, "T", lambda: calls.append(1) or 6) == 5
    assert len(calls) == 1
    e.unset_tag_value(p1, "T")
    assert e.get_tag_value(p1, "T") is None
