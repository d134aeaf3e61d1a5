"""Bucketed writer invariants (``DataFrameWriterExtensionsTest.scala:93-153``), signatures
(``FileBasedSignatureProviderTest``, ``IndexSignatureProviderTest``), explain output
(``ExplainTest.scala:65-181``), BucketUnion (``BucketUnionTest.scala:29-123``), Hybrid Scan
(``HybridScanSuite``) and the Delta source (``DeltaLakeIntegrationTest``)."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, col
from hyperspace_amd.io.writer import bucket_file_name, get_bucket_id, write_bucketed_table
from hyperspace_amd.plan import logical as L
from hyperspace_amd.plan import physical as X
from hyperspace_amd.utils import murmur3
from hyperspace_amd.utils.hashing import md5_hex

from helpers import (count_nodes, index_names_used, make_session, sample_table, scans,
                     sorted_rows, verify_index_usage, write_parquet_parts)


# ------------------------------------------------------------------------------------------------
# bucketed writer
# ------------------------------------------------------------------------------------------------
def test_bucket_file_naming_round_trip():
    n = bucket_file_name(3, "0d181aab-9773-4929-926d-5a97dbbb081a", 17, "snappy")
    assert n == "part-00003-0d181aab-9773-4929-926d-5a97dbbb081a_00017.c000.snappy.parquet"
    assert get_bucket_id(n) == 17
    assert get_bucket_id("part-00000-0d181aab-9773-4929-926d-5a97dbbb081a_00001.c000.parquet") == 1
    assert get_bucket_id("part-00000.parquet") is None


@pytest.mark.parametrize("cols", [["k"], ["s"], ["k", "s"]])
def test_bucketed_write_invariants(tmp_path, cols):
    rng = np.random.default_rng(0)
    n = 5000
    t = pa.table({"k": pa.array(rng.integers(-1000, 1000, n), pa.int64()),
                  "s": pa.array([f"v{x}" for x in rng.integers(0, 300, n)]),
                  "d": rng.random(n)})
    files = write_bucketed_table(t, str(tmp_path / "out"), 8, cols)
    seen = 0
    for f in files:
        b = get_bucket_id(os.path.basename(f))
        part = pq.read_table(f[len("file:"):] if f.startswith("file:") else f)
        seen += part.num_rows
        # every row re-hashes to the file's bucket
        assert set(murmur3.bucket_ids([part.column(c) for c in cols], 8).tolist()) == {b}
        # rows are sorted by the bucket columns inside the file
        keys = list(zip(*[part.column(c).to_pylist() for c in cols]))
        assert keys == sorted(keys)
    assert seen == n
    assert len({get_bucket_id(os.path.basename(f)) for f in files}) == len(files)


# ------------------------------------------------------------------------------------------------
# signatures
# ------------------------------------------------------------------------------------------------
def test_file_based_and_index_signatures(tmp_path):
    s = make_session(tmp_path)
    src = str(tmp_path / "src")
    write_parquet_parts(sample_table(), src, 3)
    from hyperspace_amd.index import signatures as SG
    df = s.read.parquet(src)
    plan = df.queryExecution.optimized_plan
    files = sorted(plan.collect(lambda p: isinstance(p, L.LogicalRelation))[0]
                   .relation.location.all_files(), key=lambda f: f.path)
    acc = ""
    for f in files:
        acc = md5_hex(acc + f"{f.length}{f.modification_time}{f.path}")
    fsig = SG.FileBasedSignatureProvider().signature(plan, s)
    assert fsig == md5_hex(acc)
    psig = SG.PlanSignatureProvider().signature(plan, s)
    assert psig == md5_hex("" + plan.node_name)
    assert SG.IndexSignatureProvider().signature(plan, s) == md5_hex(fsig + psig)
    assert isinstance(SG.create(SG.INDEX_SIGNATURE_PROVIDER), SG.IndexSignatureProvider)
    with pytest.raises(ValueError):
        SG.create("no.such.Provider")
    # any file change changes the signature
    write_parquet_parts(sample_table().slice(0, 1), src, 1, prefix="x")
    plan2 = s.read.parquet(src).queryExecution.optimized_plan
    assert SG.IndexSignatureProvider().signature(plan2, s) != SG.IndexSignatureProvider().signature(plan, s)


# ------------------------------------------------------------------------------------------------
# explain
# ------------------------------------------------------------------------------------------------
def test_explain_filter_highlights_index_scan(tmp_path):
    s = make_session(tmp_path)
    src = str(tmp_path / "src")
    write_parquet_parts(sample_table(), src, 2)
    hs = Hyperspace(s)
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["imprs"]))
    out = []
    hs.explain(s.read.parquet(src).filter(col("Query") == "facebook").select("Query", "imprs"),
               redirectFunc=out.append)
    text = "".join(out)
    sections = [l for l in text.splitlines() if l.endswith(":") and not l.startswith(" ")]
    assert sections == ["Plan with indexes:", "Plan without indexes:", "Indexes used:"]
    assert "<----FileScan Hyperspace(Type: CI, Name: fIdx, LogVersion: 1)" in text
    assert "<----FileScan parquet [Query#" in text
    assert text.count("---->") == 2
    assert "fIdx:" in text and "/indexes/fIdx/v__=0" in text
    assert not Hyperspace.isEnabled(s)  # explain restores the session state


def test_explain_verbose_join_operator_stats(tmp_path):
    s = make_session(tmp_path)
    src = str(tmp_path / "src")
    write_parquet_parts(sample_table(), src, 2)
    hs = Hyperspace(s)
    hs.createIndex(s.read.parquet(src), IndexConfig("jIdx", ["RGUID"], ["clicks"]))
    a = s.read.parquet(src)
    b = s.read.parquet(src)
    q = a.join(b, a["RGUID"] == b["RGUID"]).select(a["clicks"], b["clicks"])
    out = []
    hs.explain(q, verbose=True, redirectFunc=out.append)
    text = "".join(out)
    assert "Physical operator stats:" in text
    rows = {}
    for line in text.splitlines():
        parts = [p.strip() for p in line.strip("|").split("|")]
        if len(parts) == 4 and parts[0] and parts[1].lstrip("-").isdigit():
            rows[parts[0]] = tuple(int(x) for x in parts[1:])
    # ExplainTest.scala:142-172: the self-join's second exchange is a ReusedExchange
    assert rows["ShuffleExchange"] == (1, 0, -1)
    assert rows["ReusedExchange"] == (1, 0, -1)
    assert rows["Sort"] == (2, 0, -2)
    assert rows["SortMergeJoin"] == (1, 1, 0)
    assert "ReusedExchange [RGUID#" in text and "], Exchange hashpartitioning(RGUID#" in text


def test_reused_exchange_self_join_results(tmp_path):
    s = make_session(tmp_path)
    src = str(tmp_path / "src")
    write_parquet_parts(sample_table(), src, 2)
    a = s.read.parquet(src)
    b = s.read.parquet(src)
    q = a.join(b, a["RGUID"] == b["RGUID"]).select(a["clicks"], b["clicks"])
    plan = q.queryExecution.executed_plan
    assert len(plan.collect(lambda p: isinstance(p, X.ReusedExchangeExec))) == 1
    got = sorted(tuple(r) for r in q.collect())
    s.conf.set("spark.sql.exchange.reuse", "false")
    q2 = a.join(b, a["RGUID"] == b["RGUID"]).select(a["clicks"], b["clicks"])
    assert not q2.queryExecution.executed_plan.collect(
        lambda p: isinstance(p, X.ReusedExchangeExec))
    assert got == sorted(tuple(r) for r in q2.collect())


def test_explain_html_mode(tmp_path):
    s = make_session(tmp_path, spark__hyperspace__explain__displayMode="html")
    src = str(tmp_path / "src")
    write_parquet_parts(sample_table(), src, 1)
    hs = Hyperspace(s)
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["imprs"]))
    out = []
    hs.explain(s.read.parquet(src).filter(col("Query") == "x").select("imprs"),
               redirectFunc=out.append)
    text = "".join(out)
    assert text.startswith("<pre>") and text.endswith("</pre>")
    assert '<b style="background:LightGreen">' in text and "<br>" in text


# ------------------------------------------------------------------------------------------------
# BucketUnion
# ------------------------------------------------------------------------------------------------
def test_bucket_union_keeps_partitioning(tmp_path):
    s = make_session(tmp_path)
    t1 = pa.table({"id": pa.array([2, 3, 2], pa.int32()), "v": ["a", "b", "c"]})
    t2 = pa.table({"id": pa.array([3, 2], pa.int32()), "v": ["d", "e"]})
    d1 = s.createDataFrame(t1).repartition(10, "id")
    d2 = s.createDataFrame(t2).repartition(10, "id")
    bu = L.BucketUnion([d1.queryExecution.analyzed, d2.queryExecution.analyzed],
                       L.BucketSpec(10, ["id"], []))
    from hyperspace_amd.plan.dataframe import DataFrame
    s.enableHyperspace()  # registers BucketUnionStrategy
    df = DataFrame(s, bu)
    plan = df.queryExecution.executed_plan
    assert count_nodes(df, X.BucketUnionExec) == 1
    bue = plan.collect(lambda p: isinstance(p, X.BucketUnionExec))[0]
    assert bue.output_partitioning.num_partitions == 10
    rows = sorted((r.id, r.v) for r in df.collect())
    assert rows == [(2, "a"), (2, "c"), (2, "e"), (3, "b"), (3, "d")]
    # Appendix D golden vector: id=2 -> partition 4, id=3 -> partition 1
    assert list(murmur3.bucket_ids([pa.array([2, 3], pa.int32())], 10)) == [4, 1]


def test_bucket_union_rejects_mismatched_children(tmp_path):
    s = make_session(tmp_path)
    d1 = s.createDataFrame(pa.table({"id": pa.array([1], pa.int32())}))
    d2 = s.createDataFrame(pa.table({"id": pa.array([1], pa.int64()), "x": [1]}))
    with pytest.raises(Exception):
        L.BucketUnion([d1.queryExecution.analyzed, d2.queryExecution.analyzed],
                      L.BucketSpec(4, ["id"], [])).output


# ------------------------------------------------------------------------------------------------
# Hybrid Scan
# ------------------------------------------------------------------------------------------------
def _hybrid_session(tmp_path, deleted_ratio="0.9", lineage="true"):
    return make_session(tmp_path, spark__hyperspace__index__lineage__enabled=lineage,
                        spark__hyperspace__index__hybridscan__enabled="true",
                        spark__hyperspace__index__hybridscan__maxAppendedRatio="0.9",
                        spark__hyperspace__index__hybridscan__maxDeletedRatio=deleted_ratio)


def test_hybrid_scan_filter_with_appended_files(tmp_path):
    s = _hybrid_session(tmp_path)
    hs = Hyperspace(s)
    src = str(tmp_path / "src")
    write_parquet_parts(sample_table(), src, 3)
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["clicks"]))
    write_parquet_parts(sample_table().slice(0, 4), src, 1, prefix="app")
    q = lambda: s.read.parquet(src).filter(col("Query") == "facebook").select("Query", "clicks")  # noqa
    df = verify_index_usage(s, q, {"fIdx"}, index_files_only=False)
    # parquet + append-only: appended files are read in the same index scan
    sc = [x for x in scans(df) if x.relation.index is not None][0]
    assert any("/src/" in f.path for f in sc.relation.location.all_files())
    assert [r.clicks for r in sorted_rows(df)] == [20, 20, 40, 40, 70]


def test_hybrid_scan_filter_with_deleted_files_injects_lineage_filter(tmp_path):
    s = _hybrid_session(tmp_path)
    hs = Hyperspace(s)
    src = str(tmp_path / "src")
    paths = write_parquet_parts(sample_table(), src, 3)
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["clicks"]))
    os.remove(paths[0])
    q = lambda: s.read.parquet(src).filter(col("Query") == "facebook").select("Query", "clicks")  # noqa
    df = verify_index_usage(s, q, {"fIdx"})
    assert "_data_file_id" in df.queryExecution.executed_plan.tree_string()


def test_hybrid_scan_not_applied_when_ratio_exceeded_or_no_lineage(tmp_path):
    s = _hybrid_session(tmp_path, deleted_ratio="0.1")
    hs = Hyperspace(s)
    src = str(tmp_path / "src")
    paths = write_parquet_parts(sample_table(), src, 2)
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["clicks"]))
    os.remove(paths[0])  # deletes ~50% of the bytes > 10%
    Hyperspace.enable(s)
    df = s.read.parquet(src).filter(col("Query") == "facebook").select("clicks")
    assert index_names_used(df) == set()


def test_hybrid_scan_join_uses_bucket_union(tmp_path):
    s = _hybrid_session(tmp_path)
    hs = Hyperspace(s)
    src = str(tmp_path / "src")
    write_parquet_parts(sample_table(), src, 3)
    hs.createIndex(s.read.parquet(src), IndexConfig("jIdx", ["RGUID"], ["clicks"]))
    write_parquet_parts(sample_table().slice(2, 3), src, 1, prefix="app")

    def q():
        a = s.read.parquet(src)
        b = s.read.parquet(src)
        return a.join(b, a["RGUID"] == b["RGUID"]).select(a["clicks"], b["clicks"])
    df = verify_index_usage(s, q, {"jIdx"}, index_files_only=False)
    assert count_nodes(df, X.BucketUnionExec) == 2
    # only the appended rows are shuffled; the index side keeps its bucketing
    for ex in df.queryExecution.executed_plan.collect(lambda p: isinstance(p, X.ShuffleExchangeExec)):
        assert ex.partitioning.num_partitions == 4


# ------------------------------------------------------------------------------------------------
# Delta Lake source
# ------------------------------------------------------------------------------------------------
def test_delta_source_index_refresh_and_time_travel(tmp_path):
    from hyperspace_amd.sources.delta import delete_delta_files, read_snapshot, write_delta
    s = make_session(tmp_path, spark__hyperspace__index__lineage__enabled="true")
    # the Delta provider is opt-in, as in the reference (DeltaLakeIntegrationTest)
    s.conf.set("spark.hyperspace.index.sources.fileBasedBuilders",
               "com.microsoft.hyperspace.index.sources.delta.DeltaLakeFileBasedSourceBuilder,"
               "com.microsoft.hyperspace.index.sources.default.DefaultFileBasedSourceBuilder")
    hs = Hyperspace(s)
    path = str(tmp_path / "delta")
    t = sample_table()
    write_delta(t.slice(0, 5), path)
    write_delta(t.slice(5), path)
    df = s.read.format("delta").load(path)
    assert df.count() == 10
    hs.createIndex(df, IndexConfig("dIdx", ["Query"], ["clicks"]))
    q = lambda: s.read.format("delta").load(path).filter(col("Query") == "donde") \
        .select("Query", "clicks")  # noqa: E731
    verify_index_usage(s, q, {"dIdx"})
    # time travel: version 0 holds only the first five rows
    old = s.read.format("delta").option("versionAsOf", 0).load(path)
    assert old.count() == 5
    # delete a file, refresh incrementally, index stays correct
    snap = read_snapshot(path)
    delete_delta_files(path, [sorted(snap.files)[0]])
    s.disableHyperspace()
    assert index_names_used(q()) == set()
    hs.refreshIndex("dIdx", "incremental")
    verify_index_usage(s, q, {"dIdx"})
    e = hs.index("dIdx").collect()[0]
    assert e.numSourceFiles == 1


def test_dataframe_explain_extended_prints_all_plans(tmp_path, capsys):
    from hyperspace_amd import Session, col
    pq.write_table(pa.table({"a": [1, 2, 3], "b": [4.0, 5.0, 6.0]}), str(tmp_path / "t.parquet"))
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "ix"),
                      "spark.hyperspace.mi.execution.device": "cpu"})
    df = s.read.parquet(str(tmp_path / "t.parquet")).filter(col("a") > 1)
    text = df.queryExecution.explain_string(True)
    for h in ("== Analyzed Logical Plan ==", "== Optimized Logical Plan ==", "== Physical Plan =="):
        assert h in text
    df.explain(True)
    assert "== Physical Plan ==" in capsys.readouterr().out
