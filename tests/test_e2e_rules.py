"""End-to-end rule application on real Parquet/CSV/JSON (host executor), using the reference's
disabled-vs-enabled oracle and plan-shape assertions (``E2EHyperspaceRulesTest.scala``:
filter/join rule use, ``:455-479`` Exchange/Sort elimination, ``:1004-1019`` verifyIndexUsage)."""
import os

import pyarrow as pa
import pyarrow.csv as pacsv
import pyarrow.json  # noqa: F401
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, col, count
from hyperspace_amd.plan import physical as X

from helpers import (count_nodes, index_names_used, make_session, sample_table, scans,
                     sorted_rows, verify_index_usage, write_parquet_parts)


@pytest.fixture
def env(tmp_path):
    s = make_session(tmp_path)
    src = str(tmp_path / "sample")
    write_parquet_parts(sample_table(), src, parts=2)
    hs = Hyperspace(s)
    yield s, hs, src
    s.disableHyperspace()


# ------------------------------------------------------------------------------------------------
# FilterIndexRule
# ------------------------------------------------------------------------------------------------
def test_filter_index_used_for_filter_project(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["imprs", "clicks"]))
    df = verify_index_usage(
        s, lambda: s.read.parquet(src).filter(col("Query") == "facebook").select("Query", "imprs"),
        {"fIdx"})
    assert [r.imprs for r in sorted_rows(df)] == [2, 4, 7]
    # the filter path drops the bucket spec (FilterIndexRule.scala:59-65)
    assert all(not sc.use_bucketing for sc in scans(df))


def test_filter_index_range_predicates_and_sql_string(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["clicks"], ["Query"]))
    verify_index_usage(s, lambda: s.read.parquet(src).filter("clicks >= 30 AND clicks < 80")
                       .select("clicks", "Query"), {"fIdx"})
    verify_index_usage(s, lambda: s.read.parquet(src).filter(col("clicks").isin(10, 90))
                       .select("Query"), {"fIdx"})


def test_filter_index_used_for_count_star_over_filter(env):
    # COUNT(*) reads no column of its own: the scan narrows to the filter's columns, which the
    # index covers
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["clicks"], ["Query"]))
    df = verify_index_usage(
        s, lambda: s.read.parquet(src).filter((col("clicks") >= 30) & (col("Query") != "ibraco"))
        .agg(count("*").alias("n")), {"fIdx"})
    assert df.collect()[0].n > 0


def test_filter_index_not_used_without_first_indexed_column(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query", "clicks"], ["imprs"]))
    Hyperspace.enable(s)
    df = s.read.parquet(src).filter(col("clicks") == 20).select("clicks", "imprs")
    assert index_names_used(df) == set()
    df2 = s.read.parquet(src).filter((col("Query") == "facebook") & (col("clicks") == 20)) \
        .select("clicks", "imprs")
    assert index_names_used(df2) == {"fIdx"}


def test_filter_index_not_used_when_not_covering(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["imprs"]))
    Hyperspace.enable(s)
    df = s.read.parquet(src).filter(col("Query") == "donde").select("Query", "clicks")
    assert index_names_used(df) == set()


def test_filter_index_select_star_when_index_covers_all(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src),
                   IndexConfig("all", ["Query"], ["Date", "RGUID", "imprs", "clicks"]))
    verify_index_usage(s, lambda: s.read.parquet(src).filter(col("Query") == "ibraco"), {"all"})


def test_case_insensitive_column_names(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["qUeRy"], ["ImPrS"]))
    verify_index_usage(s, lambda: s.read.parquet(src).filter(col("QUERY") == "facebook")
                       .select("query", "IMPRS"), {"fIdx"})


def test_disabled_session_does_not_use_index(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["imprs"]))
    assert not Hyperspace.isEnabled(s)
    df = s.read.parquet(src).filter(col("Query") == "facebook").select("imprs")
    assert index_names_used(df) == set()
    Hyperspace.enable(s)
    Hyperspace.enable(s)  # idempotent
    assert Hyperspace.isEnabled(s)
    assert len([r for r in s.extra_optimizations if "Index" in type(r).__name__ or
                "Index" in getattr(r, "__name__", "")]) == 2
    Hyperspace.disable(s)
    assert not Hyperspace.isEnabled(s)


# ------------------------------------------------------------------------------------------------
# JoinIndexRule
# ------------------------------------------------------------------------------------------------
def test_join_index_removes_exchange_and_sort(env):
    s, hs, src = env
    df = s.read.parquet(src)
    hs.createIndex(df, IndexConfig("jIdx", ["RGUID"], ["clicks"]))

    def q():
        a = s.read.parquet(src)
        b = s.read.parquet(src)
        return a.join(b, a["RGUID"] == b["RGUID"]).select(a["RGUID"], a["clicks"], b["clicks"])
    s.disableHyperspace()
    base = q()
    # a self-join: Spark's ReuseExchange turns the second exchange into a ReusedExchange
    assert count_nodes(base, X.ShuffleExchangeExec) == 1
    assert count_nodes(base, X.ReusedExchangeExec) == 1
    assert count_nodes(base, X.SortExec) == 2
    out = verify_index_usage(s, q, {"jIdx"})
    assert count_nodes(out, X.ShuffleExchangeExec) == 0
    assert count_nodes(out, X.SortExec) == 0
    assert all(sc.use_bucketing for sc in scans(out))


def test_join_two_different_tables(env, tmp_path):
    s, hs, src = env
    dept = pa.table({"deptId": pa.array([1, 2, 3], pa.int32()),
                     "deptName": ["Sales", "R&D", "Ops"]})
    emp = pa.table({"empId": pa.array(list(range(10)), pa.int32()),
                    "empName": [f"e{i}" for i in range(10)],
                    "deptId": pa.array([1, 2, 3, 1, 2, 3, 1, 2, 4, 1], pa.int32())})
    write_parquet_parts(dept, str(tmp_path / "dept"), 1)
    write_parquet_parts(emp, str(tmp_path / "emp"), 3)
    hs.createIndex(s.read.parquet(str(tmp_path / "emp")), IndexConfig("empIdx", ["deptId"], ["empName"]))
    hs.createIndex(s.read.parquet(str(tmp_path / "dept")), IndexConfig("deptIdx", ["deptId"], ["deptName"]))

    def q():
        e = s.read.parquet(str(tmp_path / "emp"))
        d = s.read.parquet(str(tmp_path / "dept"))
        return e.join(d, e["deptId"] == d["deptId"]).select(e["empName"], d["deptName"])
    out = verify_index_usage(s, q, {"empIdx", "deptIdx"})
    assert len(out.collect()) == 9
    assert count_nodes(out, X.ShuffleExchangeExec) == 0


def test_join_index_not_used_when_indexed_cols_differ_from_keys(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("two", ["RGUID", "Query"], ["clicks"]))
    Hyperspace.enable(s)
    a = s.read.parquet(src)
    b = s.read.parquet(src)
    df = a.join(b, a["RGUID"] == b["RGUID"]).select(a["clicks"], b["clicks"])
    # JoinIndexRule does not fire (no bucketed scans, shuffles remain).  The inferred
    # isnotnull(RGUID) filters may still pick the index through FilterIndexRule, as in Spark.
    assert not any(sc.use_bucketing for sc in scans(df))
    assert count_nodes(df, X.ShuffleExchangeExec) + count_nodes(df, X.ReusedExchangeExec) == 2


def test_join_multi_column_keys(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("two", ["RGUID", "Query"], ["clicks"]))

    def q():
        a = s.read.parquet(src)
        b = s.read.parquet(src)
        return a.join(b, (a["RGUID"] == b["RGUID"]) & (a["Query"] == b["Query"])) \
            .select(a["clicks"], b["clicks"])
    verify_index_usage(s, q, {"two"})

    # order-incompatible mapping: (RGUID=Query', Query=RGUID') must not use the index
    Hyperspace.enable(s)
    a = s.read.parquet(src)
    b = s.read.parquet(src)
    df = a.join(b, (a["RGUID"] == b["Query"]) & (a["Query"] == b["RGUID"])).select(a["clicks"])
    assert not any(sc.use_bucketing for sc in scans(df))
    assert count_nodes(df, X.ShuffleExchangeExec) + count_nodes(df, X.ReusedExchangeExec) == 2


def test_join_with_filters_on_both_sides(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("jIdx", ["RGUID"], ["clicks", "Query"]))

    def q():
        a = s.read.parquet(src).filter(col("clicks") > 20)
        b = s.read.parquet(src).filter(col("Query") != "donde")
        return a.join(b, a["RGUID"] == b["RGUID"]).select(a["clicks"], b["Query"])
    verify_index_usage(s, q, {"jIdx"})


def test_join_aliased_condition_not_rewritten(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("jIdx", ["RGUID"], ["clicks"]))
    Hyperspace.enable(s)
    a = s.read.parquet(src).select("RGUID", "clicks")
    b = s.read.parquet(src).select("RGUID", "clicks").toDF("g", "c")
    df = a.join(b, col("RGUID") == col("g"))
    assert index_names_used(df) == set()
    assert len(df.collect()) == 18


def test_join_rule_applies_before_filter_rule(env):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("jIdx", ["RGUID"], ["clicks", "Query"]))
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["RGUID", "clicks"]))

    def q():
        a = s.read.parquet(src).filter(col("Query") == "facebook")
        b = s.read.parquet(src)
        return a.join(b, a["RGUID"] == b["RGUID"]).select(a["clicks"], b["clicks"])
    out = verify_index_usage(s, q, {"jIdx"})
    assert count_nodes(out, X.ShuffleExchangeExec) == 0


# ------------------------------------------------------------------------------------------------
# Other formats, partitioned data, staleness
# ------------------------------------------------------------------------------------------------
def test_csv_and_json_sources(env, tmp_path):
    s, hs, _ = env
    t = sample_table()
    os.makedirs(tmp_path / "csv")
    pacsv.write_csv(t, str(tmp_path / "csv" / "part-0.csv"))
    os.makedirs(tmp_path / "json")
    with open(tmp_path / "json" / "part-0.json", "w") as f:
        import json
        for r in t.to_pylist():
            f.write(json.dumps(r) + "\n")
    csv_df = s.read.option("header", "true").option("inferSchema", "true").csv(str(tmp_path / "csv"))
    hs.createIndex(csv_df, IndexConfig("csvIdx", ["Query"], ["clicks"]))
    verify_index_usage(s, lambda: s.read.option("header", "true").option("inferSchema", "true")
                       .csv(str(tmp_path / "csv")).filter(col("Query") == "donde")
                       .select("Query", "clicks"), {"csvIdx"})
    json_df = s.read.json(str(tmp_path / "json"))
    hs.createIndex(json_df, IndexConfig("jsonIdx", ["RGUID"], ["imprs"]))
    verify_index_usage(s, lambda: s.read.json(str(tmp_path / "json")).filter(col("RGUID") == "fd093f8a")
                       .select("RGUID", "imprs"), {"jsonIdx"})


def test_partitioned_source_with_lineage(tmp_path):
    s = make_session(tmp_path, spark__hyperspace__index__lineage__enabled="true")
    hs = Hyperspace(s)
    t = sample_table()
    for date in sorted(set(t.column("Date").to_pylist())):
        part = t.filter(pa.compute.equal(t.column("Date"), date)).drop(["Date"])
        write_parquet_parts(part, str(tmp_path / "pt" / f"Date={date}"), 1)
    df = s.read.parquet(str(tmp_path / "pt"))
    assert "Date" in df.columns
    hs.createIndex(df, IndexConfig("pIdx", ["Query"], ["clicks"]))
    entry = hs.index("pIdx").collect()[0]
    assert entry.hasLineage
    verify_index_usage(s, lambda: s.read.parquet(str(tmp_path / "pt")).filter(col("Query") == "facebook")
                       .select("Query", "clicks"), {"pIdx"})
    # index rows carry the partition column and the lineage column
    import pyarrow.parquet as pq
    idx_files = [f for f in scans(s.read.parquet(str(tmp_path / "pt")).filter(col("Query") == "facebook")
                                  .select("Query", "clicks"))[0].relation.location.all_files()]
    names = pq.read_schema(idx_files[0].path[len("file:"):]).names
    assert names == ["Query", "clicks", "Date", "_data_file_id"]


def test_stale_index_not_used_after_source_append(env, tmp_path):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["imprs"]))
    write_parquet_parts(sample_table().slice(0, 3), src, 1, prefix="extra")
    Hyperspace.enable(s)
    df = s.read.parquet(src).filter(col("Query") == "facebook").select("imprs")
    assert index_names_used(df) == set()
    hs.refreshIndex("fIdx", "full")
    df = s.read.parquet(src).filter(col("Query") == "facebook").select("imprs")
    assert index_names_used(df) == {"fIdx"}
    assert sorted(r.imprs for r in df.collect()) == [2, 2, 4, 7]


def test_index_not_used_for_non_parquet_relation_mismatch(env, tmp_path):
    """An index built on one directory is not used for a different directory."""
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["imprs"]))
    other = str(tmp_path / "other")
    write_parquet_parts(sample_table(), other, 2)
    Hyperspace.enable(s)
    df = s.read.parquet(other).filter(col("Query") == "facebook").select("imprs")
    assert index_names_used(df) == set()


def test_rule_errors_never_break_queries(env, monkeypatch):
    s, hs, src = env
    hs.createIndex(s.read.parquet(src), IndexConfig("fIdx", ["Query"], ["imprs"]))
    Hyperspace.enable(s)
    from hyperspace_amd.rules import rule_utils

    def boom(*a, **k):
        raise RuntimeError("boom")
    monkeypatch.setattr(rule_utils, "get_candidate_indexes", boom)
    df = s.read.parquet(src).filter(col("Query") == "facebook").select("imprs")
    assert sorted(r.imprs for r in df.collect()) == [2, 4, 7]
