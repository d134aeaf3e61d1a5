"""SQL over temporary views and catalog tables (hyperspace_amd/plan/sql.py, catalog.py), with
the reference's disabled-vs-enabled oracle: ports of ``E2EHyperspaceRulesTest.scala:226-341``
(joins over temp views and managed tables use both indexes; alias columns in the join keep the
plan unchanged) and ``python/hyperspace/tests/test_indexutilization.py:42-57`` (a filter query
over a temp view is explained with the index)."""
import pyarrow as pa
import pytest

from hyperspace_amd import Hyperspace, IndexConfig
from hyperspace_amd.exceptions import HyperspaceException

from helpers import (index_names_used, make_session, sample_table, sorted_rows,
                     verify_index_usage, write_parquet_parts)


@pytest.fixture
def env(tmp_path):
    s = make_session(tmp_path)
    src = str(tmp_path / "sample")
    t = sample_table().rename_columns(["c1", "c2", "c3", "c4", "c5"])
    write_parquet_parts(t, src, parts=2)
    yield s, Hyperspace(s), src
    s.disableHyperspace()


def test_join_over_temp_views_uses_both_indexes(env):
    s, hs, src = env
    left, right = s.read.parquet(src), s.read.parquet(src)
    hs.createIndex(left, IndexConfig("leftIndex", ["c3"], ["c1"]))
    hs.createIndex(right, IndexConfig("rightIndex", ["c3"], ["c4"]))
    left.createOrReplaceTempView("t1")
    right.createOrReplaceTempView("t2")
    df = verify_index_usage(s, lambda: s.sql("SELECT t1.c1, t2.c4 FROM t1, t2 WHERE t1.c3 = t2.c3"),
                            {"leftIndex", "rightIndex"})
    assert df.columns == ["c1", "c4"]
    # explicit JOIN syntax and aliases plan the same join
    verify_index_usage(s, lambda: s.sql("SELECT a.c1, b.c4 FROM t1 AS a JOIN t2 b ON a.c3 = b.c3"),
                       {"leftIndex", "rightIndex"})


def test_join_over_managed_and_external_tables(env, tmp_path):
    s, hs, src = env
    orig = s.read.parquet(src)
    orig.select("c1", "c3").write.saveAsTable("t1")                             # managed
    orig.select("c3", "c4").write.option("path", str(tmp_path / "tables" / "t2")).saveAsTable("t2")
    assert s.catalog.tableExists("t1") and s.catalog.tableExists("T2")
    left, right = s.table("t1"), s.table("t2")
    hs.createIndex(left, IndexConfig("leftIndex", ["c3"], ["c1"]))
    hs.createIndex(right, IndexConfig("rightIndex", ["c3"], ["c4"]))
    verify_index_usage(s, lambda: s.sql("SELECT t1.c1, t2.c4 FROM t1, t2 WHERE t1.c3 = t2.c3"),
                       {"leftIndex", "rightIndex"})
    with pytest.raises(HyperspaceException):
        orig.write.saveAsTable("t1")                       # errorifexists
    orig.select("c1", "c3").write.mode("overwrite").saveAsTable("t1")
    # a new session over the same warehouse sees the tables (the catalog is persisted)
    s2 = make_session(tmp_path)
    assert sorted_rows(s2.table("t2")) == sorted_rows(s.table("t2"))
    assert s.catalog.dropTable("t1") and not s.catalog.tableExists("t1")


def test_alias_columns_in_join_keep_the_plan(env):
    """Join keys that are aliases of the indexed column are not rewritten (the reference's
    verifyNoChange: JoinIndexRule leaves the optimized plan as it is)."""
    s, hs, src = env
    left, right = s.read.parquet(src), s.read.parquet(src)
    hs.createIndex(left, IndexConfig("leftIndex", ["c3"], ["c1"]))
    hs.createIndex(right, IndexConfig("rightIndex", ["c3"], ["c4"]))
    left.createOrReplaceTempView("t1")
    right.createOrReplaceTempView("t2")
    q1 = "SELECT alias, c4 FROM t2, (SELECT c3 AS alias, c1 FROM t1) WHERE t2.c3 = alias"
    q2 = "SELECT alias, c4 FROM t2, (SELECT c3, c1 AS alias FROM t1) AS newt WHERE t2.c3 = newt.c3"
    for q in (q1, q2):
        s.disableHyperspace()
        want = sorted_rows(s.sql(q))
        s.enableHyperspace()
        df = s.sql(q)
        assert "leftIndex" not in index_names_used(df)
        assert sorted_rows(df) == want


def test_filter_over_temp_view_explained_with_index(env, capsys):
    s, hs, src = env
    df = s.read.parquet(src)
    hs.createIndex(df, IndexConfig("idx1", ["c5"], ["c3", "c4"]))
    df.createOrReplaceTempView("employees")
    q = s.sql("SELECT c5, c3, c4 FROM employees WHERE employees.c5 > 26")
    Hyperspace.enable(s)
    assert index_names_used(q) == {"idx1"}
    out = []
    hs.explain(q, False, out.append)
    assert "idx1" in out[0]


def test_sql_aggregates_order_limit_union(env):
    s, _, src = env
    t = s.read.parquet(src)
    t.createOrReplaceTempView("t")
    rows = s.sql("SELECT c3, count(*) AS n, sum(c5) AS clicks FROM t WHERE c4 > 0 "
                 "GROUP BY c3 HAVING count(*) > 1 ORDER BY clicks DESC, c3 LIMIT 3").collect()
    full = sample_table().to_pylist()
    agg = {}
    for r in full:
        if r["imprs"] > 0:
            a = agg.setdefault(r["Query"], [0, 0])
            a[0] += 1
            a[1] += r["clicks"]
    want = sorted(((q, n, c) for q, (n, c) in agg.items() if n > 1), key=lambda x: (-x[2], x[0]))[:3]
    assert [tuple(r) for r in rows] == want
    # ORDER BY an input column not selected; DISTINCT; UNION (distinct) vs UNION ALL
    r2 = s.sql("SELECT c3 FROM t ORDER BY c5 DESC LIMIT 2").collect()
    top = sorted(full, key=lambda r: -r["clicks"])[:2]
    assert [r[0] for r in r2] == [r["Query"] for r in top]
    d = s.sql("SELECT DISTINCT c3 FROM t").collect()
    assert sorted(r[0] for r in d) == sorted({r["Query"] for r in full})
    u = s.sql("SELECT c3 FROM t UNION SELECT c3 FROM t").collect()
    ua = s.sql("SELECT c3 FROM t UNION ALL SELECT c3 FROM t").collect()
    assert len(u) == len(d) and len(ua) == 2 * len(full)
    star = s.sql("SELECT * FROM t WHERE c5 >= 100")
    assert star.columns == ["c1", "c2", "c3", "c4", "c5"]
    with pytest.raises(HyperspaceException):
        s.sql("SELECT nope FROM t").collect()
    with pytest.raises(HyperspaceException):
        s.sql("SELECT c1 FROM missing_view")


def test_group_by_unnamed_expression(env):
    """``GROUP BY c5 % 7`` (no alias in the GROUP BY): the partial aggregate's attribute for the
    expression is made once, so the exchange above and the final aggregate read the same one."""
    s, _, src = env
    s.read.parquet(src).createOrReplaceTempView("t")
    rows = s.sql("SELECT c5 % 7 AS m, count(*) AS n, sum(c4) AS p FROM t WHERE c5 > 0 "
                 "GROUP BY c5 % 7").collect()
    want = {}
    for r in sample_table().to_pylist():
        if r["clicks"] > 0:
            a = want.setdefault(r["clicks"] % 7, [0, 0])
            a[0] += 1
            a[1] += r["imprs"]
    assert sorted(tuple(r) for r in rows) == sorted((k, n, p) for k, (n, p) in want.items())


def test_temp_view_lifecycle(env):
    s, _, src = env
    df = s.read.parquet(src)
    df.createTempView("v")
    with pytest.raises(HyperspaceException):
        df.createTempView("v")
    df.filter("c5 > 50").createOrReplaceTempView("v")
    assert len(s.sql("SELECT * FROM v").collect()) == len(df.filter("c5 > 50").collect())
    assert "v" in s.catalog.listTables()
    assert s.catalog.dropTempView("V")
    assert not s.catalog.tableExists("v")


def test_union_order_by_limit_apply_to_the_whole_union(env):
    """A trailing ORDER BY / LIMIT after a UNION chain orders and limits the union's rows (as in
    Spark), not the last branch; a parenthesized branch keeps its own ORDER BY / LIMIT."""
    s, _, src = env
    t = s.read.parquet(src)
    t.createOrReplaceTempView("t")
    full = sample_table().to_pylist()
    clicks = sorted((r["clicks"] for r in full), reverse=True)
    got = s.sql("SELECT c5 FROM t WHERE c5 < 300 UNION ALL SELECT c5 FROM t WHERE c5 >= 300 "
                "ORDER BY c5 DESC LIMIT 4").collect()
    assert [r[0] for r in got] == clicks[:4]
    inner = s.sql("SELECT c5 FROM t UNION ALL (SELECT c5 FROM t ORDER BY c5 LIMIT 1)").collect()
    assert len(inner) == len(full) + 1
    # only Spark's default null ordering is representable: a different one is refused, not lost
    assert s.sql("SELECT c5 FROM t ORDER BY c5 ASC NULLS FIRST LIMIT 1").collect()
    with pytest.raises(HyperspaceException):
        s.sql("SELECT c5 FROM t ORDER BY c5 ASC NULLS LAST")


def test_overwrite_of_a_table_read_by_the_written_data_is_refused(env):
    s, _, src = env
    s.read.parquet(src).select("c1", "c5").write.saveAsTable("t1")
    n = len(s.table("t1").collect())
    with pytest.raises(HyperspaceException):
        s.table("t1").filter("c5 > 0").write.mode("overwrite").saveAsTable("t1")
    assert len(s.table("t1").collect()) == n          # the table survived
    with pytest.raises(HyperspaceException):
        s.read.parquet(src).write.saveAsTable("../escape")
    with pytest.raises(HyperspaceException):
        s.catalog.dropTable("a/b")
    assert not s.catalog.tableExists("../escape")
