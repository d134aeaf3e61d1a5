"""Plan shapes the Hyperspace rules produce that used to fall back to the host engine, now run on
the MI355X executor (VERDICT r4 "missing" #3), each asserted native against the host oracle:

* multi-key joins whose keys include a string column (union-dictionary codes, then packed);
* multi-key joins over a Hybrid Scan BucketUnion (packed per part);
* left / right / full outer, left semi and left anti joins over a BucketUnion (per part pair,
  match marks OR-ed over the other side's parts);
* GROUP BY an unnamed expression (SQL ``GROUP BY c % 3``);
* row ORDER BY over unsorted input (device radix sort; the row order itself is checked).

Reference: JoinIndexRule.scala:57-58,118-124 (any join type, any number of EqualTo
conjuncts), RuleUtils.scala:439-441 (BucketUnion under the join)."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_

from test_gpu_e2e import _both, _close, tpch  # noqa: F401

pytestmark = pytest.mark.gpu


def _table(rows):
    return pa.Table.from_pylist(sorted((r.asDict() for r in rows),
                                       key=lambda d: tuple((v is None, str(v)) for v in d.values())))


@pytest.fixture
def skeys(tmp_path, device):
    """Two tables joined on (region string, k int)."""
    rng = np.random.default_rng(11)
    regions = np.array([f"R{i:02d}" for i in range(12)])
    n1, n2 = 60_000, 9_000
    a = pa.table({"region": pa.array(regions[rng.integers(0, 12, n1)]),
                  "k": rng.integers(0, 700, n1).astype(np.int64),
                  "v": np.round(rng.random(n1) * 100, 3)})
    b = pa.table({"region": pa.array(regions[rng.integers(0, 10, n2)]),
                  "k": rng.integers(0, 800, n2).astype(np.int64),
                  "w": rng.integers(0, 50, n2).astype(np.int32)})
    for name, t in (("a", a), ("b", b)):
        os.makedirs(tmp_path / name)
        half = t.num_rows // 2
        pq.write_table(t.slice(0, half), tmp_path / name / "p0.parquet")
        pq.write_table(t.slice(half), tmp_path / name / "p1.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "8",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=str(tmp_path / "wh"))
    return s, str(tmp_path / "a"), str(tmp_path / "b")


def test_multi_key_join_with_string_key_native(skeys):
    s, ap, bp = skeys
    hs = Hyperspace(s)
    a, b = s.read.parquet(ap), s.read.parquet(bp)
    hs.createIndex(a, IndexConfig("a_rk", ["region", "k"], ["v"]))
    hs.createIndex(b, IndexConfig("b_rk", ["region", "k"], ["w"]))
    Hyperspace.enable(s)
    cond = (a["region"] == b["region"]) & (a["k"] == b["k"])
    q_agg = a.join(b, cond).filter("w < 30").agg(sum_("v").alias("sv"), count("*").alias("n"))
    q_rows = a.join(b, cond).filter("v > 90").select(a["region"], a["k"], "v", "w")
    for q, sort in ((q_agg, False), (q_rows, True)):
        assert "a_rk" in q.queryExecution.executed_plan.tree_string()
        g, c, path = _both(s, q, sort=sort)
        assert path == "native", s.backend().fallback_reason
        assert g.num_rows > 0
        _close(g, c)


def _hybrid(s, lpath, opath):
    for k, v in (("lineage.enabled", "true"), ("hybridscan.enabled", "true"),
                 ("hybridscan.maxAppendedRatio", "0.5"), ("hybridscan.maxDeletedRatio", "0.5")):
        s.conf.set(f"spark.hyperspace.index.{k}", v)
    hs = Hyperspace(s)
    li, od = s.read.parquet(lpath), s.read.parquet(opath)
    hs.createIndex(li, IndexConfig("li_ok", ["l_orderkey"], ["l_extendedprice", "l_discount",
                                                             "l_quantity"]))
    hs.createIndex(od, IndexConfig("ord_ok", ["o_orderkey"], ["o_orderdate", "o_shippriority"]))
    t_li = pq.read_table(os.path.join(lpath, "part-0.parquet")).slice(0, 15_000)
    t_od = pq.read_table(os.path.join(opath, "part-0.parquet")).slice(0, 3_000)
    shift = 10_000_000
    # new orders (fresh keys) plus appended lineitems of both new and existing orders
    t_od = t_od.set_column(0, "o_orderkey", pa.compute.add(t_od.column("o_orderkey"), shift))
    keys = t_li.column("l_orderkey").to_numpy()
    moved = np.where(np.arange(len(keys)) % 2 == 0, keys + shift, keys)
    t_li = t_li.set_column(0, "l_orderkey", pa.array(moved))
    pq.write_table(t_li, os.path.join(lpath, "part-app.parquet"))
    pq.write_table(t_od, os.path.join(opath, "part-app.parquet"))
    Hyperspace.enable(s)
    # per-part lowering (the merged-union fast path would hide the BucketUnion parts)
    s.conf.set("spark.hyperspace.mi.hybridMerge.enabled", "false")
    s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "false")
    return s.read.parquet(lpath), s.read.parquet(opath)


def test_outer_semi_anti_joins_over_bucket_union_native(tpch):  # noqa: F811
    s, lpath, opath = tpch
    li, od = _hybrid(s, lpath, opath)
    lf = li.filter("l_quantity < 10")
    of = od.filter("o_orderdate < DATE '1995-06-01'")
    for how in ("left", "right", "full", "leftsemi", "leftanti"):
        j = lf.join(of, lf["l_orderkey"] == of["o_orderkey"], how)
        rows = j.select(*(["l_orderkey", "l_extendedprice"] +
                          (["o_orderdate"] if how not in ("leftsemi", "leftanti") else [])))
        agg = j.agg(count("*").alias("n"), sum_("l_extendedprice").alias("p"))
        assert "BucketUnion" in agg.queryExecution.executed_plan.tree_string(), how
        for q, sort in ((agg, False), (rows, True)):
            g, c, path = _both(s, q, sort=sort)
            assert path == "native", (how, s.backend().fallback_reason)
            _close(g, c)


def test_multi_key_join_over_bucket_union_native(skeys):
    """Hybrid Scan on both sides of a (string, int) two-key join: appended files make each side
    a BucketUnion of the index and the shuffled appended rows."""
    s, ap, bp = skeys
    for k, v in (("lineage.enabled", "true"), ("hybridscan.enabled", "true"),
                 ("hybridscan.maxAppendedRatio", "0.9"), ("hybridscan.maxDeletedRatio", "0.5")):
        s.conf.set(f"spark.hyperspace.index.{k}", v)
    hs = Hyperspace(s)
    a, b = s.read.parquet(ap), s.read.parquet(bp)
    hs.createIndex(a, IndexConfig("a_rk", ["region", "k"], ["v"]))
    hs.createIndex(b, IndexConfig("b_rk", ["region", "k"], ["w"]))
    # appended rows with regions the index dictionaries have not seen
    rng = np.random.default_rng(5)
    na = pa.table({"region": pa.array([f"N{i % 3}" if i % 2 else f"R{i % 12:02d}"
                                       for i in range(4000)]),
                   "k": rng.integers(0, 700, 4000).astype(np.int64),
                   "v": np.round(rng.random(4000) * 100, 3)})
    nb = pa.table({"region": pa.array([f"N{i % 3}" for i in range(1500)]),
                   "k": rng.integers(0, 700, 1500).astype(np.int64),
                   "w": rng.integers(0, 50, 1500).astype(np.int32)})
    pq.write_table(na, os.path.join(ap, "app.parquet"))
    pq.write_table(nb, os.path.join(bp, "app.parquet"))
    Hyperspace.enable(s)
    s.conf.set("spark.hyperspace.mi.hybridMerge.enabled", "false")
    a, b = s.read.parquet(ap), s.read.parquet(bp)
    cond = (a["region"] == b["region"]) & (a["k"] == b["k"])
    for q, sort in ((a.join(b, cond).agg(count("*").alias("n"), sum_("v").alias("sv")), False),
                    (a.join(b, cond).filter("w > 40").select(a["region"], "v", "w"), True)):
        plan = q.queryExecution.executed_plan.tree_string()
        assert "BucketUnion" in plan and "a_rk" in plan, plan
        g, c, path = _both(s, q, sort=sort)
        assert path == "native", s.backend().fallback_reason
        _close(g, c)


def test_group_by_unnamed_expression_native(tpch):  # noqa: F811
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    hs.createIndex(li, IndexConfig("li_q", ["l_quantity"], ["l_discount", "l_extendedprice"]))
    Hyperspace.enable(s)
    li.createOrReplaceTempView("li")
    q = s.sql("SELECT l_quantity % 7 AS m, count(*) AS n, sum(l_extendedprice) AS p FROM li "
              "WHERE l_quantity > 5 GROUP BY l_quantity % 7")
    assert "li_q" in q.queryExecution.executed_plan.tree_string()
    g, c, path = _both(s, q)
    assert path == "native", s.backend().fallback_reason
    assert g.num_rows == 7
    _close(g, c)


def test_row_order_by_sorted_on_device(tpch):  # noqa: F811
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    hs.createIndex(li, IndexConfig("li_ship", ["l_shipdate"], ["l_discount", "l_quantity",
                                                               "l_extendedprice", "l_orderkey"]))
    Hyperspace.enable(s)
    f = li.filter("l_shipdate >= DATE '1994-01-01' AND l_shipdate < DATE '1994-03-01'")
    qs = [f.select("l_orderkey", "l_quantity", "l_extendedprice")
           .orderBy(col("l_quantity").desc(), col("l_extendedprice"), col("l_orderkey")),
          f.select("l_shipdate", "l_discount", "l_orderkey")
           .orderBy(col("l_discount"), col("l_shipdate").desc(), col("l_orderkey")).limit(500)]
    for q in qs:
        g, c, path = _both(s, q, sort=False)          # the row ORDER itself is compared
        assert path == "native", s.backend().fallback_reason
        assert g.num_rows > 100
        _close(g, c)
