"""Hash-mode GROUP BY on the device (exec/hash_agg.py + csrc/kernels/hash_agg.hip): multi-column,
high-cardinality (> 1M groups), float and string keys, ORDER BY ... LIMIT through the device
top-k, and TPC-H Q3's full shape (join + 3-column group + top 10).  Every query is checked
against the host oracle and must run native (no silent fallback)."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, avg, col, count, max_, min_, sum_

from test_gpu_e2e import _both, _close, tpch  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


def _native(s):
    b = s.backend()
    assert b.last_path == "native", b.fallback_reason


def test_multi_column_group_by_scan(tpch):  # noqa: F811
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    hs.createIndex(li, IndexConfig("li_ship", ["l_shipdate"],
                                   ["l_discount", "l_quantity", "l_returnflag", "l_orderkey"]))
    Hyperspace.enable(s)
    q = li.filter("l_shipdate >= DATE '1994-01-01'") \
        .groupBy("l_returnflag", "l_quantity").agg(sum_("l_discount").alias("d"),
                                                    count("*").alias("n"),
                                                    min_("l_discount").alias("mn"),
                                                    max_("l_shipdate").alias("mx"),
                                                    avg("l_quantity").alias("aq"))
    g, c, path = _both(s, q)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    # float group key (hash mode, raw float image)
    q2 = li.filter("l_shipdate < DATE '1993-01-01'").groupBy("l_quantity").agg(count("*").alias("c"))
    g, c, path = _both(s, q2)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    # high-cardinality single key + ORDER BY ... LIMIT (device top-k: > TOPK_MIN_GROUPS groups)
    q3 = li.filter("l_shipdate >= DATE '1992-01-01'").groupBy("l_orderkey") \
        .agg(sum_("l_quantity").alias("qty")).orderBy(col("qty").desc(), col("l_orderkey")).limit(7)
    g, c, path = _both(s, q3, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)


def test_tpch_q3_full_shape(tpch):  # noqa: F811
    """SELECT l_orderkey, sum(l_extendedprice * (1 - l_discount)) AS revenue, o_orderdate,
    o_shippriority ... GROUP BY l_orderkey, o_orderdate, o_shippriority
    ORDER BY revenue DESC, o_orderdate LIMIT 10 — over the co-located merge join."""
    s, lpath, opath = tpch
    hs = Hyperspace(s)
    li, od = s.read.parquet(lpath), s.read.parquet(opath)
    hs.createIndex(li, IndexConfig("li_ok", ["l_orderkey"], ["l_extendedprice", "l_discount",
                                                             "l_shipdate"]))
    hs.createIndex(od, IndexConfig("ord_ok", ["o_orderkey"], ["o_orderdate", "o_shippriority"]))
    Hyperspace.enable(s)
    s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "false")
    j = li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
        .filter("o_orderdate < DATE '1995-03-15' AND l_shipdate > DATE '1995-03-15'")
    q = j.groupBy("l_orderkey", "o_orderdate", "o_shippriority") \
        .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue")) \
        .orderBy(col("revenue").desc(), col("o_orderdate")).limit(10)
    from hyperspace_amd.exec import jit
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    assert g.num_rows == 10
    _close(g, c)
    # the (l_orderkey, o_orderdate, o_shippriority) groups reduce to l_orderkey's (o_orderkey is
    # unique): the run-keyed two-phase join aggregates into the hash table and the top groups'
    # orders columns are looked up afterwards
    assert jit.LAST_MJ_PATH[0] == "runs_hash"
    # whole keys went through the walk's per-wavefront top-K lists (hash_agg.TopKPlan) and the
    # table kept only keys split across walk windows; same rows as the table-only walk
    be = s.backend()
    assert be.metrics.get("run_topk") == 1
    s.conf.set("spark.hyperspace.mi.runTopK.enabled", "false")
    g1, _, path = _both(s, q, sort=False)
    s.conf.set("spark.hyperspace.mi.runTopK.enabled", "true")
    assert path == "native" and jit.LAST_MJ_PATH[0] == "runs_hash"
    _close(g1, c)
    _close(g1, g)
    # ascending order, a COUNT order key, and several literal vectors (a fresh walk each)
    for dd, asc in (("1995-03-02", True), ("1995-03-20", False), ("1994-11-30", True)):
        qa = li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
            .filter(f"o_orderdate < DATE '{dd}' AND l_shipdate > DATE '{dd}'") \
            .groupBy("l_orderkey", "o_orderdate", "o_shippriority") \
            .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue"),
                 count("*").alias("n")) \
            .orderBy(col("n").asc() if asc else col("revenue").desc(), col("l_orderkey")) \
            .limit(7)
        ga, ca, path = _both(s, qa, sort=False)
        assert path == "native", be.fallback_reason
        assert be.metrics.get("run_topk") in (0, 1)
        _close(ga, ca)
    s.conf.set("spark.hyperspace.mi.fdGroup.enabled", "false")
    g2, _, path = _both(s, q, sort=False)
    s.conf.set("spark.hyperspace.mi.fdGroup.enabled", "true")
    assert path == "native" and jit.LAST_MJ_PATH[0] == "hash"
    _close(g2, c)
    # without the LIMIT: every group comes back (multi-column packed key, no top-k)
    q_all = j.groupBy("l_orderkey", "o_orderdate", "o_shippriority") \
        .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue"),
             count("*").alias("n"))
    g, c, path = _both(s, q_all)
    assert path == "native", s.backend().fallback_reason
    assert g.num_rows > 1000
    _close(g, c)


def test_more_than_a_million_groups_and_overflow_retry(tmp_path, device):
    rng = np.random.default_rng(3)
    n = 2_600_000
    k = rng.integers(0, 1_300_000, n).astype(np.int64) * 7 + 11
    t = pa.table({"k": k, "v": rng.random(n), "w": rng.integers(0, 5, n).astype(np.int32)})
    os.makedirs(tmp_path / "t")
    pq.write_table(t.slice(0, n // 2), tmp_path / "t" / "part-0.parquet")
    pq.write_table(t.slice(n // 2), tmp_path / "t" / "part-1.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "8",
                      "spark.hyperspace.mi.execution.device": "gpu"})
    hs = Hyperspace(s)
    df = s.read.parquet(str(tmp_path / "t"))
    hs.createIndex(df, IndexConfig("ik", ["k"], ["v", "w"]))
    Hyperspace.enable(s)
    q = df.filter(col("k") >= 0).groupBy("k").agg(sum_("v").alias("sv"), count("*").alias("n"))
    be = s.backend()
    be.htables.sizes.clear()
    g, c, path = _both(s, q)
    assert path == "native", be.fallback_reason
    assert g.num_rows > 1_000_000
    _close(g, c)
    # a stale (too small) size guess overflows the probe budget; the query re-runs with a
    # larger table and stays exact
    for key in list(be.htables.sizes):
        be.htables.sizes[key] = 1 << 12
    g2, _, path = _both(s, q)
    assert path == "native"
    _close(g2, c)
    # two group columns, one from the index key
    q2 = df.filter(col("k") < 1_000_000).groupBy("w", "k").agg(max_("v").alias("mx"))
    g, c, path = _both(s, q2)
    assert path == "native", be.fallback_reason
    _close(g, c)


def test_dense_group_order_by_limit(tpch):  # noqa: F811
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    hs.createIndex(li, IndexConfig("li_ship2", ["l_shipdate"], ["l_quantity", "l_returnflag"]))
    Hyperspace.enable(s)
    q = li.filter("l_shipdate > DATE '1995-01-01'").groupBy("l_returnflag") \
        .agg(sum_("l_quantity").alias("q")).orderBy(col("q").desc()).limit(2)
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
