"""Semi-join through a key-domain bitmap (exec/gpu.py GpuBackend._semi_join_agg,
csrc/kernels/key_bitmap.hip): TPC-H Q3's three-way join (customer x orders) x lineitem, whose
second join is not index-rewritable (JoinIndexRule.scala:100-105,149-150), runs as a scan of the
lineitem index filtered by a bitmap of the (customer x orders) order keys.  Checked against the
host oracle; a build side with repeated keys takes the general join.  GPU-only."""
import datetime
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_
from hyperspace_amd.models import tpch

pytestmark = pytest.mark.gpu


@pytest.fixture
def q3data(tmp_path, device):
    data = tmp_path / "data"
    tpch.generate(str(data), 0.02, 4, workers=1)
    tpch.write_customers(str(data), 0.02, 2)
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "16",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.sql.shuffle.partitions": "8",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=str(tmp_path / "wh"))
    hs = Hyperspace(s)
    c = s.read.parquet(str(data / "customer"))
    o = s.read.parquet(str(data / "orders"))
    li = s.read.parquet(str(data / "lineitem"))
    hs.createIndex(c, IndexConfig("cust", ["c_custkey"], ["c_mktsegment"]))
    hs.createIndex(o, IndexConfig("ord_cust", ["o_custkey"],
                                  ["o_orderkey", "o_orderdate", "o_shippriority"]))
    hs.createIndex(li, IndexConfig("li_ok", ["l_orderkey"],
                                   ["l_extendedprice", "l_discount", "l_shipdate"]))
    Hyperspace.enable(s)
    return s, c, o, li


def _q3(c, o, li, seg, d):
    co = c.join(o, c["c_custkey"] == o["o_custkey"]) \
        .filter((col("c_mktsegment") == seg) & (col("o_orderdate") < d))
    return co.join(li, co["o_orderkey"] == li["l_orderkey"]).filter(col("l_shipdate") > d) \
        .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue"),
             count("*").alias("lines"))


def _run(s, df):
    s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
    g = df.to_arrow().to_pylist()
    be = s.backend()
    path = be.last_path
    s.conf.set("spark.hyperspace.mi.execution.device", "cpu")
    c = df.to_arrow().to_pylist()
    s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
    return g, c, path, be


def test_three_way_q3_semi_join_bitmap(q3data):
    s, c, o, li = q3data
    for i, seg in enumerate(["BUILDING", "MACHINERY", "HOUSEHOLD"]):
        d = datetime.date(1995, 3, 1) + datetime.timedelta(days=7 * i)
        q = _q3(c, o, li, seg, d)
        g, h, path, be = _run(s, q)
        assert path == "native", be.fallback_reason
        assert be.last_semi_join["build_keys"] > 0
        # the lineitem index is sorted by l_orderkey: one bitmap test per key run
        assert be.last_semi_join["probe"] == "runs"
        assert g[0]["lines"] == h[0]["lines"] > 0
        h0 = h
        assert abs(g[0]["revenue"] - h[0]["revenue"]) <= 1e-9 * abs(h[0]["revenue"])
        # grouped over a probe-side column as well
        s.backend().last_semi_join = None
        qg = c.join(o, c["c_custkey"] == o["o_custkey"]) \
            .filter((col("c_mktsegment") == seg) & (col("o_orderdate") < d)) \
            .join(li, o["o_orderkey"] == li["l_orderkey"]) \
            .groupBy(li["l_discount"]).agg(count("*").alias("n"))
        g, h, path, be = _run(s, qg)
        assert path == "native", be.fallback_reason
        assert be.last_semi_join is not None
        assert sorted(map(tuple, (r.values() for r in g))) == \
            sorted(map(tuple, (r.values() for r in h)))
        # the per-row bitmap scan agrees with the run form
        s.conf.set("spark.hyperspace.mi.semiRuns.enabled", "false")
        try:
            g2, _, path2, be = _run(s, q)
            assert path2 == "native" and be.last_semi_join["probe"] == "scan"
            assert g2[0]["lines"] == h0[0]["lines"]
            assert abs(g2[0]["revenue"] - h0[0]["revenue"]) <= 1e-9 * abs(h0[0]["revenue"])
        finally:
            s.conf.set("spark.hyperspace.mi.semiRuns.enabled", "true")


def test_repeated_build_keys_take_the_general_join(q3data, tmp_path):
    """Build keys that repeat (a join side that is not unique on the key) would be counted
    once by a bitmap: the executor detects the duplicate bits and runs the general join."""
    s, c, o, li = q3data
    s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
    dup = tmp_path / "dup"
    os.makedirs(dup)
    keys = np.repeat(np.arange(1, 2000, dtype=np.int64) * 32 + 1, 2)     # every key twice
    pq.write_table(pa.table({"k": keys, "x": np.arange(len(keys), dtype=np.int64)}),
                   dup / "part-0.parquet")
    t = s.read.parquet(str(dup))
    q = t.filter(col("x") >= 0).join(li, t["k"] == li["l_orderkey"]) \
        .agg(count("*").alias("n"), sum_(col("l_discount")).alias("d"))
    g, h, path, be = _run(s, q)
    assert g[0]["n"] == h[0]["n"]
    assert abs(g[0]["d"] - h[0]["d"]) <= 1e-9 * max(1.0, abs(h[0]["d"]))


def test_three_way_q3_co_partitioned_with_orders_key_index(q3data):
    """With an orders index bucketed by o_orderkey like the lineitem index (same bucket count,
    same source files, covering the orders side's columns), the (customer x orders) build
    becomes right-side predicates of a co-partitioned lineitem x orders merge join: the
    orders filters plus o_custkey in a bitmap of the customer keys (_copart_semi)."""
    s, c, o, li = q3data
    hs = Hyperspace(s)
    hs.createIndex(o, IndexConfig("ord_ok", ["o_orderkey"], ["o_custkey", "o_orderdate"]))
    for i, seg in enumerate(["BUILDING", "FURNITURE"]):
        d = datetime.date(1995, 3, 1) + datetime.timedelta(days=11 * i)
        q = _q3(c, o, li, seg, d)
        g, h, path, be = _run(s, q)
        assert path == "native", be.fallback_reason
        assert be.last_semi_join["probe"] == "copart" and be.last_semi_join["index"] == "ord_ok"
        assert g[0]["lines"] == h[0]["lines"] > 0
        assert abs(g[0]["revenue"] - h[0]["revenue"]) <= 1e-9 * abs(h[0]["revenue"])
        # grouped by a lineitem column
        qg = c.join(o, c["c_custkey"] == o["o_custkey"]) \
            .filter((col("c_mktsegment") == seg) & (col("o_orderdate") < d)) \
            .join(li, o["o_orderkey"] == li["l_orderkey"]) \
            .groupBy(li["l_discount"]).agg(count("*").alias("n"))
        g, h, path, be = _run(s, qg)
        assert path == "native" and be.last_semi_join["probe"] == "copart"
        assert sorted(map(tuple, (r.values() for r in g))) == \
            sorted(map(tuple, (r.values() for r in h)))
    # switched off: the orders-key bitmap path
    s.conf.set("spark.hyperspace.mi.coPartitionedSemiJoin.enabled", "false")
    try:
        g, h, path, be = _run(s, _q3(c, o, li, "BUILDING", datetime.date(1995, 3, 1)))
        assert path == "native" and be.last_semi_join["probe"] == "runs"
        assert g[0]["lines"] == h[0]["lines"]
    finally:
        s.conf.set("spark.hyperspace.mi.coPartitionedSemiJoin.enabled", "true")
