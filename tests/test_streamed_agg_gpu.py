"""Bucket-range streaming (exec/gpu.py GpuBackend._stream_chunks / _streamed_agg): when the
indexes a query aggregates over do not fit ``spark.hyperspace.mi.deviceCacheBytes``, the query
runs natively as one pass per bucket range, and its result equals the unbounded (one resident
pass) run and the host oracle.  Q6 (scan), Q3 (co-partitioned join through two indexes) and a
date-grouped scan.  Reference: BucketUnionExec.scala:61-74 runs bucketed plans partition by
partition.  A row-producing filter streams too.  GPU-only."""
import datetime
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, max_, min_, sum_

pytestmark = pytest.mark.gpu

BUDGET = "spark.hyperspace.mi.deviceCacheBytes"


@pytest.fixture
def env(tmp_path, device):
    rng = np.random.default_rng(9)
    n_ord = 30_000
    okeys = rng.permutation(np.arange(1, n_ord + 1, dtype=np.int64) * 4)
    od = pa.table({"o_orderkey": okeys,
                   "o_orderdate": pa.array(rng.integers(8000, 10500, n_ord).astype(np.int32))
                   .view(pa.date32()),
                   "o_shippriority": rng.integers(0, 3, n_ord).astype(np.int32)})
    lk = np.repeat(okeys, rng.integers(1, 8, n_ord))
    n = len(lk)
    li = pa.table({"l_orderkey": lk,
                   "l_quantity": rng.integers(1, 51, n).astype(np.float64),
                   "l_extendedprice": np.round(rng.random(n) * 1e5, 2),
                   "l_discount": rng.integers(0, 11, n) / 100.0,
                   "l_shipdate": pa.array(rng.integers(8000, 10600, n).astype(np.int32))
                   .view(pa.date32())})
    for name, t in (("lineitem", li), ("orders", od)):
        os.makedirs(tmp_path / name)
        pq.write_table(t, tmp_path / name / "part-0.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "16",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=str(tmp_path / "wh"))
    hs = Hyperspace(s)
    lidf = s.read.parquet(str(tmp_path / "lineitem"))
    oddf = s.read.parquet(str(tmp_path / "orders"))
    hs.createIndex(lidf, IndexConfig("li_ship", ["l_shipdate"],
                                     ["l_discount", "l_quantity", "l_extendedprice"]))
    hs.createIndex(lidf, IndexConfig("li_ok", ["l_orderkey"],
                                     ["l_extendedprice", "l_discount", "l_shipdate"]))
    hs.createIndex(oddf, IndexConfig("od_ok", ["o_orderkey"], ["o_orderdate", "o_shippriority"]))
    Hyperspace.enable(s)
    return s, lidf, oddf


def _queries(li, od):
    dd = datetime.date(1995, 3, 15)
    return {
        "q6": li.filter((col("l_shipdate") >= datetime.date(1994, 1, 1)) &
                        (col("l_shipdate") < datetime.date(1995, 1, 1)) &
                        (col("l_discount") >= 0.05) & (col("l_quantity") < 24))
        .agg(sum_(col("l_extendedprice") * col("l_discount")).alias("r"), count("*").alias("n")),
        "q3": li.join(od, li["l_orderkey"] == od["o_orderkey"])
        .filter((col("o_orderdate") < dd) & (col("l_shipdate") > dd))
        .groupBy("o_shippriority")
        .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("rev"),
             count("*").alias("n"), min_(col("l_discount")).alias("dmin")),
        "rows": li.filter(col("l_orderkey") < 4000)
        .select("l_orderkey", "l_extendedprice", "l_shipdate"),
        "by_day": li.filter(col("l_shipdate") < datetime.date(1993, 1, 1))
        .groupBy("l_shipdate")
        .agg(count("*").alias("n"), max_(col("l_extendedprice")).alias("mx")),
    }


def _norm(rows):
    return sorted(tuple(r) for r in rows)


def _close(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            if isinstance(v, float):
                assert abs(u - v) <= 1e-9 * max(1.0, abs(v)), (x, y)
            else:
                assert u == v, (x, y)


def test_streamed_aggregates_match_unbounded(env):
    s, li, od = env
    qs = _queries(li, od)
    be = s.backend()
    unbounded = {}
    for k, q in qs.items():
        unbounded[k] = _norm(q.collect())
        assert be.last_path == "native", (k, be.fallback_reason)
        assert be.last_stream_passes == 0
    s.conf.set(BUDGET, str(64 * 1024))          # far below the indexes' decoded size
    try:
        for k, q in qs.items():
            got = _norm(q.collect())
            assert be.last_path == "native", (k, be.fallback_reason)
            assert be.last_stream_passes > 1, k
            _close(got, unbounded[k])
    finally:
        s.conf.unset(BUDGET)
    s.conf.set("spark.hyperspace.mi.execution.device", "cpu")
    try:
        for k, q in qs.items():
            _close(unbounded[k], _norm(q.collect()))
    finally:
        s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
