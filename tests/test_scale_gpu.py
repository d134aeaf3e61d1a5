"""The bench's own query shapes at a scale where the multi-tile / 200-bucket / multi-launch
branches run (the two-phase join test used 8 buckets and ~480k rows, and
the bench cross-checks only its first timed step).

TPC-H SF1 (6M lineitem rows, 1.5M orders) in 8 source files, 200 buckets, the bench's three
covering indexes; Q6, the Q3 join aggregate and Q3's full shape (3-column group, top 10) each
run over several literal vectors, submitted 4 deep through ``collect_async`` like the bench's
timed loop, and every result is compared with the host oracle (Hyperspace disabled, pyarrow
engine) - the reference's enabled-vs-disabled pattern (E2EHyperspaceRulesTest.scala:1004-1019).
"""
import datetime
import os

import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sf1(tmp_path_factory):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    from hyperspace_amd.models import tpch
    root = tmp_path_factory.mktemp("sf1")
    data = str(root / "tpch")
    tpch.generate(data, 1.0, 8, workers=8)
    s = Session(conf={"spark.hyperspace.system.path": str(root / "idx"),
                      "spark.hyperspace.index.numBuckets": "200",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.sql.shuffle.partitions": "200",
                      "spark.hyperspace.mi.execution.device": "gpu",
                      "spark.hyperspace.mi.joinIndex.enabled": "false"},
                warehouse_dir=str(root / "wh"))
    hs = Hyperspace(s)
    li = s.read.parquet(os.path.join(data, "lineitem"))
    od = s.read.parquet(os.path.join(data, "orders"))
    hs.createIndex(li, IndexConfig("li_shipdate", ["l_shipdate"],
                                   ["l_discount", "l_quantity", "l_extendedprice"]))
    hs.createIndex(li, IndexConfig("li_orderkey", ["l_orderkey"],
                                   ["l_extendedprice", "l_discount", "l_shipdate"]))
    hs.createIndex(od, IndexConfig("ord_orderkey", ["o_orderkey"],
                                   ["o_orderdate", "o_shippriority"]))
    Hyperspace.enable(s)
    return s, li, od


def _q6(li, i):
    year = 1993 + i % 5
    disc = 0.02 + (i % 8) * 0.01
    return li.filter((col("l_shipdate") >= datetime.date(year, 1, 1)) &
                     (col("l_shipdate") < datetime.date(year + 1, 1, 1)) &
                     (col("l_discount") >= round(disc - 0.01, 2)) &
                     (col("l_discount") <= round(disc + 0.01, 2)) &
                     (col("l_quantity") < 24 + i % 2)) \
        .agg(sum_(col("l_extendedprice") * col("l_discount")).alias("revenue"))


def _join(li, od, i):
    dd = datetime.date(1995, 3, 1) + datetime.timedelta(days=(i * 7) % 30)
    return li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
        .filter((col("o_orderdate") < dd) & (col("l_shipdate") > dd))


def _q3(li, od, i):
    return _join(li, od, i).groupBy("o_shippriority").agg(
        sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue"),
        count("*").alias("lines"))


def _q3_full(li, od, i):
    return _join(li, od, i).groupBy("l_orderkey", "o_orderdate", "o_shippriority") \
        .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue")) \
        .orderBy(col("revenue").desc(), col("o_orderdate")).limit(10)


def _rows(rows):
    return sorted(tuple(r) for r in rows)


def _same(got, want, ordered=False):
    g, w = (list(map(tuple, got)), list(map(tuple, want))) if ordered else \
        (_rows(got), _rows(want))
    assert len(g) == len(w), (len(g), len(w))
    for a, b in zip(g, w):
        for x, y in zip(a, b):
            if isinstance(x, float):
                assert abs(x - y) <= 1e-9 * max(1.0, abs(y)), (a, b)
            else:
                assert x == y, (a, b)


def test_bench_shapes_pipelined_match_host_oracle(sf1):
    s, li, od = sf1
    backend = s.backend()
    idx = [0, 3, 5, 11]
    futs = []
    got = {}
    for i in idx:        # 4 steps in flight, as the bench's timed loop
        futs.append((i, _q6(li, i).collect_async(), _q3(li, od, i).collect_async()))
    for i, f6, f3 in futs:
        got[i] = (f6.result(), f3.result())
        assert f6.path == "native" and f3.path == "native", (f6.reason, f3.reason)
    full = {}
    for i in idx[:2]:
        full[i] = _q3_full(li, od, i).collect()
        assert backend.last_path == "native", backend.fallback_reason
    s.disableHyperspace()
    s.conf.set("spark.hyperspace.mi.execution.device", "cpu")
    try:
        for i in idx:
            _same(got[i][0], _q6(li, i).collect())
            _same(got[i][1], _q3(li, od, i).collect())
        for i in idx[:2]:
            _same(full[i], _q3_full(li, od, i).collect(), ordered=True)
    finally:
        s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
        s.enableHyperspace()
