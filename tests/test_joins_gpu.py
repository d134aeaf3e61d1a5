"""Non-inner joins on the device: left / right / full outer, left semi and left anti over the
co-located bucketed join (JoinIndexRule fires for any join type, JoinIndexRule.scala:58), as
rows and under aggregates, checked against the host oracle with the native path asserted."""
import numpy as np
import pyarrow as pa
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, col, count, sum_

from test_gpu_e2e import _both, _close, tpch  # noqa: F401  (fixture)

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("how", ["left", "right", "full", "leftsemi", "leftanti"])
def test_outer_semi_anti_joins_native(tpch, how):  # noqa: F811
    s, lpath, opath = tpch
    hs = Hyperspace(s)
    li, od = s.read.parquet(lpath), s.read.parquet(opath)
    hs.createIndex(li, IndexConfig("li_ok", ["l_orderkey"], ["l_extendedprice", "l_shipdate"]))
    hs.createIndex(od, IndexConfig("ord_ok", ["o_orderkey"], ["o_orderdate", "o_shippriority"]))
    Hyperspace.enable(s)
    # filters below the join on both sides leave unmatched rows on each side
    lf = li.filter("l_shipdate > DATE '1995-06-01'")
    of = od.filter("o_orderdate < DATE '1995-03-15'")
    j = lf.join(of, lf["l_orderkey"] == of["o_orderkey"], how)
    if how in ("leftsemi", "leftanti"):
        rows = j.select("l_orderkey", "l_extendedprice")
    else:
        rows = j.select("l_orderkey", "l_extendedprice", "o_orderkey", "o_shippriority")
    g, c, path = _both(s, rows)
    assert path == "native", s.backend().fallback_reason
    assert g.num_rows > 0
    _close(g, c)
    # an aggregate over the join result (materialized join, then the device aggregate)
    agg = j.agg(count("*").alias("n"), sum_("l_extendedprice").alias("p"))
    g, c, path = _both(s, agg, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
