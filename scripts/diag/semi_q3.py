"""Diagnose the 3-way Q3 semi-join chain on the GPU: device results with and without the
projection semi-join (``spark.hyperspace.mi.semiProject.enabled``) against pyarrow, and the
intermediate key sets (filtered orders behind the customer bitmap)."""
import datetime
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import pyarrow as pa  # noqa: E402
import pyarrow.compute as pc  # noqa: E402
import pyarrow.dataset as ds  # noqa: E402

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_  # noqa: E402
from hyperspace_amd.models import tpch  # noqa: E402
from hyperspace_amd.plan import physical as X  # noqa: E402


def main():
    tmp = tempfile.mkdtemp()
    data = os.path.join(tmp, "data")
    tpch.generate(data, 0.02, 4, workers=1)
    tpch.write_customers(data, 0.02, 2)
    s = Session(conf={"spark.hyperspace.system.path": os.path.join(tmp, "idx"),
                      "spark.hyperspace.index.numBuckets": "16",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.sql.shuffle.partitions": "8",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=os.path.join(tmp, "wh"))
    hs = Hyperspace(s)
    c = s.read.parquet(os.path.join(data, "customer"))
    o = s.read.parquet(os.path.join(data, "orders"))
    li = s.read.parquet(os.path.join(data, "lineitem"))
    hs.createIndex(c, IndexConfig("cust", ["c_custkey"], ["c_mktsegment"]))
    hs.createIndex(o, IndexConfig("ord_cust", ["o_custkey"],
                                  ["o_orderkey", "o_orderdate", "o_shippriority"]))
    hs.createIndex(li, IndexConfig("li_ok", ["l_orderkey"],
                                   ["l_extendedprice", "l_discount", "l_shipdate"]))
    Hyperspace.enable(s)
    seg, d = "BUILDING", datetime.date(1995, 3, 1)
    ct = ds.dataset(os.path.join(data, "customer")).to_table()
    ot = ds.dataset(os.path.join(data, "orders")).to_table()
    lt = ds.dataset(os.path.join(data, "lineitem")).to_table()
    cs = ct.filter(pc.equal(ct["c_mktsegment"], seg))["c_custkey"]
    ox = ot.filter(pc.and_(pc.less(ot["o_orderdate"], pa.scalar(d)),
                           pc.is_in(ot["o_custkey"], value_set=cs)))
    lx = lt.filter(pc.and_(pc.greater(lt["l_shipdate"], pa.scalar(d)),
                           pc.is_in(lt["l_orderkey"], value_set=ox["o_orderkey"])))
    print("expected customers", len(cs), "orders", ox.num_rows, "lines", lx.num_rows, flush=True)
    co = c.join(o, c["c_custkey"] == o["o_custkey"]) \
        .filter((col("c_mktsegment") == seg) & (col("o_orderdate") < d))
    q = co.join(li, co["o_orderkey"] == li["l_orderkey"]).filter(col("l_shipdate") > d) \
        .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue"),
             count("*").alias("lines"))
    for flag in ("false", "true"):
        s.conf.set("spark.hyperspace.mi.semiProject.enabled", flag)
        r = q.collect()
        be = s.backend()
        print("semiProject", flag, "->", r, be.last_path, be.last_semi_join, flush=True)
    # the inner projection's relation: orders behind the customer bitmap
    plan = q.queryExecution.executed_plan
    projs = plan.collect(lambda x: isinstance(x, X.ProjectExec))
    be = s.backend()
    for p in projs:
        sj = be._semi_project(p)
        if sj is None:
            continue
        ok = [a for a in p.output if a.name == "o_orderkey"]
        if not ok:
            continue
        got = be._materialize(sj, ok)[ok[0].expr_id].data.cpu().numpy()
        exp = np.sort(ox["o_orderkey"].to_numpy())
        print("inner semi orders", len(got), "expected", len(exp),
              "missing", len(np.setdiff1d(exp, got)), "extra", len(np.setdiff1d(got, exp)),
              flush=True)
        node = p.child
        while isinstance(node, X.FilterExec):
            node = node.child
        cside = node.left
        from hyperspace_amd.exec.gpu import _strip_exchange
        crel = be._rel(_strip_exchange(cside) or cside)
        ck = node.left_keys[0]
        dk = np.sort(be._materialize(crel, [ck])[ck.expr_id].data.cpu().numpy())
        ek = np.sort(cs.to_numpy())
        print("customers device", len(dk), "expected", len(ek), "missing",
              len(np.setdiff1d(ek, dk)), "extra", len(np.setdiff1d(dk, ek)), flush=True)
        # orders behind a bitmap of the device's own customer keys
        od = ot.filter(pc.and_(pc.less(ot["o_orderdate"], pa.scalar(d)),
                               pc.is_in(ot["o_custkey"], value_set=pa.array(dk))))
        print("orders for device customers", od.num_rows, "missing vs got",
              len(np.setdiff1d(np.sort(od["o_orderkey"].to_numpy()), got)), flush=True)
        print("crel conds", crel.conds, "dict", crel.col(
            [a for a in crel.attrs if a.name == "c_mktsegment"][0]).dictionary
            if any(a.name == "c_mktsegment" for a in crel.attrs) else None, flush=True)


if __name__ == "__main__":
    main()
