"""Host-side profile of single-query latency (TPC-H Q6 and the Q3-style join through the full
engine path, one query at a time): wall time per query with and without cProfile, and the
top functions by own time.  Run on a GPU box: ``python scripts/profile_q6.py --sf 1``."""
import argparse
import cProfile
import datetime
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=1.0)
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--data-dir", default="/tmp/hs_prof")
    args = ap.parse_args()
    import torch
    from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_
    from hyperspace_amd.models import tpch
    torch.cuda.set_device(0)
    data = os.path.join(args.data_dir, f"tpch_sf{args.sf:g}")
    tpch.generate(data, args.sf, 8)
    s = Session(conf={"spark.hyperspace.system.path": os.path.join(args.data_dir, "idx"),
                      "spark.hyperspace.index.numBuckets": "64",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.hyperspace.mi.execution.device": "gpu",
                      "spark.hyperspace.mi.joinIndex.enabled": "false"},
                warehouse_dir=os.path.join(args.data_dir, "wh"))
    hs = Hyperspace(s)
    li = s.read.parquet(os.path.join(data, "lineitem"))
    od = s.read.parquet(os.path.join(data, "orders"))
    for df, cfg in ((li, IndexConfig("li_shipdate", ["l_shipdate"],
                                     ["l_discount", "l_quantity", "l_extendedprice"])),
                    (li, IndexConfig("li_orderkey", ["l_orderkey"],
                                     ["l_extendedprice", "l_discount", "l_shipdate"])),
                    (od, IndexConfig("ord_orderkey", ["o_orderkey"],
                                     ["o_orderdate", "o_shippriority"]))):
        if not os.path.exists(os.path.join(args.data_dir, "idx", cfg.indexName)):
            hs.createIndex(df, cfg)
    Hyperspace.enable(s)
    li = s.read.parquet(os.path.join(data, "lineitem"))
    od = s.read.parquet(os.path.join(data, "orders"))

    def q6(i):
        year = 1993 + i % 5
        disc = 0.02 + (i % 8) * 0.01
        return li.filter((col("l_shipdate") >= datetime.date(year, 1, 1)) &
                         (col("l_shipdate") < datetime.date(year + 1, 1, 1)) &
                         (col("l_discount") >= round(disc - 0.01, 2)) &
                         (col("l_discount") <= round(disc + 0.01, 2)) &
                         (col("l_quantity") < 24 + i % 2)) \
            .agg(sum_(col("l_extendedprice") * col("l_discount")).alias("revenue"))

    def q3(i):
        dd = datetime.date(1995, 3, 1) + datetime.timedelta(days=(i * 7) % 30)
        j = li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
            .filter((col("o_orderdate") < dd) & (col("l_shipdate") > dd))
        return j.groupBy("o_shippriority").agg(
            sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue"),
            count("*").alias("lines"))

    for name, fn in (("q6", q6), ("q3", q3)):
        for i in range(20):
            fn(i).collect()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(args.n):
            fn(i).collect()
        el = (time.perf_counter() - t) / args.n
        # host part: build + plan + submit without waiting (the device runs behind)
        t = time.perf_counter()
        futs = [fn(i).collect_async() for i in range(200)]
        sub = (time.perf_counter() - t) / 200
        for f in futs:
            f.result()
        pr = cProfile.Profile()
        pr.enable()
        for i in range(args.n // 4):
            fn(i).collect()
        pr.disable()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(25)
        print(f"== {name}: latency {el * 1e3:.3f} ms, host submit {sub * 1e3:.3f} ms", flush=True)
        print(buf.getvalue(), flush=True)


if __name__ == "__main__":
    main()
