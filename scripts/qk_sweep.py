#!/usr/bin/env python
"""Query-kernel sweep on the bench's SF-shaped data and indexes, in one process.

Builds the bench's three covering indexes once (reusing the generated TPC-H data under
``--data-dir``), then for every configuration (a JSON dict of ``exec.jit`` module knobs, e.g.
``{"JI_VEC": 16}``) drops the generated-kernel and captured-graph caches and times Q6 (indexed
filter), Q3 (join index) and optionally Q3 via the merge-join kernel.  Per query kind it prints
the wall latency of a synchronous ``collect()`` and the per-stage device times (HS_PROFILE
stage events).  One JSON line per configuration on stdout.

    python scripts/qk_sweep.py --sf 100 --configs '[{}, {"JI_VEC": 16}]'
"""
import argparse
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT = [{}, {"VEC_PREFETCH": False}, {"WAVE_SYNC": False},
           {"VEC_PREFETCH": False, "WAVE_SYNC": False},
           {"JI_VEC": 16}, {"SCAN_VEC": 16}, {"JI_VEC": 16, "SCAN_VEC": 16},
           {"SCAN_GRID": 4096}, {"SCAN_GRID": 16384}, {"JI_VEC": 32, "SCAN_VEC": 32}]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sf", type=float, default=100)
    ap.add_argument("--buckets", type=int, default=200)
    ap.add_argument("--data-dir", default=os.environ.get("HS_BENCH_DIR", "/tmp/hs_bench"))
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--configs", default=None)
    ap.add_argument("--merge-join", action="store_true")
    ap.add_argument("--q3-full", action="store_true",
                    help="also time TPC-H Q3's full shape (3-column group + top 10) via the "
                         "merge join and the device hash aggregate")
    ap.add_argument("--only-q3-full", action="store_true")
    ap.add_argument("--only-merge", action="store_true",
                    help="time only Q3 through the merge-join kernel")
    ap.add_argument("--show-compact", action="store_true",
                    help="print every resident column's compact HBM encoding after the runs")
    ap.add_argument("--decompose", action="store_true",
                    help="also time Q3 variants without the right predicate / aggregate tail")
    ap.add_argument("--no-profile", action="store_true",
                    help="wall times without the per-stage tracer (its HIP events cost time)")
    ap.add_argument("--cprofile", type=int, default=0,
                    help="also run N queries of each kind under cProfile (top functions to "
                         "stderr)")
    args = ap.parse_args()
    if not args.no_profile:
        os.environ["HS_PROFILE"] = "1"
    # heartbeat: long silent phases (data load under a profiler) must still show progress
    import threading
    t_start = time.time()

    def beat():
        while True:
            time.sleep(30)
            print(f"[qk_sweep] alive {time.time() - t_start:.0f}s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()
    import torch
    from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_
    from hyperspace_amd.exec import jit
    from hyperspace_amd.models import tpch
    from hyperspace_amd.utils.tracing import TRACER
    torch.cuda.set_device(0)
    sf = args.sf
    nfiles = max(8, int(round(sf * 1.28)))
    data = os.path.join(args.data_dir, f"tpch_sf{sf:g}_f{nfiles}")
    tpch.generate(data, sf, nfiles, workers=16)
    idx_root = os.path.join(args.data_dir, f"sweep_indexes_sf{sf:g}_b{args.buckets}")
    fresh = not os.path.exists(idx_root)
    s = Session(conf={"spark.hyperspace.system.path": idx_root,
                      "spark.hyperspace.index.numBuckets": str(args.buckets),
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=os.path.join(args.data_dir, "wh"))
    # extra session conf for sweeps: HS_BENCH_CONF="key=value,key=value" (as bench.py)
    for kv in filter(None, os.environ.get("HS_BENCH_CONF", "").split(",")):
        k, v = kv.split("=", 1)
        s.conf.set(k.strip(), v.strip())
    hs = Hyperspace(s)
    li = s.read.parquet(os.path.join(data, "lineitem"))
    od = s.read.parquet(os.path.join(data, "orders"))
    if fresh:
        hs.createIndex(li, IndexConfig("li_shipdate", ["l_shipdate"],
                                       ["l_discount", "l_quantity", "l_extendedprice"]))
        hs.createIndex(li, IndexConfig("li_orderkey", ["l_orderkey"],
                                       ["l_extendedprice", "l_discount", "l_shipdate"]))
        hs.createIndex(od, IndexConfig("ord_orderkey", ["o_orderkey"],
                                       ["o_orderdate", "o_shippriority"]))
    Hyperspace.enable(s)
    backend = s.backend()

    def q6(i):
        year = 1993 + i % 5
        disc = 0.02 + (i % 8) * 0.01
        lo, hi = datetime.date(year, 1, 1), datetime.date(year + 1, 1, 1)
        return li.filter((col("l_shipdate") >= lo) & (col("l_shipdate") < hi) &
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

    def q3_left_count(i):      # phase 1 only: join index + left predicate, COUNT(*)
        dd = datetime.date(1995, 3, 1) + datetime.timedelta(days=(i * 7) % 30)
        return li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
            .filter(col("l_shipdate") > dd).agg(count("*").alias("lines"))

    def q3_count(i):           # phases 1 + 2: both predicates, COUNT(*)
        dd = datetime.date(1995, 3, 1) + datetime.timedelta(days=(i * 7) % 30)
        return li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
            .filter((col("o_orderdate") < dd) & (col("l_shipdate") > dd)) \
            .agg(count("*").alias("lines"))

    def q6_count(i):           # Q6 predicates, COUNT(*) (no aggregate gathers)
        year = 1993 + i % 5
        disc = 0.02 + (i % 8) * 0.01
        lo, hi = datetime.date(year, 1, 1), datetime.date(year + 1, 1, 1)
        return li.filter((col("l_shipdate") >= lo) & (col("l_shipdate") < hi) &
                         (col("l_discount") >= round(disc - 0.01, 2)) &
                         (col("l_discount") <= round(disc + 0.01, 2)) &
                         (col("l_quantity") < 24 + i % 2)).agg(count("*").alias("n"))

    def q3_full(i):
        dd = datetime.date(1995, 3, 1) + datetime.timedelta(days=(i * 7) % 30)
        j = li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
            .filter((col("o_orderdate") < dd) & (col("l_shipdate") > dd))
        return j.groupBy("l_orderkey", "o_orderdate", "o_shippriority") \
            .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue")) \
            .orderBy(col("revenue").desc(), col("o_orderdate")).limit(10)

    def timed(fn, reps):
        for i in range(3):
            fn(i).collect()
        torch.cuda.synchronize()
        TRACER.reset()
        t = time.perf_counter()
        res = None
        for i in range(reps):
            res = fn(i).collect()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t) / reps * 1e3
        rep = TRACER.report()
        stages = {k: round(v["device_ms"] / max(v["calls"], 1), 4) for k, v in rep.items()}
        host = {k: round(v["host_ms"] / max(v["calls"], 1), 4) for k, v in rep.items()}
        m = {k: v for k, v in backend.metrics.items() if k.startswith("run_topk")}
        if args.cprofile:
            import cProfile
            import io
            import pstats
            pr = cProfile.Profile()
            pr.enable()
            for i in range(args.cprofile):
                fn(i).collect()
            torch.cuda.synchronize()
            pr.disable()
            buf = io.StringIO()
            st = pstats.Stats(pr, stream=buf)
            st.sort_stats("tottime").print_stats(45)
            st.sort_stats("cumulative").print_stats(60)
            print(f"[qk_sweep] cProfile {fn.__name__} x{args.cprofile}\n{buf.getvalue()}",
                  file=sys.stderr, flush=True)
        return {"wall_ms": round(wall, 4), "stages": stages, "host_stages": host,
                "res": str(res)[:120], "metrics": m}

    if args.configs and args.configs.startswith("@"):   # @file: JSON list in a file
        with open(args.configs[1:]) as f:
            args.configs = f.read()
    configs = json.loads(args.configs) if args.configs else DEFAULT
    from hyperspace_amd.exec import kernel_config
    base = kernel_config.active()
    for cfg in configs:
        # a config names KernelConfig fields (upper- or lower-case): {"SCAN_VEC": 16}
        kernel_config.bind(base.replace(**{k.lower(): v for k, v in cfg.items()}))
        jit._KERNELS.clear()
        backend.graphs._lru.clear()
        backend.__dict__.pop("_agg_preps", None)   # prepared lowerings hold launchers
        backend._programs.clear()     # prepared re-submissions replay the previous kernels
        if args.only_merge:
            s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "false")
            out = {"cfg": cfg, "q3_merge": timed(q3, args.reps)}
            s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "true")
            print(json.dumps(out), flush=True)
            continue
        if args.only_q3_full:
            s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "false")
            out = {"cfg": cfg, "q3_full": timed(q3_full, args.reps)}
            s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "true")
            print(json.dumps(out), flush=True)
            continue
        out = {"cfg": cfg, "q6": timed(q6, args.reps), "q3": timed(q3, args.reps)}
        if args.q3_full:
            s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "false")
            out["q3_full"] = timed(q3_full, args.reps)
            s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "true")
        if args.decompose:
            for name, fn in (("q3_left_count", q3_left_count), ("q3_count", q3_count),
                             ("q6_count", q6_count)):
                out[name] = timed(fn, args.reps)
        if args.merge_join:
            s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "false")
            out["q3_merge"] = timed(q3, max(args.reps // 4, 3))
            s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "true")
        print(json.dumps(out), flush=True)
    if args.show_compact:
        for key, t in backend.cache._lru.items():
            for name, c in t.columns.items():
                comp = getattr(c, "compact", False)
                desc = "not computed" if comp is False else (
                    "none" if comp is None else f"w={comp.width} base={comp.base} scale={comp.scale}")
                print(json.dumps({"table": str(key[1]), "col": name, "dtype": str(c.data.dtype),
                                  "compact": desc}), flush=True)


if __name__ == "__main__":
    main()
