#!/usr/bin/env python
"""The BASELINE.json configurations next to the headline benchmark (``bench.py``).

    python benchmarks/configs.py --config csv10k            # CPU plumbing, no GPU
    python benchmarks/configs.py --config sf10_filter       # 1 MI355X
    python benchmarks/configs.py --config hybrid --sf 100   # SF100 index + 10% appended files
    python benchmarks/configs.py --config q3_3way --sf 100  # three-way join
    python benchmarks/configs.py --config all

One JSON line per configuration on stdout.  Every configuration checks its indexed results
against the same query with Hyperspace disabled (the reference's correctness oracle,
``E2EHyperspaceRulesTest.scala:1004-1019``) and reports which executor path ran.

* ``csv10k`` — 10k-row CSV covering index + equality lookups on the host executor.
* ``sf10_filter`` — TPC-H SF10 ``lineitem`` FilterIndexRule (``l_shipdate`` range, Q6).
* ``hybrid`` — SF-N indexes, then +10% appended Parquet files in both tables: Q6 + Q3 through
  Hybrid Scan (BucketUnion on the device), an incremental refresh, and the same queries on the
  refreshed index.
* ``q3_3way`` — the TPC-H Q3 three-way join customer ⋈ orders ⋈ lineitem (JoinIndexRule on the
  customer/orders join, device shuffle of the intermediate onto the lineitem index layout).
* ``streamed`` — the SF-N index set built and queried under small HBM budgets (default 8 GB)
  against the resident run: bucket-range build passes and streamed queries.
* ``tpcds_3way`` — BASELINE config #5: TPC-DS-shaped ``store_sales`` ⋈ ``item`` ⋈ ``date_dim``
  (``hyperspace_amd.models.tpcds``, SF300 = 864M fact rows by default, ``--tpcds-sf``) with
  covering indexes on all three tables; queries, then +10% appended fact files and an
  incremental ``refreshIndex``, then the same queries on the refreshed index.  Results are
  checked against an independent pyarrow-dataset computation (not this engine's host path).
"""
import argparse
import datetime
import json
import os
import shutil
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _session(root, device, buckets, **extra):
    from hyperspace_amd import Session
    conf = {"spark.hyperspace.system.path": os.path.join(root, "indexes"),
            "spark.hyperspace.index.numBuckets": str(buckets),
            "spark.sql.autoBroadcastJoinThreshold": "-1",
            "spark.sql.shuffle.partitions": str(buckets),
            "spark.hyperspace.mi.execution.device": device}
    conf.update(extra)
    return Session(conf=conf, warehouse_dir=os.path.join(root, "wh"))


def _sync(device):
    if device == "gpu":
        import torch
        torch.cuda.synchronize()


def _mark(device):
    """HS_CFG_MARK=1: a short spin kernel (``torch.cuda._sleep``) that brackets each timed loop
    in a kernel trace (gpu.sh cfgprof)."""
    if device == "gpu" and os.environ.get("HS_CFG_MARK"):
        import torch
        torch.cuda._sleep(1000)


def _timed_loop(fn, n, device):
    _mark(device)
    _sync(device)
    t0 = time.perf_counter()
    for i in range(n):
        fn(i)
    _sync(device)
    el = time.perf_counter() - t0
    _mark(device)
    if os.environ.get("HS_CFG_CPROFILE"):     # where the host time of the loop goes
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for i in range(n):
            fn(i)
        _sync(device)
        pr.disable()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(45)
        print(f"[cprofile] {getattr(fn, '__name__', fn)} x{n}\n{buf.getvalue()}",
              file=sys.stderr, flush=True)
    return el


def _rows(df):
    return sorted(tuple(r) for r in df.collect())


def _close(a, b):
    if len(a) != len(b):
        return False
    for x, y in zip(a, b):
        for u, v in zip(x, y):
            if isinstance(u, float) or isinstance(v, float):
                if abs(u - v) > 1e-9 * max(1.0, abs(v)):
                    return False
            elif u != v:
                return False
    return True


# ------------------------------------------------------------------------------------ csv10k
def config_csv10k(args):
    import numpy as np
    import pyarrow as pa
    import pyarrow.csv as pacsv
    from hyperspace_amd import Hyperspace, IndexConfig, col
    root = os.path.join(args.data_dir, "csv10k")
    shutil.rmtree(root, ignore_errors=True)
    os.makedirs(os.path.join(root, "src"))
    rng = np.random.default_rng(7)
    n = 10_000
    queries = np.array(["donde", "facebook", "ibraco", "miperro", "google", "bing", "yahoo"])
    t = pa.table({"Date": pa.array([f"2019-10-{d:02d}" for d in rng.integers(1, 29, n)]),
                  "RGUID": pa.array([f"{x:08x}" for x in rng.integers(0, 2**32, n)]),
                  "Query": pa.array(queries[rng.integers(0, len(queries), n)]),
                  "imprs": pa.array(rng.integers(1, 1000, n).astype(np.int32)),
                  "clicks": pa.array(rng.integers(0, 100, n).astype(np.int64))})
    for i in range(4):
        pacsv.write_csv(t.slice(i * n // 4, n // 4), os.path.join(root, "src", f"part-{i}.csv"))
    s = _session(root, "cpu", 8)
    hs = Hyperspace(s)
    df = s.read.option("header", "true").csv(os.path.join(root, "src"))
    tb = time.perf_counter()
    hs.createIndex(df, IndexConfig("csvIdx", ["Query"], ["clicks", "imprs"]))
    build_s = time.perf_counter() - tb

    def q(i):
        return df.filter(col("Query") == str(queries[i % len(queries)])).select("Query", "clicks")
    Hyperspace.enable(s)
    used = "csvIdx" in q(0).queryExecution.executed_plan.tree_string()
    on = [_rows(q(i)) for i in range(len(queries))]
    dt_on = _timed_loop(lambda i: q(i).collect(), 50, "cpu")
    s.disableHyperspace()
    off = [_rows(q(i)) for i in range(len(queries))]
    dt_off = _timed_loop(lambda i: q(i).collect(), 50, "cpu")
    return {"config": "csv10k", "device": "cpu", "rows": n, "index_build_s": round(build_s, 4),
            "lookups_per_s_indexed": round(50 / dt_on, 2),
            "lookups_per_s_no_index": round(50 / dt_off, 2),
            "index_used": used, "match": all(_close(a, b) for a, b in zip(on, off))}


# ------------------------------------------------------------------------------------ TPC-H
def _tpch(args, sf, with_customer=False):
    from hyperspace_amd.models import tpch
    nfiles = max(8, int(round(sf * 1.28)))
    data = os.path.join(args.data_dir, f"tpch_sf{sf:g}_f{nfiles}")
    tpch.generate(data, sf, nfiles, workers=min(16, os.cpu_count() or 8))
    if with_customer:
        tpch.write_customers(data, sf, max(4, nfiles // 8))
    return data, nfiles


def _build(hs, df, cfg, device):
    from hyperspace_amd.exec import device_build
    _sync(device)
    t0 = time.perf_counter()
    hs.createIndex(df, cfg)
    _sync(device)
    dt = time.perf_counter() - t0
    nbytes = device_build.LAST_BUILD_STATS.get("source_bytes", 0) if device == "gpu" else 0
    return dt, nbytes


def _q6(li, i):
    from hyperspace_amd import col, sum_
    year = 1993 + i % 5
    disc = 0.02 + (i % 8) * 0.01
    lo, hi = datetime.date(year, 1, 1), datetime.date(year + 1, 1, 1)
    return li.filter((col("l_shipdate") >= lo) & (col("l_shipdate") < hi) &
                     (col("l_discount") >= round(disc - 0.01, 2)) &
                     (col("l_discount") <= round(disc + 0.01, 2)) &
                     (col("l_quantity") < 24 + (i % 2))) \
        .agg(sum_(col("l_extendedprice") * col("l_discount")).alias("revenue"))


def _q3(li, od, i):
    from hyperspace_amd import col, count, sum_
    dd = datetime.date(1995, 3, 1) + datetime.timedelta(days=(i * 7) % 30)
    j = li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
        .filter((col("o_orderdate") < dd) & (col("l_shipdate") > dd))
    return j.groupBy("o_shippriority").agg(
        sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue"),
        count("*").alias("lines"))


def config_sf10_filter(args):
    from hyperspace_amd import Hyperspace, IndexConfig
    sf = 10.0
    data, _ = _tpch(args, sf)
    root = os.path.join(args.data_dir, "cfg_sf10")
    shutil.rmtree(root, ignore_errors=True)
    s = _session(root, args.device, args.buckets)
    hs = Hyperspace(s)
    li = s.read.parquet(os.path.join(data, "lineitem"))
    dt, nbytes = _build(hs, li, IndexConfig("li_shipdate", ["l_shipdate"],
                                            ["l_discount", "l_quantity", "l_extendedprice"]),
                        args.device)
    Hyperspace.enable(s)
    for i in range(3):
        _q6(li, 1000 + i).collect()
    k = args.steps * 5
    el = _timed_loop(lambda i: _q6(li, i).collect(), k, args.device)
    path = getattr(s.backend(), "last_path", None)
    got = _q6(li, 0).collect()[0][0]
    s.disableHyperspace()
    ref = _q6(li, 0).collect()[0][0]
    return {"config": "sf10_filter", "device": args.device, "queries_per_s": round(k / el, 2),
            "q6_ms": round(el / k * 1e3, 3), "index_build_s": round(dt, 3),
            "index_build_gbps": round(nbytes / dt / 1e9, 3) if nbytes else None,
            "path": path, "match": abs(got - ref) <= 1e-9 * abs(ref)}


def config_hybrid(args):
    import pyarrow.parquet as pq  # noqa: F401
    from hyperspace_amd import Hyperspace, IndexConfig
    from hyperspace_amd.models import tpch
    sf = args.sf
    data, nfiles = _tpch(args, sf)
    # a private copy: appending files must not disturb the shared generated data set
    work = os.path.join(args.data_dir, f"cfg_hybrid_sf{sf:g}")
    shutil.rmtree(work, ignore_errors=True)
    for t in ("lineitem", "orders"):
        os.makedirs(os.path.join(work, "data", t))
        for f in os.listdir(os.path.join(data, t)):
            os.link(os.path.join(data, t, f), os.path.join(work, "data", t, f))
    s = _session(work, args.device, args.buckets,
                 **{"spark.hyperspace.index.lineage.enabled": "true",
                    "spark.hyperspace.index.hybridscan.enabled": "true",
                    "spark.hyperspace.index.hybridscan.maxAppendedRatio": "0.3"})
    hs = Hyperspace(s)
    lpath, opath = os.path.join(work, "data", "lineitem"), os.path.join(work, "data", "orders")
    li, od = s.read.parquet(lpath), s.read.parquet(opath)
    builds = {}
    for df, cfg in ((li, IndexConfig("li_orderkey", ["l_orderkey"],
                                     ["l_extendedprice", "l_discount", "l_shipdate"])),
                    (od, IndexConfig("ord_orderkey", ["o_orderkey"],
                                     ["o_orderdate", "o_shippriority"])),
                    (li, IndexConfig("li_shipdate", ["l_shipdate"],
                                     ["l_discount", "l_quantity", "l_extendedprice"]))):
        builds[cfg.indexName] = round(_build(hs, df, cfg, args.device)[0], 3)
    # +10%: chunks nfiles.. extend the key domain (fresh orders and their lineitems)
    extra = max(1, nfiles // 10)
    for i in range(nfiles, nfiles + extra):
        tpch.write_chunk(os.path.join(work, "data"), sf, nfiles, i)
    Hyperspace.enable(s)
    li, od = s.read.parquet(lpath), s.read.parquet(opath)

    def step(i):
        _q6(li, i).collect()
        _q3(li, od, i).collect()
    plan = _q3(li, od, 0).queryExecution.executed_plan.tree_string()
    for i in range(2):
        step(1000 + i)
    from hyperspace_amd.utils.tracing import TRACER, format_report
    TRACER.reset()
    el_h = _timed_loop(step, args.steps, args.device)
    path_h = getattr(s.backend(), "last_path", None)
    merge_skip = getattr(s.backend(), "metrics", {}).get("hybrid_merge_skip")
    print(f"[hybrid] merged union skipped: {merge_skip}", file=sys.stderr, flush=True)
    if TRACER.profile:   # the filter query's plan and whether its scan pruned key ranges
        q6p = _q6(li, 0)
        q6p.collect()
        print(q6p.queryExecution.executed_plan.tree_string()[:3000], file=sys.stderr, flush=True)
        print(f"[hybrid] q6 metrics {getattr(s.backend(), 'metrics', {})}", file=sys.stderr,
              flush=True)
    if TRACER.profile:   # HS_PROFILE=1: where the Hybrid Scan steps spend their time
        print("[hybrid] hybrid-scan stage profile\n" + format_report(TRACER.report()),
              file=sys.stderr, flush=True)
        print(plan, file=sys.stderr, flush=True)
    hyb = (_q6(li, 0).collect()[0][0], _rows(_q3(li, od, 0)))
    tr = time.perf_counter()
    for name in ("li_orderkey", "ord_orderkey", "li_shipdate"):
        t1 = time.perf_counter()
        hs.refreshIndex(name, "incremental")
        _sync(args.device)
        st = {}
        if args.device == "gpu":
            from hyperspace_amd.exec import device_build
            st = {k: v for k, v in device_build.LAST_BUILD_STATS.items()
                  if isinstance(v, (int, float, str))}
        print(f"[hybrid] refresh {name}: {time.perf_counter() - t1:.3f}s {st}", file=sys.stderr,
              flush=True)
    _sync(args.device)
    refresh_s = time.perf_counter() - tr
    li, od = s.read.parquet(lpath), s.read.parquet(opath)
    for i in range(2):
        step(2000 + i)
    TRACER.reset()
    be = s.backend()
    cache0 = (be.cache.hits, be.cache.misses) if hasattr(be, "cache") else (0, 0)
    el_r = _timed_loop(step, args.steps, args.device)
    cache1 = (be.cache.hits, be.cache.misses, round(be.cache.resident_bytes / 1e9, 1)) \
        if hasattr(be, "cache") else (0, 0, 0)
    print(f"[hybrid] refreshed loop device cache hits/misses {cache0} -> {cache1}",
          file=sys.stderr, flush=True)
    if TRACER.profile:   # HS_PROFILE=1: where the refreshed-index steps spend their time
        print("[hybrid] refreshed stage profile\n" + format_report(TRACER.report()),
              file=sys.stderr, flush=True)
        for q in (_q6(li, 0), _q3(li, od, 0)):
            print(q.queryExecution.executed_plan.tree_string(), file=sys.stderr, flush=True)
    ref = (_q6(li, 0).collect()[0][0], _rows(_q3(li, od, 0)))
    match = abs(hyb[0] - ref[0]) <= 1e-9 * abs(ref[0]) and _close(hyb[1], ref[1])
    return {"config": "hybrid", "device": args.device, "sf": sf, "appended_files": extra,
            "hybrid_queries_per_s": round(2 * args.steps / el_h, 2),
            "refreshed_queries_per_s": round(2 * args.steps / el_r, 2),
            "incremental_refresh_s": round(refresh_s, 3), "index_build_s": builds,
            "bucket_union_in_plan": "BucketUnion" in plan, "path": path_h,
            "hybrid_merge_skip": merge_skip,
            "hybrid_matches_refreshed": bool(match)}


def config_q3_3way(args):
    from hyperspace_amd import Hyperspace, IndexConfig, col, count, sum_
    sf = args.sf
    data, _ = _tpch(args, sf, with_customer=True)
    root = os.path.join(args.data_dir, f"cfg_q3_sf{sf:g}")
    shutil.rmtree(root, ignore_errors=True)
    s = _session(root, args.device, args.buckets)
    hs = Hyperspace(s)
    c = s.read.parquet(os.path.join(data, "customer"))
    o = s.read.parquet(os.path.join(data, "orders"))
    li = s.read.parquet(os.path.join(data, "lineitem"))
    builds = {}
    for df, cfg in ((c, IndexConfig("cust", ["c_custkey"], ["c_mktsegment"])),
                    (o, IndexConfig("ord_cust", ["o_custkey"],
                                    ["o_orderkey", "o_orderdate", "o_shippriority"])),
                    # the orders-key index the 2-way Q3 joins: the executor's co-partitioned
                    # semi-join reads it for the (customer x orders) x lineitem join
                    (o, IndexConfig("ord_orderkey", ["o_orderkey"],
                                    ["o_custkey", "o_orderdate", "o_shippriority"])),
                    (li, IndexConfig("li_orderkey", ["l_orderkey"],
                                     ["l_extendedprice", "l_discount", "l_shipdate"]))):
        builds[cfg.indexName] = round(_build(hs, df, cfg, args.device)[0], 3)
    segs = ["BUILDING", "AUTOMOBILE", "MACHINERY", "HOUSEHOLD", "FURNITURE"]

    def q(i):
        d = datetime.date(1995, 3, 1) + datetime.timedelta(days=(i * 7) % 30)
        co = c.join(o, c["c_custkey"] == o["o_custkey"]) \
            .filter((col("c_mktsegment") == segs[i % 5]) & (col("o_orderdate") < d))
        return co.join(li, co["o_orderkey"] == li["l_orderkey"]).filter(col("l_shipdate") > d) \
            .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("revenue"),
                 count("*").alias("lines"))
    Hyperspace.enable(s)
    plan = q(0).queryExecution.executed_plan.tree_string()
    for i in range(2):
        q(1000 + i).collect()
    k = max(3, args.steps // 2)
    from hyperspace_amd.utils.tracing import TRACER, format_report
    TRACER.reset()
    el = _timed_loop(lambda i: q(i).collect(), k, args.device)
    semi = getattr(s.backend(), "last_semi_join", None)
    if TRACER.profile:   # HS_PROFILE=1: where the 3-way join's time goes
        print("[q3_3way] stage profile\n" + format_report(TRACER.report()), file=sys.stderr,
              flush=True)
        print(plan, file=sys.stderr, flush=True)
    path = getattr(s.backend(), "last_path", None)
    reason = getattr(s.backend(), "fallback_reason", None)
    got = _rows(q(0))
    s.disableHyperspace()
    t0 = time.perf_counter()
    ref = _rows(q(0))
    noidx_s = time.perf_counter() - t0
    return {"config": "q3_3way", "device": args.device, "sf": sf,
            "queries_per_s": round(k / el, 3), "q3_3way_ms": round(el / k * 1e3, 2),
            "no_index_query_s": round(noidx_s, 3), "index_build_s": builds,
            "indexes_in_plan": [n for n in ("cust", "ord_cust", "li_orderkey") if n in plan],
            "path": path, "fallback_reason": reason, "match": _close(got, ref),
            "semi_join": semi}


def config_streamed(args):
    """SURVEY §5.7 / BASELINE config #5's "beyond one GPU's HBM": the bench's SF-N index set
    built and queried under small HBM budgets (``--hbm-budget-gb``, default 8 GB for the build
    working set, ``build.hbmBudgetBytes``, and for resident index tables, ``deviceCacheBytes``)
    against the resident run on the same files: a build in bucket-range passes (GB/s), then Q6
    and Q3 that stream their index scans bucket range by bucket range (q/s).  Every streamed
    result must equal the resident one (itself the engine's oracle-checked path)."""
    from hyperspace_amd import Hyperspace, IndexConfig
    sf = args.sf
    data, _ = _tpch(args, sf)
    budget = int(args.hbm_budget_gb * (1 << 30))
    li_cfgs = (IndexConfig("li_shipdate", ["l_shipdate"],
                           ["l_discount", "l_quantity", "l_extendedprice"]),
               IndexConfig("li_orderkey", ["l_orderkey"],
                           ["l_extendedprice", "l_discount", "l_shipdate"]))
    od_cfg = IndexConfig("ord_orderkey", ["o_orderkey"], ["o_orderdate", "o_shippriority"])
    out = {"config": "streamed", "device": args.device, "sf": sf,
           "hbm_budget_gb": args.hbm_budget_gb}
    results = {}
    for mode in ("resident", "streamed"):
        root = os.path.join(args.data_dir, f"cfg_stream_{mode}")
        shutil.rmtree(root, ignore_errors=True)
        extra = {}
        if mode == "streamed":
            extra = {"spark.hyperspace.mi.build.hbmBudgetBytes": str(budget)}
        s = _session(root, args.device, args.buckets, **extra)
        hs = Hyperspace(s)
        li = s.read.parquet(os.path.join(data, "lineitem"))
        od = s.read.parquet(os.path.join(data, "orders"))
        from hyperspace_amd.exec import device_build
        bt, bb, passes = 0.0, 0, {}
        for df, cfg in ((li, li_cfgs[0]), (li, li_cfgs[1]), (od, od_cfg)):
            dt, nb = _build(hs, df, cfg, args.device)
            bt += dt
            bb += nb
            passes[cfg.indexName] = device_build.LAST_BUILD_STATS.get("passes", 1)
        if mode == "streamed":
            s.conf.set("spark.hyperspace.mi.deviceCacheBytes", str(budget))
        Hyperspace.enable(s)

        def step(i):
            _q6(li, i).collect()
            _q3(li, od, i).collect()
        for i in range(2):
            step(1000 + i)
        be = s.backend()
        el = _timed_loop(step, args.steps, args.device)
        res = [(_q6(li, i).collect()[0][0], _rows(_q3(li, od, i))) for i in range(3)]
        results[mode] = res
        out[mode] = {"queries_per_s": round(2 * args.steps / el, 2),
                     "index_build_s": round(bt, 3),
                     "index_build_gbps": round(bb / bt / 1e9, 3) if bb else None,
                     "build_passes": passes, "path": getattr(be, "last_path", None),
                     "stream_passes": getattr(be, "last_stream_passes", None)}
        # the next mode's session starts from an empty device
        del s, hs, be
        if args.device == "gpu":
            from hyperspace_amd.exec.gpu import release_process_device_memory
            release_process_device_memory()
    a, b = results["resident"], results["streamed"]
    out["match"] = all(abs(x[0] - y[0]) <= 1e-9 * abs(x[0]) and _close(x[1], y[1])
                       for x, y in zip(a, b))
    out["streamed_vs_resident_qps"] = round(out["streamed"]["queries_per_s"] /
                                            out["resident"]["queries_per_s"], 3)
    out["streamed_vs_resident_build"] = round(out["resident"]["index_build_s"] /
                                              out["streamed"]["index_build_s"], 3)
    return out


# ------------------------------------------------------------------------------------ TPC-DS
def _tpcds_query(ss, it, dd, i):
    """TPC-DS Q3-shaped star join: one manufacturer's items sold in one month of the year."""
    from hyperspace_amd import col, count, sum_
    m, moy = 1 + (i * 37) % 1000, 1 + i % 12
    items = it.filter(col("i_manufact_id") == m)
    days = dd.filter(col("d_moy") == moy)
    j = ss.join(items, ss["ss_item_sk"] == items["i_item_sk"])
    j = j.join(days, j["ss_sold_date_sk"] == days["d_date_sk"])
    return j.agg(sum_(col("ss_ext_sales_price")).alias("sales"), count("*").alias("lines"))


def _tpcds_oracle(paths, i):
    """The query computed independently with pyarrow datasets (filter pushdown, no join)."""
    import pyarrow.compute as pc
    import pyarrow.dataset as ds
    import pyarrow.parquet as pq
    m, moy = 1 + (i * 37) % 1000, 1 + i % 12
    it = pq.read_table(paths["item"], columns=["i_item_sk", "i_manufact_id"])
    items = it.filter(pc.equal(it["i_manufact_id"], m))["i_item_sk"]
    dd = pq.read_table(paths["date_dim"], columns=["d_date_sk", "d_moy"])
    days = dd.filter(pc.equal(dd["d_moy"], moy))["d_date_sk"]
    t = ds.dataset(paths["store_sales"], format="parquet").to_table(
        columns=["ss_ext_sales_price"],
        filter=ds.field("ss_item_sk").isin(items) & ds.field("ss_sold_date_sk").isin(days))
    return [(float(pc.sum(t["ss_ext_sales_price"]).as_py() or 0.0), t.num_rows)]


def config_tpcds_3way(args):
    from hyperspace_amd import Hyperspace, IndexConfig
    from hyperspace_amd.models import tpcds
    sf = args.tpcds_sf
    nfiles = max(4, int(round(sf * 1.28)))
    data = os.path.join(args.data_dir, f"tpcds_sf{sf:g}_f{nfiles}")
    tg = time.perf_counter()
    tpcds.generate(data, sf, nfiles, workers=min(16, os.cpu_count() or 8))
    gen_s = time.perf_counter() - tg
    work = os.path.join(args.data_dir, f"cfg_tpcds_sf{sf:g}")
    shutil.rmtree(work, ignore_errors=True)
    for t in ("store_sales", "item", "date_dim"):       # private links: appends stay local
        os.makedirs(os.path.join(work, "data", t))
        for f in os.listdir(os.path.join(data, t)):
            os.link(os.path.join(data, t, f), os.path.join(work, "data", t, f))
    paths = {t: os.path.join(work, "data", t) for t in ("store_sales", "item", "date_dim")}
    s = _session(work, args.device, args.buckets)
    hs = Hyperspace(s)
    ss, it, dd = (s.read.parquet(paths[t]) for t in ("store_sales", "item", "date_dim"))
    builds = {}
    for df, cfg in ((ss, IndexConfig("ss_item", ["ss_item_sk"],
                                     ["ss_sold_date_sk", "ss_ext_sales_price"])),
                    (it, IndexConfig("item_idx", ["i_item_sk"], ["i_manufact_id"])),
                    (dd, IndexConfig("date_idx", ["d_date_sk"], ["d_moy"]))):
        builds[cfg.indexName] = round(_build(hs, df, cfg, args.device)[0], 3)
    Hyperspace.enable(s)
    k = max(3, args.steps)

    def run_queries(tag):
        ss_, it_, dd_ = (s.read.parquet(paths[t]) for t in ("store_sales", "item", "date_dim"))
        plan = _tpcds_query(ss_, it_, dd_, 0).queryExecution.executed_plan.tree_string()
        for i in range(2):
            _tpcds_query(ss_, it_, dd_, 1000 + i).collect()
        from hyperspace_amd.utils.tracing import TRACER, format_report
        TRACER.reset()
        el = _timed_loop(lambda i: _tpcds_query(ss_, it_, dd_, i).collect(), k, args.device)
        if TRACER.profile:   # HS_PROFILE=1: where the star join's time goes
            print(f"[tpcds_3way:{tag}] stage profile\n" + format_report(TRACER.report()),
                  file=sys.stderr, flush=True)
            print(plan, file=sys.stderr, flush=True)
        got = _rows(_tpcds_query(ss_, it_, dd_, 0))
        ref = _tpcds_oracle(paths, 0)
        return {f"{tag}_queries_per_s": round(k / el, 3), f"{tag}_query_ms": round(el / k * 1e3, 2),
                f"{tag}_match": _close(got, ref), f"{tag}_lines": got[0][1] if got else None,
                f"{tag}_indexes_in_plan": [n for n in ("ss_item", "item_idx", "date_idx")
                                           if n in plan],
                f"{tag}_path": getattr(s.backend(), "last_path", None)}
    out = {"config": "tpcds_3way", "device": args.device, "sf": sf,
           "store_sales_rows": tpcds.store_sales_rows(sf), "source_files": nfiles,
           "datagen_s": round(gen_s, 2), "index_build_s": builds}
    out.update(run_queries("base"))
    # +10% fact rows: new files with the same domains, then an incremental refresh
    extra = max(1, nfiles // 10)
    tpcds.write_store_sales_files(os.path.join(work, "data"), sf, nfiles, first=nfiles,
                                  count=extra, workers=min(16, os.cpu_count() or 8))
    _sync(args.device)
    tr = time.perf_counter()
    hs.refreshIndex("ss_item", "incremental")
    _sync(args.device)
    out["appended_files"] = extra
    out["incremental_refresh_s"] = round(time.perf_counter() - tr, 3)
    out.update(run_queries("refreshed"))
    return out


CONFIGS = {"csv10k": config_csv10k, "sf10_filter": config_sf10_filter, "hybrid": config_hybrid,
           "q3_3way": config_q3_3way, "tpcds_3way": config_tpcds_3way,
           "streamed": config_streamed}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="all", choices=["all"] + list(CONFIGS))
    ap.add_argument("--device", default="gpu", choices=["gpu", "cpu"])
    ap.add_argument("--sf", type=float, default=100.0)
    ap.add_argument("--buckets", type=int, default=200)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--data-dir", default=os.environ.get("HS_BENCH_DIR", "/tmp/hs_bench"))
    ap.add_argument("--tpcds-sf", type=float, default=300.0)
    ap.add_argument("--hbm-budget-gb", type=float, default=8.0,
                    help="streamed: the build and resident-table HBM budgets")
    args = ap.parse_args()
    if args.device == "gpu":
        import torch
        torch.cuda.set_device(0)
    names = list(CONFIGS) if args.config == "all" else [args.config]
    for name in names:
        t0 = time.perf_counter()
        res = CONFIGS[name](args)
        res["wall_s"] = round(time.perf_counter() - t0, 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
