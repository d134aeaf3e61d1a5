"""Rank bodies for the multi-process tests (``test_distributed.py``).  Each runs in a spawned
process with ``torch.distributed`` over gloo on 127.0.0.1 and writes its observations to
``<out>/rank<r>.json`` for the parent test to check."""
from __future__ import annotations

import json
import os
import traceback


def _init(rank: int, world: int, port: int, backend: str = "gloo"):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "HS_DIST_BACKEND": backend})
    if backend == "nccl":
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    from hyperspace_amd.parallel.dist import DistContext
    if world == 1:
        import torch.distributed as dist
        import torch
        torch.cuda.set_device(0)
        dist.init_process_group(backend=backend, rank=0, world_size=1,
                                device_id=torch.device("cuda", 0))
    return DistContext.from_env(backend=backend)


def _finish(out_dir: str, rank: int, result: dict) -> None:
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(result, f)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def run(rank: int, world: int, port: int, scenario: str, out_dir: str, data_dir: str,
        backend: str = "gloo") -> None:
    result = {"rank": rank}
    try:
        ctx = _init(rank, world, port, backend)
        result.update(SCENARIOS[scenario](ctx, data_dir))
    except Exception as e:  # noqa: BLE001 — reported to the parent
        result["error"] = f"{type(e).__name__}: {e}\n{traceback.format_exc()}"
    _finish(out_dir, rank, result)


# ------------------------------------------------------------------------------------------------
def collectives(ctx, data_dir):
    import torch
    from hyperspace_amd.parallel.shuffle import exchange
    r, w = ctx.rank, ctx.world
    sums = torch.tensor([1.0 + r, 2.0], dtype=torch.float64)
    cnts = torch.tensor([1, r], dtype=torch.int64)
    mins = torch.tensor([float(r), 5.0], dtype=torch.float64)
    maxs = torch.tensor([float(r), -1.0], dtype=torch.float64)
    s, c, mn, mx = ctx.all_reduce_agg(sums, cnts, mins, maxs)
    objs = ctx.all_gather_object({"r": r})
    # uneven all-to-all: rank r sends row i to dest[i]; values encode (source rank, position)
    g = torch.Generator().manual_seed(100 + r)
    n = 50 + 17 * r
    dest = torch.randint(0, w, (n,), generator=g, dtype=torch.int32)
    vals = torch.arange(n, dtype=torch.int64) + 1000 * r
    fl = vals.double() * 0.5
    (rv, rf), counts = exchange([vals, fl], dest, w, ctx=ctx)
    import pyarrow as pa
    from hyperspace_amd.parallel.dictionary import union_sorted
    local = pa.array([f"s{r}_{i}" for i in range(r + 2)] + ["common", None])
    gd = union_sorted(local, ctx)
    return {"sums": s.tolist(), "cnts": c.tolist(), "mins": mn.tolist(), "maxs": mx.tolist(),
            "objs": objs, "recv": rv.tolist(), "recv_f": rf.tolist(), "recv_counts": counts.tolist(),
            "sent": {"dest": dest.tolist(), "vals": vals.tolist()}, "dict": gd.to_pylist()}


def _session(ctx, data_dir, **conf):
    from hyperspace_amd import Session
    from hyperspace_amd.parallel.dist import attach
    base = {"spark.hyperspace.system.path": os.path.join(data_dir, "indexes"),
            "spark.hyperspace.index.numBuckets": "4",
            "spark.sql.autoBroadcastJoinThreshold": "-1",
            "spark.sql.shuffle.partitions": "5",
            "spark.hyperspace.mi.execution.device": "cpu"}
    base.update(conf)
    s = Session(conf=base, warehouse_dir=os.path.join(data_dir, "wh"))
    attach(s, ctx)
    return s


def spmd_index(ctx, data_dir):
    """Every rank runs the same driver program (SPMD): create two indexes, query through them,
    refresh with nothing to do (a no-op everywhere), and fail a create on one rank only."""
    from hyperspace_amd import Hyperspace, IndexConfig, col, count, sum_
    from hyperspace_amd.exceptions import HyperspaceException
    s = _session(ctx, data_dir)
    hs = Hyperspace(s)
    t1 = s.read.parquet(os.path.join(data_dir, "t1"))
    t2 = s.read.parquet(os.path.join(data_dir, "t2"))
    hs.createIndex(t1, IndexConfig("i1", ["k"], ["v"]))
    hs.createIndex(t2, IndexConfig("i2", ["k"], ["w"]))
    out = {}
    try:
        hs.createIndex(t1, IndexConfig("i1", ["k"], ["v"]))
        out["dup_create"] = "no error"
    except HyperspaceException as e:
        out["dup_create"] = type(e).__name__
    hs.refreshIndex("i1", "full")  # no source change: NoChangesException -> no-op on all ranks
    s.conf.set("spark.hyperspace.mi.faultInjection", "mid_op@1")
    try:
        hs.createIndex(t2, IndexConfig("i3", ["w"], ["k"]))
        out["one_rank_fault"] = "no error"
    except HyperspaceException as e:
        out["one_rank_fault"] = type(e).__name__
    s.conf.unset("spark.hyperspace.mi.faultInjection")
    ctx.barrier()
    Hyperspace.enable(s)
    q1 = t1.filter(col("k") == 7).select("k", "v")
    j = t1.join(t2, t1["k"] == t2["k"]).groupBy(t2["w"]).agg(sum_(col("v")).alias("sv"),
                                                               count("*").alias("n"))
    out["q1"] = sorted(tuple(r.values()) for r in q1.to_arrow().to_pylist())
    out["join"] = sorted(tuple(r.values()) for r in j.to_arrow().to_pylist())
    out["join_plan"] = j.queryExecution.executed_plan.tree_string()
    ctx.barrier()
    return out


def spmd_gpu(ctx, data_dir):
    """The device executor under SPMD (ranks share cuda:0 over gloo on a 1-GPU box): distributed
    device index build (all-to-all), bucket-owner queries with all-reduced partials (grouped on
    an integer and on a string key, whose per-rank domains differ), and a non-index join whose
    hash Exchanges run as device all-to-alls."""
    from hyperspace_amd import Hyperspace, IndexConfig, col, count, sum_, min_
    s = _session(ctx, data_dir, **{"spark.hyperspace.mi.execution.device": "gpu",
                                   "spark.hyperspace.system.path":
                                       os.path.join(data_dir, "indexes_gpu")})
    hs = Hyperspace(s)
    t1 = s.read.parquet(os.path.join(data_dir, "t1"))
    t2 = s.read.parquet(os.path.join(data_dir, "t2"))
    out = {"paths": []}
    # non-index first (hash Exchange on both sides -> distributed device shuffle)
    nj = t1.join(t2, t1["k"] == t2["k"]).groupBy(t2["s"]).agg(sum_(col("v")).alias("sv"),
                                                                count("*").alias("n"))
    out["nonindex_join"] = sorted(tuple(r.values()) for r in nj.to_arrow().to_pylist())
    out["paths"].append(s.backend().last_path)
    hs.createIndex(t1, IndexConfig("i1", ["k"], ["v"]))
    hs.createIndex(t2, IndexConfig("i2", ["k"], ["w", "s"]))
    Hyperspace.enable(s)
    j = t1.join(t2, t1["k"] == t2["k"])
    q = {"join_w": j.groupBy(t2["w"]).agg(sum_(col("v")).alias("sv"), count("*").alias("n")),
         "join_s": j.groupBy(t2["s"]).agg(sum_(col("v")).alias("sv"), min_(col("v")).alias("mv")),
         "filter": t1.filter(col("k") < 20).select("k", "v")}
    q.update({
        # row-producing join over sharded buckets: device row gather across ranks
        "join_rows": j.select(t1["k"], t1["v"], t2["s"]),
        # hash-mode aggregate (two group columns) + ORDER BY ... LIMIT
        "join_multi": j.groupBy(t2["w"], t2["s"]).agg(sum_(col("v")).alias("sv")),
        "topk": j.groupBy(t1["k"]).agg(sum_(col("v")).alias("sv"))
                 .orderBy(col("sv").desc(), col("k")).limit(5),
        "left_outer": t1.join(t2.filter(col("w") < 3), t1["k"] == t2["k"], "left")
                        .select(t1["k"], t2["w"]),
        # GROUP BY (join key, right column) over a unique right key + ORDER BY ... LIMIT:
        # functional-dependency grouping, each rank's own top rows exchanged
        "fd_topk": t2.join(t1, t2["k"] == t1["k"]).groupBy(t2["k"], t1["v"])
                     .agg(sum_(col("w")).alias("sw")).orderBy(col("sw").desc(), t2["k"])
                     .limit(5)})
    # semi-join: t3 (no index, behind a hash Exchange, unique keys) x the t1 index
    t3 = s.read.parquet(os.path.join(data_dir, "t3"))
    q["semi_keys"] = t3.join(t1, t3["k"] == t1["k"]).agg(sum_(col("v")).alias("sv"),
                                                          count("*").alias("n"))
    for name, df in q.items():
        rows = [tuple(r.values()) for r in df.to_arrow().to_pylist()]
        if name == "semi_keys":
            out["semi_exchange"] = getattr(s.backend(), "last_semi_exchange", None)
        out[name] = rows if name in ("topk", "fd_topk") else sorted(rows, key=repr)
        out["paths"].append(s.backend().last_path)
        out[name + "_plan"] = df.queryExecution.executed_plan.tree_string()
    # steady state: the same queries again make no pickled (object) collective
    calls = {"n": 0}
    orig = ctx.all_gather_object

    def counting(obj):
        calls["n"] += 1
        return orig(obj)
    ctx.all_gather_object = counting
    for name, df in q.items():
        df.to_arrow()
    ctx.all_gather_object = orig
    out["steady_object_collectives"] = calls["n"]
    ctx.barrier()
    return out


def _is_sync_warning(w) -> bool:
    """A torch sync-debug-mode report of a synchronizing operation (not the mode's own notice
    that it is a prototype)."""
    return "called a synchronizing" in str(w.message)


def sync_count(ctx, data_dir):
    """Host synchronizations of warm sharded queries over RCCL (world 1 on a 1-GPU box): a
    plan-cache hit of the indexed filter and join aggregates must submit without one (no
    ``.item()`` / blocking copy / stream or event wait: counted by torch's sync debug mode and
    by wrapping the explicit waits), and reading the result costs one."""
    import datetime  # noqa: F401
    import warnings
    import torch
    from hyperspace_amd import Hyperspace, IndexConfig, col, count, sum_
    assert ctx.backend == "nccl", ctx.backend
    s = _session(ctx, data_dir, **{"spark.hyperspace.mi.execution.device": "gpu",
                                   "spark.hyperspace.system.path":
                                       os.path.join(data_dir, "indexes_sync")})
    hs = Hyperspace(s)
    t1 = s.read.parquet(os.path.join(data_dir, "t1"))
    t2 = s.read.parquet(os.path.join(data_dir, "t2"))
    t3 = s.read.parquet(os.path.join(data_dir, "t3"))
    hs.createIndex(t1, IndexConfig("i1", ["k"], ["v"]))
    hs.createIndex(t2, IndexConfig("i2", ["k"], ["w", "s"]))
    hs.createIndex(t2, IndexConfig("i2w", ["w"], ["k"]))
    hs.createIndex(t3, IndexConfig("i3", ["k"], []))
    Hyperspace.enable(s)
    be = s.backend()

    def filt(i):
        return t1.filter((col("v") >= 10 + i) & (col("v") < 300 - i)) \
            .agg(sum_(col("v")).alias("sv"), count("*").alias("n"))

    def join(i):
        return t1.join(t2, t1["k"] == t2["k"]).filter(col("w") < 3 + i % 2) \
            .groupBy(t2["w"]).agg(sum_(col("v")).alias("sv"))

    def join3(i):
        # TPC-H Q3's 3-way shape (customer x orders on custkey, filtered, then x lineitem on
        # orderkey): t3 plays customer, t2.w o_custkey, t2.k o_orderkey, t1 lineitem
        co = t3.join(t2, t3["k"] == t2["w"]).filter(t2["w"] < 3 + i % 2)
        return co.join(t1, t2["k"] == t1["k"]).agg(sum_(t1["v"]).alias("sv"),
                                                   count("*").alias("n"))

    def full(i):
        # Q3's full result shape: GROUP BY the join key, ORDER BY the aggregate, LIMIT
        return t1.join(t2, t1["k"] == t2["k"]).filter(col("w") < 3 + i % 2) \
            .groupBy(t1["k"], t2["w"]).agg(sum_(col("v")).alias("sv")) \
            .orderBy(col("sv").desc(), col("k")).limit(5)

    counts = {"wait": 0}
    waits = []
    for obj, name in ((torch.cuda, "synchronize"), (torch.cuda.Stream, "synchronize"),
                      (torch.cuda.Event, "synchronize")):
        orig = getattr(obj, name)

        def wrapped(*a, _orig=orig, _name=f"{getattr(obj, '__name__', obj)}.{name}", **k):
            counts["wait"] += 1
            import traceback
            counts.setdefault("where", []).append(
                [_name] + [f"{f.filename.rsplit('/', 1)[-1]}:{f.lineno}:{f.name}"
                           for f in traceback.extract_stack()[-6:-1]])
            return _orig(*a, **k)
        waits.append((obj, name, orig))
        setattr(obj, name, wrapped)
    out = {}
    try:
        for qname, q in (("filter", filt), ("join", join), ("join3", join3), ("full", full)):
            for i in range(3):                      # warm: lowering, kernels, program
                q(i % 2).collect()
            torch.cuda.synchronize()
            per = []
            for i in range(4):
                df = q(i % 2)
                counts["wait"] = 0
                counts["where"] = []
                with warnings.catch_warnings(record=True) as w:
                    warnings.simplefilter("always")
                    torch.cuda.set_sync_debug_mode("warn")
                    fut = df.queryExecution.to_arrow_async()   # the bench's submission
                    torch.cuda.set_sync_debug_mode("default")
                submit = counts["wait"] + sum(_is_sync_warning(x) for x in w)
                if submit:
                    out.setdefault("submit_syncs", []).append(
                        [str(x.message)[:200] + " @ " + f"{x.filename}:{x.lineno}" for x in w
                         if _is_sync_warning(x)] + counts.get("where", []))
                counts["where"] = []
                counts["wait"] = 0
                with warnings.catch_warnings(record=True) as w:
                    warnings.simplefilter("always")
                    torch.cuda.set_sync_debug_mode("warn")
                    res = fut.result()
                    torch.cuda.set_sync_debug_mode("default")
                read = counts["wait"] + sum(_is_sync_warning(x) for x in w)
                if read > 1:
                    out.setdefault("read_syncs", {}).setdefault(qname, [
                        str(x.message)[:60] + " @ " + f"{x.filename}:{x.lineno}" for x in w
                        if _is_sync_warning(x)] + counts.get("where", []))
                per.append((submit, read, fut.path, res.num_rows))
            out[qname] = per
            out.setdefault("semi", {})[qname] = getattr(be, "last_semi_join", None)
    finally:
        torch.cuda.set_sync_debug_mode("default")
        for obj, name, orig in waits:
            setattr(obj, name, orig)
    return out


def nccl_paths(ctx, data_dir):
    """Every RCCL branch of ``parallel/`` on the process group it was given (world 1 on a
    1-GPU box, more ranks on a multi-GPU node): device all-reduce / all-gather / all-to-all,
    the packed row exchange, the raw-buffer dictionary union and the one-collective aggregate
    combine."""
    import numpy as np
    import pyarrow as pa
    import torch
    from hyperspace_amd.parallel.dictionary import union_sorted
    from hyperspace_amd.parallel.exchange import RowExchange
    assert ctx.backend == "nccl", ctx.backend
    dev = ctx.device
    r, w = ctx.rank, ctx.world
    out = {}
    t = torch.tensor([1.0 + r], dtype=torch.float64, device=dev)
    ctx.all_reduce(t, "sum")
    out["allreduce"] = t.item()
    out["agree"] = ctx.agree_any([r == 0, False])
    out["max"] = ctx.all_reduce_max_float(float(r))
    g = torch.Generator().manual_seed(7 + r)
    n = 100_000 + 1234 * r
    bucket = torch.randint(0, 200, (n,), generator=g, dtype=torch.int32)
    vals = torch.arange(n, dtype=torch.int64) + (r << 40)
    f32 = (vals & ((1 << 40) - 1)).float() * 0.25
    valid = (torch.arange(n) % 3 != 0).to(torch.uint8)
    ex = RowExchange(ctx, [torch.int64, torch.float32, torch.uint8, torch.int32], dev)
    half = n // 2
    for lo, hi in ((0, half), (half, half), (half, n)):   # incl. an empty batch
        ex.add([vals[lo:hi].to(dev), f32[lo:hi].to(dev), valid[lo:hi].to(dev),
                bucket[lo:hi].to(dev)], bucket[lo:hi].to(dev))
    gv, gf, gvalid, gb = (x.cpu() for x in ex.finish())
    out["xch_rows"] = int(gv.numel())
    out["xch_owner_ok"] = bool(((gb % w) == r).all())
    out["xch_f_ok"] = bool(torch.equal(gf, (gv & ((1 << 40) - 1)).float() * 0.25))
    out["xch_valid_ok"] = bool(torch.equal(gvalid, ((gv & ((1 << 40) - 1)) % 3 != 0).to(torch.uint8)))
    out["xch_sum"] = int(gv.sum())
    gd = union_sorted(pa.array([f"k{r}", "shared", f"x{r * 7}"]), ctx)
    out["dict"] = gd.to_pylist()
    sums = torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev)
    cnts = torch.tensor([1, 2], dtype=torch.int64, device=dev)
    mins = torch.tensor([float(r), 0.0], dtype=torch.float64, device=dev)
    maxs = torch.tensor([float(r), 9.0], dtype=torch.float64, device=dev)
    s, c, mn, mx = ctx.combine_aggs_async(sums, cnts, mins, maxs)()
    out["combine"] = [s.tolist(), c.tolist(), mn.tolist(), mx.tolist()]
    ctx.barrier()
    return out


def spmd_stream_build(ctx, data_dir):
    """Multi-rank device build twice: one pass, and under a tiny HBM budget (bucket-range passes,
    every file batch exchanged per pass); the parent compares the bucket files byte for byte."""
    from hyperspace_amd import Hyperspace, IndexConfig
    from hyperspace_amd.exec import device_build
    out = {}
    for name, budget in (("one_pass", 1 << 40), ("streamed", 600_000)):
        s = _session(ctx, data_dir, **{"spark.hyperspace.mi.execution.device": "gpu",
                                       "spark.hyperspace.index.numBuckets": "16",
                                       "spark.hyperspace.system.path":
                                           os.path.join(data_dir, "ix"),
                                       "spark.hyperspace.mi.build.hbmBudgetBytes": str(budget)})
        Hyperspace(s).createIndex(s.read.parquet(os.path.join(data_dir, "src")),
                                  IndexConfig(name, ["k"], ["d", "p", "q"]))
        st = device_build.LAST_BUILD_STATS
        out[name] = {"passes": st.get("passes"), "groups": st.get("file_groups"),
                     "writer": st.get("writer"), "writer_fallback": st.get("writer_fallback")}
    ctx.barrier()
    return out


def balanced_exchange(ctx, data_dir):
    """Rows routed by a size-balanced owner map (parallel/placement.py) through the packed
    all-to-all: every row lands on its bucket's owner under that map."""
    import torch
    from hyperspace_amd.parallel.exchange import RowExchange
    from hyperspace_amd.parallel.placement import OwnerMap
    r, w = ctx.rank, ctx.world
    B = 16
    weights = [1000.0] + [10.0] * (B - 1)             # bucket 0 is heavy
    m = OwnerMap.balanced(weights, w)
    g = torch.Generator().manual_seed(7 + r)
    bucket = torch.randint(0, B, (300,), generator=g, dtype=torch.int32)
    vals = torch.arange(300, dtype=torch.int64) + 10_000 * r
    ex = RowExchange(ctx, [torch.int64, torch.int32])
    ex.add([vals, bucket], bucket, m.dest(bucket))
    rv, rb = ex.finish()
    return {"owners": m.owners.tolist(), "recv_buckets": rb.tolist(), "recv": rv.tolist(),
            "sent": vals.tolist(), "sent_b": bucket.tolist()}


def spmd_skew(ctx, data_dir):
    """Device executor over a skewed join key (ranks share cuda:0 over gloo): the same indexes
    and queries under the modulo and the size-balanced bucket placement give identical results,
    and the balanced map gives the heavy bucket a rank of its own."""
    from hyperspace_amd import Hyperspace, IndexConfig, col, count, sum_
    s = _session(ctx, data_dir, **{"spark.hyperspace.mi.execution.device": "gpu",
                                   "spark.hyperspace.index.numBuckets": "8",
                                   "spark.hyperspace.system.path":
                                       os.path.join(data_dir, "indexes_skew")})
    hs = Hyperspace(s)
    t1 = s.read.parquet(os.path.join(data_dir, "s1"))
    t2 = s.read.parquet(os.path.join(data_dir, "s2"))
    hs.createIndex(t1, IndexConfig("k1", ["k"], ["v"]))
    hs.createIndex(t2, IndexConfig("k2", ["k"], ["w"]))
    Hyperspace.enable(s)
    out = {"paths": []}
    for mode in ("modulo", "balanced"):
        s.conf.set("spark.hyperspace.mi.bucketPlacement", mode)
        j = t1.join(t2, t1["k"] == t2["k"])
        qs = {"agg": j.groupBy(t2["w"]).agg(sum_(col("v")).alias("sv"), count("*").alias("n")),
              "rows": j.filter(col("v") % 97 == 0).select(t1["k"], t1["v"], t2["w"]),
              "filter": t1.filter(col("k") < 40).groupBy(t1["k"]).agg(count("*").alias("n"))}
        res = {}
        for name, df in qs.items():
            res[name] = sorted((tuple(r.values()) for r in df.to_arrow().to_pylist()), key=repr)
            out["paths"].append(s.backend().last_path)
        out[mode] = res
        maps = s.__dict__.get("_hs_owner_maps", {})
        m = maps.get((8, ctx.world, mode))
        out[mode + "_owners"] = m.owners.tolist() if m is not None else None
    ctx.barrier()
    return out


def spmd_split(ctx, data_dir):
    """A heavy bucket of many distinct keys (ranks share cuda:0 over gloo): the balanced map
    cuts it into key ranges on several ranks (parallel/placement.py split_heavy) and the
    co-located join / filter aggregates still match the
    modulo placement; every rank's rows of that bucket lie in its key range."""
    from hyperspace_amd import Hyperspace, IndexConfig, col, count, sum_
    s = _session(ctx, data_dir, **{"spark.hyperspace.mi.execution.device": "gpu",
                                   "spark.hyperspace.index.numBuckets": "16",
                                   "spark.hyperspace.system.path":
                                       os.path.join(data_dir, "indexes_split")})
    hs = Hyperspace(s)
    t3 = s.read.parquet(os.path.join(data_dir, "s3"))
    t2 = s.read.parquet(os.path.join(data_dir, "s2"))
    hs.createIndex(t3, IndexConfig("k3", ["k"], ["v"]))
    hs.createIndex(t2, IndexConfig("k2s", ["k"], ["w"]))
    Hyperspace.enable(s)
    out = {"paths": []}
    for mode in ("modulo", "balanced"):
        s.conf.set("spark.hyperspace.mi.bucketPlacement", mode)
        j = t3.join(t2, t3["k"] == t2["k"])
        qs = {"agg": j.groupBy(t2["w"]).agg(sum_(col("v")).alias("sv"), count("*").alias("n")),
              "filter": t3.filter(col("v") % 3 == 0).agg(sum_(col("v")).alias("sv"),
                                                          count("*").alias("n"))}
        res = {}
        for name, df in qs.items():
            res[name] = sorted((tuple(r.values()) for r in df.to_arrow().to_pylist()), key=repr)
            out["paths"].append(s.backend().last_path)
        out[mode] = res
        m = s.__dict__.get("_hs_owner_maps", {}).get((16, ctx.world, mode))
        out[mode + "_splits"] = {str(b): [r.tolist(), k.tolist()]
                                 for b, (r, k) in (m.splits.items() if m is not None else [])}
    # the resident index table of this rank: rows of each cut bucket within its key range
    be = s.backend()
    m = s.__dict__["_hs_owner_maps"][(16, ctx.world, "balanced")]
    cuts = m.ranges(ctx.rank)
    ok = True
    for key, t in list(be.cache._lru.items()):
        if "k" not in t.columns or t.num_buckets != 16 or key[2][0] != "bucketed" or \
                key[2][3] != m.key:
            continue
        off = t.bucket_offsets_host
        kk = t.columns["k"].data.cpu().numpy()
        for b, (lo, hi) in cuts.items():
            seg = kk[off[b]:off[b + 1]]
            ok = ok and (lo is None or (seg >= lo).all()) and (hi is None or (seg < hi).all())
    out["cut_rows_in_range"] = bool(ok)
    out["cuts"] = {str(b): [lo, hi] for b, (lo, hi) in cuts.items()}
    ctx.barrier()
    return out


SCENARIOS = {"spmd_stream_build": spmd_stream_build, "nccl_paths": nccl_paths,
             "collectives": collectives, "spmd_index": spmd_index, "spmd_gpu": spmd_gpu,
             "balanced_exchange": balanced_exchange, "spmd_skew": spmd_skew,
             "sync_count": sync_count, "spmd_split": spmd_split}
