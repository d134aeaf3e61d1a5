"""Rank bodies for the multi-process tests (``test_distributed.py``).  Each runs in a spawned
process with ``torch.distributed`` over gloo on 127.0.0.1 and writes its observations to
``<out>/rank<r>.json`` for the parent test to check."""
from __future__ import annotations

import json
import os
import traceback


def _init(rank: int, world: int, port: int):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank),
                       "HS_DIST_BACKEND": "gloo"})
    from hyperspace_amd.parallel.dist import DistContext
    return DistContext.from_env(backend="gloo")


def _finish(out_dir: str, rank: int, result: dict) -> None:
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(result, f)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


def run(rank: int, world: int, port: int, scenario: str, out_dir: str, data_dir: str) -> None:
    result = {"rank": rank}
    try:
        ctx = _init(rank, world, port)
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
    return {"sums": s.tolist(), "cnts": c.tolist(), "mins": mn.tolist(), "maxs": mx.tolist(),
            "objs": objs, "recv": rv.tolist(), "recv_f": rf.tolist(), "recv_counts": counts.tolist(),
            "sent": {"dest": dest.tolist(), "vals": vals.tolist()}}


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
    for name, df in q.items():
        out[name] = sorted(tuple(r.values()) for r in df.to_arrow().to_pylist())
        out["paths"].append(s.backend().last_path)
        out[name + "_plan"] = df.queryExecution.executed_plan.tree_string()
    ctx.barrier()
    return out


SCENARIOS = {"collectives": collectives, "spmd_index": spmd_index, "spmd_gpu": spmd_gpu}
