"""Multi-process tests (world_size 2, 4 and 8, gloo on 127.0.0.1) for the SPMD paths: collectives and the
all-to-all row exchange (``parallel/``), and the index lifecycle under ``torch.distributed`` —
coordinator-only log writes, owner-rank bucket files, unanimous failure/no-op outcomes
(the reference has no distributed or fault-injection tests)."""
from __future__ import annotations

import json
import multiprocessing as mp
import os
import socket

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd.io.writer import get_bucket_id

WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(scenario: str, tmp_path, data_dir: str, timeout: float = 240.0, world: int = WORLD,
           backend: str = "gloo"):
    import dist_workers
    out = tmp_path / f"out_{scenario}_{world}"
    out.mkdir()
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=dist_workers.run,
                         args=(r, world, port, scenario, str(out), data_dir, backend))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
        p.join()
    assert not alive, f"{scenario}: ranks hung"
    res, errs = [], []
    for r, p in enumerate(procs):
        path = out / f"rank{r}.json"
        if not path.exists():
            errs.append(f"rank {r}: no result, exit code {p.exitcode}")
            res.append(None)
            continue
        with open(path) as f:
            d = json.load(f)
        if "error" in d:
            errs.append(f"rank {r} (exit code {p.exitcode}): {d['error']}")
        res.append(d)
    # every rank's outcome, so a rank that died (signal, OOM) is named, not just the peer that
    # saw its connection close
    assert not errs, "\n".join(errs)
    return res


@pytest.mark.parametrize("world", [2, 4, 8])
def test_collectives_and_all_to_all_exchange(tmp_path, world):
    res = _spawn("collectives", tmp_path, str(tmp_path), world=world)
    W = world
    for d in res:
        assert d["sums"] == [sum(1.0 + r for r in range(W)), 2.0 * W]
        assert d["cnts"] == [W, sum(range(W))]
        assert d["mins"] == [0.0, 5.0] and d["maxs"] == [float(W - 1), -1.0]
        assert d["objs"] == [{"r": r} for r in range(W)]
        # the dictionary union: every rank holds the same sorted union of all ranks' strings
        assert d["dict"] == sorted({f"s{r}_{i}" for r in range(W) for i in range(r + 2)} |
                                   {"common"})
    for r, d in enumerate(res):
        # rank r receives, from each source in rank order, exactly the rows addressed to it,
        # in their original order
        expect = []
        for src in res:
            expect += [v for v, dst in zip(src["sent"]["vals"], src["sent"]["dest"]) if dst == r]
        assert d["recv"] == expect
        assert d["recv_f"] == [v * 0.5 for v in expect]
        assert sum(d["recv_counts"]) == len(expect)


@pytest.fixture
def spmd_data(tmp_path):
    rng = np.random.default_rng(3)
    data = tmp_path / "data"
    k1 = rng.permutation(np.arange(200, dtype=np.int64))
    t1 = pa.table({"k": k1, "v": k1 * 2})
    k2 = np.repeat(np.arange(100, dtype=np.int64), 2)
    t2 = pa.table({"k": k2, "w": (k2 % 5).astype(np.int32),
                   "s": pa.array([f"s{x % 7}" for x in k2])})
    # unique, sparse keys over a wide domain: the sharded semi-join exchanges keys, not bitmaps
    t3 = pa.table({"k": np.concatenate([np.arange(0, 200, 3), [10_000_000]]).astype(np.int64)})
    for name, t, parts in (("t1", t1, 3), ("t2", t2, 2), ("t3", t3, 2)):
        os.makedirs(data / name)
        step = (t.num_rows + parts - 1) // parts
        for i in range(parts):
            pq.write_table(t.slice(i * step, step), data / name / f"part-{i}.parquet")
    return data, t1, t2


@pytest.mark.parametrize("world", [2, 4, 8])
def test_spmd_index_lifecycle_and_queries(tmp_path, spmd_data, world):
    """Build (packed all-to-all over gloo), filter and co-located join under 2, 4 and 8 ranks."""
    data, t1, t2 = spmd_data
    res = _spawn("spmd_index", tmp_path, str(data), world=world)
    # the index data: one file per bucket overall, each written by its owner rank, rows complete
    vdir = data / "indexes" / "i1" / "v__=0"
    files = sorted(f for f in os.listdir(vdir) if f.endswith(".parquet"))
    buckets = [get_bucket_id(f) for f in files]
    assert len(buckets) == len(set(buckets)), files
    for f in files:
        task = int(f.split("-")[1])
        assert task == get_bucket_id(f) % world, f
    assert sum(pq.read_table(vdir / f).num_rows for f in files) == t1.num_rows
    # coordinator-only log: create = 2 entries (0 CREATING, 1 ACTIVE); the no-op refresh adds none
    logs = sorted(os.listdir(data / "indexes" / "i1" / "_hyperspace_log"))
    assert logs == ["0", "1", "latestStable"], logs
    for d in res:
        assert d["dup_create"] == "HyperspaceException"
        # one rank failed mid-op: both ranks raised, the index stays in its transient state
        assert d["one_rank_fault"] in ("FaultInjected", "HyperspaceException")
        assert [tuple(x) for x in d["q1"]] == [(7, 14)]
        assert "Hyperspace(Type: CI, Name: i1" in d["join_plan"]
    i3_logs = sorted(os.listdir(data / "indexes" / "i3" / "_hyperspace_log"))
    assert i3_logs == ["0"], i3_logs
    with open(data / "indexes" / "i3" / "_hyperspace_log" / "0") as f:
        assert json.load(f)["state"] == "CREATING"
    assert res[1]["one_rank_fault"] == "FaultInjected"
    assert all(d["one_rank_fault"] == "HyperspaceException" for r, d in enumerate(res) if r != 1)
    # oracle: the join aggregate in plain pyarrow
    j = t1.join(t2, "k", join_type="inner")
    g = j.group_by("w").aggregate([("v", "sum"), ("v", "count")])
    expect = sorted(zip(g.column("w").to_pylist(), g.column("v_sum").to_pylist(),
                        g.column("v_count").to_pylist()))
    for d in res:
        assert [tuple(x) for x in d["join"]] == expect


@pytest.mark.gpu
def test_spmd_device_executor(tmp_path, spmd_data, device):
    """Two ranks share cuda:0 (gloo host-staged collectives): the device build, bucket-owner
    queries and the device shuffle must all run natively and agree with the pyarrow oracle."""
    data, t1, t2 = spmd_data
    res = _spawn("spmd_gpu", tmp_path, str(data), timeout=600.0)
    j = t1.join(t2, "k", join_type="inner")

    def oracle(key, aggs):
        g = j.group_by(key).aggregate(aggs)
        names = [key] + [f"{c}_{fn}" for c, fn in aggs]
        return sorted(zip(*[g.column(c).to_pylist() for c in names]))
    exp_s = oracle("s", [("v", "sum"), ("v", "count")])
    exp_w = oracle("w", [("v", "sum"), ("v", "count")])
    exp_sm = oracle("s", [("v", "sum"), ("v", "min")])
    flt = sorted((k, v) for k, v in zip(t1.column("k").to_pylist(), t1.column("v").to_pylist())
                 if k < 20)
    rows = sorted(zip(j.column("k").to_pylist(), j.column("v").to_pylist(),
                      j.column("s").to_pylist()), key=repr)
    gm = j.group_by(["w", "s"]).aggregate([("v", "sum")])
    exp_multi = sorted(zip(gm.column("w").to_pylist(), gm.column("s").to_pylist(),
                           gm.column("v_sum").to_pylist()), key=repr)
    gk = j.group_by("k").aggregate([("v", "sum")])
    exp_topk = sorted(zip(gk.column("k").to_pylist(), gk.column("v_sum").to_pylist()),
                      key=lambda x: (-x[1], x[0]))[:5]
    t2f = t2.filter(pa.compute.less(t2.column("w"), 3))
    lo = t1.join(t2f, "k", join_type="left outer")
    exp_lo = sorted(zip(lo.column("k").to_pylist(), lo.column("w").to_pylist()), key=repr)

    def close(a, b):
        assert len(a) == len(b), (len(a), len(b))
        for x, y in zip(a, b):
            for u, v in zip(x, y):
                assert (abs(u - v) <= 1e-9 * max(1.0, abs(v))) if isinstance(v, float) else u == v
    jf = t2.join(t1, "k", join_type="inner")
    gf = jf.group_by(["k", "v"]).aggregate([("w", "sum")])
    exp_fd = sorted(zip(gf.column("k").to_pylist(), gf.column("v").to_pylist(),
                        gf.column("w_sum").to_pylist()), key=lambda x: (-x[2], x[0]))[:5]
    k3 = set(range(0, 200, 3))
    exp_semi = [(sum(2 * k for k in k3), len(k3))]
    for d in res:
        assert d["paths"] == ["native"] * 10, d["paths"]
        assert [tuple(x) for x in d["semi_keys"]] == exp_semi
        assert d["semi_exchange"] == "keys"
        assert [tuple(x) for x in d["fd_topk"]] == exp_fd
        assert [tuple(x) for x in d["nonindex_join"]] == exp_s
        assert [tuple(x) for x in d["join_w"]] == exp_w
        assert [tuple(x) for x in d["join_s"]] == exp_sm
        assert sorted((tuple(x) for x in d["filter"]), key=repr) == sorted(flt, key=repr)
        assert "Name: i1" in d["join_w_plan"]
        close(sorted((tuple(x) for x in d["join_rows"]), key=repr), rows)
        close(sorted((tuple(x) for x in d["join_multi"]), key=repr), exp_multi)
        close([tuple(x) for x in d["topk"]], exp_topk)
        assert sorted((tuple(x) for x in d["left_outer"]), key=repr) == exp_lo
        assert d["steady_object_collectives"] == 0


def test_bench_two_ranks_reports_both_placements(tmp_path):
    """bench.py under torch.distributed (2 gloo ranks, host engine, tiny scale factor): one JSON
    line from rank 0 with the sharded (strong scaling: one query stream over co-partitioned
    buckets, the same placement and label as at N = 1) headline value and the replicated numbers
    (weak scaling: one query stream per rank over read replicas) as a side key, and the indexed
    results cross-checked against the un-indexed plan."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(29000 + os.getpid() % 2000),
           os.path.join(root, "bench.py"), "--gpus", "2", "--device", "cpu", "--sf", "0.02",
           "--steps", "2", "--warmup", "1", "--buckets", "4", "--data-dir", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["config"]["placement"] == "sharded" and out["scaling"] == "strong"
    assert out["config"]["parallelism"] == "cpu-host"
    assert out["replicated"]["scaling"] == "weak" and out["replicated"]["value"] > 0
    assert "bytes_over_xgmi" in out
    assert out["steps"] == 2 and out["crosscheck"]["index_vs_full_scan_match"]


def _check_nccl_paths(res, world):
    total = 0
    for r, d in enumerate(res):
        assert d["allreduce"] == sum(1.0 + k for k in range(world))
        assert d["agree"] == [True, False] and d["max"] == float(world - 1)
        assert d["xch_owner_ok"] and d["xch_f_ok"] and d["xch_valid_ok"]
        assert d["dict"] == sorted({f"k{k}" for k in range(world)} | {"shared"} |
                                   {f"x{k * 7}" for k in range(world)})
        s, c, mn, mx = d["combine"]
        assert s == [1.5 * world, 2.5 * world] and c == [world, 2 * world]
        assert mn == [0.0, 0.0] and mx == [float(world - 1), 9.0]
        total += d["xch_rows"]
    assert total == sum(100_000 + 1234 * k for k in range(world))


@pytest.mark.gpu
def test_rccl_branches_single_rank(tmp_path, device):
    """The nccl (RCCL) branches of parallel/dist.py, exchange.py and dictionary.py on a
    world-size-1 RCCL process group: runs on any 1-GPU MI355X box."""
    res = _spawn("nccl_paths", tmp_path, str(tmp_path), world=1, backend="nccl", timeout=300)
    _check_nccl_paths(res, 1)


@pytest.mark.gpu
def test_warm_sharded_queries_submit_without_host_syncs(tmp_path, spmd_data, device):
    """A warm sharded query (plan-cache hit of the indexed filter / join aggregate, the 3-way
    join with a key semi-join, and the grouped-by-key ORDER BY / LIMIT shape over an RCCL
    process group) submits with no host synchronization; reading its result is the one wait
    (torch's sync debug mode plus wrapped stream / event / device waits count them)."""
    data, t1, t2 = spmd_data
    res = _spawn("sync_count", tmp_path, str(data), world=1, backend="nccl", timeout=300)
    d = res[0]
    print({q: d[q] for q in ("filter", "join", "join3", "full")}, d.get("semi"),
          d.get("submit_syncs"), d.get("read_syncs"))
    for q in ("filter", "join", "join3", "full"):
        for submit, read, path, rows in d[q]:
            assert path == "native" and rows > 0, (q, d[q])
            assert submit == 0, (q, d)
            if q != "full":     # the top-k result's key lookup reads back after the wait
                assert read <= 1, (q, d)


def _gpu_count() -> int:
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001
        return 0


@pytest.mark.gpu
@pytest.mark.skipif(_gpu_count() < 2, reason="needs >= 2 GPUs (one rank per device id)")
def test_rccl_two_devices(tmp_path, spmd_data):
    """Two ranks on two device ids over RCCL: the packed exchange and collectives, then the
    device build (batched all-to-all), bucket-owner filter and co-located join — runs unchanged
    whenever torch.cuda.device_count() >= 2."""
    res = _spawn("nccl_paths", tmp_path, str(tmp_path), world=2, backend="nccl", timeout=300)
    _check_nccl_paths(res, 2)
    data, t1, t2 = spmd_data
    res = _spawn("spmd_gpu", tmp_path, str(data), world=2, backend="nccl", timeout=600)
    j = t1.join(t2, "k", join_type="inner")
    g = j.group_by("w").aggregate([("v", "sum"), ("v", "count")])
    exp_w = sorted(zip(g.column("w").to_pylist(), g.column("v_sum").to_pylist(),
                       g.column("v_count").to_pylist()))
    flt = sorted((k, v) for k, v in zip(t1.column("k").to_pylist(), t1.column("v").to_pylist())
                 if k < 20)
    for d in res:
        assert d["paths"] == ["native"] * 4, d["paths"]
        assert [tuple(x) for x in d["join_w"]] == exp_w
        assert sorted((tuple(x) for x in d["filter"]), key=repr) == sorted(flt, key=repr)


@pytest.mark.gpu
def test_multi_rank_streaming_build_writes_same_files(tmp_path, device):
    """Two ranks (gloo, sharing cuda:0): a build forced into bucket-range passes under a tiny
    HBM budget writes the same bucket files as the one-pass multi-rank build: the same rows in
    the same order, row groups and schema (CreateActionBase.scala:129-130).
    Files are compared decoded: the device writer picks dictionary vs PLAIN per column from the
    distinct values of the buckets one encode call covers, so a column with many distinct values
    overall but few per bucket is PLAIN in the one-pass files and dictionary-encoded in the
    one-bucket passes (both lossless)."""
    rng = np.random.default_rng(3)
    src = tmp_path / "data" / "src"
    src.mkdir(parents=True)
    for i in range(6):
        n = 30_000 + 1_000 * i
        t = pa.table({"k": pa.array(rng.integers(0, 4_000, n)),
                      "d": pa.array(rng.integers(8000, 11000, n).astype(np.int32)),
                      "p": pa.array(np.round(rng.random(n) * 1e4, 2)),
                      "q": pa.array(np.where(rng.random(n) < 0.1, None,
                                             rng.integers(0, 50, n)).tolist(), pa.int64())})
        pq.write_table(t, src / f"part-{i}.parquet", row_group_size=16_000)
    res = _spawn("spmd_stream_build", tmp_path, str(tmp_path / "data"), timeout=600.0)
    assert res[0]["one_pass"]["passes"] is None
    assert res[0]["streamed"]["passes"] >= 2, res

    def files(name):
        out = {}
        for root, _, fs in os.walk(tmp_path / "data" / "ix" / name):
            for f in fs:
                if f.endswith(".parquet"):
                    out[get_bucket_id(f)] = open(os.path.join(root, f), "rb").read()
        return out
    one, many = files("one_pass"), files("streamed")
    assert sorted(one) == sorted(many) and len(one) == 16
    bad = []
    for b in one:
        fx, fy = pq.ParquetFile(pa.BufferReader(one[b])), pq.ParquetFile(pa.BufferReader(many[b]))
        same = fx.read().equals(fy.read()) and fx.schema_arrow.equals(fy.schema_arrow) and \
            [fx.metadata.row_group(g).num_rows for g in range(fx.num_row_groups)] == \
            [fy.metadata.row_group(g).num_rows for g in range(fy.num_row_groups)]
        if not same:
            bad.append(b)
    assert not bad, (bad, [r["one_pass"] for r in res], [r["streamed"] for r in res])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_balanced_owner_map_routes_rows(tmp_path, world):
    """The packed all-to-all routes every row to its bucket's owner under a size-balanced map
    (parallel/placement.py): the heavy bucket's owner holds no other bucket."""
    res = _spawn("balanced_exchange", tmp_path, str(tmp_path), world=world)
    owners = res[0]["owners"]
    assert all(d["owners"] == owners for d in res)
    heavy = owners[0]
    assert owners.count(heavy) == 1
    for r, d in enumerate(res):
        assert all(owners[b] == r for b in d["recv_buckets"])
        expect = []
        for src in res:
            expect += [v for v, b in zip(src["sent"], src["sent_b"]) if owners[b] == r]
        assert d["recv"] == expect


@pytest.fixture
def skew_data(tmp_path):
    rng = np.random.default_rng(9)
    data = tmp_path / "data"
    k1 = np.concatenate([np.full(6000, 7, np.int64), rng.integers(0, 400, 4000)])
    t1 = pa.table({"k": k1, "v": np.arange(len(k1), dtype=np.int64)})
    k2 = np.arange(400, dtype=np.int64)
    t2 = pa.table({"k": k2, "w": (k2 % 6).astype(np.int32)})
    # s3: 70% of the rows in one bucket of 16 (many distinct keys < 400), the rest spread
    from hyperspace_amd.utils import murmur3
    cand = np.arange(400, dtype=np.int64)
    bid = np.asarray(murmur3.bucket_ids([pa.array(cand)], 16))
    hot = cand[bid == 5]
    k3 = np.concatenate([np.repeat(hot, 7000 // len(hot) + 1)[:7000],
                         rng.integers(0, 400, 3000)])
    t3 = pa.table({"k": k3, "v": np.arange(len(k3), dtype=np.int64)})
    for name, t, parts in (("s1", t1, 4), ("s2", t2, 2), ("s3", t3, 4)):
        os.makedirs(data / name)
        step = (t.num_rows + parts - 1) // parts
        for i in range(parts):
            pq.write_table(t.slice(i * step, step), data / name / f"part-{i}.parquet")
    return data, t1, t2


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_heavy_bucket_cut_into_key_ranges(tmp_path, skew_data, device, world):
    """A bucket holding 70% of the rows over many keys is cut into key ranges on distinct ranks
    (parallel/placement.py split_heavy); the co-located join aggregate and a filter aggregate
    return the modulo placement's (and the oracle's) result, and every rank's resident rows of
    the cut bucket lie in its range."""
    data, _, t2 = skew_data
    t3 = pq.read_table(data / "s3")
    res = _spawn("spmd_split", tmp_path, str(data), timeout=600.0, world=world)
    j = t3.join(t2, "k", join_type="inner")
    g = j.group_by("w").aggregate([("v", "sum"), ("v", "count")])
    exp = sorted(zip(g.column("w").to_pylist(), g.column("v_sum").to_pylist(),
                     g.column("v_count").to_pylist()))
    for d in res:
        assert d["paths"] == ["native"] * 4, d["paths"]
        assert d["modulo"] == d["balanced"]
        assert [tuple(x) for x in d["balanced"]["agg"]] == exp
        assert d["modulo_splits"] == {}
        sp = d["balanced_splits"]
        assert "5" in sp and len(sp["5"][0]) == len(set(sp["5"][0])) >= 2, sp
        assert d["cut_rows_in_range"]
    assert sum(1 for d in res if "5" in d["cuts"]) == len(res[0]["balanced_splits"]["5"][0])


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_balanced_placement_matches_modulo_on_skewed_key(tmp_path, skew_data, device, world):
    """Ranks share cuda:0 (gloo): a skewed join key (60% of the rows on one key) gives one
    heavy bucket; the size-balanced placement gives it a rank of its own, and every query
    (co-located join aggregate, join rows, filter) returns exactly the modulo placement's result
    and the pyarrow oracle's."""
    data, t1, t2 = skew_data
    res = _spawn("spmd_skew", tmp_path, str(data), timeout=600.0, world=world)
    j = t1.join(t2, "k", join_type="inner")
    g = j.group_by("w").aggregate([("v", "sum"), ("v", "count")])
    exp = sorted(zip(g.column("w").to_pylist(), g.column("v_sum").to_pylist(),
                     g.column("v_count").to_pylist()))
    for d in res:
        assert d["paths"] == ["native"] * 6, d["paths"]
        assert d["modulo"] == d["balanced"]
        assert [tuple(x) for x in d["balanced"]["agg"]] == exp
        assert d["modulo_owners"] == [b % world for b in range(8)]
        ow = d["balanced_owners"]
        assert ow != d["modulo_owners"]
        from hyperspace_amd.utils import murmur3
        heavy = int(murmur3.bucket_ids([pa.array([7], pa.int64())], 8)[0])
        assert ow.count(ow[heavy]) == 1          # the hot key's bucket alone on its rank
