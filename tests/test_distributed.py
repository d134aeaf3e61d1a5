"""Multi-process tests (world_size 2, gloo on 127.0.0.1) for the SPMD paths: collectives and the
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


def _spawn(scenario: str, tmp_path, data_dir: str, timeout: float = 240.0):
    import dist_workers
    out = tmp_path / f"out_{scenario}"
    out.mkdir()
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=dist_workers.run,
                         args=(r, WORLD, port, scenario, str(out), data_dir)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout)
    alive = [p for p in procs if p.is_alive()]
    for p in alive:
        p.kill()
        p.join()
    assert not alive, f"{scenario}: ranks hung"
    res = []
    for r in range(WORLD):
        with open(out / f"rank{r}.json") as f:
            d = json.load(f)
        assert "error" not in d, d["error"]
        res.append(d)
    return res


def test_collectives_and_all_to_all_exchange(tmp_path):
    res = _spawn("collectives", tmp_path, str(tmp_path))
    for d in res:
        assert d["sums"] == [1.0 + 2.0, 4.0]
        assert d["cnts"] == [2, 1]
        assert d["mins"] == [0.0, 5.0] and d["maxs"] == [1.0, -1.0]
        assert d["objs"] == [{"r": 0}, {"r": 1}]
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
    for name, t, parts in (("t1", t1, 3), ("t2", t2, 2)):
        os.makedirs(data / name)
        step = (t.num_rows + parts - 1) // parts
        for i in range(parts):
            pq.write_table(t.slice(i * step, step), data / name / f"part-{i}.parquet")
    return data, t1, t2


def test_spmd_index_lifecycle_and_queries(tmp_path, spmd_data):
    data, t1, t2 = spmd_data
    res = _spawn("spmd_index", tmp_path, str(data))
    # the index data: one file per bucket overall, each written by its owner rank, rows complete
    vdir = data / "indexes" / "i1" / "v__=0"
    files = sorted(f for f in os.listdir(vdir) if f.endswith(".parquet"))
    buckets = [get_bucket_id(f) for f in files]
    assert len(buckets) == len(set(buckets)), files
    for f in files:
        task = int(f.split("-")[1])
        assert task == get_bucket_id(f) % WORLD, f
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
    assert res[0]["one_rank_fault"] == "HyperspaceException"
    assert res[1]["one_rank_fault"] == "FaultInjected"
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
    for d in res:
        assert d["paths"] == ["native"] * 4, d["paths"]
        assert [tuple(x) for x in d["nonindex_join"]] == exp_s
        assert [tuple(x) for x in d["join_w"]] == exp_w
        assert [tuple(x) for x in d["join_s"]] == exp_sm
        assert [tuple(x) for x in d["filter"]] == flt
        assert "Name: i1" in d["join_w_plan"]


def test_bench_two_ranks_reports_both_placements(tmp_path):
    """bench.py under torch.distributed (2 gloo ranks, host engine, tiny scale factor): one JSON
    line from rank 0 with the replicated (weak-scaling) value and the sharded numbers, and the
    indexed results cross-checked against the un-indexed plan."""
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
    assert out["config"]["placement"] == "replicated" and out["scaling"] == "weak"
    assert out["sharded"]["scaling"] == "strong" and out["sharded"]["value"] > 0
    assert out["steps"] == 2 and out["crosscheck"]["index_vs_full_scan_match"]
