"""End-to-end: index build + indexed queries through the MI355X executor, checked against the
host oracle (the reference's disabled-vs-enabled pattern, E2EHyperspaceRulesTest.scala:1004-1019).
GPU-only; asserts the HIP path actually ran (no silent fallback)."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_, avg, max_, min_

pytestmark = pytest.mark.gpu


@pytest.fixture
def tpch(tmp_path, device):
    rng = np.random.default_rng(7)
    n_ord = 40_000
    okeys = rng.permutation(np.arange(1, n_ord + 1, dtype=np.int64) * 4)
    od = pa.table({"o_orderkey": okeys,
                   "o_orderdate": pa.array(rng.integers(8000, 10500, n_ord).astype(np.int32)).view(pa.date32()),
                   "o_priority": pa.array([f"{k}-PRI" for k in rng.integers(1, 6, n_ord)]),
                   "o_shippriority": rng.integers(0, 3, n_ord).astype(np.int32)})
    lk = np.repeat(okeys, rng.integers(1, 8, n_ord))
    n = len(lk)
    li = pa.table({"l_orderkey": lk,
                   "l_quantity": rng.integers(1, 51, n).astype(np.float64),
                   "l_extendedprice": np.round(rng.random(n) * 1e5, 2),
                   "l_discount": rng.integers(0, 11, n) / 100.0,
                   "l_shipdate": pa.array(rng.integers(8000, 10600, n).astype(np.int32)).view(pa.date32()),
                   "l_returnflag": pa.array(rng.choice(["A", "N", "R"], n))})
    for name, t, parts in (("lineitem", li, 5), ("orders", od, 3)):
        os.makedirs(tmp_path / name)
        step = (t.num_rows + parts - 1) // parts
        for i in range(parts):
            pq.write_table(t.slice(i * step, step), tmp_path / name / f"part-{i}.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "16",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.sql.shuffle.partitions": "8",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=str(tmp_path / "wh"))
    return s, str(tmp_path / "lineitem"), str(tmp_path / "orders")


def _both(s, df, sort=True):
    s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
    g = df.to_arrow()
    path = s.backend().last_path
    s.conf.set("spark.hyperspace.mi.execution.device", "cpu")
    c = df.to_arrow()
    s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
    if sort and g.num_rows:
        keys = [(n, "ascending") for n in g.column_names]
        g = g.sort_by(keys)
        c = c.sort_by(keys)
    return g, c, path


def _close(g: pa.Table, c: pa.Table):
    assert g.num_rows == c.num_rows, (g.num_rows, c.num_rows)
    for a, b in zip(g.columns, c.columns):
        av, bv = a.to_pylist(), b.to_pylist()
        for x, y in zip(av, bv):
            if isinstance(x, float) and isinstance(y, float):
                assert abs(x - y) <= 1e-6 * max(1.0, abs(y)), (x, y)
            else:
                assert x == y, (x, y)


def test_device_build_matches_host_build(tpch, tmp_path):
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    hs.createIndex(li, IndexConfig("li_ok", ["l_orderkey"], ["l_extendedprice", "l_returnflag"]))
    s.conf.set("spark.hyperspace.mi.execution.device", "cpu")
    s.conf.set("spark.hyperspace.system.path", str(tmp_path / "idx_cpu"))
    hs.createIndex(li, IndexConfig("li_ok", ["l_orderkey"], ["l_extendedprice", "l_returnflag"]))
    from hyperspace_amd.io.writer import get_bucket_id
    def load(root):
        out = {}
        vdir = os.path.join(root, "li_ok", "v__=0")
        for f in os.listdir(vdir):
            out[get_bucket_id(f)] = pq.read_table(os.path.join(vdir, f))
        return out
    g, c = load(str(tmp_path / "idx")), load(str(tmp_path / "idx_cpu"))
    assert g.keys() == c.keys()
    for b in g:
        assert g[b].column("l_orderkey").to_pylist() == c[b].column("l_orderkey").to_pylist()
        assert np.allclose(g[b].column("l_extendedprice").to_numpy(),
                           c[b].column("l_extendedprice").to_numpy())
        # included string column: dictionary pages + device remap (device_build._dictionary_codes)
        assert g[b].column("l_returnflag").cast(pa.string()).to_pylist() == \
            c[b].column("l_returnflag").cast(pa.string()).to_pylist()


def test_q6_filter_aggregate_native(tpch):
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    hs.createIndex(li, IndexConfig("li_ship", ["l_shipdate"],
                                   ["l_discount", "l_quantity", "l_extendedprice"]))
    Hyperspace.enable(s)
    q = li.filter("l_shipdate >= DATE '1994-01-01' AND l_shipdate < DATE '1995-01-01' AND "
                  "l_discount >= 0.05 AND l_discount <= 0.07 AND l_quantity < 24") \
        .agg(sum_(col("l_extendedprice") * col("l_discount")).alias("revenue"), count("*").alias("n"))
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    assert "Hyperspace(Type: CI, Name: li_ship" in q.queryExecution.executed_plan.tree_string()


def test_q6_graph_replays_with_new_literals(tpch):
    """The captured hipGraph of the scan pipeline replays with each query's literals."""
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    hs.createIndex(li, IndexConfig("li_ship", ["l_shipdate"],
                                   ["l_discount", "l_quantity", "l_extendedprice"]))
    Hyperspace.enable(s)
    backend = s.backend()
    for year, disc, qty in ((1994, 0.06, 24), (1995, 0.03, 25), (1993, 0.09, 24),
                            (1994, 0.06, 24), (1997, 0.05, 30)):
        q = li.filter(f"l_shipdate >= DATE '{year}-01-01' AND l_shipdate < DATE '{year + 1}-01-01'"
                      f" AND l_discount >= {disc - 0.01:.2f} AND l_discount <= {disc + 0.01:.2f}"
                      f" AND l_quantity < {qty}") \
            .agg(sum_(col("l_extendedprice") * col("l_discount")).alias("revenue"),
                 count("*").alias("n"), max_("l_quantity").alias("mq"))
        g, c, path = _both(s, q, sort=False)
        assert path == "native", s.backend().fallback_reason
        _close(g, c)
    assert len(backend.graphs) == 1
    graph = next(iter(backend.graphs._lru.values()))
    assert graph.replays >= 3
    # disabling graphs runs the eager launch sequence with identical results
    s.conf.set("spark.hyperspace.mi.hipGraph.enabled", "false")
    g2, c2, _ = _both(s, q, sort=False)
    _close(g2, c2)
    _close(g2, g)


def test_side_stream_scans_pipelined_with_joins(tpch):
    """Warm scan pipelines replay on the engine's side stream while merge joins queue on the
    query stream (several queries in flight, fresh literals each): every result equals the
    same query run with side-stream scans off, one at a time."""
    s, lpath, opath = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    od = s.read.parquet(opath)
    hs.createIndex(li, IndexConfig("li_ship2", ["l_shipdate"],
                                   ["l_discount", "l_quantity", "l_extendedprice"]))
    hs.createIndex(li, IndexConfig("li_ok2", ["l_orderkey"],
                                   ["l_extendedprice", "l_discount", "l_shipdate"]))
    hs.createIndex(od, IndexConfig("od_ok2", ["o_orderkey"], ["o_orderdate", "o_shippriority"]))
    Hyperspace.enable(s)
    s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "false")

    def q6(i):
        y = 1993 + i % 5
        return li.filter(f"l_shipdate >= DATE '{y}-01-01' AND l_shipdate < DATE '{y + 1}-01-01'"
                         f" AND l_discount >= 0.0{i % 5 + 1} AND l_quantity < {20 + i % 7}") \
            .agg(sum_(col("l_extendedprice") * col("l_discount")).alias("revenue"))

    def q3(i):
        dd = f"1995-03-{10 + i % 15:02d}"
        return li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
            .filter(f"o_orderdate < DATE '{dd}' AND l_shipdate > DATE '{dd}'") \
            .groupBy("o_shippriority").agg(sum_("l_extendedprice").alias("rev"),
                                           count("*").alias("n"))
    backend = s.backend()
    futs = []
    for i in range(10):
        futs.append((q6(i).collect_async(), q3(i).collect_async()))
    got = [(a.result(), b.result()) for a, b in futs]
    assert all(g.path == "native" for pair in futs for g in pair), backend.fallback_reason
    assert any(g.on_side for g in backend.graphs._lru.values())
    s.conf.set("spark.hyperspace.mi.sideStreamScans.enabled", "false")

    def table(rows):
        return pa.Table.from_pylist(sorted((r.asDict() for r in rows),
                                           key=lambda d: tuple(d.values())))
    for i, (g6, g3) in enumerate(got):
        _close(table(g6), table(q6(i).collect()))
        _close(table(g3), table(q3(i).collect()))


def test_two_phase_join_graph_replays_with_new_literals(tpch):
    """Plan-cache hits of the run-keyed two-phase merge join replay ONE captured hipGraph
    (graphs.TwoPhaseGraph: params H2D, tags, bits scan, final fold, D2H) with each query's
    literals - ungrouped and grouped by a right-side key, several queries in flight - equal to
    the host oracle and to the eager launches (hipGraph off)."""
    s, lpath, opath = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    od = s.read.parquet(opath)
    hs.createIndex(li, IndexConfig("li_ok3", ["l_orderkey"],
                                   ["l_extendedprice", "l_discount", "l_shipdate"]))
    hs.createIndex(od, IndexConfig("od_ok3", ["o_orderkey"], ["o_orderdate", "o_shippriority"]))
    Hyperspace.enable(s)
    s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "false")

    def q(i, grouped):
        dd = f"1995-03-{1 + (i * 7) % 28:02d}"
        j = li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
            .filter(f"o_orderdate < DATE '{dd}' AND l_shipdate > DATE '{dd}'")
        aggs = (sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("rev"),
                count("*").alias("n"))
        return j.groupBy("o_shippriority").agg(*aggs) if grouped else j.agg(*aggs)
    from hyperspace_amd.exec import jit_runs
    backend = s.backend()
    for grouped in (False, True):
        futs = [q(i, grouped).collect_async() for i in range(8)]
        got = [f.result() for f in futs]
        assert all(f.path == "native" for f in futs), backend.fallback_reason
        preps = [pr for pr in backend._agg_preps.values()
                 if isinstance(getattr(pr, "launcher", None), jit_runs.TwoPhaseLauncher)]
        assert preps and any(pr.launcher.graph is not None and pr.launcher.graph.replays >= 4
                             for pr in preps), "two-phase join did not replay a graph"
        # plan-cache hits with a known literal vector take the prepared program (no plan walk)
        futs = [q(i, grouped).collect_async() for i in range(8)]
        again = [f.result() for f in futs]
        assert any(pg[1].n > 0 for pg in backend._programs.values()), "no prepared submission"
        for a, b in zip(again, got):    # same literals: equal up to summation order
            _close(pa.Table.from_pylist(sorted((r.asDict() for r in a), key=lambda d: tuple(d.values()))),
                   pa.Table.from_pylist(sorted((r.asDict() for r in b), key=lambda d: tuple(d.values()))))
        s.conf.set("spark.hyperspace.mi.execution.device", "cpu")
        want = [q(i, grouped).collect() for i in range(8)]
        s.conf.set("spark.hyperspace.mi.hipGraph.enabled", "false")
        s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
        eager = [q(i, grouped).collect() for i in range(8)]
        s.conf.set("spark.hyperspace.mi.hipGraph.enabled", "true")

        def table(rows):
            return pa.Table.from_pylist(sorted((r.asDict() for r in rows),
                                               key=lambda d: tuple(d.values())))
        for a, b, c in zip(got, want, eager):
            _close(table(a), table(b))
            _close(table(c), table(b))


def test_side_stream_scan_survives_table_eviction(tpch):
    """A warm scan pipeline replays on the side stream; the device cache then drops the table
    (and with it the compact codes the generated kernel reads) before the result is fetched,
    and the query stream reuses that memory at once.  The replay must still read the old codes:
    every buffer whose pointer is in the args block is marked in use by the side stream
    (ADVICE r3)."""
    import torch
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    hs.createIndex(li, IndexConfig("li_ship_ev", ["l_shipdate"],
                                   ["l_discount", "l_quantity", "l_extendedprice"]))
    Hyperspace.enable(s)

    def q6(i):
        y = 1993 + i % 5
        return li.filter(f"l_shipdate >= DATE '{y}-01-01' AND l_shipdate < DATE '{y + 1}-01-01'"
                         f" AND l_quantity < {20 + i % 7}") \
            .agg(sum_(col("l_extendedprice") * col("l_discount")).alias("revenue"),
                 count("*").alias("n"))
    backend = s.backend()
    want = [q6(i).collect() for i in range(4)]      # warm: later replays go to the side stream
    for i in range(4):
        f = q6(i).collect_async()
        backend.cache.clear()                       # drops the table's last references
        junk = [torch.full((1 << 22,), -7, dtype=torch.int32, device="cuda") for _ in range(16)]
        got = f.result()
        del junk
        assert f.path == "native", backend.fallback_reason
        assert got[0][1] == want[i][0][1]
        assert abs(got[0][0] - want[i][0][0]) <= 1e-9 * abs(want[i][0][0])
    assert any(g.on_side for g in backend.graphs._lru.values())


def test_filter_rows_and_group_by_native(tpch):
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    hs.createIndex(li, IndexConfig("li_ship", ["l_shipdate"],
                                   ["l_discount", "l_quantity", "l_returnflag"]))
    Hyperspace.enable(s)
    q = li.filter("l_shipdate = DATE '1995-03-01'").select("l_shipdate", "l_discount", "l_returnflag")
    g, c, path = _both(s, q)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    q2 = li.filter("l_shipdate > DATE '1996-01-01' AND l_returnflag = 'R'") \
        .groupBy("l_returnflag").agg(sum_("l_quantity").alias("q"), avg("l_discount").alias("d"),
                                      min_("l_quantity").alias("mn"), max_("l_shipdate").alias("mx"))
    g, c, path = _both(s, q2)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    q3 = li.filter("l_shipdate < DATE '1993-01-01'").groupBy("l_quantity").agg(count("*").alias("c"))
    g, c, path = _both(s, q3)
    assert path == "native", s.backend().fallback_reason   # float key: hash-mode aggregate
    _close(g, c)


def test_join_index_aggregate_and_rows_native(tpch):
    s, lpath, opath = tpch
    hs = Hyperspace(s)
    li, od = s.read.parquet(lpath), s.read.parquet(opath)
    hs.createIndex(li, IndexConfig("li_ok", ["l_orderkey"], ["l_extendedprice", "l_discount", "l_shipdate"]))
    hs.createIndex(od, IndexConfig("ord_ok", ["o_orderkey"], ["o_orderdate", "o_shippriority"]))
    Hyperspace.enable(s)
    j = li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
        .filter("o_orderdate < DATE '1995-03-15' AND l_shipdate > DATE '1995-03-15'")
    q = j.groupBy("o_shippriority").agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("rev"),
                                       count("*").alias("n"))
    plan = q.queryExecution.executed_plan.tree_string()
    assert "Exchange hashpartitioning(l_orderkey" not in plan and "Sort [" not in plan
    g, c, path = _both(s, q)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    rows = j.select("l_orderkey", "l_extendedprice", "o_orderdate")
    g, c, path = _both(s, rows)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)


def test_non_index_join_device_shuffle(tpch):
    s, lpath, opath = tpch
    li, od = s.read.parquet(lpath), s.read.parquet(opath)
    q = li.join(od, li["l_orderkey"] == od["o_orderkey"]).filter("o_shippriority = 1") \
        .agg(sum_("l_quantity").alias("q"), count("*").alias("n"))
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)


def test_hybrid_scan_join_and_filter_on_device(tpch, tmp_path):
    """BASELINE config #4 shape: indexes + appended Parquet files, served by Hybrid Scan on
    the device (BucketUnion parts joined pairwise; appended rows shuffled on the GPU)."""
    s, lpath, opath = tpch
    for k, v in (("lineage.enabled", "true"), ("hybridscan.enabled", "true"),
                 ("hybridscan.maxAppendedRatio", "0.5"), ("hybridscan.maxDeletedRatio", "0.5")):
        s.conf.set(f"spark.hyperspace.index.{k}", v)
    hs = Hyperspace(s)
    li, od = s.read.parquet(lpath), s.read.parquet(opath)
    hs.createIndex(li, IndexConfig("li_ok", ["l_orderkey"], ["l_extendedprice", "l_discount"]))
    hs.createIndex(od, IndexConfig("ord_ok", ["o_orderkey"], ["o_orderdate"]))
    hs.createIndex(li, IndexConfig("li_ship", ["l_shipdate"], ["l_discount", "l_quantity"]))
    # append ~10% new rows to both tables (fresh order keys so the join has new matches)
    t_li = pq.read_table(os.path.join(lpath, "part-0.parquet")).slice(0, 20_000)
    t_od = pq.read_table(os.path.join(opath, "part-0.parquet")).slice(0, 4_000)
    shift = 10_000_000
    t_od = t_od.set_column(0, "o_orderkey", pa.compute.add(t_od.column("o_orderkey"), shift))
    t_li = t_li.set_column(0, "l_orderkey", pa.compute.add(t_li.column("l_orderkey"), shift))
    pq.write_table(t_li, os.path.join(lpath, "part-app.parquet"))
    pq.write_table(t_od, os.path.join(opath, "part-app.parquet"))
    Hyperspace.enable(s)
    li, od = s.read.parquet(lpath), s.read.parquet(opath)
    q = li.join(od, li["l_orderkey"] == od["o_orderkey"]).filter("o_orderdate < DATE '1996-01-01'") \
        .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("rev"), count("*").alias("n"))
    plan = q.queryExecution.executed_plan.tree_string()
    assert "BucketUnion" in plan
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    q2 = li.filter("l_shipdate >= DATE '1994-01-01' AND l_shipdate < DATE '1995-01-01'") \
        .agg(sum_(col("l_quantity") * col("l_discount")).alias("r"))
    g, c, path = _both(s, q2, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    # the unions ran as merged single tables (GpuBackend._merged_union); the per-part
    # lowering gives the same answers
    assert s.backend().__dict__.get("_hybrid_unions"), s.backend().metrics.get("hybrid_merge_skip")
    s.conf.set("spark.hyperspace.mi.hybridMerge.enabled", "false")
    try:
        for qq in (q, q2):
            g2, c2, path = _both(s, qq, sort=False)
            assert path == "native", s.backend().fallback_reason
            _close(g2, c2)
    finally:
        s.conf.set("spark.hyperspace.mi.hybridMerge.enabled", "true")
    # the filter query's UNION ALL (index + appended files): per-branch fused aggregates
    # (GpuBackend._union_agg) equal the materialize-and-concatenate path
    plan2 = q2.queryExecution.executed_plan.tree_string()
    if "Union" not in plan2:
        # same-scan appended files: one resident table of the index buckets plus the appended
        # rows sorted by the key as one more range (GpuBackend._hybrid_scan); without it the
        # index files scan bucket-sorted and the appended files flat
        # (GpuBackend._mixed_index_agg); both equal one flat table of all the files
        assert s.backend().metrics.get("hybrid_scan_merged"), plan2
        s.conf.set("spark.hyperspace.mi.hybridScanMerge.enabled", "false")
        try:
            g4, c4, path = _both(s, q2, sort=False)
            assert path == "native", s.backend().fallback_reason
            assert s.backend().metrics.get("mixed_scan_agg"), plan2
            _close(g4, c4)
            _close(g4, g)
            s.conf.set("spark.hyperspace.mi.mixedScanAgg.enabled", "false")
            g3, c3, path = _both(s, q2, sort=False)
            assert path == "native", s.backend().fallback_reason
            _close(g3, c3)
            _close(g3, g)
        finally:
            s.conf.set("spark.hyperspace.mi.mixedScanAgg.enabled", "true")
            s.conf.set("spark.hyperspace.mi.hybridScanMerge.enabled", "true")
    if "Union" in plan2 and "BucketUnion" not in plan2:
        s.conf.set("spark.hyperspace.mi.unionAgg.enabled", "false")
        try:
            g3, c3, path = _both(s, q2, sort=False)
            assert path == "native", s.backend().fallback_reason
            _close(g3, c3)
            _close(g3, g)
        finally:
            s.conf.set("spark.hyperspace.mi.unionAgg.enabled", "true")


def test_incremental_refresh_with_deletes_on_device(tpch, tmp_path):
    s, lpath, _ = tpch
    s.conf.set("spark.hyperspace.index.lineage.enabled", "true")
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    hs.createIndex(li, IndexConfig("li_ok", ["l_orderkey"], ["l_quantity"]))
    os.remove(os.path.join(lpath, "part-1.parquet"))
    hs.refreshIndex("li_ok", "incremental")
    Hyperspace.enable(s)
    li2 = s.read.parquet(lpath)
    q = li2.filter("l_orderkey > 1000 AND l_orderkey < 50000").agg(sum_("l_quantity").alias("q"))
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    assert "li_ok" in q.queryExecution.executed_plan.tree_string()


def _bucket_files_sorted(index_dir: str, key: str) -> int:
    """Every bucket file of the latest version is sorted by ``key``; returns the file count."""
    vers = sorted(d for d in os.listdir(index_dir) if d.startswith("v__="))
    vdir = os.path.join(index_dir, vers[-1])
    files = [f for f in os.listdir(vdir) if f.endswith(".parquet")]
    for f in files:
        k = pq.read_table(os.path.join(vdir, f), columns=[key]).column(key).to_numpy()
        assert np.all(k[:-1] <= k[1:]), f
    return len(files)


def test_delete_only_rewrite_is_sort_free_and_sorted(tpch, tmp_path):
    from hyperspace_amd.exec import device_build
    s, lpath, _ = tpch
    s.conf.set("spark.hyperspace.index.lineage.enabled", "true")
    hs = Hyperspace(s)
    hs.createIndex(s.read.parquet(lpath), IndexConfig("li_ok", ["l_orderkey"], ["l_quantity"]))
    os.remove(os.path.join(lpath, "part-3.parquet"))
    hs.refreshIndex("li_ok", "incremental")
    # one file per bucket + deletes only: the stable device compaction keeps the sorted order
    assert device_build.LAST_BUILD_STATS.get("rewrite_presorted") is True
    assert _bucket_files_sorted(str(tmp_path / "idx" / "li_ok"), "l_orderkey") <= 16
    Hyperspace.enable(s)
    q = s.read.parquet(lpath).filter("l_orderkey > 0").agg(sum_("l_quantity").alias("q"),
                                                           count("*").alias("n"))
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)


def test_optimize_full_on_device_merges_bucket_files(tpch, tmp_path):
    from hyperspace_amd.exec import device_build
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    hs.createIndex(s.read.parquet(lpath), IndexConfig("li_ok", ["l_orderkey"], ["l_quantity"]))
    rng = np.random.default_rng(3)
    extra = pa.table({"l_orderkey": rng.integers(1, 160_000, 3000).astype(np.int64),
                      "l_quantity": rng.integers(1, 51, 3000).astype(np.float64),
                      "l_extendedprice": np.round(rng.random(3000) * 1e5, 2),
                      "l_discount": rng.integers(0, 11, 3000) / 100.0,
                      "l_shipdate": pa.array(rng.integers(8000, 10600, 3000).astype(np.int32))
                      .view(pa.date32()),
                      "l_returnflag": pa.array(rng.choice(["A", "N", "R"], 3000))})
    pq.write_table(extra, os.path.join(lpath, "part-9.parquet"))
    hs.refreshIndex("li_ok", "incremental")       # appended rows: a second file per bucket
    hs.optimizeIndex("li_ok", "full")
    assert device_build.LAST_BUILD_STATS.get("rewrite_presorted") is False
    # K6: the bucket's two sorted files are merged (merge path), not radix re-sorted
    assert device_build.LAST_BUILD_STATS.get("rewrite_sort") == "merge-path"
    assert _bucket_files_sorted(str(tmp_path / "idx" / "li_ok"), "l_orderkey") <= 16
    Hyperspace.enable(s)
    q = s.read.parquet(lpath).filter("l_orderkey > 0").agg(sum_("l_quantity").alias("q"),
                                                           count("*").alias("n"))
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    assert "li_ok" in q.queryExecution.executed_plan.tree_string()


def test_selective_dimension_join_probes_key_runs(tmp_path, device):
    """A fact index joined with a dimension filtered down to a few keys: the executor probes
    the fact index's key runs (hs_probe_ranges) instead of scanning it, and the rows match the
    host oracle."""
    rng = np.random.default_rng(11)
    n_item, n_fact = 20_000, 1_500_000
    item = pa.table({"i_sk": np.arange(n_item, dtype=np.int64),
                     "i_manu": rng.integers(0, 500, n_item).astype(np.int32)})
    fact = pa.table({"s_item": rng.integers(0, n_item, n_fact).astype(np.int64),
                     "s_date": rng.integers(0, 365, n_fact).astype(np.int32),
                     "s_price": np.round(rng.random(n_fact) * 100, 2)})
    for name, t, parts in (("item", item, 2), ("fact", fact, 4)):
        os.makedirs(tmp_path / name)
        step = (t.num_rows + parts - 1) // parts
        for i in range(parts):
            pq.write_table(t.slice(i * step, step), tmp_path / name / f"p{i}.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "16",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.hyperspace.mi.execution.device": "gpu"})
    hs = Hyperspace(s)
    f, it = s.read.parquet(str(tmp_path / "fact")), s.read.parquet(str(tmp_path / "item"))
    hs.createIndex(f, IndexConfig("f_item", ["s_item"], ["s_date", "s_price"]))
    hs.createIndex(it, IndexConfig("i_idx", ["i_sk"], ["i_manu"]))
    Hyperspace.enable(s)
    sel = it.filter(col("i_manu") == 7)
    q = f.join(sel, f["s_item"] == sel["i_sk"]).select(f["s_date"], f["s_price"], sel["i_sk"])
    g, c, path = _both(s, q)
    assert path == "native", s.backend().fallback_reason
    assert 0 < getattr(s.backend(), "last_join_probes", 0) <= n_item
    _close(g, c)
    assert g.num_rows == c.num_rows > 0


def test_join_key_domain_pruning_matches_oracle(tmp_path, device):
    """The right side's join keys cover only the top of the left's key domain (as appended
    orders do in a Hybrid Scan): the left ranges are cut to that domain before the join, and
    the aggregate and the rows still match the host oracle."""
    rng = np.random.default_rng(5)
    n = 1_200_000
    left = pa.table({"k": rng.integers(0, 1_000_000, n).astype(np.int64),
                     "v": np.round(rng.random(n) * 10, 2)})
    right = pa.table({"rk": np.arange(900_000, 1_100_000, dtype=np.int64),
                      "w": rng.integers(0, 5, 200_000).astype(np.int32)})
    for name, t in (("l", left), ("r", right)):
        os.makedirs(tmp_path / name)
        pq.write_table(t, tmp_path / name / "p0.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "16",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.hyperspace.mi.execution.device": "gpu"})
    hs = Hyperspace(s)
    lt, rt = s.read.parquet(str(tmp_path / "l")), s.read.parquet(str(tmp_path / "r"))
    hs.createIndex(lt, IndexConfig("l_k", ["k"], ["v"]))
    hs.createIndex(rt, IndexConfig("r_k", ["rk"], ["w"]))
    Hyperspace.enable(s)
    j = lt.join(rt, lt["k"] == rt["rk"])
    q = j.agg(sum_(col("v")).alias("s"), count("*").alias("n"))
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    rows = j.filter(col("w") == 3).select(lt["k"], lt["v"])
    g, c, path = _both(s, rows)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)


def test_first_query_after_build_uses_the_build_hbm_columns(tpch):
    """The device build's sorted bucket-major columns seed the device table cache: the first
    query of a new index reads no index file back (cold latency), and is exact."""
    from hyperspace_amd.exec import device_cache as DC
    s, lpath, _ = tpch
    hs = Hyperspace(s)
    li = s.read.parquet(lpath)
    before = dict(DC.SEED_STATS)
    hs.createIndex(li, IndexConfig("li_seed", ["l_shipdate"], ["l_discount", "l_quantity"]))
    assert DC.SEED_STATS["registered"] == before["registered"] + 1
    Hyperspace.enable(s)
    q = li.filter("l_shipdate >= DATE '1994-01-01' AND l_shipdate < DATE '1995-01-01'") \
        .agg(sum_("l_quantity").alias("q"), count("*").alias("n"))
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    assert DC.SEED_STATS["hits"] == before["hits"] + 1
    _close(g, c)
    # the seed was consumed by that first hit (it pins no HBM outside the cache budget)
    assert not any(k[0] and "li_seed" in k[0][0][0] for k in DC._SEEDS)
