"""Cached join index (exec/join_index.py): joins of two resident index tables run as a streaming
scan + gather.  Results are checked against the host oracle and against the merge-join kernels
(join index disabled); the index itself is checked row by row against a numpy merge."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, max_, min_, sum_

pytestmark = pytest.mark.gpu


@pytest.fixture
def data(tmp_path, device):
    rng = np.random.default_rng(11)
    n_ord = 30_000
    okeys = rng.permutation(np.arange(1, n_ord + 1, dtype=np.int64) * 4)
    od = pa.table({"o_orderkey": okeys,
                   "o_orderdate": pa.array(rng.integers(8000, 10500, n_ord).astype(np.int32)),
                   "o_shippriority": rng.integers(0, 5, n_ord).astype(np.int32)})
    # lineitem keys: FK into orders plus keys with no order (no match) and nulls
    lk = np.concatenate([np.repeat(okeys, rng.integers(1, 8, n_ord)),
                         rng.integers(0, n_ord, 3000) * 4 + 2])
    n = len(lk)
    valid = rng.random(n) > 0.01
    li = pa.table({"l_orderkey": pa.array(lk, mask=~valid),
                   "l_extendedprice": np.round(rng.random(n) * 1e5, 2),
                   "l_discount": rng.integers(0, 11, n) / 100.0,
                   "l_shipdate": pa.array(rng.integers(8000, 10600, n).astype(np.int32))})
    # a right side with duplicate keys (not eligible: merge-join kernels)
    dup = pa.table({"d_key": np.repeat(okeys[:5000], 2),
                    "d_val": rng.integers(0, 100, 10000).astype(np.int32)})
    for name, t, parts in (("lineitem", li, 4), ("orders", od, 2), ("dup", dup, 1)):
        os.makedirs(tmp_path / name)
        step = (t.num_rows + parts - 1) // parts
        for i in range(parts):
            pq.write_table(t.slice(i * step, step), tmp_path / name / f"part-{i}.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "16",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=str(tmp_path / "wh"))
    hs = Hyperspace(s)
    li_df = s.read.parquet(str(tmp_path / "lineitem"))
    od_df = s.read.parquet(str(tmp_path / "orders"))
    dup_df = s.read.parquet(str(tmp_path / "dup"))
    hs.createIndex(li_df, IndexConfig("li_ok", ["l_orderkey"],
                                      ["l_extendedprice", "l_discount", "l_shipdate"]))
    hs.createIndex(od_df, IndexConfig("od_ok", ["o_orderkey"], ["o_orderdate", "o_shippriority"]))
    hs.createIndex(dup_df, IndexConfig("dup_k", ["d_key"], ["d_val"]))
    Hyperspace.enable(s)
    return s, li_df, od_df, dup_df


def _run(s, df, device="gpu", join_index=True):
    s.conf.set("spark.hyperspace.mi.execution.device", device)
    s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "true" if join_index else "false")
    t = df.to_arrow()
    path = s.backend().last_path if device == "gpu" else "cpu"
    s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
    s.conf.set("spark.hyperspace.mi.joinIndex.enabled", "true")
    return t.sort_by([(n, "ascending") for n in t.column_names]) if t.num_rows else t, path


def _close(a: pa.Table, b: pa.Table):
    assert a.num_rows == b.num_rows
    for x, y in zip(a.columns, b.columns):
        for u, v in zip(x.to_pylist(), y.to_pylist()):
            if isinstance(u, float):
                assert abs(u - v) <= 1e-9 * max(1.0, abs(v)), (u, v)
            else:
                assert u == v, (u, v)


def _q3(li, od, dd):
    return li.join(od, li["l_orderkey"] == od["o_orderkey"]) \
        .filter((col("o_orderdate") < dd) & (col("l_shipdate") > dd)) \
        .groupBy("o_shippriority") \
        .agg(sum_(col("l_extendedprice") * (1 - col("l_discount"))).alias("rev"),
             count("*").alias("n"), min_(col("o_orderdate")).alias("mn"),
             max_(col("l_shipdate")).alias("mx"))


def test_join_index_q3_matches_oracle_and_merge_join(data):
    s, li, od, _ = data
    from hyperspace_amd.exec.jit import _KERNELS
    for dd in (9000, 9300, 10000):
        q = _q3(li, od, dd)
        g, p = _run(s, q)
        assert p == "native", s.backend().fallback_reason
        m, p2 = _run(s, q, join_index=False)
        assert p2 == "native"
        c, _ = _run(s, q, device="cpu")
        _close(g, c)
        _close(m, c)
    assert any(k[0] == "join_index_agg" for k in _KERNELS), "join-index kernel did not run"


def test_join_index_ungrouped_and_left_range_pruned(data):
    s, li, od, _ = data
    j = li.join(od, li["l_orderkey"] == od["o_orderkey"])
    for q in (j.filter(col("o_orderdate") < 9500).agg(sum_(col("l_extendedprice")).alias("s")),
              j.filter((col("l_orderkey") > 20000) & (col("l_orderkey") <= 80000))
               .agg(count("*").alias("n"), sum_(col("o_shippriority")).alias("p"))):
        g, p = _run(s, q)
        assert p == "native", s.backend().fallback_reason
        c, _ = _run(s, q, device="cpu")
        _close(g, c)


def test_join_index_matches_numpy_merge(data):
    """Every left row's index entry is the first right row with an equal key, or -1."""
    s, li, od, _ = data
    q = li.join(od, li["l_orderkey"] == od["o_orderkey"]).agg(count("*").alias("n"))
    _run(s, q)
    be = s.backend()
    tables = [t for t in be.cache._lru.values() if "_join_index" in t.__dict__]
    assert tables, "no join index was built"
    lt = tables[0]
    (rref, lcol, rcol, ji), = lt._join_index.values()
    jidx = ji.decoded(lt.num_rows)
    lk = lcol.data.cpu().numpy()
    lv = lcol.valid.cpu().numpy().astype(bool) if lcol.valid is not None else np.ones(len(lk), bool)
    rk = rcol.data.cpu().numpy()
    rt = rref()
    j = jidx.cpu().numpy()[:lt.num_rows]
    loff, roff = lt.bucket_offsets_host, rt.bucket_offsets_host
    for b in range(len(loff) - 1):
        seg = rk[roff[b]:roff[b + 1]]
        for i in range(loff[b], loff[b + 1]):
            pos = np.searchsorted(seg, lk[i])
            want = roff[b] + pos if lv[i] and pos < len(seg) and seg[pos] == lk[i] else -1
            assert j[i] == want, (b, i, j[i], want)


def test_duplicate_right_keys_keep_merge_join(data):
    s, li, _, dup = data
    q = li.join(dup, li["l_orderkey"] == dup["d_key"]).groupBy("d_val") \
        .agg(count("*").alias("n"), sum_(col("l_discount")).alias("d"))
    g, p = _run(s, q)
    assert p == "native", s.backend().fallback_reason
    c, _ = _run(s, q, device="cpu")
    _close(g, c)


@pytest.mark.parametrize("coded,codings", [(True, ((1, 7),)), (True, ((2, 8),)), (False, ())])
def test_join_index_encodings(data, monkeypatch, coded, codings):
    """uint8 / uint16 block-coded and plain int32 join indexes give the oracle's answer."""
    from hyperspace_amd.exec import join_index
    s, li, od, _ = data
    monkeypatch.setattr(join_index, "CODED", coded)
    monkeypatch.setattr(join_index, "CODINGS", codings)
    for t in s.backend().cache._lru.values():
        t.__dict__.pop("_join_index", None)
    q = _q3(li, od, 9400)
    g, p = _run(s, q)
    assert p == "native", s.backend().fallback_reason
    c, _ = _run(s, q, device="cpu")
    _close(g, c)
    widths = {ji.width for t in s.backend().cache._lru.values()
              for (_, _, _, ji) in t.__dict__.get("_join_index", {}).values()}
    assert widths == {codings[0][0] if coded else 4}


def test_string_join_keys_on_device(tmp_path, device):
    """Joins on string keys run natively: both sides' dictionary codes are remapped into the
    sorted union of the two dictionaries (order-preserving), then the join index applies."""
    rng = np.random.default_rng(2)
    names = np.array([f"cust#{i:06d}" for i in rng.permutation(5000)])
    cust = pa.table({"c_name": names, "c_seg": pa.array(rng.choice(["AUTO", "BUILD", "MACH"], 5000))})
    on = rng.choice(names, 20000)
    on[:300] = [f"ghost#{i}" for i in range(300)]              # keys with no customer
    valid = rng.random(20000) > 0.02
    ords = pa.table({"o_cname": pa.array(on, mask=~valid),
                     "o_total": np.round(rng.random(20000) * 1e4, 2)})
    for name, t in (("cust", cust), ("ords", ords)):
        os.makedirs(tmp_path / name)
        pq.write_table(t, tmp_path / name / "p0.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "8",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=str(tmp_path / "wh"))
    hs = Hyperspace(s)
    c = s.read.parquet(str(tmp_path / "cust"))
    o = s.read.parquet(str(tmp_path / "ords"))
    hs.createIndex(c, IndexConfig("c_name_idx", ["c_name"], ["c_seg"]))
    hs.createIndex(o, IndexConfig("o_cname_idx", ["o_cname"], ["o_total"]))
    Hyperspace.enable(s)
    for lim in (2000.0, 7000.0):
        q = o.join(c, o["o_cname"] == c["c_name"]).filter(col("o_total") < lim) \
            .groupBy("c_seg").agg(sum_(col("o_total")).alias("t"), count("*").alias("n"))
        g, p = _run(s, q)
        assert p == "native", s.backend().fallback_reason
        cpu, _ = _run(s, q, device="cpu")
        _close(g, cpu)


def test_multi_key_join_on_device(tmp_path, device):
    """(k1, k2) equi-joins of two indexes bucketed and sorted by (k1, k2) run natively on a packed
    order-preserving 64-bit key (here through the join index: the right pairs are unique)."""
    rng = np.random.default_rng(4)
    n_ps = 20000
    pk = rng.integers(1, 3000, n_ps).astype(np.int64)
    sk = rng.integers(1, 50, n_ps).astype(np.int32)
    pairs = np.unique(np.stack([pk, sk.astype(np.int64)], 1), axis=0)
    ps = pa.table({"ps_partkey": pairs[:, 0], "ps_suppkey": pairs[:, 1].astype(np.int32),
                   "ps_cost": np.round(rng.random(len(pairs)) * 100, 2)})
    pick = rng.integers(0, len(pairs), 60000)
    lpk, lsk = pairs[pick, 0].copy(), pairs[pick, 1].astype(np.int32)
    lsk[:500] = 99                                        # pairs with no partsupp row
    li = pa.table({"l_partkey": lpk, "l_suppkey": pa.array(lsk, mask=rng.random(60000) < 0.01),
                   "l_qty": rng.integers(1, 50, 60000).astype(np.float64)})
    for name, t in (("ps", ps), ("li", li)):
        os.makedirs(tmp_path / name)
        pq.write_table(t, tmp_path / name / "p0.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "8",
                      "spark.sql.autoBroadcastJoinThreshold": "-1",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=str(tmp_path / "wh"))
    hs = Hyperspace(s)
    a = s.read.parquet(str(tmp_path / "li"))
    b = s.read.parquet(str(tmp_path / "ps"))
    hs.createIndex(a, IndexConfig("li_ps", ["l_partkey", "l_suppkey"], ["l_qty"]))
    hs.createIndex(b, IndexConfig("ps_ps", ["ps_partkey", "ps_suppkey"], ["ps_cost"]))
    Hyperspace.enable(s)
    j = a.join(b, (a["l_partkey"] == b["ps_partkey"]) & (a["l_suppkey"] == b["ps_suppkey"]))
    for q in (j.filter(col("ps_cost") < 50).agg(sum_(col("l_qty") * col("ps_cost")).alias("v"),
                                                 count("*").alias("n")),
              j.filter(col("l_qty") > 25).select("l_partkey", "l_suppkey", "ps_cost")):
        g, p = _run(s, q)
        assert p == "native", s.backend().fallback_reason
        c, _ = _run(s, q, device="cpu")
        _close(g, c)
