"""String keys on the device: Spark Murmur3 of dictionary-coded strings on the GPU (bucket ids of
the device shuffle match the host hash bit for bit), a Hybrid Scan join on a string key (the
reference's canonical E2E case indexes and joins on the string column c3,
E2EHyperspaceRulesTest.scala:184-189; appended rows are shuffled by the index bucket spec,
RuleUtils.scala:519-578), and a non-index string-key join through the device shuffle."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_

from test_gpu_e2e import _both, _close

pytestmark = pytest.mark.gpu


def test_dictionary_string_hash_matches_spark_murmur3(device):
    import torch
    from hyperspace_amd.exec.device_table import DeviceColumn
    from hyperspace_amd.ops import kernels as K
    from hyperspace_amd.utils import murmur3
    rng = np.random.default_rng(5)
    words = ["", "a", "ab", "abc", "abcd", "abcde", "héllo wörld", "x" * 37, "日本語", "\x00\x7f\x80"]
    vals = [words[i] if i < len(words) else None for i in rng.integers(0, len(words) + 2, 5000)]
    arr = pa.array(vals, pa.string())
    d = pa.compute.unique(arr.drop_null()).sort()
    codes = pa.compute.index_in(arr, value_set=d).fill_null(0).to_numpy().astype(np.int32)
    valid = torch.from_numpy(np.array([v is not None for v in vals], np.uint8)).to(device)
    c = DeviceColumn(torch.from_numpy(codes).to(device), valid, pa.string(), d)
    ints = pa.array(rng.integers(-5, 5, 5000).astype(np.int32))
    ci = DeviceColumn(torch.from_numpy(ints.to_numpy()).to(device), None, pa.int32())
    for cols, host in (([c], [arr]), ([ci, c], [ints, arr]), ([c, ci], [arr, ints])):
        dev, _ = K.murmur3_bucket(cols, 200)
        want = murmur3.bucket_ids(host, 200)
        assert np.array_equal(dev.cpu().numpy(), np.asarray(want)), cols


@pytest.fixture
def strs(tmp_path, device):
    rng = np.random.default_rng(11)
    n_dim = 5000
    keys = np.array([f"key-{i:05d}-{'x' * (i % 7)}" for i in range(n_dim)])
    dim = pa.table({"c3": pa.array(keys), "w": rng.integers(0, 100, n_dim).astype(np.int64)})
    fk = keys[rng.integers(0, n_dim, 60_000)]
    fact = pa.table({"c3": pa.array(fk), "v": rng.random(len(fk)),
                     "q": rng.integers(1, 10, len(fk)).astype(np.int64)})
    for name, t, parts in (("fact", fact, 3), ("dim", dim, 2)):
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
    return s, str(tmp_path / "fact"), str(tmp_path / "dim"), keys, rng


def test_hybrid_scan_join_on_string_key_native(strs):
    s, fpath, dpath, keys, rng = strs
    for k, v in (("hybridscan.enabled", "true"), ("hybridscan.maxAppendedRatio", "0.5")):
        s.conf.set(f"spark.hyperspace.index.{k}", v)
    hs = Hyperspace(s)
    fact, dim = s.read.parquet(fpath), s.read.parquet(dpath)
    from hyperspace_amd.exec import device_build
    hs.createIndex(fact, IndexConfig("f_c3", ["c3"], ["v", "q"]))
    # the string key's dictionary-encoded pages decoded on the device, not through pyarrow
    assert "c3" in device_build.LAST_BUILD_STATS["device_decoded"]
    assert device_build.LAST_BUILD_STATS["host_decoded"] == []
    hs.createIndex(dim, IndexConfig("d_c3", ["c3"], ["w"]))
    # appended files: new keys (not in either index dictionary) and existing ones
    newk = np.array([f"new-{i}" for i in range(300)])
    app_f = pa.table({"c3": pa.array(np.concatenate([newk[rng.integers(0, 300, 3000)],
                                                      keys[rng.integers(0, len(keys), 3000)]])),
                      "v": rng.random(6000), "q": rng.integers(1, 10, 6000).astype(np.int64)})
    app_d = pa.table({"c3": pa.array(newk), "w": rng.integers(0, 100, 300).astype(np.int64)})
    pq.write_table(app_f, os.path.join(fpath, "part-app.parquet"))
    pq.write_table(app_d, os.path.join(dpath, "part-app.parquet"))
    Hyperspace.enable(s)
    fact, dim = s.read.parquet(fpath), s.read.parquet(dpath)
    j = fact.join(dim, fact["c3"] == dim["c3"])
    q = j.filter(col("w") < 50).agg(sum_("v").alias("sv"), count("*").alias("n"))
    plan = q.queryExecution.executed_plan.tree_string()
    assert "BucketUnion" in plan and "Name: f_c3" in plan and "Name: d_c3" in plan
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    # grouped by the string key (dense dictionary group, or hash mode over the union)
    q2 = j.groupBy(fact["c3"]).agg(sum_("q").alias("sq"))
    g, c, path = _both(s, q2)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
    # rows of the join: every (index part, appended part) pair joins on its own, the row sets
    # concatenate, string columns re-coded over one dictionary
    q3 = j.filter(col("w") < 20).select(fact["c3"], "v", "w")
    g, c, path = _both(s, q3)
    assert path == "native", s.backend().fallback_reason
    assert g.num_rows > 0
    _close(g, c)


def test_non_index_string_join_device_shuffle(strs):
    s, fpath, dpath, _, _ = strs
    fact, dim = s.read.parquet(fpath), s.read.parquet(dpath)
    q = fact.join(dim, fact["c3"] == dim["c3"]).filter(col("w") > 20) \
        .agg(sum_("v").alias("sv"), count("*").alias("n"))
    plan = q.queryExecution.executed_plan.tree_string()
    assert "Exchange hashpartitioning(c3" in plan
    g, c, path = _both(s, q, sort=False)
    assert path == "native", s.backend().fallback_reason
    _close(g, c)
