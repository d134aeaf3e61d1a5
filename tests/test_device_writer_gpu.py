"""General device Parquet writer (exec/pq_encode.py, csrc/runtime/hs_parquet_write.cpp
hs_pq_write_file2): an index over nullable double / boolean / timestamp / decimal / int16 /
string columns is written by the device encoder (``LAST_BUILD_STATS["writer"] == "device"``),
its files round-trip through pyarrow, and a cold load of the index files (no build seed)
decodes them on the device, pages included.  Reference: DataFrameWriterExtensions.scala:49-67
writes any Spark schema.  GPU-only."""
import decimal
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_, min_, max_

pytestmark = pytest.mark.gpu


@pytest.fixture
def mixed(tmp_path, device):
    rng = np.random.default_rng(21)
    n = 120_000
    k = rng.integers(0, 50_000, n).astype(np.int64)

    def nulls(p):
        return rng.random(n) < p
    t = pa.table({
        "k": k,
        "x": pa.array(np.round(rng.random(n) * 100, 3), mask=nulls(0.1)),
        "b": pa.array(rng.random(n) < 0.4, mask=nulls(0.2)),
        "ts": pa.array(rng.integers(0, 2 * 10**15, n), type=pa.timestamp("us"),
                       mask=nulls(0.05)),
        "dec": pa.array([decimal.Decimal(int(v)).scaleb(-2) for v in
                         rng.integers(-10**9, 10**9, n)], type=pa.decimal128(12, 2)),
        "i16": pa.array(rng.integers(-30000, 30000, n).astype(np.int16)),
        "s": pa.array(rng.choice(["red", "green", "blue", "cyan"], n), mask=nulls(0.15))})
    os.makedirs(tmp_path / "src")
    for i in range(3):
        pq.write_table(t.slice(i * n // 3, n // 3 + (1 if i == 2 else 0) * (n % 3)),
                       tmp_path / "src" / f"p{i}.parquet")
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "8",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=str(tmp_path / "wh"))
    return s, t, str(tmp_path / "src")


def _rows(t: pa.Table):
    return sorted((tuple(r.values()) for r in t.to_pylist()), key=repr)


def test_device_writer_covers_nullable_and_typed_columns(mixed, tmp_path):
    from hyperspace_amd.exec import device_build, device_cache, pq_encode, staging
    s, src, path = mixed
    pq_encode.PAGE_ROWS = 4096          # several data pages per column chunk
    try:
        hs = Hyperspace(s)
        df = s.read.parquet(path)
        hs.createIndex(df, IndexConfig("mixed", ["k"], ["x", "b", "ts", "dec", "i16", "s"]))
    finally:
        pq_encode.PAGE_ROWS = 1 << 16
    st = device_build.LAST_BUILD_STATS
    assert st.get("writer") == "device", st.get("writer_fallback")
    files = []
    for root, _, fs in os.walk(tmp_path / "idx" / "mixed"):
        files += [os.path.join(root, f) for f in fs if f.endswith(".parquet")]
    assert files
    got = pa.concat_tables([pq.read_table(f) for f in files])
    assert got.schema.field("ts").type == pa.timestamp("us")
    assert got.schema.field("dec").type == pa.decimal128(12, 2)
    assert got.schema.field("i16").type == pa.int16()
    assert _rows(got.select(src.column_names)) == _rows(src)
    md = pq.ParquetFile(files[0]).metadata
    assert md.created_by == pq_encode.CREATED_BY
    # queries over the index, first from the build's HBM columns, then after a cold load
    Hyperspace.enable(s)
    q = df.filter(col("k") < 20_000).groupBy("s").agg(
        count("*").alias("n"), sum_(col("x")).alias("sx"), min_(col("ts")).alias("t0"),
        max_(col("i16")).alias("m16"), count(col("b")).alias("nb"))
    want = None
    for cold in (False, True):
        if cold:
            device_cache.clear_seeds()
            s.backend().cache.clear()
            staging.HOST_DECODED.clear()
            staging.DEVICE_DECODED.clear()
        s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
        g = q.to_arrow()
        path_ = s.backend().last_path
        s.conf.set("spark.hyperspace.mi.execution.device", "cpu")
        c = q.to_arrow()
        s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
        assert path_ == "native", s.backend().fallback_reason
        gr, cr = _rows(g), _rows(c)
        assert len(gr) == len(cr)
        for a, b in zip(gr, cr):
            for u, v in zip(a, b):
                if isinstance(v, float):
                    assert abs(u - v) <= 1e-9 * max(1.0, abs(v))
                else:
                    assert u == v
        if cold:
            # the paged index files decoded on the device (no pyarrow fallback for them)
            assert not ({"k", "x", "b", "ts", "s"} & staging.HOST_DECODED), staging.HOST_DECODED
        want = gr
    assert want


def test_file_dicts_match_numpy(device):
    """Per-file dictionaries (hs_pq_dict_mark / hs_pq_dict_remap): codes into a job-wide
    dictionary become ranks among the codes each file uses; files of 0 rows, of one row, and
    spanning several 4096-row mark chunks; a 16-bit wide dictionary."""
    import torch
    from hyperspace_amd.exec import pq_encode as PE
    rng = np.random.default_rng(5)
    for n_dict, sizes in ((11, [0, 1, 5000, 9000, 3, 4096, 12000]),
                          (40_000, [70_000, 10, 0, 33_333])):
        fo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        codes = rng.integers(0, n_dict, int(fo[-1])).astype(np.int32)
        d = torch.from_numpy(codes.copy()).to(device)
        subsets = PE._file_dicts(d, n_dict, fo, device)
        got = d.cpu().numpy()
        for f in range(len(sizes)):
            c = codes[fo[f]:fo[f + 1]]
            u = np.unique(c)
            assert np.array_equal(subsets[f], u)
            assert np.array_equal(got[fo[f]:fo[f + 1]], np.searchsorted(u, c))
