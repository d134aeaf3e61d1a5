"""PLAIN BYTE_ARRAY pages on the device (csrc/kernels/parquet_decode.hip eb-16 pages,
csrc/kernels/strings.hip, io/native_parquet.StringCodes.finish_plain): an index build over
source files whose string columns are PLAIN-encoded (no dictionary pages; nulls, empty and
long values, a high-cardinality column, one file dictionary-encoded to mix both kinds) decodes
every column on the device (``host_decoded == []``) and writes the same rows as the source;
queries grouping by those strings match the host oracle.  Reference: SURVEY K1 "BYTE_ARRAY
offsets"; E2EHyperspaceRulesTest.scala:184-189 (string-keyed indexes).  GPU-only."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, Session, col, count, sum_

pytestmark = pytest.mark.gpu


@pytest.fixture
def plain(tmp_path, device):
    rng = np.random.default_rng(31)
    n = 90_000
    words = ["", "a", "MAIL", "SHIP", "TRUCK", "AIR", "REG AIR", "FOB", "ünïcødé",
             "x" * 100, "y" * 7, "z" * 8, "w" * 9]
    t = pa.table({
        "k": rng.integers(0, 20_000, n).astype(np.int64),
        "mode": pa.array(rng.choice(words, n), mask=rng.random(n) < 0.1),
        "tag": pa.array([f"tag-{v:06d}" for v in rng.integers(0, 30_000, n)]),
        "x": np.round(rng.random(n) * 100, 2)})
    os.makedirs(tmp_path / "src")
    for i in range(3):
        part = t.slice(i * (n // 3), n // 3)
        # files 0 and 1 PLAIN (no dictionary), file 2 dictionary-encoded
        pq.write_table(part, tmp_path / "src" / f"p{i}.parquet", use_dictionary=(i == 2),
                       data_page_size=64 * 1024)
    s = Session(conf={"spark.hyperspace.system.path": str(tmp_path / "idx"),
                      "spark.hyperspace.index.numBuckets": "8",
                      "spark.hyperspace.mi.execution.device": "gpu"},
                warehouse_dir=str(tmp_path / "wh"))
    return s, t, str(tmp_path / "src")


def _rows(t: pa.Table):
    return sorted((tuple(r.values()) for r in t.to_pylist()), key=repr)


def test_plain_string_pages_decode_on_device(plain, tmp_path):
    from hyperspace_amd.exec import device_build, staging
    s, src, path = plain
    for f in ("p0", "p1"):
        md = pq.ParquetFile(os.path.join(path, f + ".parquet")).metadata
        encs = md.row_group(0).column(1).encodings
        assert "PLAIN_DICTIONARY" not in encs and "RLE_DICTIONARY" not in encs, encs
    hs = Hyperspace(s)
    df = s.read.parquet(path)
    staging.DEVICE_DECODED.clear()
    hs.createIndex(df, IndexConfig("strs", ["k"], ["mode", "tag", "x"]))
    st = device_build.LAST_BUILD_STATS
    assert st.get("host_decoded") == [], st.get("host_decoded")
    assert {"mode", "tag"} <= staging.DEVICE_DECODED
    files = []
    for root, _, fs in os.walk(tmp_path / "idx" / "strs"):
        files += [os.path.join(root, f) for f in fs if f.endswith(".parquet")]
    got = pa.concat_tables([pq.read_table(f) for f in files])
    assert _rows(got.select(src.column_names)) == _rows(src)
    Hyperspace.enable(s)
    q = df.filter(col("k") < 15_000).groupBy("mode").agg(count("*").alias("n"),
                                                         sum_(col("x")).alias("sx"))
    g = q.to_arrow()
    assert s.backend().last_path == "native", s.backend().fallback_reason
    s.conf.set("spark.hyperspace.mi.execution.device", "cpu")
    c = q.to_arrow()
    s.conf.set("spark.hyperspace.mi.execution.device", "gpu")
    gr, cr = _rows(g), _rows(c)
    assert len(gr) == len(cr) == len({w for w in src.column("mode").to_pylist()})
    for a, b in zip(gr, cr):
        assert a[0] == b[0] and a[1] == b[1] and abs(a[2] - b[2]) <= 1e-9 * max(1.0, abs(b[2]))


def test_plain_strings_upload_matches_pyarrow(plain, device):
    """The upload layer itself: PLAIN string chunks -> codes over a dictionary equal to the
    pyarrow-decoded values, row for row (nulls included)."""
    import torch
    from hyperspace_amd.exec import staging
    _, src, path = plain
    files = [os.path.join(path, f"p{i}.parquet") for i in range(3)]
    rows = [pq.ParquetFile(f).metadata.num_rows for f in files]
    schema = pa.schema([src.schema.field("mode"), src.schema.field("tag")])
    staging.HOST_DECODED.clear()
    up = staging.upload_files(lambda p, cols=None: pq.read_table(p, columns=cols or schema.names),
                              files, rows, schema, device, parquet_local=files,
                              device_pages=True)
    cols = dict(up.columns)
    staging.finish_strings(up, cols, device, None)
    torch.cuda.synchronize()
    assert not ({"mode", "tag"} & staging.HOST_DECODED), staging.HOST_DECODED
    want = pa.concat_tables([pq.read_table(f, columns=["mode", "tag"]) for f in files])
    for name in ("mode", "tag"):
        dc = cols[name]
        codes = dc.data.cpu().numpy()
        valid = dc.valid.cpu().numpy().astype(bool) if dc.valid is not None else \
            np.ones(len(codes), bool)
        vals = dc.dictionary.take(pa.array(codes)).to_pylist()
        exp = want.column(name).to_pylist()
        assert [v if ok else None for v, ok in zip(vals, valid)] == exp
        assert dc.dictionary.equals(dc.dictionary.sort())   # job-global sorted dictionary
