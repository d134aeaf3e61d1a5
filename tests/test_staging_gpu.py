"""Pipelined host<->HBM staging used by the device index build (exec/staging.py)."""
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

pytestmark = pytest.mark.gpu


def test_upload_download_round_trip(tmp_path, device):
    from hyperspace_amd.exec import staging
    rng = np.random.default_rng(4)
    files, tables = [], []
    for i in range(5):
        n = int(rng.integers(1, 50_000))
        t = pa.table({
            "k": pa.array(rng.integers(0, 1 << 40, n), pa.int64()),
            "d": pa.array(rng.integers(0, 20_000, n).astype(np.int32)).view(pa.date32()),
            "x": pa.array(rng.random(n), mask=rng.random(n) < 0.1),
            "s": pa.array([f"s{v}" for v in rng.integers(0, 100, n)]),
            "b": pa.array(rng.random(n) < 0.5),
        })
        p = str(tmp_path / f"f{i}.parquet")
        pq.write_table(t, p)
        files.append(p)
        tables.append(t)
    counts = [pq.ParquetFile(f).metadata.num_rows for f in files]
    schema = tables[0].schema
    up = staging.upload_files(lambda f: pq.read_table(f), files, counts, schema, device,
                              lineage_ids=[10, 11, 12, 13, 14], lineage_name="_lin")
    full = pa.concat_tables(tables)
    assert up.num_rows == full.num_rows
    assert np.array_equal(up.columns["k"].data.cpu().numpy(), full.column("k").to_numpy())
    assert np.array_equal(up.columns["d"].data.cpu().numpy(),
                          full.column("d").combine_chunks().view(pa.int32()).to_numpy())
    xv = up.columns["x"].valid.cpu().numpy().astype(bool)
    assert np.array_equal(xv, full.column("x").is_valid().to_numpy())
    exp_lin = np.repeat([10, 11, 12, 13, 14], counts)
    assert np.array_equal(up.columns["_lin"].data.cpu().numpy(), exp_lin)
    assert [len(c) for c in up.host_strings["s"]] == counts

    # download: pretend rows are bucket-major with 7 buckets
    off = np.linspace(0, full.num_rows, 8).astype(np.int64)
    names = ["k", "d", "x", "b"]
    written = {}

    def write(t, b):
        written[b] = t
        return f"bucket{b}"
    paths = staging.download_buckets([up.columns[n] for n in names], names, full.select(names).schema,
                                     off, write, device, chunk_bytes=64 << 10)
    assert sorted(paths) == sorted(f"bucket{b}" for b in range(7) if off[b + 1] > off[b])
    back = pa.concat_tables([written[b] for b in sorted(written)])
    assert back.equals(full.select(names))
