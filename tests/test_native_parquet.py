"""Native Parquet page layer (csrc/runtime/hs_parquet.cpp): footer and page-header parsing,
Snappy, and RLE/bit-packed run tables, checked on the CPU against pyarrow for many writer
configurations.  The run tables are expanded with the numpy oracle (``expand_host``) — the same
contract the HIP expansion kernels implement (GPU tier: test_native_parquet_gpu)."""
from __future__ import annotations

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq
import pytest

from hyperspace_amd.io import native_parquet as NP

np_types = {"i32": (pa.int32(), np.int32), "i64": (pa.int64(), np.int64),
            "f32": (pa.float32(), np.float32), "f64": (pa.float64(), np.float64),
            "d32": (pa.date32(), np.int32)}


def _table(n, rng, nulls: bool):
    cols = {}
    for name, (t, nd) in np_types.items():
        if name.startswith("f"):
            vals = np.round(rng.random(n) * 100, 2).astype(nd)
        else:
            vals = rng.integers(0, 50 if name == "i32" else 10_000_000, n).astype(nd)
        mask = (rng.random(n) < 0.1) if nulls else None
        arr = pa.array(vals, mask=mask)
        cols[name] = arr.view(t) if t == pa.date32() else arr.cast(t)
    # sorted low-cardinality column: long RLE runs of dictionary indices
    cols["sorted"] = pa.array(np.sort(rng.integers(0, 30, n)).astype(np.int64))
    cols["s"] = pa.array([f"v{x}" for x in rng.integers(0, 5, n)])
    return pa.table(cols)


def _check_file(path, t):
    with NP.PqFile(str(path)) as f:
        assert f.ok, f.error
        assert f.num_rows == t.num_rows
        rg_rows = [f.row_group_rows(g) for g in range(f.num_row_groups)]
        assert sum(rg_rows) == t.num_rows
        for name in t.column_names:
            c = f.column(name)
            assert c >= 0
            if name == "s":
                assert f.read_chunk_host(0, c)[0] == NP.UNSUPPORTED
                continue
            nd = np_types[name][1] if name in np_types else np.int64
            start = 0
            for g, rows in enumerate(rg_rows):
                rc, buf, info, vr, lr = f.read_chunk_host(g, c)
                assert rc == NP.OK, (name, g, rc)
                dense, valid = NP.expand_host(buf, info, vr, lr, np.dtype(nd))
                ref = t.column(name).slice(start, rows).combine_chunks()
                if ref.type == pa.date32():
                    ref = ref.view(pa.int32())
                ref_valid = np.asarray(ref.is_valid())
                assert info.num_values == rows
                assert info.num_nonnull == ref_valid.sum()
                np.testing.assert_array_equal(dense, ref.drop_null().to_numpy())
                if ref.null_count:
                    assert valid is not None
                    np.testing.assert_array_equal(valid.astype(bool), ref_valid)
                start += rows


@pytest.mark.parametrize("compression", ["none", "snappy"])
@pytest.mark.parametrize("dictionary", [True, False])
@pytest.mark.parametrize("page_version", ["1.0", "2.0"])
@pytest.mark.parametrize("nulls", [False, True])
def test_page_layer_matches_pyarrow(tmp_path, compression, dictionary, page_version, nulls):
    rng = np.random.default_rng(5)
    t = _table(20_000, rng, nulls)
    path = tmp_path / "t.parquet"
    pq.write_table(t, path, compression=compression, use_dictionary=dictionary,
                   data_page_version=page_version, row_group_size=7_000, data_page_size=4096)
    _check_file(path, t)


def test_dictionary_fallback_to_plain_pages(tmp_path):
    """High-cardinality columns overflow the dictionary and switch to PLAIN pages mid-chunk."""
    rng = np.random.default_rng(6)
    t = _table(60_000, rng, False)
    path = tmp_path / "t.parquet"
    pq.write_table(t, path, compression="snappy", dictionary_pagesize_limit=2048,
                   data_page_size=8192)
    md = pq.ParquetFile(path).metadata.row_group(0)
    encs = {md.column(i).path_in_schema: md.column(i).encodings for i in range(md.num_columns)}
    assert "PLAIN" in encs["i64"] and "RLE_DICTIONARY" in encs["i64"]
    _check_file(path, t)


def test_tpch_datagen_files(tmp_path):
    from hyperspace_amd.models import tpch
    tpch.write_chunk(str(tmp_path), 0.01, 2, 0)
    path = tmp_path / "lineitem" / "part-00000.parquet"
    t = pq.read_table(path)
    with NP.PqFile(str(path)) as f:
        for name in ("l_orderkey", "l_quantity", "l_extendedprice", "l_discount", "l_shipdate",
                     "l_linenumber"):
            c = f.column(name)
            rc, buf, info, vr, lr = f.read_chunk_host(0, c)
            assert rc == NP.OK
            nd = np.int32 if name in ("l_shipdate", "l_linenumber") else \
                (np.int64 if name == "l_orderkey" else np.float64)
            dense, _ = NP.expand_host(buf, info, vr, lr, np.dtype(nd))
            ref = t.column(name).combine_chunks()
            if ref.type == pa.date32():
                ref = ref.view(pa.int32())
            np.testing.assert_array_equal(dense, ref.to_numpy())
            # dictionary-encoded low-cardinality doubles cross PCIe as narrow indices
            if name == "l_quantity":
                assert info.dict_encoded and set(vr["bit_width"]) <= {6, 0}


def test_unsupported_codec_and_missing_file(tmp_path):
    t = pa.table({"a": pa.array(np.arange(100, dtype=np.int64))})
    path = tmp_path / "z.parquet"
    pq.write_table(t, path, compression="zstd")
    with NP.PqFile(str(path)) as f:
        assert f.ok
        assert f.read_chunk_host(0, f.column("a"))[0] == NP.UNSUPPORTED
    with NP.PqFile(str(tmp_path / "nope.parquet")) as f:
        assert not f.ok and f.error
    bad = tmp_path / "bad.parquet"
    bad.write_bytes(b"PAR1" + b"\0" * 64)
    with NP.PqFile(str(bad)) as f:
        assert not f.ok


def test_snappy_decompress_matches_pyarrow():
    L = NP.lib()
    rng = np.random.default_rng(1)
    for data in (b"", b"a", bytes(rng.integers(0, 4, 100_000).astype(np.uint8)),
                 bytes(rng.integers(0, 256, 50_000).astype(np.uint8)), b"abcd" * 20_000):
        comp = pa.compress(data, codec="snappy", asbytes=True)
        out = np.zeros(len(data) + 16, dtype=np.uint8)
        src = np.frombuffer(comp, dtype=np.uint8)
        got = L.hs_pq_snappy_decompress(src.ctypes.data, len(comp), out.ctypes.data, len(out))
        assert got == len(data)
        assert out[:got].tobytes() == data
    # truncated input is rejected, not overrun
    comp = pa.compress(b"xyz" * 1000, codec="snappy", asbytes=True)
    src = np.frombuffer(comp[:-5], dtype=np.uint8)
    out = np.zeros(4000, dtype=np.uint8)
    assert L.hs_pq_snappy_decompress(src.ctypes.data, len(src), out.ctypes.data, len(out)) == -1


@pytest.mark.gpu
def test_native_parquet_gpu_decode_matches_pyarrow(tmp_path, device):
    """The HIP expansion kernels + staging path against pyarrow, incl. nulls and PLAIN pages."""
    import torch
    from hyperspace_amd.exec import staging
    rng = np.random.default_rng(9)
    files, tables = [], []
    for i, (comp, dic, ver, nulls) in enumerate([("snappy", True, "1.0", False),
                                                 ("none", False, "2.0", True),
                                                 ("snappy", True, "2.0", True)]):
        t = _table(30_000 + i * 1000, rng, nulls)
        path = tmp_path / f"p{i}.parquet"
        pq.write_table(t, path, compression=comp, use_dictionary=dic, data_page_version=ver,
                       row_group_size=11_000, data_page_size=8192)
        files.append(str(path))
        tables.append(t)
    full = pa.concat_tables(tables)
    schema = full.schema
    counts = [t.num_rows for t in tables]

    def read_file(p, cols=None):
        return pq.read_table(p, columns=cols)
    up = staging.upload_files(read_file, files, counts, schema, device, parquet_local=files)
    torch.cuda.synchronize()
    for name in np_types:
        col = up.columns[name]
        ref = full.column(name).combine_chunks()
        if ref.type == pa.date32():
            ref = ref.view(pa.int32())
        vals = col.data.cpu().numpy()
        valid = np.asarray(ref.is_valid())
        if ref.null_count:
            assert col.valid is not None
            np.testing.assert_array_equal(col.valid.cpu().numpy().astype(bool), valid)
        np.testing.assert_array_equal(vals[valid], ref.drop_null().to_numpy())
    assert "s" in up.host_strings  # strings still come back through pyarrow
