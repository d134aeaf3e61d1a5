"""Native Parquet page layer (csrc/runtime/hs_parquet.cpp): footer and page-header parsing,
Snappy, and RLE/bit-packed run tables, checked on the CPU against pyarrow for many writer
configurations.  The run tables are expanded with the numpy oracle (``expand_host``) — the same
contract the HIP expansion kernels implement (GPU tier: test_native_parquet_gpu)."""
from __future__ import annotations

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
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


def _plan_and_decode_host(path, names):
    """Device page plan of ``names`` (hs_pq_plan_chunk) consumed by the host reference decoder
    (NP.decode_plan_host): {name: values} plus the fields the plan refused."""
    with NP.PqFile(str(path)) as f:
        assert f.ok, f.error
        plan = []
        for name in names:
            c = f.column(name)
            ptype, _, eb = f.column_info(c)
            if ptype == 0:               # BOOLEAN: one byte per value on the device path
                eb = 1
            plan.append((pa.field(name, pa.int64()), c, eb))
        cap = sum(int(f.L.hs_pq_chunk_raw_bytes(f.h, g, c)) + 16
                  for _, c, _ in plan for g in range(f.num_row_groups)) + 64
        raw = np.zeros(cap, dtype=np.uint8)
        hcap = sum(int(f.L.hs_pq_chunk_host_bound(f.h, g, c)) + 16
                   for _, c, _ in plan for g in range(f.num_row_groups))
        hd = np.zeros(hcap, dtype=np.uint8)
        pages, chunks, raw_used, scratch, host_used, skipped = NP.plan_file(
            f, plan, cap, raw.ctypes.data, hcap, hd.ctypes.data)
        assert raw_used <= cap and host_used <= hcap
        rg_off = np.concatenate([[0], np.cumsum([f.row_group_rows(g)
                                                 for g in range(f.num_row_groups)])])
        out = {fld.name: np.zeros(f.num_rows, dtype={1: np.uint8, 4: np.uint32}.get(eb, np.uint64))
               for fld, _, eb in plan}
        valid = {fld.name: np.ones(f.num_rows, dtype=np.uint8) for fld, _, _ in plan}
        targets, vtargets = {}, {}
        for fld, g, p0, n in chunks:
            for i in range(p0, p0 + n):
                p = pages[i]
                pages[i]["out"] = i + 1
                r0 = int(rg_off[g] + p["row"])
                targets[i + 1] = out[fld.name][r0:r0 + int(p["nvals"])]
                if p["nulls"]:
                    pages[i]["valid"] = i + 1
                    vtargets[i + 1] = valid[fld.name][r0:r0 + int(p["nvals"])]
        NP.decode_plan_host(raw, pages, targets, hd, vtargets)
        # every data page starts at its row; pages tile the chunk
        for fld, g, p0, n in chunks:
            data = pages[p0:p0 + n][pages[p0:p0 + n]["kind"] != 2]
            assert int(data["nvals"].sum()) == f.row_group_rows(g)
            assert (data["dst"] % 16 == 0).all()
        _plan_and_decode_host.valid = {k: v for k, v in valid.items() if k not in skipped}
        return {k: v for k, v in out.items() if k not in skipped}, skipped


@pytest.mark.parametrize("compression", ["none", "snappy"])
@pytest.mark.parametrize("dictionary", [True, False])
@pytest.mark.parametrize("page_version", ["1.0", "2.0"])
def test_device_page_plan_matches_pyarrow(tmp_path, compression, dictionary, page_version):
    """The device-decode page plan (host pread + page headers only) decodes to pyarrow's values;
    chunks with nulls decode their definition levels too (validity bytes, values spread to
    their rows with 0 at nulls)."""
    rng = np.random.default_rng(8)
    t = _table(23_000, rng, False)
    t = t.append_column("n64", pa.array(np.where(rng.random(t.num_rows) < 0.05, None,
                                                 rng.integers(0, 9, t.num_rows))))
    path = tmp_path / "t.parquet"
    pq.write_table(t, path, compression=compression, use_dictionary=dictionary,
                   data_page_version=page_version, row_group_size=9_000, data_page_size=4096)
    names = list(np_types) + ["sorted", "n64"]
    vals, skipped = _plan_and_decode_host(path, names)
    assert not skipped
    for name in names[:-1]:
        ref = t.column(name).combine_chunks()
        if ref.type == pa.date32():
            ref = ref.view(pa.int32())
        nd = ref.to_numpy()
        np.testing.assert_array_equal(vals[name].view(nd.dtype), nd)
    ref = t.column("n64").combine_chunks()
    np.testing.assert_array_equal(_plan_and_decode_host.valid["n64"],
                                  ref.is_valid().to_numpy(zero_copy_only=False).astype(np.uint8))
    np.testing.assert_array_equal(vals["n64"].view(np.int64),
                                  ref.fill_null(0).to_numpy().astype(np.int64))


def test_device_page_plan_refuses_nulls_when_disabled(tmp_path):
    """HS_PQ_DEVICE_NULLS=0 (hs_pq_set_device_nulls(0)): chunks with nulls are refused by the
    device plan and take the host page layer."""
    rng = np.random.default_rng(12)
    n = 9_000
    t = pa.table({"k": pa.array(rng.integers(0, 9, n)),
                  "n": pa.array(np.where(rng.random(n) < 0.1, None, rng.integers(0, 9, n)))})
    path = tmp_path / "n.parquet"
    pq.write_table(t, path)
    L = NP.lib()
    L.hs_pq_set_device_nulls(0)
    try:
        _, skipped = _plan_and_decode_host(path, ["k", "n"])
    finally:
        L.hs_pq_set_device_nulls(1)
    assert skipped == {"n"}


@pytest.mark.parametrize("page_version", ["1.0", "2.0"])
def test_device_page_plan_nullable_strings_and_bools(tmp_path, page_version):
    """Nullable dictionary-encoded strings (codes through the chunk's code table) and nullable
    booleans plan for the device; all-null pages and runs of nulls included."""
    rng = np.random.default_rng(14)
    n = 30_000
    words = np.array(["alpha", "beta", "gamma", "delta", "eps"])
    nulls = rng.random(n) < 0.2
    nulls[5_000:9_000] = True                       # whole pages of nulls
    s = pa.array(np.where(nulls, None, words[rng.integers(0, 5, n)]).tolist(), pa.string())
    b = pa.array(np.where(rng.random(n) < 0.3, None, rng.random(n) < 0.5).tolist(), pa.bool_())
    t = pa.table({"s": s, "b": b})
    path = tmp_path / "s.parquet"
    pq.write_table(t, path, data_page_version=page_version, row_group_size=12_000,
                   data_page_size=1024, use_dictionary=["s"])
    vals, skipped = _plan_and_decode_host(path, ["b"])
    assert not skipped
    vb = _plan_and_decode_host.valid["b"]
    np.testing.assert_array_equal(vb, b.is_valid().to_numpy(zero_copy_only=False).astype(np.uint8))
    np.testing.assert_array_equal(vals["b"][vb == 1],
                                  b.drop_null().to_numpy(zero_copy_only=False).astype(np.uint8))
    assert (vals["b"][vb == 0] == 0).all()


@pytest.mark.parametrize("compression", ["none", "snappy"])
@pytest.mark.parametrize("encoding", ["PLAIN", "RLE"])
@pytest.mark.parametrize("page_version", ["1.0", "2.0"])
def test_device_page_plan_booleans(tmp_path, compression, encoding, page_version):
    """BOOLEAN chunks (bit-packed PLAIN and length-prefixed RLE pages, v1 and v2) plan for the
    device and decode to one byte per value; runs of equal values exercise the RLE runs."""
    rng = np.random.default_rng(3)
    n = 50_000
    runs = np.repeat(rng.random(n // 100) < 0.5, 100)
    t = pa.table({"b": pa.array(rng.random(n) < 0.3), "r": pa.array(runs),
                  "k": pa.array(rng.integers(0, 9, n))})
    path = tmp_path / "b.parquet"
    pq.write_table(t, path, compression=compression, use_dictionary=False,
                   column_encoding={"b": encoding, "r": encoding, "k": "PLAIN"},
                   data_page_version=page_version, row_group_size=20_000, data_page_size=2048)
    vals, skipped = _plan_and_decode_host(path, ["b", "r", "k"])
    assert not skipped
    for name in ("b", "r"):
        np.testing.assert_array_equal(vals[name], t.column(name).to_numpy().astype(np.uint8))


def test_device_page_plan_large_dictionary(tmp_path):
    """Snappy dictionary pages over 64 KiB and pages Snappy compressed (tag-dense) are inflated
    by the planner (codec 2) and still decode exactly."""
    rng = np.random.default_rng(4)
    n = 60_000
    t = pa.table({"big": pa.array(rng.integers(0, 1 << 40, n)),
                  "dbl": pa.array(np.round(rng.random(n) * 1e5, 2))})
    path = tmp_path / "d.parquet"
    pq.write_table(t, path, compression="snappy", row_group_size=40_000,
                   dictionary_pagesize_limit=1 << 21)
    vals, skipped = _plan_and_decode_host(path, ["big", "dbl"])
    assert not skipped
    for name in ("big", "dbl"):
        nd = t.column(name).to_numpy()
        np.testing.assert_array_equal(vals[name].view(nd.dtype), nd)


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
    staging.DEVICE_DECODED.clear()
    up = staging.upload_files(read_file, files, counts, schema, device, parquet_local=files)
    torch.cuda.synchronize()
    # null-free chunks were inflated and expanded on the device (file 0 has no nulls at all)
    assert set(np_types) | {"sorted"} <= staging.DEVICE_DECODED
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
    # strings: the dictionary-encoded files decode on the device (codes through the parsed
    # dictionary pages), the PLAIN-encoded file 1 through pyarrow; one global dictionary
    assert "s" in staging.DEVICE_DECODED
    # the PLAIN-encoded file's string pages decode on the device too (length-prefix walk)
    assert all(c is None for c in up.host_strings.get("s", []))
    cols = dict(up.columns)
    staging.finish_strings(up, cols, device, None)
    got = cols["s"].dictionary.take(pa.array(cols["s"].data.cpu().numpy()))
    assert got.equals(full.column("s").combine_chunks())
    assert cols["s"].dictionary.equals(pc.unique(full.column("s").combine_chunks()).sort())


@pytest.mark.gpu
def test_device_string_decode_matches_pyarrow(tmp_path, device):
    """Dictionary-encoded BYTE_ARRAY chunks decode on the device to codes over one global
    sorted dictionary: v1 and v2 pages, Snappy and uncompressed, many row groups with different
    dictionaries, a large dictionary, empty strings and multi-byte UTF-8, and a file with nulls
    (definition levels decoded on the device); the file without a dictionary (PLAIN pages)
    decodes on the device as well (value addresses from the page walk, hashed into codes)."""
    import torch
    from hyperspace_amd.exec import staging
    rng = np.random.default_rng(21)
    words = np.array(["", "a", "zz", "été", "日本", "x" * 300] +
                     [f"w{i:05d}" for i in range(20_000)], dtype=object)
    files, tables = [], []
    specs = [("snappy", True, "1.0", 6), ("none", True, "2.0", 20_006), ("snappy", True, "2.0", 40),
             ("snappy", False, "1.0", 50), ("snappy", True, "1.0", 9)]
    for i, (comp, dic, ver, card) in enumerate(specs):
        n = 25_000 + 1000 * i
        vals = words[rng.integers(0, card, n)]
        mask = (rng.random(n) < 0.05) if i == 4 else None
        t = pa.table({"s": pa.array(list(vals), pa.string(), mask=mask),
                      "k": pa.array(rng.integers(0, 1 << 40, n))})
        path = tmp_path / f"s{i}.parquet"
        pq.write_table(t, path, compression=comp, use_dictionary=dic, data_page_version=ver,
                       row_group_size=7_000, data_page_size=4096)
        files.append(str(path))
        tables.append(t)
    full = pa.concat_tables(tables)

    def read_file(p, cols=None):
        return pq.read_table(p, columns=cols)
    staging.DEVICE_DECODED.clear()
    up = staging.upload_files(read_file, files, [t.num_rows for t in tables], full.schema,
                              device, parquet_local=files)
    torch.cuda.synchronize()
    assert "s" in staging.DEVICE_DECODED
    assert all(c is None for c in up.host_strings.get("s", []))
    cols = dict(up.columns)
    staging.finish_strings(up, cols, device, None)
    c = cols["s"]
    ref = full.column("s").combine_chunks()
    assert c.dictionary.equals(pc.unique(ref.drop_null()).sort())
    valid = np.asarray(ref.is_valid())
    assert c.valid is not None
    np.testing.assert_array_equal(c.valid.cpu().numpy().astype(bool), valid)
    got = c.dictionary.take(pa.array(c.data.cpu().numpy()))
    assert got.filter(pa.array(valid)).equals(ref.drop_null())


@pytest.mark.gpu
@pytest.mark.parametrize("dictionary", [True, False])
def test_device_inflate_expand_matches_pyarrow(tmp_path, device, dictionary):
    """hs_pq_decode_pages (Snappy inflate + expand on the GPU) on streams with long overlapping
    copies (repeated 8/16-byte patterns), literal-only pages, large pages and large (host
    inflated) dictionaries."""
    import torch
    from hyperspace_amd.exec import staging
    rng = np.random.default_rng(12)
    n = 200_000
    t = pa.table({"rep": pa.array(np.tile(np.array([7, 7, 7, 9], np.int64), n // 4)),
                  "pat": pa.array(np.tile(rng.integers(0, 1 << 40, 37), n // 37 + 1)[:n]),
                  "rnd": pa.array(rng.integers(-(1 << 62), 1 << 62, n)),
                  "f": pa.array(rng.random(n).astype(np.float32)),
                  "d": pa.array(np.repeat(rng.integers(0, 1000, n // 100), 100).astype(np.int32)),
                  "const": pa.array(np.full(n, 123456789, np.int64)),
                  "mix": pa.array(np.where(rng.random(n) < 0.9, 5, rng.integers(0, 1 << 30, n))),
                  "hicard": pa.array(np.round(rng.random(n) * 1e6, 2))})
    path = tmp_path / "r.parquet"
    pq.write_table(t, path, compression="snappy", use_dictionary=dictionary,
                   row_group_size=70_000, data_page_size=1 << 20)
    staging.DEVICE_DECODED.clear()
    up = staging.upload_files(lambda p, cols=None: pq.read_table(p, columns=cols), [str(path)],
                              [n], t.schema, device, parquet_local=[str(path)])
    torch.cuda.synchronize()
    assert staging.DEVICE_DECODED == set(t.column_names)
    for name in t.column_names:
        np.testing.assert_array_equal(up.columns[name].data.cpu().numpy(),
                                      t.column(name).to_numpy())


# ------------------------------------------------------------------------------------------------
# Writer framing (csrc/runtime/hs_parquet_write.cpp) with host-packed payloads
def _pack_host(codes: np.ndarray, bw: int) -> bytes:
    """LSB-first bit-packing in groups of 8 (the contract of the hs_pq_pack kernel)."""
    n = len(codes)
    pad = (-n) % 8
    c = np.concatenate([codes.astype(np.uint64), np.zeros(pad, np.uint64)])
    bits = ((c[:, None] >> np.arange(bw, dtype=np.uint64)) & 1).astype(np.uint8).reshape(-1)
    return np.packbits(bits, bitorder="little").tobytes()


def _snappy_elements_host(raw: bytes) -> bytes:
    """Snappy elements (no preamble) of ``raw`` in 64 KiB chunks: the device kernel's output
    contract, produced by the host build of the same match finder."""
    from hyperspace_amd.ops import _lib as NL
    L = NL.lib()
    a = np.frombuffer(raw, dtype=np.uint8)
    ch = L.hs_snappy_chunk_bytes()
    out = []
    for s in range(0, len(a), ch):
        piece = np.ascontiguousarray(a[s:s + ch])
        buf = np.empty(L.hs_snappy_max_compressed(len(piece)), dtype=np.uint8)
        k = L.hs_snappy_compress_host(piece.ctypes.data, len(piece), buf.ctypes.data)
        assert k >= 0
        out.append(buf[:k].tobytes())
    return b"".join(out)


def test_snappy_compressor_round_trips_through_pyarrow():
    from hyperspace_amd.exec import pq_encode as PE
    rng = np.random.default_rng(9)
    cases = [b"", b"abc", bytes(range(256)) * 300,
             rng.integers(0, 256, 200_000).astype(np.uint8).tobytes(),       # incompressible
             np.repeat(rng.integers(0, 5, 9000), 37).astype(np.uint8).tobytes(),
             np.sort(rng.integers(0, 10**6, 50_000)).astype(np.int64).tobytes()]
    for raw in cases:
        z = PE.snappy_stream_host(np.frombuffer(raw, dtype=np.uint8))
        got = pa.decompress(z.tobytes(), len(raw), codec="snappy", asbytes=True) if raw else b""
        assert got == raw
        # element streams of independently compressed chunks concatenate
        el = _snappy_elements_host(raw)
        assert PE._varint(len(raw)) + el == z.tobytes()
    assert len(PE.snappy_stream_host(np.zeros(1 << 16, np.uint8))) < 4000


@pytest.mark.parametrize("codec", ["none", "snappy"])
def test_native_writer_round_trips_through_pyarrow_and_native_reader(tmp_path, codec):
    import ctypes as C
    from hyperspace_amd.exec import pq_encode as PE
    rng = np.random.default_rng(4)
    rgs = [1000, 777]
    n = sum(rgs)
    plain = rng.integers(-10**12, 10**12, n).astype(np.int64)
    dvals = np.array([0.0, -0.0, 0.05, 0.1, np.nan], dtype=np.float64)
    dcodes = rng.integers(0, len(dvals), n)
    dates = np.sort(rng.integers(8000, 8050, n)).astype(np.int32)
    ddict = np.unique(dates)
    date_codes = np.searchsorted(ddict, dates)
    sdict = pa.array(["A", "N", "R", "long string value"])
    scodes = rng.integers(0, len(sdict), n)
    sd_page = PE._string_dict_page(sdict)
    keep = []

    def buf(b: bytes):
        a = np.frombuffer(b, dtype=np.uint8).copy()
        keep.append(a)
        return a.ctypes.data, a.nbytes

    L = PE._writer()
    cols = (PE.WCol * (4 * len(rgs)))()
    start = 0
    for g, rows in enumerate(rgs):
        sl = slice(start, start + rows)
        specs = [("k", 2, 0, 0, 0, None, 0, plain[sl].tobytes()),
                 ("d", 5, 0, 1, 3, dvals.tobytes(), len(dvals), _pack_host(dcodes[sl], 3)),
                 ("t", 1, 1, 1, 6, ddict.tobytes(), len(ddict), _pack_host(date_codes[sl], 6)),
                 ("s", 6, 2, 1, 2, sd_page.tobytes(), len(sdict), _pack_host(scodes[sl], 2))]
        for c, (name, pt, lg, dic, bw, dpage, dcount, payload) in enumerate(specs):
            w = cols[g * 4 + c]
            w.name, w.ptype, w.logical, w.dict, w.bit_width = name.encode(), pt, lg, dic, bw
            w.codec = PE.CODEC_IDS[codec]
            if dic:
                w.dict_raw_bytes = len(dpage)
                if codec == "snappy":
                    dpage = PE.snappy_stream_host(np.frombuffer(dpage, np.uint8)).tobytes()
                w.dict_page, w.dict_bytes = buf(dpage)
                w.dict_count = dcount
            w.payload_raw_bytes = len(payload)
            if codec == "snappy":
                payload = _snappy_elements_host(payload)
            w.payload, w.payload_bytes = buf(payload)
        start += rows
    path = tmp_path / "native.parquet"
    rg = (C.c_int64 * len(rgs))(*rgs)
    assert L.hs_pq_write_file(str(path).encode(), 4, len(rgs), rg, cols, b"test") == 0
    t = pq.read_table(path)
    assert t.schema.field("t").type == pa.date32() and t.schema.field("s").type == pa.string()
    np.testing.assert_array_equal(t.column("k").to_numpy(), plain)
    got_d = t.column("d").to_numpy()
    np.testing.assert_array_equal(got_d.view(np.int64), dvals[dcodes].view(np.int64))  # bit-exact
    np.testing.assert_array_equal(t.column("t").cast(pa.int32()).to_numpy(), dates)
    assert t.column("s").to_pylist() == sdict.take(pa.array(scodes)).to_pylist()
    md = pq.ParquetFile(path).metadata
    assert md.num_row_groups == 2
    assert md.row_group(0).column(0).compression == ("SNAPPY" if codec == "snappy" else
                                                     "UNCOMPRESSED")
    st = md.row_group(0).column(0).statistics
    assert st is not None and st.has_null_count and st.null_count == 0
    # the native reader decodes the same file (dictionary + bit-packed pages)
    with NP.PqFile(str(path)) as f:
        rc, b, info, vr, lr = f.read_chunk_host(1, f.column("d"))
        assert rc == NP.OK and info.dict_encoded
        dense, _ = NP.expand_host(b, info, vr, lr, np.dtype(np.float64))
        np.testing.assert_array_equal(dense.view(np.int64), dvals[dcodes[1000:]].view(np.int64))


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["none", "snappy"])
def test_device_encoded_bucket_files(tmp_path, device, codec):
    """pq_encode: device dictionary build (sample + full-unique fallback), HIP bit-packing and
    the native writer produce bucket files pyarrow reads back bit-exactly."""
    import torch
    from hyperspace_amd.exec import pq_encode as PE
    from hyperspace_amd.exec.device_table import DeviceColumn
    rng = np.random.default_rng(12)
    n = 300_000
    dvals = np.array([0.0, -0.0, 0.05, 0.1, np.nan, 1e300], dtype=np.float64)
    data = {"plain": rng.integers(-10**15, 10**15, n).astype(np.int64),
            "lowcard": dvals[rng.integers(0, len(dvals), n)],
            # rare values the sample misses: forces the full device unique
            "rare": np.where(rng.random(n) < 0.0005, rng.integers(100, 2000, n),
                             rng.integers(0, 8, n)).astype(np.int32),
            "date": rng.integers(8000, 8100, n).astype(np.int32)}
    sdict = pa.array(sorted({f"s{i}" for i in range(37)}))
    scodes = rng.integers(0, len(sdict), n).astype(np.int32)
    cols = {k: DeviceColumn(torch.from_numpy(v).to(device), None,
                            pa.date32() if k == "date" else pa.from_numpy_dtype(v.dtype))
            for k, v in data.items()}
    cols["str"] = DeviceColumn(torch.from_numpy(scodes).to(device), None, pa.string(), sdict)
    names = list(cols)
    schema = pa.schema([pa.field(k, cols[k].atype) for k in names])
    counts = rng.multinomial(n, np.ones(16) / 16)
    counts[3] = 0
    counts[0] += n - counts.sum()
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    paths = PE.write_buckets(cols, names, schema, off,
                             lambda b: str(tmp_path / f"b{b:03d}.parquet"), 7_000, device,
                             codec=codec)
    assert paths is not None and len(paths) == 15
    for b in range(16):
        lo, hi = int(off[b]), int(off[b + 1])
        p = tmp_path / f"b{b:03d}.parquet"
        if hi == lo:
            assert not p.exists()
            continue
        t = pq.read_table(p)
        assert t.num_rows == hi - lo
        np.testing.assert_array_equal(t.column("plain").to_numpy(), data["plain"][lo:hi])
        np.testing.assert_array_equal(t.column("lowcard").to_numpy().view(np.int64),
                                      data["lowcard"][lo:hi].view(np.int64))
        np.testing.assert_array_equal(t.column("rare").to_numpy(), data["rare"][lo:hi])
        np.testing.assert_array_equal(t.column("date").cast(pa.int32()).to_numpy(),
                                      data["date"][lo:hi])
        assert t.column("str").to_pylist() == sdict.take(pa.array(scodes[lo:hi])).to_pylist()
        md = pq.ParquetFile(p).metadata
        assert md.num_row_groups == (hi - lo + 6_999) // 7_000
        assert "RLE_DICTIONARY" in md.row_group(0).column(1).encodings
        assert md.row_group(0).column(0).compression == ("SNAPPY" if codec == "snappy" else
                                                         "UNCOMPRESSED")
        # the native page layer + device decode read the same files back
        with NP.PqFile(str(p)) as f:
            rc, bb, info, vr, lr = f.read_chunk_host(0, f.column("date"))
            assert rc == NP.OK
            dense, _ = NP.expand_host(bb, info, vr, lr, np.dtype(np.int32))
            np.testing.assert_array_equal(dense[:min(7_000, hi - lo)],
                                          data["date"][lo:lo + min(7_000, hi - lo)])


@pytest.mark.gpu
def test_device_timestamp_decode_matches_pyarrow(tmp_path, device):
    """INT64 timestamps (micro- and milliseconds, with and without a dictionary, one file with
    nulls) decode through the native page layer as raw int64 in the arrow type's unit."""
    import torch
    from hyperspace_amd.exec import staging
    rng = np.random.default_rng(4)
    files, tables = [], []
    for i, (dic, nulls) in enumerate([(True, False), (False, False), (True, True)]):
        n = 20_000
        us = rng.integers(0, 2_000_000_000_000_000, n)
        mask = (rng.random(n) < 0.1) if nulls else None
        t = pa.table({"tu": pa.array(us, pa.timestamp("us"), mask=mask),
                      "tm": pa.array(us // 1000 % 1000, pa.int64()).cast(pa.timestamp("ms")),
                      "k": pa.array(rng.integers(0, 100, n))})
        path = tmp_path / f"t{i}.parquet"
        pq.write_table(t, path, use_dictionary=dic, row_group_size=6000)
        files.append(str(path))
        tables.append(pq.read_table(path))
    full = pa.concat_tables(tables)

    def read_file(p, cols=None):
        return pq.read_table(p, columns=cols)
    staging.DEVICE_DECODED.clear()
    staging.HOST_DECODED.clear()
    up = staging.upload_files(read_file, files, [t.num_rows for t in tables], full.schema,
                              device, parquet_local=files)
    torch.cuda.synchronize()
    assert {"tu", "tm"} <= staging.DEVICE_DECODED | (staging.HOST_DECODED - {"tu", "tm"})
    assert "tm" not in staging.HOST_DECODED
    for name in ("tu", "tm"):
        ref = full.column(name).combine_chunks()
        valid = np.asarray(ref.is_valid())
        got = up.columns[name].data.cpu().numpy()
        np.testing.assert_array_equal(got[valid], ref.view(pa.int64()).drop_null().to_numpy())
        if ref.null_count:
            np.testing.assert_array_equal(up.columns[name].valid.cpu().numpy().astype(bool), valid)


@pytest.mark.gpu
def test_device_boolean_decode_matches_pyarrow(tmp_path, device):
    """BOOLEAN columns (PLAIN and RLE pages, v1 and v2, one file with nulls) decode on the device
    to one byte per row; the file with nulls takes the host page layer."""
    import torch
    from hyperspace_amd.exec import staging
    rng = np.random.default_rng(6)
    files, tables = [], []
    for i, (enc, ver, nulls) in enumerate([("PLAIN", "1.0", False), ("RLE", "2.0", False),
                                           ("RLE", "1.0", False), ("PLAIN", "2.0", True)]):
        n = 30_000
        runs = np.repeat(rng.random(n // 50) < 0.5, 50)
        mask = (rng.random(n) < 0.1) if nulls else None
        t = pa.table({"b": pa.array(rng.random(n) < 0.4, mask=mask), "r": pa.array(runs),
                      "k": pa.array(rng.integers(0, 100, n))})
        path = tmp_path / f"b{i}.parquet"
        pq.write_table(t, path, use_dictionary=False, row_group_size=12_000,
                       column_encoding={"b": enc, "r": enc, "k": "PLAIN"},
                       data_page_version=ver, data_page_size=4096, compression="snappy")
        files.append(str(path))
        tables.append(pq.read_table(path))
    full = pa.concat_tables(tables)

    def read_file(p, cols=None):
        return pq.read_table(p, columns=cols)
    staging.DEVICE_DECODED.clear()
    staging.HOST_DECODED.clear()
    up = staging.upload_files(read_file, files, [t.num_rows for t in tables], full.schema,
                              device, parquet_local=files)
    torch.cuda.synchronize()
    assert "r" in staging.DEVICE_DECODED and "r" not in staging.HOST_DECODED
    assert "b" in staging.DEVICE_DECODED
    for name in ("b", "r"):
        ref = full.column(name).combine_chunks()
        valid = np.asarray(ref.is_valid())
        got = up.columns[name].data.cpu().numpy()
        np.testing.assert_array_equal(got[valid], ref.drop_null().to_numpy(zero_copy_only=False).astype(np.uint8))
        if ref.null_count:
            np.testing.assert_array_equal(up.columns[name].valid.cpu().numpy().astype(bool), valid)


@pytest.mark.parametrize("codec", ["none", "snappy"])
def test_native_writer_v2_nullable_types_and_pages(tmp_path, codec):
    """hs_pq_write_file2 (exec/pq_encode.py write_buckets): several data pages per column
    chunk, definition levels of nullable columns as one bit-packed run per page, only non-null
    values encoded; BOOLEAN bits, INT16 (INT32 + INT logical), TIMESTAMP(us, UTC), DECIMAL(12,2)
    as INT64, dictionary strings with nulls.  Pages built on the host with the device kernels'
    byte contracts; read back with pyarrow (and the null counts in the footer)."""
    import ctypes as C
    import datetime
    from hyperspace_amd.exec import pq_encode as PE
    rng = np.random.default_rng(12)
    rgs, page_rows = [2500, 1333], 700
    n = sum(rgs)
    valid = {c: rng.random(n) > p for c, p in (("x", 0.2), ("b", 0.3), ("ts", 0.1), ("dec", 0.0),
                                                  ("i16", 0.05), ("s", 0.25))}
    x = rng.random(n)
    b = rng.random(n) < 0.5
    ts = rng.integers(0, 2 * 10**15, n).astype(np.int64)
    dec = rng.integers(-10**11, 10**11, n).astype(np.int64)       # unscaled, scale 2
    i16 = rng.integers(-30000, 30000, n).astype(np.int32)
    sdict = pa.array(["aa", "b", "ccc"])
    scodes = rng.integers(0, 3, n)
    keep = []

    def buf(raw: bytes):
        a = np.frombuffer(raw, dtype=np.uint8).copy() if raw else np.zeros(1, np.uint8)
        keep.append(a)
        return a.ctypes.data, len(raw)

    # name, ptype, logical, lp0, lp1, values (full length), eb / "bits" / ("dict", bw)
    specs = [("x", 5, 0, 0, 0, x.view(np.int64), 8),
             ("b", 0, 0, 0, 0, b.astype(np.int64), "bits"),
             ("ts", 2, 4, 1, 1, ts, 8),
             ("dec", 2, 5, 12, 2, dec, 8),
             ("i16", 1, 3, 16, 1, i16.astype(np.int64), 4),
             ("s", 6, 2, 0, 0, scodes, ("dict", 2))]
    L = PE._writer()
    ncols = len(specs)
    cols = (PE.WCol2 * (ncols * len(rgs)))()
    start = 0
    for g, rows in enumerate(rgs):
        for c, (name, pt, lg, lp0, lp1, vals, how) in enumerate(specs):
            w = cols[g * ncols + c]
            w.name, w.ptype, w.logical, w.lp0, w.lp1 = name.encode(), pt, lg, lp0, lp1
            w.codec = PE.CODEC_IDS[codec]
            vm = valid[name][start:start + rows]
            w.nullable = int(not vm.all())
            w.null_count = int((~vm).sum())
            if isinstance(how, tuple):
                dp = PE._string_dict_page(sdict).tobytes()
                w.dict, w.bit_width, w.dict_count, w.dict_raw_bytes = 1, how[1], 3, len(dp)
                if codec == "snappy":
                    dp = PE.snappy_stream_host(np.frombuffer(dp, np.uint8)).tobytes()
                w.dict_page, w.dict_bytes = buf(dp)
            npg = (rows + page_rows - 1) // page_rows
            pgs = (PE.WPage * npg)()
            for q in range(npg):
                r0 = start + q * page_rows
                r1 = min(r0 + page_rows, start + rows)
                pv = valid[name][r0:r1]
                nn = vals[r0:r1][pv]
                if how == "bits":
                    raw = _pack_host(nn, 1)
                elif isinstance(how, tuple):
                    raw = _pack_host(nn, how[1])
                else:
                    raw = nn.astype({8: np.int64, 4: np.int32}[how]).tobytes()
                lev = _pack_host(pv.astype(np.int64), 1)
                pg = pgs[q]
                pg.nvals, pg.nonnull = r1 - r0, int(pv.sum())
                pg.payload_raw, pg.levels_raw = len(raw), len(lev)
                if codec == "snappy":
                    raw, lev = _snappy_elements_host(raw), _snappy_elements_host(lev)
                pg.payload, pg.payload_bytes = buf(raw)
                pg.levels, pg.levels_bytes = buf(lev)
            keep.append(pgs)
            w.pages = C.cast(pgs, C.POINTER(PE.WPage))
            w.npages = npg
        start += rows
    path = tmp_path / "v2.parquet"
    rg = (C.c_int64 * len(rgs))(*rgs)
    assert L.hs_pq_write_file2(str(path).encode(), ncols, len(rgs), rg, cols, b"test") == 0
    t = pq.read_table(path)
    sch = t.schema
    assert sch.field("b").type == pa.bool_()
    assert sch.field("ts").type == pa.timestamp("us", tz="UTC")
    assert sch.field("dec").type == pa.decimal128(12, 2)
    assert sch.field("i16").type == pa.int16()

    def expect(name, arr):
        return [v if ok else None for v, ok in zip(arr, valid[name])]
    assert t.column("x").to_pylist() == expect("x", x.tolist())
    assert t.column("b").to_pylist() == expect("b", b.tolist())
    assert t.column("ts").cast(pa.int64()).to_pylist() == expect("ts", ts.tolist())
    import decimal
    assert t.column("dec").to_pylist() == expect(
        "dec", [decimal.Decimal(int(v)).scaleb(-2) for v in dec])
    assert t.column("i16").to_pylist() == expect("i16", i16.tolist())
    assert t.column("s").to_pylist() == expect("s", sdict.take(pa.array(scodes)).to_pylist())
    md = pq.ParquetFile(path).metadata
    assert md.num_row_groups == 2
    for g in range(2):
        for c, (name, *_rest) in enumerate(specs):
            st = md.row_group(g).column(c).statistics
            lo = sum(rgs[:g])
            assert st.null_count == int((~valid[name][lo:lo + rgs[g]]).sum())
    # the native reader's page layer walks the multi-page chunks (level + value runs)
    from hyperspace_amd.io import native_parquet as NP
    with NP.PqFile(str(path)) as f:
        for name, dt, vals in (("x", np.dtype(np.float64), x), ("ts", np.dtype(np.int64), ts)):
            rc, bb, info, vr, lr = f.read_chunk_host(1, f.column(name))
            assert rc == NP.OK
            dense, vmask = NP.expand_host(bb, info, vr, lr, dt)
            sl = slice(rgs[0], n)
            np.testing.assert_array_equal(vmask.astype(bool), valid[name][sl])
            np.testing.assert_array_equal(dense.view(np.int64),
                                          vals[sl][valid[name][sl]].view(np.int64))
    assert datetime  # noqa
