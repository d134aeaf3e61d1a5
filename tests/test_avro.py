"""Avro source (``DefaultFileBasedSource.scala:43-48`` lists avro among the default formats):
the container layout pinned by a hand-assembled file from the Avro 1.x spec, round trips through
the native block decoder (null / deflate / snappy codecs, nullable unions, logical types), and a
covering index built on an Avro source used by FilterIndexRule (disabled-vs-enabled oracle)."""
import datetime
import json
import os
import struct
import zlib

import pyarrow as pa
import pytest

from hyperspace_amd import Hyperspace, IndexConfig, col
from hyperspace_amd.exceptions import HyperspaceException
from hyperspace_amd.io import avro

from helpers import make_session, verify_index_usage


@pytest.fixture(scope="module", autouse=True)
def _runtime():
    from hyperspace_amd.exec import jit
    if not os.path.exists(jit.RUNTIME_PATH):
        pytest.skip("runtime library not built")


def _zz(n):
    return avro._zz(n)


def _container(schema: dict, blocks, codec=b"null", sync=b"S" * 16) -> bytes:
    meta = {b"avro.schema": json.dumps(schema).encode(), b"avro.codec": codec}
    out = bytearray(b"Obj\x01")
    out += _zz(len(meta))
    for k, v in meta.items():
        out += _zz(len(k)) + k + _zz(len(v)) + v
    out += _zz(0) + sync
    for count, payload in blocks:
        out += _zz(count) + _zz(len(payload)) + payload + sync
    return bytes(out)


def test_hand_assembled_container(tmp_path):
    # record {a: long, s: ["null", "string"]}: (1, "x"), (-2, null), (300, "héllo")
    schema = {"type": "record", "name": "r",
              "fields": [{"name": "a", "type": "long"}, {"name": "s", "type": ["null", "string"]}]}
    rec = (b"\x02" + b"\x02\x02x" +                       # a=1 (zigzag 2); branch 1, len 1, "x"
           b"\x03" + b"\x00" +                            # a=-2 (zigzag 3); branch 0 = null
           b"\xd8\x04" + b"\x02" + _zz(6) + "héllo".encode())   # a=300 (zigzag 600)
    p = tmp_path / "golden.avro"
    p.write_bytes(_container(schema, [(3, rec)]))
    t = avro.read_avro(str(p))
    assert t.schema == pa.schema([pa.field("a", pa.int64(), nullable=False),
                                  pa.field("s", pa.string())])
    assert t.column("a").to_pylist() == [1, -2, 300]
    assert t.column("s").to_pylist() == ["x", None, "héllo"]


def test_snappy_codec_block_with_crc(tmp_path):
    schema = {"type": "record", "name": "r", "fields": [{"name": "v", "type": "int"}]}
    raw = b"".join(_zz(v) for v in (7, -1, 123456))
    # literal-only snappy stream: varint length, then a literal tag (len - 1) << 2
    comp = bytes([len(raw)]) + bytes([(len(raw) - 1) << 2]) + raw
    crc = struct.pack(">I", zlib.crc32(raw) & 0xFFFFFFFF)
    p = tmp_path / "s.avro"
    p.write_bytes(_container(schema, [(3, comp + crc)], codec=b"snappy"))
    assert avro.read_avro(str(p)).column("v").to_pylist() == [7, -1, 123456]
    bad = comp + struct.pack(">I", (zlib.crc32(raw) + 1) & 0xFFFFFFFF)
    p.write_bytes(_container(schema, [(3, bad)], codec=b"snappy"))
    with pytest.raises(HyperspaceException, match="CRC"):
        avro.read_avro(str(p))


def test_hostile_block_lengths_are_errors_not_allocations(tmp_path):
    """A Snappy preamble claiming 2^35 bytes, and a deflate bomb past the ~1032:1 DEFLATE bound,
    are rejected before any allocation of that size."""
    schema = {"type": "record", "name": "r", "fields": [{"name": "v", "type": "int"}]}
    huge = bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x7F])     # varint ~2^35
    body = huge + bytes([0]) + b"\x00" * 4
    p = tmp_path / "h.avro"
    p.write_bytes(_container(schema, [(1, body)], codec=b"snappy"))
    with pytest.raises(HyperspaceException, match="snappy"):
        avro.read_avro(str(p))
    # valid raw-deflate stream whose output exceeds the DEFLATE expansion bound for its size:
    # impossible for real data, so truncate a legit stream's output claim by corrupting it
    co = zlib.compressobj(9, zlib.DEFLATED, -15)
    bomb = co.compress(b"\x00" * (8 << 20)) + co.flush()
    assert len(bomb) * 1032 + 4096 > (8 << 20)      # a genuine stream stays inside the bound
    p2 = tmp_path / "d.avro"
    p2.write_bytes(_container(schema, [(1, bomb[: len(bomb) // 2])], codec=b"deflate"))
    with pytest.raises(HyperspaceException, match="deflate"):
        avro.read_avro(str(p2))


@pytest.mark.parametrize("codec", ["null", "deflate"])
def test_round_trip_all_types(tmp_path, codec):
    n = 10_000
    t = pa.table({
        "b": pa.array([i % 3 == 0 if i % 7 else None for i in range(n)], pa.bool_()),
        "i": pa.array([i - 5000 if i % 11 else None for i in range(n)], pa.int32()),
        "l": pa.array([(i * 7919) << 20 for i in range(n)], pa.int64()),
        "f": pa.array([i / 4.0 for i in range(n)], pa.float32()),
        "d": pa.array([i * 0.01 if i % 5 else None for i in range(n)], pa.float64()),
        "s": pa.array([f"k{i % 97}" if i % 13 else None for i in range(n)], pa.string()),
        "y": pa.array([bytes([i % 256, 0, 1]) for i in range(n)], pa.binary()),
        "dt": pa.array([datetime.date(2000, 1, 1) + datetime.timedelta(days=i) for i in range(n)]),
        "ts": pa.array([datetime.datetime(2020, 1, 1) + datetime.timedelta(microseconds=37 * i)
                        for i in range(n)], pa.timestamp("us")),
    })
    p = str(tmp_path / f"rt_{codec}.avro")
    avro.write_avro(p, t, codec=codec, block_rows=777)
    back = avro.read_avro(p)
    for name in t.column_names:
        assert back.column(name).to_pylist() == t.column(name).to_pylist(), name
    assert back.column("dt").type == pa.date32() and back.column("ts").type == pa.timestamp("us")


def test_corrupt_sync_marker_is_an_error(tmp_path):
    p = str(tmp_path / "c.avro")
    avro.write_avro(p, pa.table({"x": pa.array([1, 2, 3], pa.int64())}))
    data = bytearray(open(p, "rb").read())
    data[-1] ^= 0xFF
    open(p, "wb").write(bytes(data))
    with pytest.raises(HyperspaceException, match="sync"):
        avro.read_avro(p)


def test_covering_index_on_avro_source(tmp_path):
    src = tmp_path / "avro_src"
    src.mkdir()
    rows = 2_000
    for part in range(3):
        ids = list(range(part * rows, (part + 1) * rows))
        avro.write_avro(str(src / f"part-{part}.avro"), pa.table({
            "id": pa.array(ids, pa.int64()),
            "name": pa.array([f"n{i % 50}" for i in ids]),
            "score": pa.array([float(i % 17) for i in ids])}), codec="deflate")
    s = make_session(tmp_path)
    df = s.read.format("avro").load(str(src))
    assert df.count() == 3 * rows
    hs = Hyperspace(s)
    hs.createIndex(df, IndexConfig("avroIdx", ["name"], ["score"]))
    verify_index_usage(s, lambda: s.read.avro(str(src)).filter(col("name") == "n7")
                       .select("name", "score"), {"avroIdx"})
