"""Avro object-container files as a source format (``session.read.format("avro")``).

The reference's default source provider accepts ``avro`` (``DefaultFileBasedSource.scala:43-48``;
``IndexConstants`` default formats ``avro,csv,json,orc,parquet,text``) through Spark's Avro data
source.  Here the container header (magic, metadata map, sync marker) and the schema JSON are
parsed in Python, and the data blocks are decoded natively (``csrc/runtime/hs_avro.cpp``:
null / deflate / snappy codecs) straight into columnar buffers that become Arrow arrays.

Supported schemas: a top-level record whose fields are primitives (boolean, int, long, float,
double, bytes, string) or ``["null", primitive]`` unions, with the logical types ``date``,
``timestamp-millis`` and ``timestamp-micros`` (mapped as Spark maps them: DateType and
microsecond TimestampType).  ``write_avro`` writes the same subset (tests, examples).
"""
from __future__ import annotations

import ctypes as C
import json
import os
import struct
import threading
import zlib
from typing import List, Optional, Tuple

import numpy as np
import pyarrow as pa

from ..exceptions import HyperspaceException

MAGIC = b"Obj\x01"
_PRIM = {"null": 0, "boolean": 1, "int": 2, "long": 3, "float": 4, "double": 5, "bytes": 6,
         "string": 7}
_CODECS = {"null": 0, "deflate": 1, "snappy": 2}

_L = None
_lock = threading.Lock()


def _lib():
    global _L
    if _L is None:
        with _lock:
            if _L is None:
                from ..exec.jit import runtime
                L = runtime()
                P, I, I64 = C.c_void_p, C.c_int, C.c_int64
                L.hs_avro_decode.restype = P
                L.hs_avro_decode.argtypes = [P, I64, P, I, I, P, P]
                L.hs_avro_error.restype = C.c_char_p
                L.hs_avro_error.argtypes = [P]
                L.hs_avro_rows.restype = I64
                L.hs_avro_rows.argtypes = [P]
                L.hs_avro_buffer.restype = P
                L.hs_avro_buffer.argtypes = [P, I, I, C.POINTER(C.c_int64)]
                L.hs_avro_free.restype = None
                L.hs_avro_free.argtypes = [P]
                _L = L
    return _L


# ---------------------------------------------------------------------------------- encoding
def _zz(n: int) -> bytes:
    v = (n << 1) ^ (n >> 63)
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_long(buf: bytes, pos: int) -> Tuple[int, int]:
    v, shift = 0, 0
    while True:
        if pos >= len(buf):
            raise HyperspaceException("avro: truncated varint")
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            break
        shift += 7
    return (v >> 1) ^ -(v & 1), pos


def _read_bytes(buf: bytes, pos: int) -> Tuple[bytes, int]:
    n, pos = _read_long(buf, pos)
    return buf[pos:pos + n], pos + n


# ---------------------------------------------------------------------------------- header
def read_header(buf: bytes) -> Tuple[dict, bytes, int]:
    """(metadata, sync marker, offset of the first data block) of a container."""
    if buf[:4] != MAGIC:
        raise HyperspaceException("not an Avro object container file")
    pos, meta = 4, {}
    while True:
        n, pos = _read_long(buf, pos)
        if n == 0:
            break
        if n < 0:
            n = -n
            _, pos = _read_long(buf, pos)          # block byte size
        for _ in range(n):
            k, pos = _read_bytes(buf, pos)
            v, pos = _read_bytes(buf, pos)
            meta[k.decode()] = v
    return meta, buf[pos:pos + 16], pos + 16


def _field_type(t) -> Tuple[int, int, pa.DataType, Optional[str]]:
    """(program type, null branch or -1, arrow type, logical type) of a field schema."""
    null_branch = -1
    if isinstance(t, list):
        branches = [b if isinstance(b, str) else b.get("type") for b in t]
        if len(t) != 2 or "null" not in branches:
            raise HyperspaceException(f"avro: unsupported union {t}")
        null_branch = branches.index("null")
        t = t[1 - null_branch]
    logical = None
    if isinstance(t, dict):
        logical = t.get("logicalType")
        t = t.get("type")
    if not isinstance(t, str) or t not in _PRIM:
        raise HyperspaceException(f"avro: unsupported field type {t}")
    code = _PRIM[t]
    arrow = {1: pa.bool_(), 2: pa.int32(), 3: pa.int64(), 4: pa.float32(), 5: pa.float64(),
             6: pa.binary(), 7: pa.string(), 0: pa.null()}[code]
    if logical == "date" and code == 2:
        arrow = pa.date32()
    elif logical in ("timestamp-millis", "timestamp-micros") and code == 3:
        arrow = pa.timestamp("us")
    elif logical == "decimal":
        raise HyperspaceException("avro: decimal logical type is not supported")
    return code, null_branch, arrow, logical


def schema_of(meta: dict) -> Tuple[list, pa.Schema]:
    js = json.loads(meta["avro.schema"].decode())
    if not isinstance(js, dict) or js.get("type") != "record":
        raise HyperspaceException("avro: top-level schema must be a record")
    fields, arrow = [], []
    for f in js["fields"]:
        code, nb, at, logical = _field_type(f["type"])
        fields.append((f["name"], code, nb, logical))
        arrow.append(pa.field(f["name"], at, nullable=nb >= 0))
    return fields, pa.schema(arrow)


# ---------------------------------------------------------------------------------- read
def read_avro(path: str, columns: Optional[List[str]] = None) -> pa.Table:
    with open(path, "rb") as f:
        buf = f.read()
    meta, sync, start = read_header(buf)
    codec = meta.get("avro.codec", b"null").decode()
    if codec not in _CODECS:
        raise HyperspaceException(f"avro: unsupported codec {codec}")
    fields, schema = schema_of(meta)
    L = _lib()
    body = np.frombuffer(buf, dtype=np.uint8)[start:]
    types = np.array([f[1] for f in fields], dtype=np.int32)
    nulls = np.array([f[2] for f in fields], dtype=np.int32)
    syncb = np.frombuffer(sync, dtype=np.uint8)
    h = L.hs_avro_decode(body.ctypes.data if len(body) else None, len(body), syncb.ctypes.data,
                         _CODECS[codec], len(fields), types.ctypes.data, nulls.ctypes.data)
    try:
        err = L.hs_avro_error(h)
        if err:
            raise HyperspaceException(f"avro: {path}: {err.decode()}")
        rows = int(L.hs_avro_rows(h))
        arrays = []
        for i, (name, code, nb, logical) in enumerate(fields):
            arrays.append(_to_arrow(L, h, i, code, nb, logical, schema.field(i).type, rows))
    finally:
        L.hs_avro_free(h)
    t = pa.Table.from_arrays(arrays, schema=schema)
    if columns is not None:
        t = t.select([c for c in columns if c in t.column_names])
    return t


def _buf(L, h, i: int, which: int) -> np.ndarray:
    n = C.c_int64(0)
    p = L.hs_avro_buffer(h, i, which, C.byref(n))
    if n.value == 0:
        return np.zeros(0, dtype=np.uint8)
    return np.ctypeslib.as_array((C.c_uint8 * n.value).from_address(p)).copy()


def _to_arrow(L, h, i, code, nb, logical, atype, rows) -> pa.Array:
    valid = _buf(L, h, i, 1).astype(bool)
    mask = None if nb < 0 else ~valid
    if code == 0:
        return pa.nulls(rows)
    if code in (6, 7):
        offs = _buf(L, h, i, 2).view(np.int64)
        chars = _buf(L, h, i, 0)
        big = pa.large_binary() if code == 6 else pa.large_string()
        vb = None
        if mask is not None and mask.any():
            vb = pa.py_buffer(np.packbits(valid, bitorder="little"))
        arr = pa.Array.from_buffers(big, rows, [vb, pa.py_buffer(offs), pa.py_buffer(chars)])
        return arr.cast(atype)
    dt = {1: np.bool_, 2: np.int32, 3: np.int64, 4: np.float32, 5: np.float64}[code]
    vals = _buf(L, h, i, 0).view(dt)
    if logical == "timestamp-millis":
        vals = vals * 1000
    if atype == pa.date32():
        return pa.array(vals, type=pa.int32(), mask=mask).cast(pa.date32())
    if pa.types.is_timestamp(atype):
        return pa.array(vals, type=pa.int64(), mask=mask).cast(atype)
    return pa.array(vals, type=atype, mask=mask)


# ---------------------------------------------------------------------------------- write
def _avro_type(t: pa.DataType):
    if pa.types.is_boolean(t):
        return "boolean"
    if pa.types.is_int8(t) or pa.types.is_int16(t) or pa.types.is_int32(t):
        return "int"
    if pa.types.is_int64(t):
        return "long"
    if pa.types.is_float32(t):
        return "float"
    if pa.types.is_float64(t):
        return "double"
    if pa.types.is_date32(t):
        return {"type": "int", "logicalType": "date"}
    if pa.types.is_timestamp(t):
        return {"type": "long", "logicalType": "timestamp-micros"}
    if pa.types.is_string(t) or pa.types.is_large_string(t):
        return "string"
    if pa.types.is_binary(t) or pa.types.is_large_binary(t):
        return "bytes"
    raise HyperspaceException(f"avro: cannot write {t}")


def _encode_value(v, at) -> bytes:
    base = at if isinstance(at, str) else at["type"]
    if base == "boolean":
        return b"\x01" if v else b"\x00"
    if base in ("int", "long"):
        if isinstance(at, dict) and at.get("logicalType") == "date":
            import datetime as _dt
            v = (v - _dt.date(1970, 1, 1)).days
        elif isinstance(at, dict) and at.get("logicalType") == "timestamp-micros":
            import datetime as _dt
            v = (v - _dt.datetime(1970, 1, 1)) // _dt.timedelta(microseconds=1)
        return _zz(int(v))
    if base == "float":
        return struct.pack("<f", v)
    if base == "double":
        return struct.pack("<d", v)
    b = v.encode() if base == "string" else bytes(v)
    return _zz(len(b)) + b


def write_avro(path: str, table: pa.Table, codec: str = "null", block_rows: int = 4096,
               sync: Optional[bytes] = None) -> None:
    """Write ``table`` as an Avro container (every field a ``["null", T]`` union)."""
    if codec not in ("null", "deflate"):
        raise HyperspaceException(f"avro writer: codec {codec} not supported")
    fields = [{"name": f.name, "type": ["null", _avro_type(f.type)]} for f in table.schema]
    schema = {"type": "record", "name": "topLevelRecord", "fields": fields}
    sync = sync or os.urandom(16)
    meta = {"avro.schema": json.dumps(schema).encode(), "avro.codec": codec.encode()}
    out = bytearray(MAGIC)
    out += _zz(len(meta))
    for k, v in meta.items():
        out += _zz(len(k)) + k.encode() + _zz(len(v)) + v
    out += _zz(0) + sync
    cols = [table.column(i).to_pylist() for i in range(table.num_columns)]
    for s in range(0, table.num_rows, block_rows):
        e = min(table.num_rows, s + block_rows)
        blk = bytearray()
        for r in range(s, e):
            for c, f in zip(cols, fields):
                v = c[r]
                if v is None:
                    blk += _zz(0)
                else:
                    blk += _zz(1) + _encode_value(v, f["type"][1])
        data = bytes(blk)
        if codec == "deflate":
            co = zlib.compressobj(6, zlib.DEFLATED, -15)
            data = co.compress(data) + co.flush()
        out += _zz(e - s) + _zz(len(data)) + data + sync
    with open(path, "wb") as f:
        f.write(bytes(out))
