"""Spark-compatible Murmur3_x86_32 bucketing — vectorized numpy reference implementation.

This is the CPU oracle for the HIP kernel ``hs_murmur3_bucket`` (csrc/kernels/hash_partition.hip)
and the CPU executor's shuffle.  Semantics follow Spark's ``Murmur3Hash(children, seed=42)``
as used by ``HashPartitioning.partitionIdExpression = pmod(hash, numPartitions)``
(reference call sites: ``CreateActionBase.scala:129-130``, ``DataFrameWriterExtensions.scala:57-66``):

* columns chain: the running hash of column i is the seed of column i+1; a null leaves it as is;
* int/short/byte/bool/date -> ``hashInt``; long/timestamp -> ``hashLong``;
* float/double hash their IEEE bits (``floatToIntBits`` / ``doubleToLongBits``: canonical NaN,
  -0.0 keeps its sign bit — Spark 2.4.2, the version the reference pins (``build.sbt:19``); the
  -0.0 -> 0.0 rewrite inside hash expressions is Spark 3.x);
* decimal(p <= 18) hashes its unscaled long; timestamps hash microseconds (floor for ns);
* strings -> ``hashUnsafeBytes`` with Spark's non-standard tail (each trailing byte is mixed as
  its own sign-extended int).

Golden vectors: ``BucketUnionTest.scala:101-122`` (h(2)=1765031574 -> bucket 4 of 10,
h(3)=-1823081949 -> bucket 1 of 10).
"""
from __future__ import annotations

import numpy as np

SEED = 42
C1 = np.uint32(0xCC9E2D51)
C2 = np.uint32(0x1B873593)
M5 = np.uint32(5)
N1 = np.uint32(0xE6546B64)
F1 = np.uint32(0x85EBCA6B)
F2 = np.uint32(0xC2B2AE35)


def _rotl(x, r):
    return (x << np.uint32(r)) | (x >> np.uint32(32 - r))


def _mix_k1(k1):
    k1 = k1 * C1
    k1 = _rotl(k1, 15)
    return k1 * C2


def _mix_h1(h1, k1):
    h1 = h1 ^ k1
    h1 = _rotl(h1, 13)
    return h1 * M5 + N1


def _fmix(h1, length):
    h1 = h1 ^ np.uint32(length) if np.isscalar(length) else h1 ^ length.astype(np.uint32)
    h1 = h1 ^ (h1 >> np.uint32(16))
    h1 = h1 * F1
    h1 = h1 ^ (h1 >> np.uint32(13))
    h1 = h1 * F2
    return h1 ^ (h1 >> np.uint32(16))


def hash_int(values, seed):
    with np.errstate(over="ignore"):
        v = np.asarray(values).astype(np.int64).astype(np.uint32)
        s = np.asarray(seed).astype(np.int64).astype(np.uint32)
        return _fmix(_mix_h1(s, _mix_k1(v)), 4)


def hash_long(values, seed):
    with np.errstate(over="ignore"):
        v = np.asarray(values).astype(np.int64).view(np.uint64) if np.asarray(values).dtype == np.int64 \
            else np.asarray(values).astype(np.int64).view(np.uint64)
        lo = (v & np.uint64(0xFFFFFFFF)).astype(np.uint32)
        hi = (v >> np.uint64(32)).astype(np.uint32)
        s = np.asarray(seed).astype(np.int64).astype(np.uint32)
        h1 = _mix_h1(s, _mix_k1(lo))
        h1 = _mix_h1(h1, _mix_k1(hi))
        return _fmix(h1, 8)


def hash_bytes(b: bytes, seed: int) -> int:
    """Scalar ``hashUnsafeBytes`` (Spark tail semantics). Returns uint32."""
    with np.errstate(over="ignore"):
        h1 = np.uint32(seed & 0xFFFFFFFF)
        n = len(b)
        aligned = n - n % 4
        if aligned:
            words = np.frombuffer(b[:aligned], dtype="<u4")
            for w in words:
                h1 = _mix_h1(h1, _mix_k1(np.uint32(w)))
        for i in range(aligned, n):
            byte = b[i] - 256 if b[i] > 127 else b[i]
            h1 = _mix_h1(h1, _mix_k1(np.uint32(byte & 0xFFFFFFFF)))
        return int(_fmix(h1, n))


def _to_signed(u32):
    return np.asarray(u32, dtype=np.uint32).view(np.int32)


def hash_column(arr, seed):
    """Hash one pyarrow/numpy column with per-row seeds; returns uint32 array.

    ``arr`` is a pyarrow Array/ChunkedArray (preferred, carries type+nulls) or numpy array.
    Nulls keep the incoming seed.
    """
    import pyarrow as pa
    import pyarrow.compute as pc

    if isinstance(arr, pa.ChunkedArray):
        arr = arr.combine_chunks()
    n = len(arr)
    seed = np.broadcast_to(np.asarray(seed, dtype=np.uint32), (n,)).copy()
    if not isinstance(arr, pa.Array):
        arr = pa.array(arr)
    t = arr.type
    valid = None
    if arr.null_count:
        valid = np.asarray(arr.is_valid().to_numpy(zero_copy_only=False), dtype=bool)
    if pa.types.is_dictionary(t):
        arr = arr.cast(t.value_type)
        t = arr.type
    if pa.types.is_boolean(t):
        vals = np.asarray(arr.fill_null(False).to_numpy(zero_copy_only=False)).astype(np.int32)
        h = hash_int(vals, seed)
    elif pa.types.is_integer(t) and t.bit_width <= 32:
        h = hash_int(np.asarray(arr.fill_null(0).to_numpy()).astype(np.int32), seed)
    elif pa.types.is_integer(t):
        h = hash_long(np.asarray(arr.fill_null(0).to_numpy()).astype(np.int64), seed)
    elif pa.types.is_date32(t):
        h = hash_int(np.asarray(arr.cast(pa.int32()).fill_null(0).to_numpy()), seed)
    elif pa.types.is_timestamp(t):
        raw = np.asarray(arr.view(pa.int64()).fill_null(0).to_numpy(zero_copy_only=False),
                         dtype=np.int64)
        k = {"s": 6, "ms": 3, "us": 0, "ns": -3}[t.unit]
        micros = raw * (10 ** k) if k >= 0 else np.floor_divide(raw, 10 ** -k)
        h = hash_long(micros, seed)
    elif pa.types.is_float32(t):
        f = np.asarray(arr.fill_null(0).to_numpy(), dtype=np.float32).copy()
        bits = f.view(np.int32).copy()
        bits[np.isnan(f)] = 0x7FC00000
        h = hash_int(bits, seed)
    elif pa.types.is_float64(t):
        f = np.asarray(arr.fill_null(0).to_numpy(), dtype=np.float64).copy()
        bits = f.view(np.int64).copy()
        bits[np.isnan(f)] = 0x7FF8000000000000
        h = hash_long(bits, seed)
    elif pa.types.is_decimal(t) and t.precision <= 18:
        scaled = [None if v is None else int(v.scaleb(t.scale).to_integral_value())
                  for v in arr.to_pylist()]
        h = hash_long(np.array([0 if v is None else v for v in scaled], dtype=np.int64), seed)
    elif pa.types.is_string(t) or pa.types.is_large_string(t) or pa.types.is_binary(t) \
            or pa.types.is_large_binary(t):
        h = hash_strings(arr, seed)
    else:
        raise TypeError(f"murmur3: unsupported column type {t}")
    h = np.asarray(h, dtype=np.uint32)
    if valid is not None:
        h = np.where(valid, h, seed)
    return h


def hash_strings(arr, seed):
    """Vectorized ``hashUnsafeBytes`` over a pyarrow string/binary array (per-row seed)."""
    import pyarrow as pa
    if pa.types.is_large_string(arr.type) or pa.types.is_large_binary(arr.type):
        offs_dtype = np.int64
    else:
        offs_dtype = np.int32
    arr = arr.fill_null("") if pa.types.is_string(arr.type) or pa.types.is_large_string(arr.type) \
        else arr.fill_null(b"")
    bufs = arr.buffers()
    offsets = np.frombuffer(bufs[1], dtype=offs_dtype)[arr.offset:arr.offset + len(arr) + 1].astype(np.int64)
    data = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else np.zeros(0, np.uint8)
    n = len(arr)
    lens = offsets[1:] - offsets[:-1]
    offsets = offsets[:-1]
    h1 = np.asarray(seed, dtype=np.uint32).copy()
    maxlen = int(lens.max()) if n else 0
    padded = np.concatenate([data, np.zeros(8, np.uint8)])
    with np.errstate(over="ignore"):
        for i in range(0, maxlen - maxlen % 4 + 4, 4):
            active = lens - lens % 4 > i
            if not active.any():
                break
            idx = offsets[active] + i
            w = (padded[idx].astype(np.uint32) | (padded[idx + 1].astype(np.uint32) << np.uint32(8))
                 | (padded[idx + 2].astype(np.uint32) << np.uint32(16))
                 | (padded[idx + 3].astype(np.uint32) << np.uint32(24)))
            h1[active] = _mix_h1(h1[active], _mix_k1(w))
        for j in range(3):
            active = (lens % 4) > j
            if not active.any():
                continue
            idx = offsets[active] + (lens[active] - lens[active] % 4) + j
            b = padded[idx].astype(np.int8).astype(np.int32).astype(np.uint32)
            h1[active] = _mix_h1(h1[active], _mix_k1(b))
        return _fmix(h1, lens.astype(np.uint32))


def hash_columns(columns, seed: int = SEED):
    """Chain-hash a list of pyarrow columns (row-wise), returns int32 hash values."""
    n = len(columns[0])
    h = np.full(n, seed & 0xFFFFFFFF, dtype=np.uint32)
    for c in columns:
        h = hash_column(c, h)
    return _to_signed(h)


def pmod(h, n: int):
    return np.mod(np.asarray(h, dtype=np.int64), n).astype(np.int32)


def bucket_ids(columns, num_buckets: int):
    return pmod(hash_columns(columns), num_buckets)
