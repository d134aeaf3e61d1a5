"""Device-resident columnar tables (HBM) for the MI355X executor.

A ``DeviceColumn`` is a 1-D torch tensor on the GPU (fixed-width values) plus an optional uint8
validity mask.  Strings live on the device as int32 codes into a host-side *sorted* dictionary, so
code order == string order and range/equality predicates on strings become integer predicates.
Raw string bytes (offsets + chars) are uploaded only where Spark-compatible hashing needs them.

A ``DeviceTable`` optionally carries bucket offsets (``B+1`` int64, device + host copies): rows of
bucket ``b`` are ``[off[b], off[b+1])`` and sorted by the index's indexed columns.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc

from ..ops import _lib as NL


def _torch():
    import torch
    return torch


_NP_TO_HS = {np.dtype(np.int8): NL.I8, np.dtype(np.int16): NL.I16, np.dtype(np.int32): NL.I32,
             np.dtype(np.int64): NL.I64, np.dtype(np.float32): NL.F32,
             np.dtype(np.float64): NL.F64, np.dtype(np.uint8): NL.BOOL,
             np.dtype(np.uint32): NL.U32, np.dtype(np.uint64): NL.U64}
_HS_OF_TORCH: dict = {}     # torch dtype -> HS type (DeviceColumn.hs_type)


def storage_numpy_dtype(t: pa.DataType) -> np.dtype:
    if pa.types.is_boolean(t):
        return np.dtype(np.uint8)
    if pa.types.is_date32(t):
        return np.dtype(np.int32)
    if pa.types.is_date64(t) or pa.types.is_timestamp(t) or pa.types.is_duration(t):
        return np.dtype(np.int64)
    if pa.types.is_string(t) or pa.types.is_large_string(t) or pa.types.is_dictionary(t):
        return np.dtype(np.int32)
    if pa.types.is_decimal(t):
        return np.dtype(np.float64)
    return np.dtype(t.to_pandas_dtype())


def is_string(t: pa.DataType) -> bool:
    return pa.types.is_string(t) or pa.types.is_large_string(t) or (
        pa.types.is_dictionary(t) and (pa.types.is_string(t.value_type) or
                                        pa.types.is_large_string(t.value_type)))


def h2d(a: np.ndarray, device):
    torch = _torch()
    # arrow-backed numpy views are read-only: np.require copies those (torch needs writable)
    t = torch.from_numpy(np.require(a, requirements=["C", "W"]))
    if t.numel() >= (1 << 20):
        t = t.pin_memory()
        return t.to(device, non_blocking=True)
    return t.to(device)


class DeviceColumn:
    __slots__ = ("data", "valid", "atype", "dictionary", "offsets", "chars", "compact", "dupkeys",
                 "hs_transient")

    def __init__(self, data, valid, atype: pa.DataType, dictionary: Optional[pa.Array] = None,
                 offsets=None, chars=None):
        self.data = data
        self.valid = valid
        self.atype = atype
        self.dictionary = dictionary
        self.offsets = offsets
        self.chars = chars
        self.compact = False  # exec.encoding.compact_of: False = not computed, None = n/a
        self.dupkeys = None   # exec.jit.key_has_dups: None = not computed
        self.hs_transient = False   # a per-query intermediate (never compacted)

    def __len__(self):
        return int(self.data.shape[0])

    @property
    def hs_type(self) -> int:
        dt = self.data.dtype
        t = _HS_OF_TORCH.get(dt)      # on every lowering's path: one dict hit per call
        if t is None:
            t = _HS_OF_TORCH[dt] = _NP_TO_HS[np.dtype(str(dt).replace("torch.", ""))]
        return t

    @property
    def is_float(self) -> bool:
        return self.hs_type in (NL.F32, NL.F64)

    def desc(self) -> NL.ColDesc:
        return NL.ColDesc(self.data.data_ptr(), self.valid.data_ptr() if self.valid is not None else 0,
                          self.hs_type, 0)

    def nbytes(self) -> int:
        n = self.data.numel() * self.data.element_size()
        if self.valid is not None:
            n += self.valid.numel()
        return n

    # -- conversions -----------------------------------------------------------------------------
    @staticmethod
    def from_arrow(arr, device, dictionary: Optional[pa.Array] = None, raw_strings: bool = False):
        if isinstance(arr, pa.ChunkedArray):
            arr = arr.combine_chunks() if arr.num_chunks != 1 else arr.chunk(0)
        t = arr.type
        valid = None
        if arr.null_count:
            valid = h2d(np.asarray(arr.is_valid().to_numpy(zero_copy_only=False), dtype=np.uint8), device)
        if is_string(t):
            if pa.types.is_dictionary(t):
                arr = arr.cast(t.value_type)
            if dictionary is None:
                dictionary = pc.unique(arr.drop_null()).sort()
            codes = pc.index_in(arr, value_set=dictionary).fill_null(0)
            data = h2d(np.asarray(codes.to_numpy(zero_copy_only=False), dtype=np.int32), device)
            col = DeviceColumn(data, valid, pa.string(), dictionary)
            if raw_strings:
                a2 = arr.cast(pa.large_string()).fill_null("")
                bufs = a2.buffers()
                offs = np.frombuffer(bufs[1], dtype=np.int64)[a2.offset:a2.offset + len(a2) + 1]
                chars = np.frombuffer(bufs[2], dtype=np.uint8) if bufs[2] is not None else \
                    np.zeros(1, np.uint8)
                col.offsets = h2d(offs - offs[0], device)
                col.chars = h2d(chars[offs[0]:offs[-1]].copy() if len(chars) else chars, device)
            return col
        nd = storage_numpy_dtype(t)
        if pa.types.is_boolean(t):
            np_vals = np.asarray(arr.fill_null(False).to_numpy(zero_copy_only=False), dtype=np.uint8)
        elif pa.types.is_decimal(t):
            np_vals = np.asarray(arr.cast(pa.float64()).fill_null(0).to_numpy(), dtype=np.float64)
        elif pa.types.is_date32(t) or pa.types.is_timestamp(t) or pa.types.is_date64(t):
            st = pa.int32() if pa.types.is_date32(t) else pa.int64()
            np_vals = np.asarray(arr.view(st).fill_null(0).to_numpy(zero_copy_only=False), dtype=nd)
        else:
            if arr.null_count:
                arr = arr.fill_null(0)
            np_vals = np.asarray(arr.to_numpy(zero_copy_only=False), dtype=nd)
        return DeviceColumn(h2d(np_vals, device), valid, t)

    def to_arrow(self) -> pa.Array:
        vals = self.data.cpu().numpy()
        mask = None
        if self.valid is not None:
            mask = self.valid.cpu().numpy() == 0
        t = self.atype
        if self.dictionary is not None:
            idx = pa.array(vals, pa.int32(), mask=mask)
            return self.dictionary.take(idx).cast(t) if len(self.dictionary) else \
                pa.nulls(len(vals), t)
        if pa.types.is_boolean(t):
            return pa.array(vals.astype(bool), pa.bool_(), mask=mask)
        if pa.types.is_date32(t):
            return pa.array(vals.astype(np.int32), pa.int32(), mask=mask).view(pa.date32())
        if pa.types.is_timestamp(t) or pa.types.is_date64(t):
            return pa.array(vals.astype(np.int64), pa.int64(), mask=mask).view(t)
        if pa.types.is_decimal(t):
            return pa.array(vals, pa.float64(), mask=mask).cast(t)
        return pa.array(vals, t, mask=mask)


class DeviceTable:
    def __init__(self, columns: Dict[str, DeviceColumn], num_rows: int,
                 bucket_offsets=None, bucket_offsets_host: Optional[np.ndarray] = None):
        self.columns = dict(columns)
        self.num_rows = int(num_rows)
        self.bucket_offsets = bucket_offsets
        self.bucket_offsets_host = bucket_offsets_host

    @property
    def num_buckets(self) -> int:
        return 0 if self.bucket_offsets_host is None else len(self.bucket_offsets_host) - 1

    def column(self, name: str) -> DeviceColumn:
        return self.columns[name]

    def nbytes(self) -> int:
        return sum(c.nbytes() for c in self.columns.values())

    def resident_bytes(self) -> int:
        """Columns plus the structures queries derive from this table and keep on it:
        compacted copies (exec/encoding.py), join indexes (exec/join_index.py), packed
        multi-key and remapped string-key tables (exec/gpu.py) — what stays in HBM with it."""
        n = 0
        for c in self.columns.values():
            n += c.nbytes()
            comp = getattr(c, "compact", None)
            if comp:
                n += comp.nbytes()
        d = self.__dict__
        for (_, _, _, ji) in d.get("_join_index", {}).values():
            n += ji.nbytes()
        for t in d.get("_packed_keys", {}).values():
            n += t.columns["__hs_jkey"].nbytes() + sum(
                ji.nbytes() for (_, _, _, ji) in t.__dict__.get("_join_index", {}).values())
        for t in d.get("_repart", {}).values():
            n += t.resident_bytes()
        for (_, t) in d.get("_remap", {}).values():
            n += sum(c.nbytes() for k, c in t.columns.items() if c is not self.columns.get(k))
            n += sum(ji.nbytes() for (_, _, _, ji) in t.__dict__.get("_join_index", {}).values())
        return n

    @staticmethod
    def from_arrow(t: pa.Table, device, dictionaries: Optional[dict] = None) -> "DeviceTable":
        cols = {}
        for name, c in zip(t.column_names, t.columns):
            cols[name] = DeviceColumn.from_arrow(c, device, (dictionaries or {}).get(name))
        return DeviceTable(cols, t.num_rows)

    def to_arrow(self, names: Optional[List[str]] = None) -> pa.Table:
        names = names or list(self.columns)
        return pa.Table.from_arrays([self.columns[n].to_arrow() for n in names], names=names)
