"""ctypes binding to ``libhs_kernels.so`` (the HIP/CDNA4 kernels in ``csrc/kernels``).

The C structs are mirrored with ``ctypes.Structure`` and their sizes are checked against the
library at load time, so an ABI drift fails loudly instead of corrupting kernel arguments.
On a machine with a GPU a missing library is an error (never a silent host fallback).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_HERE, "_native", "libhs_kernels.so")

MAX_COLS = 16
MAX_PREDS = 16
MAX_AGGS = 8
MAX_TERMS = 3
HASH_MAX_COLS = 8
GATHER_MAX_COLS = 32

# HsType
I8, I16, I32, I64, F32, F64, BOOL, U32, U64 = range(9)
STR = 100
STRDICT = 101   # int32 codes hashed through the dictionary's bytes (hash_partition.hip)
# PredKind
PK_INT_LIT, PK_FLT_LIT, PK_INT_COL, PK_FLT_COL, PK_IS_NULL, PK_NOT_NULL, PK_IN_SET, PK_BITMAP, \
    PK_TRUE = range(9)
# CmpOp
OP_EQ, OP_NE, OP_LT, OP_LE, OP_GT, OP_GE = range(6)
# AggKind
AK_SUM, AK_COUNT, AK_MIN, AK_MAX, AK_COUNT_STAR = range(5)


class ColDesc(C.Structure):
    _fields_ = [("data", C.c_void_p), ("valid", C.c_void_p), ("type", C.c_int32),
                ("pad", C.c_int32)]


class HashCol(C.Structure):
    _fields_ = [("data", C.c_void_p), ("valid", C.c_void_p), ("offsets", C.c_void_p),
                ("aux", C.c_void_p), ("type", C.c_int32), ("xform", C.c_int32)]


# HashCol.xform (csrc/kernels/hash_partition.hip): value transform before hashing
XF_NONE, XF_DECIMAL, XF_MUL, XF_FDIV = 0, 0x100, 0x200, 0x300


class HashParams(C.Structure):
    _fields_ = [("cols", HashCol * HASH_MAX_COLS), ("ncols", C.c_int32),
                ("num_buckets", C.c_int32), ("seed", C.c_uint32), ("pad", C.c_int32)]


class Pred(C.Structure):
    _fields_ = [("kind", C.c_int32), ("op", C.c_int32), ("col", C.c_int32), ("col2", C.c_int32),
                ("group", C.c_int32), ("set_len", C.c_int32), ("ilit", C.c_int64),
                ("flit", C.c_double), ("set", C.c_void_p)]


class AggSpec(C.Structure):
    _fields_ = [("kind", C.c_int32), ("nterms", C.c_int32), ("col", C.c_int32 * MAX_TERMS),
                ("pad", C.c_int32), ("alpha", C.c_double * MAX_TERMS),
                ("beta", C.c_double * MAX_TERMS)]


class ScanParams(C.Structure):
    _fields_ = [("cols", ColDesc * MAX_COLS), ("preds", Pred * MAX_PREDS),
                ("aggs", AggSpec * MAX_AGGS), ("npreds", C.c_int32), ("naggs", C.c_int32),
                ("group_col", C.c_int32), ("num_groups", C.c_int32), ("group_base", C.c_int64)]


class JoinParams(C.Structure):
    _fields_ = [("cols", ColDesc * MAX_COLS), ("preds", Pred * MAX_PREDS),
                ("aggs", AggSpec * MAX_AGGS), ("npreds", C.c_int32), ("nlp", C.c_int32),
                ("naggs", C.c_int32), ("lkey", C.c_int32), ("rkey", C.c_int32),
                ("group_col", C.c_int32), ("num_groups", C.c_int32), ("key_is_float", C.c_int32),
                ("group_base", C.c_int64)]


class SortKeySpec(C.Structure):
    _fields_ = [("col", ColDesc), ("kmin", C.c_uint64), ("bits", C.c_int32),
                ("has_nulls", C.c_int32)]


MERGE_MAX_KEYS = 8


class MergeKeys(C.Structure):
    _fields_ = [("col", ColDesc * MERGE_MAX_KEYS), ("kmin", C.c_uint64 * MERGE_MAX_KEYS),
                ("bits", C.c_int32 * MERGE_MAX_KEYS), ("nullable", C.c_int32 * MERGE_MAX_KEYS),
                ("nkeys", C.c_int32), ("pad", C.c_int32)]


class GatherCol(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("src_valid", C.c_void_p),
                ("dst_valid", C.c_void_p), ("elem_bytes", C.c_int32), ("pad", C.c_int32)]


class GatherParams(C.Structure):
    _fields_ = [("cols", GatherCol * GATHER_MAX_COLS), ("ncols", C.c_int32),
                ("idx_is_u32", C.c_int32)]


XCH_MAX_COLS = 32
XCH_MAX_DEST = 64


class XchParams(C.Structure):
    _fields_ = [("src", C.c_void_p * XCH_MAX_COLS), ("elem_bytes", C.c_int32 * XCH_MAX_COLS),
                ("ncols", C.c_int32), ("world", C.c_int32)]


class XchCopy(C.Structure):
    _fields_ = [("src", C.c_void_p), ("dst", C.c_void_p), ("count", C.c_int64),
                ("elem_bytes", C.c_int32), ("pad", C.c_int32)]


_lib = None


class NativeMissing(RuntimeError):
    pass


def _sig(fn, restype, *args):
    fn.restype = restype
    fn.argtypes = list(args)


def bind_hip_runtime() -> None:
    """Load torch (and with it the HIP runtime torch ships) before any of our libraries.

    Our .so files need ``libamdhip64.so.7``; torch bundles its own copy with the same SONAME.
    Whichever loads first is the one the process uses, and two HIP runtimes must never be
    mixed (torch's streams, allocations and contexts belong to its copy): loading ours first
    made a later torch share /opt/rocm's runtime and launches failed with hipErrorNoDevice."""
    import torch  # noqa: F401


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeMissing(f"{LIB_PATH} not built; run `python -m hyperspace_amd._native.build`")
    bind_hip_runtime()
    L = C.CDLL(LIB_PATH)
    P, I, I64, U64 = C.c_void_p, C.c_int, C.c_int64, C.c_uint64
    for name, st in (("hs_hash_params_size", HashParams), ("hs_scan_params_size", ScanParams),
                     ("hs_join_params_size", JoinParams), ("hs_sort_key_spec_size", SortKeySpec),
                     ("hs_gather_params_size", GatherParams), ("hs_xch_params_size", XchParams),
                     ("hs_xch_copy_size", XchCopy), ("hs_merge_keys_size", MergeKeys)):
        f = getattr(L, name)
        f.restype = C.c_int
        if f() != C.sizeof(st):
            raise RuntimeError(f"ABI mismatch for {st.__name__}: lib {f()} vs ctypes {C.sizeof(st)}")
    _sig(L.hs_murmur3_bucket, I, P, I64, P, P, P)
    _sig(L.hs_murmur3_hash, I, P, I64, P, P)
    _sig(L.hs_sort_workspace_bytes, I64, I64)
    _sig(L.hs_sort_columns, I, P, I, I64, P, I, P, I64, P)
    _sig(L.hs_merge_make_keys, I, P, I64, P, P)
    _sig(L.hs_merge_round, I, P, P, P, P, P, I, I64, P)
    _sig(L.hs_scan_tmp_elems, I64, I64)
    _sig(L.hs_exclusive_scan_i64, I, P, P, I64, P, I64, P)
    _sig(L.hs_exclusive_scan_u32, I, P, P, I64, P, I64, P)
    _sig(L.hs_gather, I, P, P, I64, P)
    _sig(L.hs_gather_packed, I, P, I, I, I64, P, P, I64, P)
    _sig(L.hs_bucket_offsets, I, P, I64, I, P, P)
    _sig(L.hs_scan_tile_rows, I)
    _sig(L.hs_scan_grid, I)
    _sig(L.hs_join_tile_rows, I)
    _sig(L.hs_range_search, I, P, P, P, I, I, U64, I, I, U64, I, P, P, P, P)
    _sig(L.hs_range_search_dev, I, P, P, P, I, P, P, P, P, P)
    _sig(L.hs_ranges_to_tiles, I, P, I, I, P, P)
    _sig(L.hs_ranges_to_tiles_aligned, I, P, P, I, I, I64, P, P)
    _sig(L.hs_scan_agg, I, P, P, P, I, P, I, P, P, P, P, P, P, P, P, P)
    _sig(L.hs_scan_count, I, P, P, P, I, P, I, P, P)
    _sig(L.hs_scan_select, I, P, P, P, I, P, P, I, P, P)
    _sig(L.hs_scan_bitmap, I, P, P, P, I, P, I, I, I64, I64, P, P)
    _sig(L.hs_join_agg, I, P, P, P, P, P, I, P, I64, P, I, P, P, P, P, P, P, P, P, P)
    _sig(L.hs_agg_final, I, P, P, P, P, I, I, P, P, P, P, P)
    _sig(L.hs_join_count, I, P, P, P, P, P, I, P, I64, P, I, P, P)
    _sig(L.hs_join_emit, I, P, I, P, P, I, P, P, P, P)
    _sig(L.hs_join_spans, I, P, P, P, P, P, I, P, I64, P, I, P)
    _sig(L.hs_join_spans_sampled, I, P, P, P, P, P, P, I, I64, P, I, P, I64, P, I, I, P)
    _sig(L.hs_join_sample_stride, I)
    _sig(L.hs_join_index, I, P, I, P, P, I, P, P)
    _sig(L.hs_pq_decode_values, I, P, P, I64, I64, I64, I, P, P)
    _sig(L.hs_pq_decode_levels, I, P, P, I64, P, P)
    _sig(L.hs_pq_pack, I, P, P, I, I64, I, P, P, P)
    _sig(L.hs_pq_dict_mark, I, P, P, I, I64, I, P, P)
    _sig(L.hs_pq_dict_remap, I, P, P, I, I64, I, P, P, P)
    _sig(L.hs_pq_warmup, I, P)
    _sig(L.hs_pq_decode_pages, I, P, P, P, I, P, P)
    _sig(L.hs_pq_page_struct_size, I)
    _sig(L.hs_pq_dict_codes, I, P, I64, I, P, I, P, P, P)
    _sig(L.hs_histogram, I, P, I64, I, P, P)
    _sig(L.hs_xch_tile_rows, I)
    _sig(L.hs_xch_pack, I, P, P, I64, P, P, P, P)
    _sig(L.hs_xch_unpack, I, P, I, I64, P)
    _sig(L.hs_probe_ranges, I, P, P, P, P, I, P, P, P, P)
    _sig(L.hs_compact_result_size, I)
    _sig(L.hs_compact_probe, I, P, P, I64, I, I, P, P, P)
    _sig(L.hs_compact_probe_ws_elems, I64)
    _sig(L.hs_compact_encode, I, P, P, I64, I, I, I64, I64, I, P, P)
    _sig(L.hs_key_runs_mask, I, P, I64, P, P, P)
    _sig(L.hs_key_runs_fill, I, P, I64, P, P, P, P, P)
    _sig(L.hs_tile_runs, I, P, I, P, P, P, I64, P, P)
    _sig(L.hs_run_rowmask, I, P, P, P, I64, I64, P, P)
    _sig(L.hs_run_bitmap_tags, I, P, I64, I64, P, I64, P, P)
    _sig(L.hs_key_bitmap, I, P, I64, I64, I64, P, P, P)
    _sig(L.hs_bitmap_popcount, I, P, I64, P, P)
    _sig(L.hs_str_hash64, I, P, P, I64, P, P)
    _sig(L.hs_str_gather, I, P, P, P, I64, P, P)
    _sig(L.hs_str_differ, I, P, P, P, P, I64, P, P)
    _sig(L.hs_snappy_max_compressed, I64, I64)
    _sig(L.hs_snappy_chunk_bytes, I)
    _sig(L.hs_snappy_compress, I, P, I, P, I64, P, P)
    _sig(L.hs_snappy_pack, I, P, I64, P, P, I, P, P)
    _sig(L.hs_snappy_compress_host, I64, P, I64, P)
    _sig(L.hs_mark_rows, I, P, I64, P, P)
    _sig(L.hs_select_marked_blocks, I64, I64)
    _sig(L.hs_select_marked, I, P, I64, P, I, P, P, P, P)
    _sig(L.hs_topk_levels, I)
    _sig(L.hs_topk_bins, I)
    _sig(L.hs_hagg_init, I, P, P, P, P, P, I64, I, P)
    _sig(L.hs_hagg_extract_blocks, I64, I64)
    _sig(L.hs_hagg_extract, I, P, P, P, P, P, I64, I, I, I, P, P, P, I64, P, P, P, P, P, P, P)
    _sig(L.hs_hagg_merge, I, P, P, P, P, P, P, I64, I64, P, P, P, P, P, I64, I, P, P)
    _sig(L.hs_topk_images, I, P, P, P, P, P, P, I64, I64, I, I, I, I, U64, I, I, P, P)
    _sig(L.hs_topk_select, I, P, I64, I64, P, P, P, P, P)
    _sig(L.hs_topk_runs_threshold, I, P, P, I64, P, P)
    _sig(L.hs_topk_runs_fd, I, P, I, I, I64, I, U64, P, P, I, P, I, P, P)
    _sig(L.hs_topk_runs_images, I, P, P, P, I64, U64, P, P, P, I64, I, I, I, I, P, P)
    _sig(L.hs_topk_runs_gather, I, P, P, I, P, P, P, P, I64, U64, P, P, P, P, I64, P, P, I, P,
         P)
    _sig(L.hs_hagg_take, I, P, I64, P, P, P, P, P, P, I, I64, I64, P, P, P, P, P, P, P)
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with code {rc}")


def raw_stream() -> int:
    """The current HIP stream of the current device as an integer handle, without building a
    ``torch.cuda.Stream`` (every kernel launch and graph replay asks for it)."""
    import torch
    return torch._C._cuda_getCurrentRawStream(torch._C._cuda_getDevice())


def stream_ptr():
    return C.c_void_p(raw_stream())


def ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def available() -> bool:
    try:
        lib()
        return True
    except (NativeMissing, OSError):
        return False
