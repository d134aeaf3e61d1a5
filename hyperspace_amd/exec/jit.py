"""Whole-stage code generation for the MI355X executor (hipRTC; ``csrc/runtime/hs_jit.cpp``).

The AOT kernels in ``csrc/kernels`` interpret a predicate/aggregate *description* (``Pred`` /
``AggSpec`` structs) per row batch.  That keeps one binary for every query, but the compiler
cannot see which columns a query touches: each predicate is a separate, serialized load round
trip, and the interpreter's register footprint caps occupancy.  This module emits one
straight-line HIP kernel per query *shape* instead — exact column types, the CNF as a boolean
expression, every load visible to the scheduler so all predicate columns of a row batch are in
flight at once — and compiles it with hipRTC for gfx950.  Literals (filter constants, affine
coefficients, IN-set pointers) are kernel arguments, so a shape compiles once and every later
query of that shape (e.g. TPC-H Q6 with new dates) reuses the code object.

The generated kernels write the same per-block partials as the AOT ones and share the AOT
deterministic final reduction (``hs_agg_final``), and the join kernel consumes the AOT per-tile
span records (``hs_join_spans_sampled``: cached sparse samples + galloping): codegen only
replaces the per-row inner loops.

Kernel arguments are one by-value struct whose fields are all 8 bytes wide, packed here with
``struct``; the runtime passes it with ``HIP_LAUNCH_PARAM_BUFFER_POINTER``.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import struct
import threading
from typing import Dict, List, Optional, Tuple

from ..ops import _lib as NL

ARCH = os.environ.get("HS_OFFLOAD_ARCH", "gfx950")
_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RUNTIME_PATH = os.path.join(_HERE, "_native", "libhs_runtime.so")
# in-tree cache travels with the repo snapshot; override with HS_JIT_CACHE
CACHE_DIR = os.environ.get("HS_JIT_CACHE", os.path.join(_HERE, "_native", "jitcache"))

BLOCK = 256
# Code-generation tunables: the fields of ONE frozen exec.kernel_config.KernelConfig (defaults,
# measurements and meaning are documented there), bound into these names by
# kernel_config.bind(); generated kernel shape keys include them.
from . import kernel_config as _KC  # noqa: E402
_CFG = _KC.active()
SCAN_ITEMS, SCAN_GRID, SCAN_VEC = _CFG.scan_items, _CFG.scan_grid, _CFG.scan_vec
SCAN_COMPACT, SCAN_EAGER = _CFG.scan_compact, _CFG.scan_eager
JOIN_ITEMS, JOIN_BLOCK, JOIN_LDS_KEYS, JOIN_GRID = (_CFG.join_items, _CFG.join_block,
                                                    _CFG.join_lds_keys, _CFG.join_grid)
JOIN_EAGER, JOIN_STAGE_RIGHT, JOIN_PIPELINE = (_CFG.join_eager, _CFG.join_stage_right,
                                               _CFG.join_pipeline)
JOIN_DIRECT, JOIN_DIRECT_SLOTS = _CFG.join_direct, _CFG.join_direct_slots
JI_ITEMS, JI_VEC, JI_COMPACT, JI_STAGE, JI_BITMAP = (_CFG.ji_items, _CFG.ji_vec, _CFG.ji_compact,
                                                     _CFG.ji_stage, _CFG.ji_bitmap)
MJ_ITEMS, MJ_LDS_KEYS, MJ_GRID, MJ_STEPS = (_CFG.mj_items, _CFG.mj_lds_keys, _CFG.mj_grid,
                                            _CFG.mj_steps)
MJ_STAGE_UNROLL, MJ_BLOCK = _CFG.mj_stage_unroll, _CFG.mj_block
MJ_DBUF, MJ_PREFETCH, MJ_RPF, MJ_EAGER = (_CFG.mj_dbuf, _CFG.mj_prefetch, _CFG.mj_rpf,
                                          _CFG.mj_eager)
MJ_SPARSE, MJ_HASH_LANEMAJOR = _CFG.mj_sparse, _CFG.mj_hash_lanemajor
MJ_KEY32, MJ_KEY16 = _CFG.mj_key32, _CFG.mj_key16
MJ_RUNS, MJ_RUNS_HASH, MJ_RUNS_ITEMS, MJ_RUNS_PREFETCH = (_CFG.mj_runs, _CFG.mj_runs_hash,
                                                          _CFG.mj_runs_items,
                                                          _CFG.mj_runs_prefetch)
VEC_PREFETCH, WAVE_SYNC = _CFG.vec_prefetch, _CFG.wave_sync

_CTYPE = {NL.I8: "signed char", NL.I16: "short", NL.I32: "int", NL.I64: "long long",
          NL.F32: "float", NL.F64: "double", NL.BOOL: "unsigned char", NL.U32: "unsigned int",
          NL.U64: "unsigned long long"}
_OPSTR = {NL.OP_EQ: "==", NL.OP_NE: "!=", NL.OP_LT: "<", NL.OP_LE: "<=", NL.OP_GT: ">",
          NL.OP_GE: ">="}
_CODE_T = {1: "signed char", 2: "short", 4: "int"}   # exec.encoding code widths
_SIZEOF = {"signed char": 1, "unsigned char": 1, "short": 2, "unsigned short": 2, "int": 4,
           "unsigned int": 4, "float": 4, "long long": 8, "unsigned long long": 8, "double": 8}

_rt = None
_rt_lock = threading.Lock()


def runtime():
    global _rt
    if _rt is None:
        with _rt_lock:
            if _rt is None:
                if not os.path.exists(RUNTIME_PATH):
                    raise RuntimeError(f"{RUNTIME_PATH} missing: run python -m hyperspace_amd._native.build")
                NL.bind_hip_runtime()
                L = C.CDLL(RUNTIME_PATH)
                L.hs_jit_get.restype = C.c_void_p
                L.hs_jit_get.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_char_p,
                                         C.POINTER(C.c_int)]
                L.hs_jit_launch.restype = C.c_int
                L.hs_jit_launch.argtypes = [C.c_void_p, C.c_uint, C.c_uint, C.c_uint, C.c_void_p,
                                            C.c_void_p, C.c_size_t]
                L.hs_jit_compile_to_cache.restype = C.c_int
                L.hs_jit_compile_to_cache.argtypes = [C.c_char_p] * 4
                L.hs_jit_last_error.restype = C.c_char_p
                L.hs_host_alloc.restype = C.c_void_p
                L.hs_host_alloc.argtypes = [C.c_size_t]
                L.hs_host_free.restype = None
                L.hs_host_free.argtypes = [C.c_void_p]
                L.hs_memcpy_async.restype = C.c_int
                L.hs_memcpy_async.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int,
                                              C.c_void_p]
                L.hs_stream_sync.restype = C.c_int
                L.hs_stream_sync.argtypes = [C.c_void_p]
                # captured pipelines with per-replay kernel arguments (csrc/runtime/hs_graph.cpp)
                L.hs_graph_capture_begin.restype = C.c_int
                L.hs_graph_capture_begin.argtypes = [C.c_void_p]
                L.hs_graph_capture_end.restype = C.c_void_p
                L.hs_graph_capture_end.argtypes = [C.c_void_p, C.POINTER(C.c_void_p), C.c_int]
                L.hs_graph_set_args.restype = C.c_int
                L.hs_graph_set_args.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_size_t]
                L.hs_graph_launch.restype = C.c_int
                L.hs_graph_launch.argtypes = [C.c_void_p, C.c_void_p]
                L.hs_graph_destroy.restype = None
                L.hs_graph_destroy.argtypes = [C.c_void_p]
                L.hs_graph_replay.restype = C.c_int
                L.hs_graph_replay.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                              C.c_void_p, C.c_void_p]
                L.hs_event_create.restype = C.c_void_p
                L.hs_event_create.argtypes = []
                L.hs_event_record.restype = C.c_int
                L.hs_event_record.argtypes = [C.c_void_p, C.c_void_p]
                L.hs_event_query.restype = C.c_int
                L.hs_event_query.argtypes = [C.c_void_p]
                L.hs_event_sync.restype = C.c_int
                L.hs_event_sync.argtypes = [C.c_void_p]
                L.hs_event_destroy.restype = None
                L.hs_event_destroy.argtypes = [C.c_void_p]
                L.hs_graph_last_error.restype = C.c_char_p
                _rt = L
    return _rt


# ------------------------------------------------------------------------------------------------
# Argument struct
# ------------------------------------------------------------------------------------------------
class Args:
    """Ordered 8-byte kernel argument slots: ('p'|'q'|'d', name, C type)."""

    def __init__(self):
        self.slots: List[Tuple[str, str, str]] = []
        self._index: Dict[str, int] = {}
        self._layout = None    # (struct format, [(name, is_double)]) once the slots are final

    def add(self, kind: str, name: str, ctype: str) -> str:
        if name not in self._index:
            self._index[name] = len(self.slots)
            self.slots.append((kind, name, ctype))
            self._layout = None
        return f"a.{name}"

    def struct_src(self) -> str:
        body = "".join(f"  {ct} {n};\n" for _, n, ct in self.slots)
        return "struct Args {\n" + body + "};\n"

    def offset(self, name: str) -> int:
        """Byte offset of slot ``name`` in the packed block (every slot is 8 bytes)."""
        return 8 * self._index[name]

    def _lay(self):
        lay = self._layout
        if lay is None:
            lay = self._layout = (
                "<" + "".join("q" if k in ("p", "q") else "d" for k, _, _ in self.slots),
                [(n, k == "d") for k, n, _ in self.slots])
        return lay

    def pack(self, values: Dict[str, object], default=None) -> bytes:
        """The argument block of ``values`` (every slot; ``default`` fills missing ones)."""
        fmt, names = self._lay()
        if default is None:
            vals = [float(values[n]) if d else int(values[n] or 0) for n, d in names]
        else:
            vals = [float(values.get(n, default)) if d else int(values.get(n, default) or 0)
                    for n, d in names]
        return struct.pack(fmt, *vals)

    def patch(self, block: bytearray, values: Dict[str, object]) -> bytearray:
        """``block`` (a packed template) with the slots named in ``values`` rewritten (names
        that are not slots of this kernel are skipped): a new literal vector re-packs only its
        literal slots."""
        idx = self._index
        slots = self.slots
        for n, v in values.items():
            i = idx.get(n)
            if i is None:
                continue
            if slots[i][0] == "d":
                struct.pack_into("<d", block, 8 * i, float(v))
            else:
                struct.pack_into("<q", block, 8 * i, int(v or 0))
        return block


# kernels this process compiled with hipRTC / loaded from the on-disk code-object cache
JIT_STATS = {"compiled": 0, "loaded": 0}
# committed kernel sources compiled ahead of time by aot_compile() (__graft_entry__.build)
AOT_DIR = os.path.join(_HERE, "_native", "aot")


def _record_source(directory: str, name: str, src: str) -> None:
    import hashlib
    os.makedirs(directory, exist_ok=True)
    h = hashlib.sha1(src.encode()).hexdigest()[:16]
    path = os.path.join(directory, f"{name}.{h}.hip")
    if not os.path.exists(path):
        with open(path, "w") as f:
            f.write(src)


def aot_compile(src_dir: str = AOT_DIR, cache_dir: str = None, workers: int = 8) -> int:
    """Compile every recorded kernel source in ``src_dir`` (``<kernel>.<hash>.hip``, the exact
    text the planner generates: HS_JIT_RECORD) into the code-object cache, so the first query
    of those shapes loads a code object instead of running hipRTC.  Needs no GPU.  Returns the
    number of sources."""
    import concurrent.futures as cf
    cache_dir = cache_dir or CACHE_DIR
    if not os.path.isdir(src_dir):
        return 0
    files = sorted(f for f in os.listdir(src_dir) if f.endswith(".hip"))
    L = runtime()

    def one(f):
        with open(os.path.join(src_dir, f)) as fh:
            src = fh.read()
        name = f.split(".")[0]
        rc = L.hs_jit_compile_to_cache(src.encode(), name.encode(), ARCH.encode(),
                                       cache_dir.encode())
        if rc != 0:
            raise RuntimeError(f"AOT compile of {f} failed: {L.hs_jit_last_error().decode()}")
    with cf.ThreadPoolExecutor(max_workers=max(1, workers)) as ex:
        list(ex.map(one, files))
    return len(files)


class Kernel:
    def __init__(self, src: str, name: str, args: Args, lds_bytes: int = 0, block: int = 256):
        self.src = src
        self.name = name
        self.args = args
        self.lds_bytes = lds_bytes
        self.block = block
        self._fn = None

    def function(self):
        if self._fn is None:
            L = runtime()
            dump = os.environ.get("HS_JIT_DUMP")
            if dump:   # generated sources for inspection / offline ISA (hipcc --save-temps)
                import hashlib
                os.makedirs(dump, exist_ok=True)
                h = hashlib.md5(self.src.encode()).hexdigest()[:10]
                with open(os.path.join(dump, f"{self.name}_{h}.hip"), "w") as f:
                    f.write("#include <hip/hip_runtime.h>\n" + self.src)
            rec = os.environ.get("HS_JIT_RECORD")
            if rec:    # kernel sources of a workload, for the ahead-of-time set (aot_compile)
                _record_source(rec, self.name, self.src)
            compiled = C.c_int(0)
            fn = L.hs_jit_get(self.src.encode(), self.name.encode(), ARCH.encode(),
                              CACHE_DIR.encode(), C.byref(compiled))
            if not fn:
                raise RuntimeError(f"JIT compile/load failed: {L.hs_jit_last_error().decode()}")
            JIT_STATS["compiled" if compiled.value == 1 else "loaded"] += 1
            self._fn = fn
        return self._fn

    def launch_packed(self, grid: int, buf, stream_ptr: int, shmem: int = 0) -> None:
        """Launch with an already packed argument block (``Args.pack`` bytes / bytearray, or a
        ctypes buffer used as is)."""
        cbuf = buf if isinstance(buf, C.Array) else C.create_string_buffer(bytes(buf), len(buf))
        rc = runtime().hs_jit_launch(self.function(), grid, self.block, shmem or self.lds_bytes,
                                     stream_ptr, cbuf, len(buf))
        if rc != 0:
            raise RuntimeError(f"JIT launch failed: {runtime().hs_jit_last_error().decode()}")

    def launch(self, grid: int, values: Dict[str, object], stream_ptr: int, shmem: int = 0) -> None:
        buf = self.args.pack(values)
        cbuf = C.create_string_buffer(buf, len(buf))
        rc = runtime().hs_jit_launch(self.function(), grid, self.block, shmem or self.lds_bytes,
                                     stream_ptr, cbuf, len(buf))
        if rc != 0:
            raise RuntimeError(f"JIT launch failed: {runtime().hs_jit_last_error().decode()}")


# ------------------------------------------------------------------------------------------------
# Shared source fragments
# ------------------------------------------------------------------------------------------------
_PRELUDE = r"""
typedef long long i64;
typedef unsigned long long u64;
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ i64 wsumi(i64 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wmin(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wmax(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ bool in_set(const i64* s, int n, i64 x) {
  int lo = 0, hi = n;
  while (lo < hi) { const int m = (lo + hi) >> 1; if (s[m] < x) lo = m + 1; else hi = m; }
  return lo < n && s[lo] == x;
}
__device__ __forceinline__ bool bit_test(const u64* w, i64 nbits, i64 x) {
  return x >= 0 && x < nbits && ((w[x >> 6] >> (x & 63)) & 1ull);
}
// V consecutive elements starting at an index that is a multiple of V (so the address is
// aligned to V * sizeof(T) for a 16-byte aligned base): one dwordx4 per 16 bytes
template <typename T, int V>
__device__ __forceinline__ void vload(const T* __restrict__ p, long long i, T (&x)[V]) {
  constexpr int B = (int)sizeof(T) * V;
  if constexpr (B % 16 == 0) {
    const uint4* q = reinterpret_cast<const uint4*>(p + i);
#pragma unroll
    for (int k = 0; k < B / 16; ++k) reinterpret_cast<uint4*>(x)[k] = q[k];
  } else if constexpr (B == 8) {
    *reinterpret_cast<uint2*>(x) = *reinterpret_cast<const uint2*>(p + i);
  } else if constexpr (B == 4) {
    *reinterpret_cast<unsigned*>(x) = *reinterpret_cast<const unsigned*>(p + i);
  } else {
#pragma unroll
    for (int k = 0; k < V; ++k) x[k] = p[i + k];
  }
}
// NW dwords of a wavefront-uniform window through a raw buffer resource: the base is uniform
// (scalar registers), the range check of the buffer unit returns 0 for bytes at or past
// ``nbytes`` - so the table's last, partial group loads with the same dwordx4s as a full one
// instead of a per-element edge path (which doubled the kernel's register footprint)
typedef unsigned hs_v4u __attribute__((ext_vector_type(4)));
// two 16-bit codes' range test at once: per half, (x - lo) | (hi - x) with saturation (the
// sign survives clamping), so bits 15 and 31 are the two rows' fail bits
typedef short hs_s2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned hs_rng2(unsigned x, int lo, int hi) {
  const hs_s2 v = __builtin_bit_cast(hs_s2, x);
  const hs_s2 l = {(short)lo, (short)lo}, h = {(short)hi, (short)hi};
  return __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(v, l)) |
         __builtin_bit_cast(unsigned, __builtin_elementwise_sub_sat(h, v));
}
// [lo, hi] clamped to int16 for hs_rng2: a range wholly outside int16 becomes the empty
// (32767, -32768), which every code fails (clamping it bound by bound would keep an endpoint)
__device__ __forceinline__ int hs_c16lo(long long lo, long long hi) {
  return (hi < -32768ll || lo > 32767ll) ? 32767 : (int)(lo < -32768ll ? -32768ll : lo);
}
__device__ __forceinline__ int hs_c16hi(long long lo, long long hi) {
  return (hi < -32768ll || lo > 32767ll) ? -32768 : (int)(hi > 32767ll ? 32767ll : hi);
}
// bits 0..15 of x to the even, 16..31 to the odd positions (row order of a 2-rows-per-word mask)
__device__ __forceinline__ unsigned hs_unzip16(unsigned x) {
  unsigned a = x & 0xFFFFu, b = x >> 16;
  a = (a | (a << 8)) & 0x00FF00FFu; a = (a | (a << 4)) & 0x0F0F0F0Fu;
  a = (a | (a << 2)) & 0x33333333u; a = (a | (a << 1)) & 0x55555555u;
  b = (b | (b << 8)) & 0x00FF00FFu; b = (b | (b << 4)) & 0x0F0F0F0Fu;
  b = (b | (b << 2)) & 0x33333333u; b = (b | (b << 1)) & 0x55555555u;
  return a | (b << 1);
}
// a code bound clamped to +-2^20: narrow (<= 16-bit) codes against it never overflow int32
__device__ __forceinline__ int hs_c20(long long v) {
  return (int)(v < -1048576ll ? -1048576ll : (v > 1048576ll ? 1048576ll : v));
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hs_rsrc(const void* base, long long nbytes) {
  const u64 a_ = (u64)base;
  const unsigned lo_ = __builtin_amdgcn_readfirstlane((unsigned)a_);
  const unsigned hi_ = __builtin_amdgcn_readfirstlane((unsigned)(a_ >> 32));
  const long long n_ = nbytes < 0 ? 0 : (nbytes > 0x7fffffffll ? 0x7fffffffll : nbytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((u64)hi_ << 32) | lo_), (short)0,
                                           __builtin_amdgcn_readfirstlane((int)n_), 0x00020000);
}
template <int NW>
__device__ __forceinline__ void bload(__amdgpu_buffer_rsrc_t r, unsigned off, unsigned (&x)[NW]) {
  static_assert(NW % 4 == 0, "bload: whole dwordx4s");
#pragma unroll
  for (int k = 0; k < NW / 4; ++k) {
    const hs_v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * k, 0, 0);
    x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
  }
}
// the same window read lane-coalesced: instruction k of the wavefront covers 1 KB contiguous
// (lane l: 16 bytes at (64 k + l) * 16), so lane l holds 16-byte chunks of other lanes' rows;
// hs_lds_t then moves every chunk to its owner through the wavefront's LDS slab (chunk j of
// lane g at slot g * NJ + (j ^ (g % NJ)): both the stores and the loads hit distinct banks)
template <int NW>
__device__ __forceinline__ void bload_t(__amdgpu_buffer_rsrc_t r, int ln, unsigned (&x)[NW]) {
  static_assert(NW % 4 == 0, "bload_t: whole dwordx4s");
#pragma unroll
  for (int k = 0; k < NW / 4; ++k) {
    const hs_v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)((64 * k + ln) * 16), 0, 0);
    x[4 * k] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
  }
}
template <int NW>
__device__ __forceinline__ void hs_lds_t(hs_v4u* slab, int ln, unsigned (&x)[NW]) {
  constexpr int NJ = NW / 4;
#pragma unroll
  for (int k = 0; k < NJ; ++k) {
    const int c = 64 * k + ln, g = c / NJ, j = c % NJ;
    hs_v4u v; v.x = x[4 * k]; v.y = x[4 * k + 1]; v.z = x[4 * k + 2]; v.w = x[4 * k + 3];
    slab[g * NJ + (j ^ (g % NJ))] = v;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const hs_v4u v = slab[ln * NJ + (j ^ (ln % NJ))];
    x[4 * j] = v.x; x[4 * j + 1] = v.y; x[4 * j + 2] = v.z; x[4 * j + 3] = v.w;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ void lds_min(double* p, double v) {
  u64* a = (u64*)p; u64 old = *a, as;
  do { as = old; if (__longlong_as_double((i64)as) <= v) break;
       old = atomicCAS(a, as, (u64)__double_as_longlong(v)); } while (as != old);
}
__device__ __forceinline__ void lds_max(double* p, double v) {
  u64* a = (u64*)p; u64 old = *a, as;
  do { as = old; if (__longlong_as_double((i64)as) >= v) break;
       old = atomicCAS(a, as, (u64)__double_as_longlong(v)); } while (as != old);
}
// order-preserving signed image of a double (top-K thresholds published with atomicMax)
__device__ __forceinline__ long long hs_dimg(double d) {
  const long long u = __double_as_longlong(d);
  return u >= 0 ? u : u ^ 0x7fffffffffffffffll;
}
__device__ __forceinline__ double hs_dimg_inv(long long i) {
  return __longlong_as_double(i >= 0 ? i : i ^ 0x7fffffffffffffffll);
}
// hash-mode grouping (exec/hash_agg.py, csrc/kernels/hash_agg.hip): probe hash and the bit
// images of float group keys (-0.0 -> 0.0, one NaN)
__device__ __forceinline__ u64 hs_mix64(u64 h) {
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull; h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull;
  return h ^ (h >> 33);
}
__device__ __forceinline__ u64 hs_f64key(double d) {
  d = d == 0.0 ? 0.0 : d;
  return d != d ? 0x7ff8000000000000ull : (u64)__double_as_longlong(d);
}
__device__ __forceinline__ u64 hs_f32key(float f) {
  f = f == 0.0f ? 0.0f : f;
  return f != f ? 0x7fc00000ull : (u64)(unsigned)__float_as_uint(f);
}
"""


def _ident(kind: int) -> str:
    return "__builtin_inf()" if kind == NL.AK_MIN else (
        "-__builtin_inf()" if kind == NL.AK_MAX else "0.0")


class _Gen:
    """Expression builder over column slots of one or two row variables."""

    def __init__(self, args: Args, cols: Dict[int, tuple], split: int, rows: Tuple[str, str],
                 approx=frozenset(), intpred: bool = False):
        self.a = args
        self.cols = cols          # slot -> (hs_type, has_valid, compact signature or None)
        self.split = split
        self.rows = rows          # row variable for slot < split / >= split
        # decimal-scaled compact slots read only by SUM/COUNT: decode with a reciprocal
        # multiply (<= 1 ulp) instead of an exact f64 division (~12 VALU instructions)
        self.approx = approx
        # predicates on decimal-scaled compact columns compare the integer q = base + code with
        # host-computed integer bounds (exact, no f64 division); needs the q<s> registers the
        # phase-major generators emit
        self.intpred = intpred

    def row(self, slot: int) -> str:
        return self.rows[1] if slot >= self.split else self.rows[0]

    def ptr(self, slot: int) -> str:
        return self.a.add("p", f"c{slot}", f"const {self.raw_type(slot)}*")

    def vptr(self, slot: int) -> Optional[str]:
        hv = self.cols[slot][1]
        return self.a.add("p", f"v{slot}", "const unsigned char*") if hv else None

    def value(self, slot: int, row: str) -> str:
        """Logical value of column ``slot`` at ``row`` (decodes compact columns in registers)."""
        return self.decode(slot, f"{self.ptr(slot)}[{row}]")

    def raw_type(self, slot: int) -> str:
        """C type of the stored element (the code type for compact columns; grouped 16-bit
        codes, encoding.GroupedCompact, are unsigned)."""
        t, _, enc = self.cols[slot]
        if enc and len(enc) > 2 and enc[2] == 64:
            return "unsigned short"
        return _CODE_T[enc[0]] if enc else _CTYPE[t]

    def decode(self, slot: int, raw: str) -> str:
        """Logical value of a stored element expression ``raw`` of column ``slot``."""
        t, _, enc = self.cols[slot]
        if not enc:
            return raw
        ct = _CTYPE[t]
        base = self.a.add("q", f"B{slot}", "long long")
        if enc[1]:
            if slot in self.approx:
                inv = self.a.add("d", f"R{slot}", "double")
                return f"({ct})((double)({base} + (i64){raw}) * {inv})"
            scale = self.a.add("d", f"Q{slot}", "double")
            return f"({ct})((double)({base} + (i64){raw}) / {scale})"
        return f"({ct})({base} + (i64){raw})"

    def ok(self, slot: int) -> str:
        return f"n{slot}" if self.cols[slot][1] else "true"

    def load(self, slot: int, guard: str, out: List[str], ind: str) -> None:
        t = self.cols[slot][0]
        ct = _CTYPE[t]
        r = self.row(slot)
        out.append(f"{ind}const {ct} x{slot} = ({guard}) ? {self.value(slot, r)} : ({ct})0;")
        if self.cols[slot][1]:
            out.append(f"{ind}const bool n{slot} = ({guard}) && {self.vptr(slot)}[{r}] != 0;")

    def leaf(self, k: int, p: NL.Pred) -> str:
        kind, op = p.kind, p.op
        if kind == NL.PK_TRUE:
            return "true"
        c = p.col
        if kind == NL.PK_IS_NULL:
            return f"(!{self.ok(c)})"
        if kind == NL.PK_NOT_NULL:
            return f"({self.ok(c)})"
        enc = self.cols[c][2]
        if self.intpred and enc and (kind == NL.PK_INT_LIT and not enc[1] or
                                     kind == NL.PK_FLT_LIT and enc[1]):
            # compact column: compare the stored code with host-computed 32-bit code bounds
            # (exact: code_bounds), no decode and no 64-bit compare
            lo = self.a.add("q", f"CL{k}", "long long")
            hi = self.a.add("q", f"CH{k}", "long long")
            inside = f"(r{c} >= (int){lo} && r{c} <= (int){hi})"
            return f"({self.ok(c)} && {'!' if op == NL.OP_NE else ''}{inside})"
        if kind == NL.PK_INT_LIT:
            lit = self.a.add("q", f"L{k}", "long long")
            return f"({self.ok(c)} && ((i64)x{c} {_OPSTR[op]} {lit}))"
        if kind == NL.PK_FLT_LIT:
            if self.intpred and enc and enc[1]:
                lo = self.a.add("q", f"T{k}", "long long")
                hi = self.a.add("q", f"U{k}", "long long")
                inside = f"(q{c} >= {lo} && q{c} <= {hi})"
                return f"({self.ok(c)} && {'!' if op == NL.OP_NE else ''}{inside})"
            lit = self.a.add("d", f"F{k}", "double")
            return f"({self.ok(c)} && ((double)x{c} {_OPSTR[op]} {lit}))"
        if kind in (NL.PK_INT_COL, NL.PK_FLT_COL):
            c2 = p.col2
            cast = "i64" if kind == NL.PK_INT_COL else "double"
            return (f"({self.ok(c)} && {self.ok(c2)} && "
                    f"(({cast})x{c} {_OPSTR[op]} ({cast})x{c2}))")
        if kind == NL.PK_IN_SET:
            sp = self.a.add("p", f"S{k}", "const long long*")
            sn = self.a.add("q", f"N{k}", "long long")
            neg = "" if op == NL.OP_EQ else "!"
            return f"({self.ok(c)} && {neg}in_set({sp}, (int){sn}, (i64)x{c}))"
        if kind == NL.PK_BITMAP:
            # bit (value - base) of a key-domain bitmap (base = ilit: a semi-join's build keys)
            sp = self.a.add("p", f"S{k}", "const unsigned long long*")
            sn = self.a.add("q", f"N{k}", "long long")
            base = self.a.add("q", f"L{k}", "long long")
            neg = "" if op == NL.OP_EQ else "!"
            return f"({self.ok(c)} && {neg}bit_test({sp}, {sn} * 64, (i64)x{c} - {base}))"
        raise ValueError(f"pred kind {kind}")

    def sign_leaf(self, k: int, p: NL.Pred) -> Optional[str]:
        """``leaf`` as an int32 whose sign bit is set iff the row fails it, with no compare
        (no lane-mask registers, no select of per-bit constants): a range test of a narrow
        compact code is ``(r - lo) | (hi - r)``.  None when the leaf has no such form."""
        kind, op = p.kind, p.op
        if kind == NL.PK_TRUE:
            return "0"
        c = p.col
        hv = self.cols[c][1]
        if kind == NL.PK_IS_NULL:
            return f"(-(int){self.ok(c)})" if hv else "(-1)"
        if kind == NL.PK_NOT_NULL:
            return f"((int){self.ok(c)} - 1)" if hv else "0"
        enc = self.cols[c][2]
        if not (self.intpred and enc and (kind == NL.PK_INT_LIT and not enc[1] or
                                          kind == NL.PK_FLT_LIT and enc[1])):
            return None
        if _SIZEOF.get(self.raw_type(c), 8) > 2:
            return None
        lo = self.a.add("q", f"CL{k}", "long long")
        hi = self.a.add("q", f"CH{k}", "long long")
        s = f"((r{c} - hs_c20({lo})) | (hs_c20({hi}) - r{c}))"
        if op == NL.OP_NE:
            s = f"(~{s})"
        return f"({s} | ((int){self.ok(c)} - 1))" if hv else s

    def cnf_sign2(self, preds: List[Tuple[int, NL.Pred]], word: str,
                  offset: Optional[str] = None) -> Optional[str]:
        """``cnf_sign`` over two rows at once for 16-bit signed codes without validity: the
        dword ``word.format(slot)`` holds both rows' codes, the result's bits 15 / 31 are their
        fail bits (``hs_rng2``).  None when a leaf has no such form."""
        groups: Dict[int, List[str]] = {}
        order: List[int] = []
        for k, p in preds:
            kind, op = p.kind, p.op
            if kind == NL.PK_TRUE:
                leaf = "0u"
            else:
                c = p.col
                if self.cols[c][1] or self.raw_type(c) != "short":
                    return None
                enc = self.cols[c][2]
                if kind == NL.PK_NOT_NULL:
                    leaf = "0u"
                elif kind == NL.PK_IS_NULL:
                    leaf = "0xFFFFFFFFu"
                elif self.intpred and enc and (kind == NL.PK_INT_LIT and not enc[1] or
                                               kind == NL.PK_FLT_LIT and enc[1]):
                    lo = self.a.add("q", f"CL{k}", "long long")
                    hi = self.a.add("q", f"CH{k}", "long long")
                    if offset is not None:      # the words hold code - offset
                        o = offset.format(c)
                        lo, hi = f"({lo} - {o})", f"({hi} - {o})"
                    leaf = (f"hs_rng2({word.format(c)}, hs_c16lo({lo}, {hi}), "
                            f"hs_c16hi({lo}, {hi}))")
                    if op == NL.OP_NE:
                        leaf = f"(~{leaf})"
                else:
                    return None
            if p.group not in groups:
                groups[p.group] = []
                order.append(p.group)
            groups[p.group].append(leaf)
        if not order:
            return "0u"
        return "(" + " | ".join("(" + " & ".join(groups[g]) + ")" for g in order) + ")"

    def cnf_sign(self, preds: List[Tuple[int, NL.Pred]]) -> Optional[str]:
        """``cnf`` as a sign word (negative iff the row fails), or None: a group (OR) fails
        when every leaf fails (AND of the words), the conjunction when any group fails (OR)."""
        if not preds:
            return "0"
        groups: Dict[int, List[str]] = {}
        order: List[int] = []
        for k, p in preds:
            leaf = self.sign_leaf(k, p)
            if leaf is None:
                return None
            if p.group not in groups:
                groups[p.group] = []
                order.append(p.group)
            groups[p.group].append(leaf)
        return "(" + " | ".join("(" + " & ".join(groups[g]) + ")" for g in order) + ")"

    def cnf(self, preds: List[Tuple[int, NL.Pred]]) -> str:
        if not preds:
            return "true"
        groups: Dict[int, List[str]] = {}
        order: List[int] = []
        for k, p in preds:
            if p.group not in groups:
                groups[p.group] = []
                order.append(p.group)
            groups[p.group].append(self.leaf(k, p))
        return " && ".join("(" + " || ".join(groups[g]) + ")" for g in order)

    def agg_value(self, i: int, a: NL.AggSpec) -> Tuple[str, str]:
        """(value expr, validity expr) of aggregate i."""
        if a.kind == NL.AK_COUNT_STAR:
            return "1.0", "true"
        terms, oks = [], []
        for t in range(a.nterms):
            c = a.col[t]
            al = self.a.add("d", f"A{i}_{t}", "double")
            be = self.a.add("d", f"B{i}_{t}", "double")
            terms.append(f"({al} + {be} * (double)x{c})")
            if self.cols[c][1]:
                oks.append(f"n{c}")
        return " * ".join(terms) or "1.0", " && ".join(oks) or "true"


def _sum_only_slots(preds, aggs, group_col: int = -1, cols=None) -> frozenset:
    """Slots whose decoded value is read only as a term of SUM / COUNT aggregates: it may carry
    a 1-ulp decode error, which a floating-point sum's own rounding already dominates.
    Predicates (except literal compares on decimal-scaled compact columns, which run on the
    integer codes), MIN/MAX and the group key keep exact decoding."""
    exact = set()
    for _, p in preds:
        enc = (cols or {}).get(p.col, (None, None, None))[2]
        if p.kind in (NL.PK_IS_NULL, NL.PK_NOT_NULL, NL.PK_TRUE):
            continue
        if p.kind == NL.PK_FLT_LIT and enc and enc[1]:
            continue
        exact.add(p.col)
        if p.kind in (NL.PK_INT_COL, NL.PK_FLT_COL):
            exact.add(p.col2)
    if group_col >= 0:
        exact.add(group_col)
    summed = set()
    for a in aggs:
        cols = [a.col[t] for t in range(a.nterms)]
        if a.kind in (NL.AK_SUM, NL.AK_COUNT):
            summed.update(cols)
        elif a.kind != NL.AK_COUNT_STAR:
            exact.update(cols)
    return frozenset(summed - exact)


def _pred_slots(preds) -> List[int]:
    s = []
    for _, p in preds:
        if p.kind == NL.PK_TRUE:
            continue
        s.append(p.col)
        if p.kind in (NL.PK_INT_COL, NL.PK_FLT_COL):
            s.append(p.col2)
    return list(dict.fromkeys(s))


def _agg_slots(aggs) -> List[int]:
    s = []
    for a in aggs:
        if a.kind != NL.AK_COUNT_STAR:
            s += [a.col[t] for t in range(a.nterms)]
    return list(dict.fromkeys(s))


def _accumulate(gen: _Gen, aggs, grouped: bool, pass_var: str, gvar: str, ind: str) -> List[str]:
    out = []
    for i, a in enumerate(aggs):
        v, ok = gen.agg_value(i, a)
        out.append(f"{ind}{{ const bool ok = {pass_var} && {ok}; const double v = ok ? {v} : 0.0;")
        if not grouped:
            if a.kind == NL.AK_MIN:
                out.append(f"{ind}  if (ok) {{ acc{i} = fmin(acc{i}, v); cnt{i} += 1u; }} }}")
            elif a.kind == NL.AK_MAX:
                out.append(f"{ind}  if (ok) {{ acc{i} = fmax(acc{i}, v); cnt{i} += 1u; }} }}")
            else:   # v is 0.0 when !ok: no branch
                out.append(f"{ind}  acc{i} += v; cnt{i} += ok ? 1u : 0u; }}")
            continue
        # wave-peeled grouped accumulation into LDS (one atomic per distinct group per wave)
        out.append(f"{ind}  bool todo = ok;")
        out.append(f"{ind}  while (true) {{")
        out.append(f"{ind}    const u64 act = __ballot(todo); if (act == 0ull) break;")
        out.append(f"{ind}    const int ld = __ffsll((unsigned long long)act) - 1;")
        out.append(f"{ind}    const int g0 = __shfl({gvar}, ld, 64);")
        out.append(f"{ind}    const bool mine = todo && {gvar} == g0;")
        out.append(f"{ind}    const u64 cm = __ballot(mine);")
        if a.kind == NL.AK_MIN:
            out.append(f"{ind}    const double r = wmin(mine ? v : __builtin_inf());")
        elif a.kind == NL.AK_MAX:
            out.append(f"{ind}    const double r = wmax(mine ? v : -__builtin_inf());")
        else:
            out.append(f"{ind}    const double r = wsum(mine ? v : 0.0);")
        out.append(f"{ind}    if ((int)(threadIdx.x & 63) == ld) {{")
        out.append(f"{ind}      const int s = g0 * NA + {i};")
        if a.kind == NL.AK_MIN:
            out.append(f"{ind}      lds_min(&gmn[s], r);")
        elif a.kind == NL.AK_MAX:
            out.append(f"{ind}      lds_max(&gmx[s], r);")
        elif a.kind == NL.AK_SUM:
            out.append(f"{ind}      atomicAdd(&gsum[s], r);")
        out.append(f"{ind}      atomicAdd(&gcnt[s], (unsigned long long)__popcll(cm));")
        out.append(f"{ind}    }}")
        out.append(f"{ind}    todo = todo && !mine;")
        out.append(f"{ind}  }} }}")
    return out


def _acc_decls(aggs, grouped: bool, args: Args) -> List[str]:
    out = [f"  constexpr int NA = {len(aggs)};"]
    if grouped:
        out += ["  extern __shared__ __attribute__((aligned(16))) double glds[];",
                "  const int GA = (int)a.num_groups * NA;",
                "  double* gsum = glds; double* gmn = glds + GA; double* gmx = glds + 2 * GA;",
                "  unsigned long long* gcnt = (unsigned long long*)(glds + 3 * GA);",
                "  for (int i = threadIdx.x; i < GA; i += blockDim.x) {",
                "    gsum[i] = 0.0; gmn[i] = __builtin_inf(); gmx[i] = -__builtin_inf(); gcnt[i] = 0ull; }",
                "  __syncthreads();"]
        args.add("q", "num_groups", "long long")
        args.add("q", "group_base", "long long")
    else:
        for i, a in enumerate(aggs):
            out.append(f"  double acc{i} = {_ident(a.kind)}; unsigned cnt{i} = 0u;")
    return out


def _flush(aggs, grouped: bool, block: int = None) -> List[str]:
    BLOCK = block or globals()["BLOCK"]  # noqa: N806 — waves per block of this kernel
    out = []
    if grouped:
        out += ["  __syncthreads();",
                "  for (int i = threadIdx.x; i < GA; i += blockDim.x) {",
                "    const i64 o = (i64)blockIdx.x * GA + i;",
                "    a.psum[o] = gsum[i]; a.pcnt[o] = (i64)gcnt[i]; a.pmin[o] = gmn[i]; a.pmax[o] = gmx[i];",
                "  }"]
        return out
    out += [f"  __shared__ double rv[{BLOCK // 64}][NA]; __shared__ i64 rc[{BLOCK // 64}][NA];",
            "  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;"]
    for i, a in enumerate(aggs):
        red = "wmin" if a.kind == NL.AK_MIN else ("wmax" if a.kind == NL.AK_MAX else "wsum")
        out.append(f"  {{ const double r = {red}(acc{i}); const i64 c = wsumi((i64)cnt{i});"
                   f" if (lane == 0) {{ rv[w][{i}] = r; rc[w][{i}] = c; }} }}")
    out.append("  __syncthreads();")
    out.append("  if (threadIdx.x == 0) {")
    for i, a in enumerate(aggs):
        comb = "fmin(t, rv[k][{i}])" if a.kind == NL.AK_MIN else (
            "fmax(t, rv[k][{i}])" if a.kind == NL.AK_MAX else "t + rv[k][{i}]")
        comb = comb.format(i=i)
        out.append(f"    {{ double t = {_ident(a.kind)}; i64 c = 0;")
        out.append(f"      for (int k = 0; k < {BLOCK // 64}; ++k) {{ t = {comb}; c += rc[k][{i}]; }}")
        out.append(f"      const i64 o = (i64)blockIdx.x * NA + {i};")
        is_mm = a.kind in (NL.AK_MIN, NL.AK_MAX)
        out.append(f"      a.psum[o] = {'0.0' if is_mm else 't'}; a.pcnt[o] = c;")
        out.append(f"      a.pmin[o] = {'t' if a.kind == NL.AK_MIN else '__builtin_inf()'};"
                   f" a.pmax[o] = {'t' if a.kind == NL.AK_MAX else '-__builtin_inf()'}; }}")
    out.append("  }")
    return out


def _common_args(args: Args) -> None:
    for n in ("psum", "pmin", "pmax"):
        args.add("p", n, "double*")
    args.add("p", "pcnt", "long long*")


# ------------------------------------------------------------------------------------------------
# Scan + filter + aggregate
# ------------------------------------------------------------------------------------------------
def _col_specs(p, compacts) -> Dict[int, tuple]:
    """slot -> (hs_type, has_valid, compact signature | None)."""
    out = {}
    for s in range(NL.MAX_COLS):
        if p.cols[s].data:
            c = (compacts or {}).get(s)
            out[s] = (p.cols[s].type, bool(p.cols[s].valid), c.signature() if c else None)
    return out


def scan_agg_shape(p: NL.ScanParams, compacts=None, vec: int = 0, hk=None) -> tuple:
    cols = tuple(sorted(_col_specs(p, compacts).items()))
    preds = tuple((p.preds[k].kind, p.preds[k].op, p.preds[k].col, p.preds[k].col2,
                   p.preds[k].group) for k in range(p.npreds))
    aggs = tuple((p.aggs[i].kind, p.aggs[i].nterms, tuple(p.aggs[i].col[:p.aggs[i].nterms]))
                 for i in range(p.naggs))
    return ("scan_agg", cols, preds, aggs, p.group_col, SCAN_ITEMS, SCAN_EAGER, vec,
            SCAN_COMPACT, WAVE_SYNC, VEC_PREFETCH, hk.shape() if hk is not None else None)


def gen_scan_agg(p: NL.ScanParams, compacts=None, vec: int = 0, hk=None) -> Kernel:
    """Filter + aggregate over row ranges, phase-major over the SCAN_ITEMS rows of each thread
    and branch-free: (1) the predicate columns of every item are loaded together; (2) the
    aggregate inputs (and group column) of every item, where rows that failed the predicates
    read the tile's first row instead of branching around the load — their lanes coalesce into
    one line, so only passing rows cost HBM bytes; (3) accumulate.  SCAN_EAGER loads every
    column in phase 1."""
    args = Args()
    for n, ct in (("rstart", "const long long*"), ("rlen", "const long long*"),
                  ("tile_prefix", "const long long*")):
        args.add("p", n, ct)
    args.add("q", "R", "long long")
    _common_args(args)
    cols = _col_specs(p, compacts)
    preds = [(k, p.preds[k]) for k in range(p.npreds)]
    aggs = [p.aggs[i] for i in range(p.naggs)]
    grouped = p.group_col >= 0
    assert not (grouped and hk is not None)
    pslots = _pred_slots(preds)
    aslots = [s for s in _agg_slots(aggs) if s not in pslots]
    if grouped and p.group_col not in pslots and p.group_col not in aslots:
        aslots.append(p.group_col)
    for s in (hk.slots if hk is not None else []):
        if s not in pslots and s not in aslots:
            aslots.append(s)
    if SCAN_EAGER:
        pslots, aslots = pslots + aslots, []
    allslots = pslots + aslots
    approx = _sum_only_slots(preds, aggs, p.group_col, cols) - set(hk.slots if hk else [])
    NI = vec or SCAN_ITEMS
    T = BLOCK * NI
    if vec:
        args.add("q", "nrows", "long long")
    b: List[str] = []
    b += _acc_decls(aggs, grouped, args)
    if grouped:
        base = args.add("q", "group_base", "long long")
        ng = args.add("q", "num_groups", "long long")
    ind = "    "
    g0_ = _Gen(args, cols, NL.MAX_COLS, ("row0", "row0"), approx, True)
    compact = SCAN_COMPACT and bool(aslots)

    def body(b: List[str], full: Optional[bool]) -> None:
        """Tile body; ``full`` = vectorized full tile / vectorized last tile / None (scalar)."""
        if full is not None:     # raw vector arrays come from the tile loop (_vec_tiles)
            _vec_load_slots(b, g0_, pslots, NI, ind)
        else:
            b.extend(["    const i64 tb0 = a.rstart[r] + off;",
                      f"    const i64 rows = a.rlen[r] - off < {T} ? a.rlen[r] - off : {T};"])
            for it in range(NI):
                b.extend([f"{ind}const bool act{it} = {it * BLOCK} + (i64)threadIdx.x < rows;",
                          f"{ind}const i64 row{it} = tb0 + (act{it} ? {it * BLOCK} + (i64)threadIdx.x : 0);"])
            for it in range(NI):
                g1 = _Gen(args, cols, NL.MAX_COLS, (f"row{it}", f"row{it}"), approx, True)
                for s in pslots:
                    _uload(g1, s, it, b, ind)
        for it in range(NI):
            g1 = _Gen(args, cols, NL.MAX_COLS, (f"row{it}", f"row{it}"), approx, True)
            b.append(f"{ind}bool pass{it} = act{it} && {_rename(g1.cnf(preds), allslots, it)};")
        if compact:
            b.extend(_compacted_tail(args, cols, NL.MAX_COLS, approx, aggs, grouped, p.group_col,
                                     aslots, allslots, NI, ind, with_j=False, hk=hk))
            return
        if aslots:
            for it in range(NI):
                b.append(f"{ind}const i64 lq{it} = pass{it} ? row{it} : tb0;")
            for it in range(NI):
                g2 = _Gen(args, cols, NL.MAX_COLS, (f"lq{it}", f"lq{it}"), approx, True)
                for s in aslots:
                    _uload(g2, s, it, b, ind)
        for it in range(NI):
            g2 = _Gen(args, cols, NL.MAX_COLS, (f"row{it}", f"row{it}"), approx, True)
            gvar = f"gi{it}"
            if grouped:
                g = p.group_col
                b.append(f"{ind}const i64 gl{it} = (i64){_rename(f'x{g}', allslots, it)} - {base};")
                b.append(f"{ind}pass{it} = pass{it} && {_rename(g2.ok(g), allslots, it)} && "
                         f"gl{it} >= 0 && gl{it} < {ng};")
                b.append(f"{ind}const int {gvar} = pass{it} ? (int)gl{it} : 0;")
            if hk is not None:
                b.extend(_rename(x, allslots, it) for x in
                         JH._hash_accumulate(g2, aggs, hk, f"pass{it}", ind))
                continue
            b.extend(_rename(x, allslots, it) for x in
                     _accumulate(g2, aggs, grouped, f"pass{it}", gvar, ind))

    if vec:
        _vec_tiles(b, T, NI, ind, _vec_loads(g0_, pslots), [], body)
    else:
        _tile_loop(b, T, NI, 0)
        body(b, None)
    b += ["  }"]
    if hk is None:
        b += _flush(aggs, grouped)
    if compact:
        W = BLOCK // 64
        b.insert(0, f"  typedef {_crow_t(T)} crow_t; __shared__ crow_t crow_s[{W}][{64 * NI}];")
        b.insert(1, "  const int cln = threadIdx.x & 63, wv = threadIdx.x >> 6;")
    src = (_PRELUDE + args.struct_src() +
           f'extern "C" __global__ __launch_bounds__({BLOCK}) void hs_jit_scan_agg(Args a) {{\n' +
           "\n".join(b) + "\n}\n")
    lds = (len(aggs) * p.num_groups * 32) if grouped else 0
    return Kernel(src, "hs_jit_scan_agg", args, lds)


def scan_agg_values(p: NL.ScanParams, rstart, rlen, tile_prefix, parts,
                    compacts=None) -> Dict[str, object]:
    v = {"rstart": rstart.data_ptr(), "rlen": rlen.data_ptr(), "tile_prefix": tile_prefix.data_ptr(),
         "R": rstart.numel(), "psum": parts[0].data_ptr(), "pcnt": parts[1].data_ptr(),
         "pmin": parts[2].data_ptr(), "pmax": parts[3].data_ptr(),
         "num_groups": p.num_groups, "group_base": p.group_base}
    _fill_common(v, p.cols, [(k, p.preds[k]) for k in range(p.npreds)],
                 [p.aggs[i] for i in range(p.naggs)], compacts)
    return v


_BIG = 1 << 62


def _int_lit_bounds(op: int, lit: int) -> Tuple[int, int]:
    """Inclusive [lo, hi] of the integer values v with ``v OP lit`` (EQ and NE: [lit, lit])."""
    lit = int(lit)
    if op == NL.OP_LT:
        return (-_BIG, lit - 1)
    if op == NL.OP_LE:
        return (-_BIG, lit)
    if op == NL.OP_GT:
        return (lit + 1, _BIG)
    if op == NL.OP_GE:
        return (lit, _BIG)
    return (lit, lit)


def code_bounds(lo: int, hi: int, base: int) -> Tuple[int, int]:
    """Value bounds [lo, hi] mapped to the stored codes (value = base + code) of a compact
    column and clamped to int32, the widest code: exact, since every code lies in int32; an
    empty range stays empty ((1, 0))."""
    clo = max(int(lo) - int(base), -(1 << 31))
    chi = min(int(hi) - int(base), (1 << 31) - 1)
    return (clo, chi) if clo <= chi else (1, 0)


def int_bounds(op: int, lit: float, scale: float) -> Tuple[int, int]:
    """[T, U] such that, for every integer q of a decimal-scaled column (value = q / scale,
    correctly rounded), ``q / scale OP lit`` holds iff ``T <= q <= U`` (``NE``: iff not).
    Exact: thresholds are found with the same IEEE double division the decode uses."""
    import math
    if lit != lit:                                   # NaN compares false (NE: true)
        return (_BIG, -_BIG)
    if math.isinf(lit):
        below = lit > 0                              # every finite value is below +inf
        if op in (NL.OP_LT, NL.OP_LE):
            return (-_BIG, _BIG) if below else (_BIG, -_BIG)
        if op in (NL.OP_GT, NL.OP_GE):
            return (_BIG, -_BIG) if below else (-_BIG, _BIG)
        return (_BIG, -_BIG)

    def first(pred) -> int:                          # smallest integer t with pred(t / scale)
        t = math.floor(lit * scale) - 4
        while not pred(t / scale):
            t += 1
        return t
    ge = first(lambda x: x >= lit)
    gt = first(lambda x: x > lit)
    if op == NL.OP_GE:
        return (ge, _BIG)
    if op == NL.OP_GT:
        return (gt, _BIG)
    if op == NL.OP_LE:
        return (-_BIG, gt - 1)
    if op == NL.OP_LT:
        return (-_BIG, ge - 1)
    return (ge, gt - 1)                              # EQ / NE


def _fill_common(v: Dict[str, object], cols, preds, aggs, compacts=None) -> None:
    _fill_cols(v, cols, compacts)
    fill_preds_aggs(v, preds, aggs, compacts)


def _fill_cols(v: Dict[str, object], cols, compacts=None) -> None:
    """Column argument slots (pointers, compact bases / scales): fixed for a resident table,
    so a prepared query fills them once."""
    for s in range(NL.MAX_COLS):
        if cols[s].data:
            c = (compacts or {}).get(s)
            v[f"c{s}"] = c.codes.data_ptr() if c else cols[s].data
            v[f"v{s}"] = cols[s].valid or 0
            if c:
                v[f"B{s}"] = c.base
                v[f"Q{s}"] = c.scale or 1.0
                v[f"R{s}"] = 1.0 / (c.scale or 1.0)
                gb = getattr(c, "gbase", None)
                if gb is not None:
                    v[f"G{s}"] = gb.data_ptr()
                    v[f"W{s}"] = c.wide.data_ptr()
                rk = getattr(c, "runkeys", None)
                if rk is not None:
                    v[f"RK{s}"] = rk.data_ptr()
                    v[f"GM{s}"] = c.gmask.data_ptr()
                    v[f"GR{s}"] = c.gruns.data_ptr()


def fill_preds_aggs(v: Dict[str, object], preds, aggs, compacts=None) -> None:
    """Literal-dependent argument slots: predicate values / code bounds and aggregate terms."""
    for k, p in preds:
        v[f"L{k}"] = p.ilit
        v[f"F{k}"] = p.flit
        c = (compacts or {}).get(p.col)
        if p.kind == NL.PK_FLT_LIT and c is not None and c.scale:
            v[f"T{k}"], v[f"U{k}"] = int_bounds(p.op, p.flit, c.scale)
            v[f"CL{k}"], v[f"CH{k}"] = code_bounds(v[f"T{k}"], v[f"U{k}"], c.base)
        elif p.kind == NL.PK_INT_LIT and c is not None and not c.scale:
            v[f"CL{k}"], v[f"CH{k}"] = code_bounds(*_int_lit_bounds(p.op, p.ilit), c.base)
        v[f"S{k}"] = p.set or 0
        v[f"N{k}"] = p.set_len
    for i, a in enumerate(aggs):
        for t in range(a.nterms):
            v[f"A{i}_{t}"] = a.alpha[t]
            v[f"B{i}_{t}"] = a.beta[t]


# ------------------------------------------------------------------------------------------------
# Co-located join + aggregate
# ------------------------------------------------------------------------------------------------
def join_agg_shape(p: NL.JoinParams, compacts=None) -> tuple:
    cols = tuple(sorted(_col_specs(p, compacts).items()))
    preds = tuple((p.preds[k].kind, p.preds[k].op, p.preds[k].col, p.preds[k].col2,
                   p.preds[k].group) for k in range(p.npreds))
    aggs = tuple((p.aggs[i].kind, p.aggs[i].nterms, tuple(p.aggs[i].col[:p.aggs[i].nterms]))
                 for i in range(p.naggs))
    return ("join_agg", cols, preds, p.nlp, aggs, p.group_col, p.lkey, p.rkey, p.key_is_float,
            JOIN_ITEMS, JOIN_LDS_KEYS, JOIN_EAGER, JOIN_BLOCK, JOIN_STAGE_RIGHT, JOIN_PIPELINE,
            JOIN_DIRECT, JOIN_DIRECT_SLOTS)


def _key_expr(var: str, is_float: bool) -> str:
    if is_float:
        return (f"({{ double d_ = (double){var}; d_ = d_ == 0.0 ? 0.0 : d_; "
                f"const u64 b_ = (u64)__double_as_longlong(d_); "
                f"(b_ & 0x8000000000000000ull) ? ~b_ : (b_ | 0x8000000000000000ull); }})")
    return f"((u64)(i64){var} ^ 0x8000000000000000ull)"


def gen_join_agg(p: NL.JoinParams, compacts=None) -> Kernel:
    """Co-located join + aggregate over 512-row left tiles (see module docstring).

    The kernel is latency-bound (rows in flight per CU x dependent HBM round trips per tile), so
    the code is scheduled to minimise round trips on each tile's critical path:

    1. the next tile's span record is prefetched while the current tile runs;
    2. every left column the query needs (key, left predicates, left aggregate inputs, group) and
       this thread's share of the right key span are loaded in ONE batch;
    3. LDS stage + barrier + LDS binary search of the keys;
    4. one batch of right-column loads at the matched rows, then accumulate.

    With ``JOIN_EAGER`` off, left aggregate inputs are loaded only for matched rows instead
    (fewer bytes, one more round trip)."""
    BLOCK = JOIN_BLOCK  # noqa: N806 — workgroup size of this kernel
    LDS_KEYS = join_lds_keys()  # noqa: N806
    args = Args()
    args.add("p", "tile_prefix", "const long long*")
    args.add("q", "R", "long long")
    args.add("p", "spans", "const long long*")
    _common_args(args)
    cols = _col_specs(p, compacts)
    split = 8
    gen = _Gen(args, cols, split, ("lrow", "j"))
    lpreds = [(k, p.preds[k]) for k in range(p.nlp)]
    rpreds = [(k, p.preds[k]) for k in range(p.nlp, p.npreds)]
    aggs = [p.aggs[i] for i in range(p.naggs)]
    grouped = p.group_col >= 0
    fl = bool(p.key_is_float)
    lk, rk = p.lkey, p.rkey
    need = _pred_slots(lpreds) + _pred_slots(rpreds) + _agg_slots(aggs) + \
        ([p.group_col] if grouped else [])
    left_all = list(dict.fromkeys([lk] + [s for s in need if s < split]))
    right_all = list(dict.fromkeys([s for s in need if s >= split]))
    lpred_slots = list(dict.fromkeys([lk] + [s for s in _pred_slots(lpreds) if s < split]))
    if JOIN_EAGER:
        left_first, left_late = left_all, []
    else:
        left_first = lpred_slots
        left_late = [s for s in left_all if s not in lpred_slots]
    NI = JOIN_ITEMS
    KEYS_PER_THREAD = 1   # typical spans (~4 right rows per 16 left rows) fit one key per thread
    b: List[str] = []
    b += _acc_decls(aggs, grouped, args)
    b += [f"  __shared__ u64 skeys[{LDS_KEYS}];",
          "  const i64 ntiles = a.tile_prefix[a.R];",
          "  const i64 per = (ntiles + gridDim.x - 1) / gridDim.x;",
          "  const i64 t0 = (i64)blockIdx.x * per;",
          "  const i64 t1 = ntiles < t0 + per ? ntiles : t0 + per;",
          "  i64 n_row0 = 0, n_rows = 0, n_rs = 0, n_re = 0;",
          "  if (t0 < t1) { n_row0 = a.spans[4 * t0]; n_rows = a.spans[4 * t0 + 1];",
          "                 n_rs = a.spans[4 * t0 + 2]; n_re = a.spans[4 * t0 + 3]; }",
          "  for (i64 t = t0; t < t1; ++t) {",
          "    const i64 row0 = n_row0, rows = n_rows, rs = n_rs, re = n_re;",
          "    if (t + 1 < t1) { n_row0 = a.spans[4 * t + 4]; n_rows = a.spans[4 * t + 5];",
          "                      n_rs = a.spans[4 * t + 6]; n_re = a.spans[4 * t + 7]; }",
          f"    const bool staged = re - rs <= {LDS_KEYS};"]
    ind = "    "
    for it in range(NI):
        b.append(f"{ind}const i64 lr{it} = row0 + {it * BLOCK} + threadIdx.x;")
        b.append(f"{ind}const bool la{it} = {it * BLOCK} + (i64)threadIdx.x < rows;")
    # (1) left batch + this thread's right keys, issued together.  `batch` collects the loads
    # and `fields` the registers they fill, so the pipelined variant can issue the NEXT tile's
    # batch while this tile searches and gathers.
    batch: List[str] = []
    fields: List[Tuple[str, str]] = []
    for it in range(NI):
        g2 = _Gen(args, cols, split, (f"lr{it}", "j"))
        blk: List[str] = []
        for s in left_first:
            g2.load(s, f"la{it}", blk, ind)
            fields.append((_CTYPE[cols[s][0]], f"x{s}_{it}"))
            if cols[s][1]:
                fields.append(("bool", f"n{s}_{it}"))
        batch += [_rename(x, left_first, it) for x in blk]
    # right columns of the span are staged in LDS with the keys (one coalesced batch), so the
    # match rounds read them from LDS instead of a dependent HBM gather at j
    staged_cols = right_all if JOIN_STAGE_RIGHT else []
    for s in staged_cols:
        ct = _CTYPE[cols[s][0]]
        b.insert(1, f"  __shared__ {ct} sv{s}[{LDS_KEYS}];")
        if cols[s][1]:
            b.insert(1, f"  __shared__ unsigned char sn{s}[{LDS_KEYS}];")
    for q in range(KEYS_PER_THREAD):
        off = f"{q * BLOCK} + (i64)threadIdx.x"
        batch.append(f"{ind}const bool sa{q} = staged && {off} < re - rs;")
        batch.append(f"{ind}const u64 sk{q} = sa{q} ? "
                     f"{_key_expr(gen.value(rk, f'rs + {off}'), fl)} : 0ull;")
        fields += [("bool", f"sa{q}"), ("u64", f"sk{q}")]
        for s in staged_cols:
            ct = _CTYPE[cols[s][0]]
            batch.append(f"{ind}const {ct} svv{s}_{q} = sa{q} ? {gen.value(s, f'rs + {off}')} : ({ct})0;")
            fields.append((ct, f"svv{s}_{q}"))
            if cols[s][1]:
                batch.append(f"{ind}const unsigned char snv{s}_{q} = sa{q} ? {gen.vptr(s)}[rs + {off}] : 0;")
                fields.append(("unsigned char", f"snv{s}_{q}"))
    direct = JOIN_DIRECT and not fl
    if direct:
        # first / last right key of the span (uniform loads): a span of integer keys whose
        # value range fits DT slots gets a direct-address LDS table instead of a binary search
        batch.append(f"{ind}const u64 dbk = (staged && re > rs) ? "
                     f"{_key_expr(gen.value(rk, 'rs'), fl)} : 0ull;")
        batch.append(f"{ind}const u64 dek = (staged && re > rs) ? "
                     f"{_key_expr(gen.value(rk, 're - 1'), fl)} : 0ull;")
        fields += [("u64", "dbk"), ("u64", "dek")]
        b.insert(1, f"  __shared__ short dtab[{JOIN_DIRECT_SLOTS}];")
    pre: List[str] = []
    if JOIN_PIPELINE:
        b, pre = _pipeline_tiles(b, batch, fields, NI, BLOCK, LDS_KEYS)
    else:
        b += batch
    for it in range(NI):
        g2 = _Gen(args, cols, split, (f"lr{it}", "j"))
        cond = _rename(g2.cnf(lpreds), left_first, it)
        okk = f"n{lk}_{it}" if cols[lk][1] else "true"
        b.append(f"{ind}bool m{it} = la{it} && {okk} && {cond};")
        b.append(f"{ind}const u64 k{it} = {_key_expr(f'x{lk}_{it}', fl)};")
    if direct:
        b.append(f"{ind}const bool dense = staged && re > rs && dek - dbk < {JOIN_DIRECT_SLOTS}ull;")
    for q in range(KEYS_PER_THREAD):
        idx = f"{q * BLOCK} + threadIdx.x"
        b.append(f"{ind}if (sa{q}) {{ skeys[{idx}] = sk{q};")
        if direct:
            b.append(f"{ind}  if (dense) dtab[sk{q} - dbk] = (short)({idx});")
        for s in staged_cols:
            b.append(f"{ind}  sv{s}[{idx}] = svv{s}_{q};")
            if cols[s][1]:
                b.append(f"{ind}  sn{s}[{idx}] = snv{s}_{q};")
        b.append(f"{ind}}}")
    b += [f"{ind}if (staged) {{",
          f"{ind}  for (i64 q = {KEYS_PER_THREAD * BLOCK} + threadIdx.x; q < re - rs; q += {BLOCK}) {{",
          f"{ind}    const u64 kq = {_key_expr(gen.value(rk, 'rs + q'), fl)};",
          f"{ind}    skeys[q] = kq;"]
    if direct:
        b.append(f"{ind}    if (dense) dtab[kq - dbk] = (short)q;")
    for s in staged_cols:
        b.append(f"{ind}    sv{s}[q] = {gen.value(s, 'rs + q')};")
        if cols[s][1]:
            b.append(f"{ind}    sn{s}[q] = {gen.vptr(s)}[rs + q];")
    b += [f"{ind}  }}", f"{ind}}}", f"{ind}__syncthreads();"]
    # (2) first match per row (LDS binary search; global search for oversized spans)
    for it in range(NI):
        b += [f"    i64 j{it} = rs;",
              f"    if (m{it}) {{"]
        if direct:
            # slot hit verified against the staged key (stale slots from earlier tiles fail the
            # check); duplicates walk back to their first occurrence
            b += ["      if (dense) {",
                  f"        const u64 d = k{it} - dbk; m{it} = false;",
                  f"        if (d < {JOIN_DIRECT_SLOTS}ull) {{ i64 q = dtab[d];",
                  f"          if (q >= 0 && q < re - rs && skeys[q] == k{it}) {{",
                  f"            while (q > 0 && skeys[q - 1] == k{it}) --q;",
                  f"            j{it} = rs + q; m{it} = true; }} }}",
                  "      } else"]
        b += ["      if (staged) { i64 lo = 0, hi = re - rs;",
              f"        while (lo < hi) {{ const i64 md = (lo + hi) >> 1; if (skeys[md] < k{it}) lo = md + 1; else hi = md; }}",
              f"        j{it} = rs + lo; m{it} = j{it} < re && skeys[lo] == k{it};",
              "      } else { i64 lo = rs, hi = re;",
              f"        while (lo < hi) {{ const i64 md = (lo + hi) >> 1; const bool nv = {_valid_expr(gen, rk, 'md')};",
              f"          if (nv || {_key_expr(gen.value(rk, 'md'), fl)} < k{it}) lo = md + 1; else hi = md; }}",
              f"        j{it} = lo; m{it} = lo < re && {_key_expr(gen.value(rk, 'lo'), fl)} == k{it}; }}",
              "    }"]
    # (3) match rounds: right columns at j, residual predicates, accumulate
    anym = " || ".join(f"m{it}" for it in range(NI))
    b.append(f"    while (__any({anym})) {{")
    allslots = left_all + right_all
    for it in range(NI):
        g2 = _Gen(args, cols, split, (f"lr{it}", f"j{it}"))
        blk = []
        for s in right_all:
            if s in staged_cols:
                ct = _CTYPE[cols[s][0]]
                blk.append(f"      const {ct} x{s} = m{it} ? (staged ? sv{s}[j{it} - rs] : "
                           f"{g2.value(s, f'j{it}')}) : ({ct})0;")
                if cols[s][1]:
                    blk.append(f"      const bool n{s} = m{it} && (staged ? sn{s}[j{it} - rs] : "
                               f"{g2.vptr(s)}[j{it}]) != 0;")
            else:
                g2.load(s, f"m{it}", blk, "      ")
        b += [_rename(x, right_all, it) for x in blk]
        cond = _rename(g2.cnf(rpreds), allslots, it)
        b.append(f"      bool ps{it} = m{it} && {cond};")
        if left_late:
            blk = []
            for s in left_late:
                g2.load(s, f"ps{it}", blk, "      ")
            b += [_rename(x, left_late, it) for x in blk]
        gvar = f"gi{it}"
        if grouped:
            g = p.group_col
            base = args.add("q", "group_base", "long long")
            ng = args.add("q", "num_groups", "long long")
            b.append(f"      const i64 gl{it} = (i64)x{g}_{it} - {base};")
            okg = f"n{g}_{it}" if cols[g][1] else "true"
            b.append(f"      ps{it} = ps{it} && {okg} && gl{it} >= 0 && gl{it} < {ng};")
            b.append(f"      const int {gvar} = ps{it} ? (int)gl{it} : 0;")
        acc = _accumulate(g2, aggs, grouped, f"ps{it}", gvar, "      ")
        b += [_rename(x, allslots, it) for x in acc]
        b += [f"      if (m{it}) {{ ++j{it};",
              f"        m{it} = j{it} < re && (staged ? skeys[j{it} - rs] : "
              f"{_key_expr(gen.value(rk, f'j{it}'), fl)}) == k{it}; }}"]
    b += ["    }", "    __syncthreads();", "  }"]
    b += _flush(aggs, grouped, BLOCK)
    src = (_PRELUDE + args.struct_src() + "\n".join(pre) +
           f'extern "C" __global__ __launch_bounds__({BLOCK}) void hs_jit_join_agg(Args a) {{\n' +
           "\n".join(b) + "\n}\n")
    lds = (len(aggs) * p.num_groups * 32) if grouped else 0
    return Kernel(src, "hs_jit_join_agg", args, lds, BLOCK)


def _pipeline_tiles(b: List[str], batch: List[str], fields, NI: int, BLOCK: int,  # noqa: N803
                    LDS_KEYS: int):  # noqa: N803
    """Software-pipeline the tile loop: tile t+1's left batch and right keys are loaded while
    tile t runs its LDS search and match rounds, which takes one dependent HBM round trip off
    every tile's critical path.  Vector-memory loads retire in issue order, so the prefetch
    (issued first) never delays the current tile's own gathers.

    ``b`` holds the kernel prologue up to and including the per-tile ``lr/la`` lines; the
    batch loads move into a device function returning a register struct, and the tile body
    reads the current struct's fields under their usual names."""
    head = b[:b.index("  for (i64 t = t0; t < t1; ++t) {")]
    body_la = [x for x in b[len(head):] if x.lstrip().startswith(("const i64 lr",
                                                                   "const bool la"))]
    pre = ["struct Batch {"] + [f"  {ct} {n};" for ct, n in fields] + ["};",
           "__device__ __forceinline__ Batch load_batch(const Args& a, i64 row0, i64 rows, "
           "i64 rs, i64 re) {",
           f"  const bool staged = re - rs <= {LDS_KEYS};"]
    pre += [x.replace("    ", "  ", 1) for x in body_la + batch]
    pre += ["  Batch B_;"] + [f"  B_.{n} = {n};" for _, n in fields] + ["  return B_;", "}", ""]
    out = list(head)
    out += ["  i64 c_row0 = n_row0, c_rows = n_rows, c_rs = n_rs, c_re = n_re;",
            "  if (t0 + 1 < t1) { n_row0 = a.spans[4 * t0 + 4]; n_rows = a.spans[4 * t0 + 5];",
            "                     n_rs = a.spans[4 * t0 + 6]; n_re = a.spans[4 * t0 + 7]; }",
            "  Batch cur = load_batch(a, c_row0, c_rows, c_rs, c_re);",
            "  for (i64 t = t0; t < t1; ++t) {",
            "    const i64 row0 = c_row0, rows = c_rows, rs = c_rs, re = c_re;",
            f"    const bool staged = re - rs <= {LDS_KEYS};",
            "    Batch nxt = cur;",
            "    if (t + 1 < t1) nxt = load_batch(a, n_row0, n_rows, n_rs, n_re);",
            "    c_row0 = n_row0; c_rows = n_rows; c_rs = n_rs; c_re = n_re;",
            "    if (t + 2 < t1) { n_row0 = a.spans[4 * t + 8]; n_rows = a.spans[4 * t + 9];",
            "                      n_rs = a.spans[4 * t + 10]; n_re = a.spans[4 * t + 11]; }"]
    out += body_la
    out += [f"    const {ct} {n} = cur.{n};" for ct, n in fields]
    out += ["    cur = nxt;"]
    return out, pre


def join_lds_keys() -> int:
    """LDS key slots per join workgroup: 2x the tile (FK joins stage ~tile/4 keys), capped."""
    return max(256, min(JOIN_LDS_KEYS, 2 * JOIN_BLOCK * JOIN_ITEMS))


def _valid_expr(gen: _Gen, slot: int, row: str) -> str:
    vp = gen.vptr(slot)
    return f"({vp}[{row}] == 0)" if vp else "false"


def _rename(line: str, slots, it: int) -> str:
    """Suffix per-row-slot variables x<s>/n<s> with the batch item index."""
    import re
    for s in sorted(set(slots), reverse=True):
        line = re.sub(rf"\b([xnqr]){s}\b", rf"\g<1>{s}_{it}", line)
    return line


_SOFF: Dict[int, tuple] = {}


# ------------------------------------------------------------------------------------------------
# Join through a cached join index (exec/join_index.py)
# ------------------------------------------------------------------------------------------------
def join_index_agg_shape(p: NL.JoinParams, compacts=None, vec: int = 0, jw: int = 4,
                         jlog: int = 0, stage: bool = False, bitmap: bool = False) -> tuple:
    cols = tuple(sorted(_col_specs(p, compacts).items()))
    preds = tuple((p.preds[k].kind, p.preds[k].op, p.preds[k].col, p.preds[k].col2,
                   p.preds[k].group) for k in range(p.npreds))
    aggs = tuple((p.aggs[i].kind, p.aggs[i].nterms, tuple(p.aggs[i].col[:p.aggs[i].nterms]))
                 for i in range(p.naggs))
    return ("join_index_agg", cols, preds, p.nlp, aggs, p.group_col, JI_ITEMS, vec, BLOCK, jw,
            jlog, JI_COMPACT, WAVE_SYNC, bool(stage and vec), bool(bitmap), VEC_PREFETCH)


def _uload_raw(gen: _Gen, slot: int, it, raw: str, vraw: str, out: List[str], ind: str) -> None:
    """``_uload``'s registers for column ``slot`` / item ``it`` from an already loaded stored
    element ``raw`` (and validity byte ``vraw``)."""
    ct = _CTYPE[gen.cols[slot][0]]
    enc = gen.cols[slot][2]
    if enc:
        out.append(f"{ind}const int r{slot}_{it} = (int){raw};")
        if enc[1]:
            base = gen.a.add("q", f"B{slot}", "long long")
            out.append(f"{ind}const i64 q{slot}_{it} = {base} + (i64){raw};")
    out.append(f"{ind}const {ct} x{slot}_{it} = {gen.decode(slot, raw)};")
    if gen.cols[slot][1]:
        out.append(f"{ind}const bool n{slot}_{it} = {vraw} != 0;")


def _uload(gen: _Gen, slot: int, it: int, out: List[str], ind: str) -> None:
    """Unconditional load of column ``slot`` for batch item ``it`` at the generator's row
    variable (callers redirect rows that do not need the value to an always-valid shared row, so
    the load needs no branch and the wavefront's redirected lanes coalesce into one line)."""
    ct = _CTYPE[gen.cols[slot][0]]
    r = gen.row(slot)
    enc = gen.cols[slot][2]
    if enc:
        out.append(f"{ind}const {gen.raw_type(slot)} w{slot}_{it} = {gen.ptr(slot)}[{r}];")
        out.append(f"{ind}const int r{slot}_{it} = (int)w{slot}_{it};")
        if enc[1]:
            base = gen.a.add("q", f"B{slot}", "long long")
            out.append(f"{ind}const i64 q{slot}_{it} = {base} + (i64)w{slot}_{it};")
        out.append(f"{ind}const {ct} x{slot}_{it} = {gen.decode(slot, f'w{slot}_{it}')};")
    else:
        out.append(f"{ind}const {ct} x{slot}_{it} = {gen.value(slot, r)};")
    if gen.cols[slot][1]:
        out.append(f"{ind}const bool n{slot}_{it} = {gen.vptr(slot)}[{r}] != 0;")


def _crow_t(T: int) -> str:
    """Element type of the compaction lists' tile-relative row offsets."""
    return "unsigned short" if T + 8 <= 65536 else "int"


def _wave_sync(force: bool = False) -> str:
    """Barrier that orders the per-wavefront LDS compaction lists: each wavefront owns its own
    list, and a wavefront's LDS operations execute in order, so only the compiler has to be kept
    from moving accesses across (a block-wide barrier would make the block's wavefronts wait for
    each other's memory round trips)."""
    return ("__builtin_amdgcn_fence(__ATOMIC_RELEASE, \"wavefront\"); "
            "__builtin_amdgcn_wave_barrier(); "
            "__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, \"wavefront\");") if (WAVE_SYNC or force) \
        else "__syncthreads();"


def _vec_rows(b: List[str], NI: int, ind: str) -> None:
    """Row mapping of a vectorized tile: the tile covers range r from its start rounded down to
    a multiple of NI, each thread owns NI consecutive rows at an aligned index ``g0``; rows
    outside [rs, re) are inactive (their ``row`` is never read: every use is guarded by the
    item's ``act``/``pass``).  Activity is two 32-bit compares per item against the thread's
    clamped item bounds [alo, ahi)."""
    b += ["    const i64 rs = a.rstart[r], re = rs + a.rlen[r];",
          f"    const i64 tb0 = (rs & ~(i64){NI - 1}) + off;",
          f"    const i64 g0 = tb0 + (i64)threadIdx.x * {NI};"]
    _vec_act(b, NI, ind)


def _vec_act(b: List[str], NI: int, ind: str) -> None:
    """Per-item activity and rows of a vectorized tile from its geometry ``rs re g0``."""
    b += [f"    const i64 dlo_ = rs - g0, dhi_ = re - g0;",
          f"    const int alo = dlo_ <= 0 ? 0 : (dlo_ >= {NI} ? {NI} : (int)dlo_);",
          f"    const int ahi = dhi_ <= 0 ? 0 : (dhi_ >= {NI} ? {NI} : (int)dhi_);"]
    for it in range(NI):
        b += [f"{ind}const bool act{it} = {it} >= alo && {it} < ahi;",
              f"{ind}const i64 row{it} = g0 + {it};"]


def _vec_loads(gen: "_Gen", slots, extra=()) -> List[Tuple[str, str, str]]:
    """(array name, C type, pointer) of every streamed vector load of a tile: ``extra`` raw
    arrays, the stored elements of ``slots`` and their validity bytes."""
    loads = list(extra) + [(f"x{s}", gen.raw_type(s), gen.ptr(s)) for s in slots]
    for s in slots:
        if gen.cols[s][1]:
            loads.append((f"n{s}", "unsigned char", gen.vptr(s)))
    return loads


_TILE_HEAD = ["  const i64 ntiles = a.tile_prefix[a.R];",
              "  const i64 per = (ntiles + gridDim.x - 1) / gridDim.x;",
              "  const i64 t0 = (i64)blockIdx.x * per;",
              "  const i64 t1 = ntiles < t0 + per ? ntiles : t0 + per;",
              "  int r = 0;",
              "  if (t0 < t1) { int lo = 0, hi = (int)a.R;",
              "    while (hi - lo > 1) { const int m = (lo + hi) >> 1; if (a.tile_prefix[m] <= t0) lo = m; else hi = m; }",
              "    r = lo; }"]


def _tile_loop(b: List[str], T: int, NI: int, vec: int, ind: str = "    ") -> None:
    """Header of the persistent tile loop of the streaming kernels: each block owns a contiguous
    run of ``T``-row tiles and ``r`` tracks the row range of the tile.  Vectorized tiles
    (``vec``) also get the row geometry ``rs re tb0 g0 act<k> row<k>``."""
    b += _TILE_HEAD
    b += ["  for (i64 t = t0; t < t1; ++t) {",
          "    while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= t) ++r;",
          f"    const i64 off = (t - a.tile_prefix[r]) * {T};"]
    if vec:
        _vec_rows(b, NI, ind)


def _vec_tiles(b: List[str], T: int, NI: int, ind: str, loads, scalars, body,
               tscalars=()) -> None:
    """Tile loops of a vectorized streaming kernel (``body(b, mode)`` emits one tile's work;
    ``loads`` = (name, C type, pointer) vector arrays, ``scalars`` = (name, C type, expression
    over ``G0``) per-thread values loaded with them).

    Tiles that end inside the table (``tb0 + T <= nrows``: every tile but the table's last few)
    read their columns with unconditional aligned vector loads, the rest element-wise, behind a
    wavefront-uniform test — a per-thread ``if (vok) vector else elements`` merge makes the
    compiler wait for each vector load before the merge, one round trip per column.

    With VEC_PREFETCH the full tiles run software pipelined: tile t+1's vector loads are issued
    at the top of tile t, before t's predicates, gathers and aggregate tail, so each wavefront
    keeps the next tile's stream in flight across this tile's dependent round trips.  Full
    tiles precede partial ones in a block's run, so the pipelined loop runs first and the
    element-wise loop finishes the run.  ``tscalars`` = (name, C type, expression over ``{t}``)
    per-tile values (span bounds, run windows) prefetched the same way."""
    if not VEC_PREFETCH:
        _tile_loop(b, T, NI, 1, ind)
        for name, ct, expr in tscalars:
            b.append(f"{ind}const {ct} {name} = {expr.format(t='t')};")
        b.append(f"{ind}if (tb0 + {T} <= a.nrows) {{")
        _vec_issue(b, loads, NI, ind, True)
        for name, ct, expr in scalars:
            b.append(f"{ind}const {ct} {name} = {expr.replace('G0', 'g0')};")
        body(b, True)
        b.append(f"{ind}}} else {{")
        _vec_issue(b, loads, NI, ind, False)
        for name, ct, expr in scalars:
            b.append(f"{ind}const {ct} {name} = {expr.replace('G0', 'g0')};")
        body(b, False)
        b.append(f"{ind}}}")
        return
    b += _TILE_HEAD

    def geom(texpr: str, i2: str) -> None:
        b.extend([f"{i2}while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= {texpr}) ++r;",
                  f"{i2}{{ const i64 off_ = ({texpr} - a.tile_prefix[r]) * {T};",
                  f"{i2}  rsP = a.rstart[r]; reP = rsP + a.rlen[r];",
                  f"{i2}  tb0P = (rsP & ~(i64){NI - 1}) + off_;",
                  f"{i2}  g0P = tb0P + (i64)threadIdx.x * {NI}; }}",
                  f"{i2}fullP = tb0P + {T} <= a.nrows;"])
        for name, ct, expr in tscalars:
            b.append(f"{i2}{name}P = {expr.format(t=texpr)};")
        b.append(f"{i2}if (fullP) {{")
        for name, ct, ptr in loads:
            b.append(f"{i2}  vload<{ct}, {NI}>({ptr}, g0P, {name}vP);")
        for name, ct, expr in scalars:
            b.append(f"{i2}  {name}P = {expr.replace('G0', 'g0P')};")
        b.append(f"{i2}}}")

    b.append("  i64 rsP = 0, reP = 0, tb0P = 0, g0P = 0; bool fullP = false;")
    for name, ct, _ in loads:
        b.append(f"  {ct} {name}vP[{NI}];")
    for name, ct, _ in list(scalars) + list(tscalars):
        b.append(f"  {ct} {name}P = ({ct})0;")
    b.append("  i64 t = t0;")
    b.append("  if (t < t1) {")
    geom("t", "    ")
    b.append("  }")
    b += ["  for (; t < t1 && fullP; ++t) {",
          "    const i64 rs = rsP, re = reP, tb0 = tb0P, g0 = g0P;"]
    for name, ct, _ in loads:
        b.append(f"{ind}{ct} {name}v[{NI}]; " +
                 " ".join(f"{name}v[{k}] = {name}vP[{k}];" for k in range(NI)))
    for name, ct, _ in list(scalars) + list(tscalars):
        b.append(f"{ind}const {ct} {name} = {name}P;")
    b.append(f"{ind}if (t + 1 < t1) {{")
    geom("(t + 1)", ind + "  ")
    b.append(f"{ind}}} else fullP = false;")
    _vec_act(b, NI, ind)
    body(b, True)
    b.append("  }")
    b += ["  for (; t < t1; ++t) {",
          "    while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= t) ++r;",
          f"    const i64 off = (t - a.tile_prefix[r]) * {T};"]
    _vec_rows(b, NI, ind)
    for name, ct, expr in tscalars:
        b.append(f"{ind}const {ct} {name} = {expr.format(t='t')};")
    _vec_issue(b, loads, NI, ind, False)
    for name, ct, expr in scalars:
        b.append(f"{ind}const {ct} {name} = {expr.replace('G0', 'g0')};")
    body(b, False)


def _vec_issue(b: List[str], loads, NI: int, ind: str, full: bool) -> None:
    """Loads of the NI consecutive rows at ``g0`` into ``<name>v`` for every (name, C type,
    pointer) of ``loads``: aligned vector loads in full tiles, guarded element loads otherwise."""
    for name, ct, ptr in loads:
        b.append(f"{ind}{ct} {name}v[{NI}];")
        if full:
            b.append(f"{ind}vload<{ct}, {NI}>({ptr}, g0, {name}v);")
        else:
            b.append(f"{ind}" + " ".join(
                f"{name}v[{k}] = act{k} ? {ptr}[g0 + {k}] : ({ct})0;" for k in range(NI)))


def _vec_load_slots(b: List[str], gen: "_Gen", slots, NI: int, ind: str) -> None:
    """Per-item registers x<s>_<k> / n<s>_<k> (decoded) of the raw vector arrays the tile loop
    loaded for ``slots``."""
    for it in range(NI):
        for s in slots:
            ct = _CTYPE[gen.cols[s][0]]
            enc = gen.cols[s][2]
            if enc:
                b.append(f"{ind}const int r{s}_{it} = (int)x{s}v[{it}];")
            if enc and enc[1]:
                base = gen.a.add("q", f"B{s}", "long long")
                b.append(f"{ind}const i64 q{s}_{it} = {base} + (i64)x{s}v[{it}];")
            b.append(f"{ind}const {ct} x{s}_{it} = {gen.decode(s, f'x{s}v[{it}]')};")
            if gen.cols[s][1]:
                b.append(f"{ind}const bool n{s}_{it} = n{s}v[{it}] != 0;")


def _vec_aligned_ptrs(ptrs) -> bool:
    return all(int(x) % 16 == 0 for x in ptrs if x)


def _compacted_tail(args, cols, split, approx, aggs, grouped, group_col, third, allslots,
                    NI: int, ind: str, with_j: bool = True, pass_fmt: str = "pass{it}",
                    j_fmt: str = "j{it}", dump: bool = False, hk=None,
                    jgroup: bool = False) -> List[str]:
    """Phase 3 over the passing rows only.  A join like TPC-H Q3 keeps a few percent of its
    rows, so decoding and accumulating all NI x 64 rows of a wavefront (branch-free) is mostly
    wasted VALU work: instead each lane appends its passing (row, j) pairs to a per-wavefront
    LDS list (positions from per-item ballots), and the wavefront walks the list 64
    entries at a time — aggregate loads, decode and accumulation run once per passing row."""
    # list position of a passing item: item-major order (all lanes' item 0, then item 1, ...),
    # from one ballot + mbcnt per item instead of a 6-step cross-lane prefix sum
    b = [f"{ind}int wtot = 0;"]
    for it in range(NI):
        pv = pass_fmt.format(it=it)
        cj = f"cj_s[wv][pos{it}] = (int)({j_fmt.format(it=it)}); " if with_j else ""
        b += [f"{ind}{{ const bool pz = {pv}; const u64 bm = __ballot(pz);",
              f"{ind}  const int pos{it} = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), "
              f"__builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));"]
        if dump:
            # branch-free: failing lanes write their own slot past the list (crow_s/cj_s carry
            # 64 extra entries per wavefront), so no exec-mask save/restore per item
            b += [f"{ind}  const int wp{it} = pz ? pos{it} : {64 * NI} + cln;",
                  f"{ind}  crow_s[wv][wp{it}] = (crow_t)(row{it} - tb0); " +
                  cj.replace(f"[pos{it}]", f"[wp{it}]")]
        else:
            b += [f"{ind}  if (pz) {{ crow_s[wv][pos{it}] = (crow_t)(row{it} - tb0); {cj}}}"]
        b += [f"{ind}  wtot += __popcll(bm); }}"]
    b += [f"{ind}{_wave_sync()}",
          f"{ind}for (int cb = 0; cb < wtot; cb += 64) {{",
          f"{ind}  const int ce = cb + cln;",
          f"{ind}  bool cok = ce < wtot;",
          f"{ind}  const i64 crow = tb0 + (cok ? crow_s[wv][ce] : 0);",
          f"{ind}  const i64 cj = cok ? (i64)cj_s[wv][ce] : 0;" if with_j else
          f"{ind}  const i64 cj = crow;"]
    ind2 = ind + "  "
    g = _Gen(args, cols, split, ("crow", "cj"), approx, True)
    # every slot the aggregates and the group key read, re-loaded at the listed rows (the
    # phase-1/2 registers belong to the original, uncompacted rows)
    tail = list(dict.fromkeys(_agg_slots(aggs) + ([group_col] if grouped and not jgroup else []) +
                              (hk.slots if hk is not None else [])))
    for sl in tail:
        _uload(g, sl, "c", b, ind2)
    gvar = "gic"
    if jgroup:
        # the listed j is the row's group index itself (jit_runs: a right-side group key's code
        # carried in the run tag)
        b.append(f"{ind2}const int {gvar} = cok ? (int)cj : 0;")
    elif grouped:
        base = args.add("q", "group_base", "long long")
        ng = args.add("q", "num_groups", "long long")
        b.append(f"{ind2}const i64 glc = (i64){_rename(f'x{group_col}', allslots, 'c')} - {base};")
        b.append(f"{ind2}cok = cok && {_rename(g.ok(group_col), allslots, 'c')} && "
                 f"glc >= 0 && glc < {ng};")
        b.append(f"{ind2}const int {gvar} = cok ? (int)glc : 0;")
    if hk is not None:
        b += [_rename(x, allslots, "c") for x in JH._hash_accumulate(g, aggs, hk, "cok", ind2)]
    else:
        b += [_rename(x, allslots, "c") for x in _accumulate(g, aggs, grouped, "cok", gvar, ind2)]
    b += [f"{ind}}}", f"{ind}{_wave_sync()}"]
    return b


def gen_join_index_agg(p: NL.JoinParams, compacts=None, vec: int = 0, jw: int = 4,
                       jlog: int = 0, stage: Optional[bool] = None,
                       bitmap: bool = False) -> Kernel:
    """Fused join + aggregate as a streaming scan of the left table's row ranges that reads
    ``jidx[row]`` — the matching right row from the cached join index (exec/join_index.py) — and
    gathers right-side columns there.

    The kernel is latency-bound on its chain of dependent loads, so the code is phase-major over
    the JI_ITEMS rows of each thread (every row's loads of one phase are in flight together) and
    branch-free (rows that do not need a value load it from a shared, always-valid row instead
    of branching around the load):

    1. ``jidx`` and the left predicate columns of all items;
    2. right predicate columns at ``j`` (non-matching rows read right row 0);
    3. aggregate inputs and the group column (failing rows read the tile's first row).

    Right rows of consecutive left rows are monotone (both sides sorted by key per bucket), so
    the gathers of a wavefront hit a few adjacent cache lines."""
    args = Args()
    jct = {4: "int", 2: "unsigned short", 1: "unsigned char"}[jw]
    sent = {2: "0xFFFF", 1: "0xFF"}.get(jw)
    for n, ct in (("rstart", "const long long*"), ("rlen", "const long long*"),
                  ("tile_prefix", "const long long*"), ("jidx", f"const {jct}*")):
        args.add("p", n, ct)
    if jw < 4:
        # block-coded join index (exec/join_index.py): j = jbase[row >> jlog] + code
        args.add("p", "jbase", "const int*")
    args.add("q", "R", "long long")
    _common_args(args)
    cols = _col_specs(p, compacts)
    split = 8
    lpreds = [(k, p.preds[k]) for k in range(p.nlp)]
    rpreds = [(k, p.preds[k]) for k in range(p.nlp, p.npreds)]
    aggs = [p.aggs[i] for i in range(p.naggs)]
    grouped = p.group_col >= 0
    first = _pred_slots(lpreds)
    second = [s for s in _pred_slots(rpreds) if s not in first]
    third = [s for s in _agg_slots(aggs) + ([p.group_col] if grouped else [])
             if s not in first and s not in second]
    third = list(dict.fromkeys(third))
    allslots = first + second + third
    approx = _sum_only_slots(lpreds + rpreds, aggs, p.group_col, cols)
    NI = vec or JI_ITEMS
    T = BLOCK * NI
    if vec:
        args.add("q", "nrows", "long long")
    b: List[str] = []
    b += _acc_decls(aggs, grouped, args)
    if grouped:
        base = args.add("q", "group_base", "long long")
        ng = args.add("q", "num_groups", "long long")
    ind = "    "
    g1 = _Gen(args, cols, split, ("row0", "row0"), approx, True)
    compact = JI_COMPACT and bool(third)
    # the bitmap replaces phase 2 only when the aggregate tail re-loads what it needs
    bitmap = bool(bitmap and second and compact and _right_only(p, split))
    stage = bool(vec and second and not bitmap and (JI_STAGE if stage is None else stage))

    def phase2_global(b: List[str]) -> None:
        for it in range(NI):
            g2 = _Gen(args, cols, split, (f"row{it}", f"j{it}"), approx, True)
            for s in second:
                _uload(g2, s, it, b, ind)

    def body(b: List[str], full: Optional[bool]) -> None:
        """Tile body; ``full`` = vectorized full tile / vectorized last tile / None (scalar)."""
        if full is not None:     # raw vector arrays and jb come from the tile loop
            _vec_load_slots(b, g1, first, NI, ind)
            for it in range(NI):
                if jw < 4:
                    b.append(f"{ind}const int jr{it} = act{it} && jrv[{it}] != {sent} ? "
                             f"jb + (int)jrv[{it}] : -1;")
                else:
                    b.append(f"{ind}const int jr{it} = act{it} ? jrv[{it}] : -1;")
        else:
            b.extend(["    const i64 tb0 = a.rstart[r] + off;",
                      f"    const i64 rows = a.rlen[r] - off < {T} ? a.rlen[r] - off : {T};"])
            for it in range(NI):
                b.extend([f"{ind}const bool act{it} = {it * BLOCK} + (i64)threadIdx.x < rows;",
                          f"{ind}const i64 row{it} = tb0 + (act{it} ? {it * BLOCK} + (i64)threadIdx.x : 0);"])
            # phase 1: join index + left predicate columns of every item
            for it in range(NI):
                if jw < 4:
                    b.append(f"{ind}const {jct} jc{it} = a.jidx[row{it}];")
                    b.append(f"{ind}const int jr{it} = jc{it} != {sent} ? "
                             f"a.jbase[row{it} >> {jlog}] + (int)jc{it} : -1;")
                else:
                    b.append(f"{ind}const int jr{it} = a.jidx[row{it}];")
                g1i = _Gen(args, cols, split, (f"row{it}", f"row{it}"), approx, True)
                for s in first:
                    _uload(g1i, s, it, b, ind)
        for it in range(NI):
            g1i = _Gen(args, cols, split, (f"row{it}", f"row{it}"), approx, True)
            cond = _rename(g1i.cnf(lpreds), allslots, it)
            b.append(f"{ind}bool pass{it} = act{it} && jr{it} >= 0 && {cond};")
            b.append(f"{ind}const i64 j{it} = pass{it} ? (i64)jr{it} : 0;")
        # phase 2: right predicate columns at the matched rows
        if bitmap:
            _bitmap_phase2(b, args, NI, ind)
            b.extend(_compacted_tail(args, cols, split, approx, aggs, grouped, p.group_col,
                                     third, allslots, NI, ind))
            return
        if stage:
            _ji_stage_phase2(b, g1, args, cols, split, approx, second, NI, stage, ind,
                             phase2_global)
        else:
            phase2_global(b)
        for it in range(NI):
            g2 = _Gen(args, cols, split, (f"row{it}", f"j{it}"), approx, True)
            b.append(f"{ind}pass{it} = pass{it} && {_rename(g2.cnf(rpreds), allslots, it)};")
        if compact:
            b.extend(_compacted_tail(args, cols, split, approx, aggs, grouped, p.group_col,
                                     third, allslots, NI, ind))
            return
        # phase 3: aggregate inputs (rows that failed read the tile's first row / right row 0)
        if third:
            for it in range(NI):
                b.extend([f"{ind}const i64 lq{it} = pass{it} ? row{it} : tb0;",
                          f"{ind}const i64 jq{it} = pass{it} ? j{it} : 0;"])
            for it in range(NI):
                g3 = _Gen(args, cols, split, (f"lq{it}", f"jq{it}"), approx, True)
                for s in third:
                    _uload(g3, s, it, b, ind)
        for it in range(NI):
            g3 = _Gen(args, cols, split, (f"lq{it}", f"jq{it}"), approx, True)
            gvar = f"gi{it}"
            if grouped:
                g = p.group_col
                gx = _rename(f"x{g}", allslots, it)
                ok = _rename(g3.ok(g), allslots, it)
                b.append(f"{ind}const i64 gl{it} = (i64){gx} - {base};")
                b.append(f"{ind}pass{it} = pass{it} && {ok} && gl{it} >= 0 && gl{it} < {ng};")
                b.append(f"{ind}const int {gvar} = pass{it} ? (int)gl{it} : 0;")
            b.extend(_rename(x, allslots, it) for x in
                     _accumulate(g3, aggs, grouped, f"pass{it}", gvar, ind))

    if vec:
        # NI | block size and g0 % NI == 0: the thread's rows share one join-index block
        sc = [("jb", "int", f"a.jbase[G0 >> {jlog}]")] if jw < 4 else []
        _vec_tiles(b, T, NI, ind, _vec_loads(g1, first, extra=[("jr", jct, "a.jidx")]), sc, body)
    else:
        _tile_loop(b, T, NI, 0)
        body(b, None)
    b += ["  }"]
    b += _flush(aggs, grouped)
    W = BLOCK // 64
    pre = []
    if compact:
        pre.append(f"  typedef {_crow_t(T)} crow_t; __shared__ crow_t crow_s[{W}][{64 * NI}]; "
                   f"__shared__ int cj_s[{W}][{64 * NI}];")
    if stage:
        for s in second:
            pre.append(f"  __shared__ __attribute__((aligned(16))) {g1.raw_type(s)} st{s}_s[{W}][512];")
            if cols[s][1]:
                pre.append(f"  __shared__ unsigned char sn{s}_s[{W}][512];")
    if compact or stage:
        pre.append("  const int cln = threadIdx.x & 63, wv = threadIdx.x >> 6;")
    b = pre + b
    src = (_PRELUDE + args.struct_src() +
           f'extern "C" __global__ __launch_bounds__({BLOCK}) void hs_jit_join_index_agg(Args a) {{\n' +
           "\n".join(b) + "\n}\n")
    lds = (len(aggs) * p.num_groups * 32) if grouped else 0
    return Kernel(src, "hs_jit_join_index_agg", args, lds)


def _bitmap_phase2(b: List[str], args: Args, NI: int, ind: str) -> None:
    """Phase 2 of the join-index kernel as bit tests on the right side's predicate bitmap
    (``gen_pred_bitmap``).  A thread's NI rows are consecutive and the join index is monotone
    within a bucket, so the matched right rows of its passing items fall in at most two bitmap
    words (loaded once each, unconditionally: word 0 stands in when nothing passes); an item
    whose word is neither (a gap of over 64 right rows) loads its own."""
    bm = args.add("p", "rbm", "const unsigned long long*")
    lo = " ".join(f"if (pass{it} && (int)j{it} < mlo) mlo = (int)j{it};" for it in range(NI))
    hi = " ".join(f"if (pass{it} && (int)j{it} > mhi) mhi = (int)j{it};" for it in range(NI))
    b += [f"{ind}int mlo = 0x7fffffff, mhi = -1; {lo} {hi}",
          f"{ind}const int wlo = mhi >= 0 ? (mlo >> 6) : 0, whi = mhi >= 0 ? (mhi >> 6) : 0;",
          f"{ind}const u64 bw0 = {bm}[wlo], bw1 = {bm}[whi];"]
    for it in range(NI):
        b += [f"{ind}if (pass{it}) {{ const int wi = (int)j{it} >> 6;",
              f"{ind}  const u64 w = wi == wlo ? bw0 : (wi == whi ? bw1 : {bm}[wi]);",
              f"{ind}  pass{it} = ((w >> ((int)j{it} & 63)) & 1ull) != 0ull; }}"]


def _right_only(p: NL.JoinParams, split: int = 8) -> bool:
    """Every right-side predicate reads right columns only (no left/right column compares)."""
    for k in range(p.nlp, p.npreds):
        pr = p.preds[k]
        if pr.kind == NL.PK_TRUE:
            continue
        if pr.col < split or (pr.kind in (NL.PK_INT_COL, NL.PK_FLT_COL) and pr.col2 < split):
            return False
    return True


def pred_bitmap_shape(p: NL.JoinParams, compacts=None) -> tuple:
    cols = tuple((s, c) for s, c in sorted(_col_specs(p, compacts).items()) if s >= 8)
    preds = tuple((p.preds[k].kind, p.preds[k].op, p.preds[k].col, p.preds[k].col2,
                   p.preds[k].group) for k in range(p.nlp, p.npreds))
    return ("pred_bitmap", cols, preds, p.nlp)


BITMAP_ITEMS = 4


def gen_pred_bitmap(p: NL.JoinParams, compacts=None) -> Kernel:
    """Semi-join bitmap of the right side of a join: bit r of ``rbm`` = the right-side
    predicates (``preds[nlp:]``) hold on right row r.  Each wavefront writes whole 64-bit words
    (one ballot per word, BITMAP_ITEMS words in flight per wavefront); an SF100 orders table is
    150M rows -> 18.75 MB of bitmap, resident in the Infinity Cache for the join kernel."""
    args = Args()
    args.add("p", "rbm", "unsigned long long*")
    args.add("q", "rnrows", "long long")
    cols = {s: c for s, c in _col_specs(p, compacts).items() if s >= 8}
    rpreds = [(k, p.preds[k]) for k in range(p.nlp, p.npreds)]
    slots = _pred_slots(rpreds)
    NI = BITMAP_ITEMS
    b = ["  const int lane = threadIdx.x & 63;",
         "  const i64 nw = (a.rnrows + 63) >> 6;",
         f"  const i64 wstep = (i64)gridDim.x * {BLOCK // 64 * NI};",
         f"  for (i64 w0 = ((i64)blockIdx.x * {BLOCK // 64} + (threadIdx.x >> 6)) * {NI}; w0 < nw; "
         "w0 += wstep) {"]
    ind = "    "
    for it in range(NI):
        b += [f"{ind}const i64 row{it} = ((w0 + {it}) << 6) + lane;",
              f"{ind}const bool act{it} = row{it} < a.rnrows;",
              f"{ind}const i64 jr{it} = act{it} ? row{it} : 0;"]
    for it in range(NI):
        g = _Gen(args, cols, 8, (f"jr{it}", f"jr{it}"), frozenset(), True)
        for sl in slots:
            _uload(g, sl, it, b, ind)
    for it in range(NI):
        g = _Gen(args, cols, 8, (f"jr{it}", f"jr{it}"), frozenset(), True)
        b += [f"{ind}{{ const u64 m = __ballot(act{it} && {_rename(g.cnf(rpreds), slots, it)});",
              f"{ind}  if (lane == 0 && w0 + {it} < nw) a.rbm[w0 + {it}] = m; }}"]
    b.append("  }")
    src = (_PRELUDE + args.struct_src() +
           f'extern "C" __global__ __launch_bounds__({BLOCK}) void hs_jit_pred_bitmap(Args a) {{\n' +
           "\n".join(b) + "\n}\n")
    return Kernel(src, "hs_jit_pred_bitmap", args)


def pred_bitmap(p: NL.JoinParams, compacts, rnrows: int, device):
    """Launch the right side's predicate bitmap (``gen_pred_bitmap``) on the current stream."""
    import torch
    nw = (int(rnrows) + 63) // 64
    bm = torch.empty(max(nw, 1), dtype=torch.int64, device=device)
    k = kernel_for(pred_bitmap_shape(p, compacts), lambda: gen_pred_bitmap(p, compacts))
    v = {"rbm": bm.data_ptr(), "rnrows": int(rnrows)}
    _fill_common(v, p.cols, [(i, p.preds[i]) for i in range(p.npreds)], [], compacts)
    per_block = BLOCK // 64 * BITMAP_ITEMS
    grid = max(1, min((nw + per_block - 1) // per_block, 8192))
    k.launch(grid, v, NL.stream_ptr())
    return bm


def _ji_stage_phase2(b: List[str], g1: "_Gen", args, cols, split, approx, second, NI: int,
                     stage: int, ind: str, fallback) -> None:
    """Phase 2 of the join-index kernel through LDS: the matched right rows of a wavefront's
    passing items are one short, monotone run (both sides sorted by key within a bucket, the
    wavefront's rows consecutive), so the wavefront copies the 8-byte aligned window of every
    right predicate column that holds the run [jlo, jhi] into its own LDS slice — one coalesced
    ``dwordx2`` per lane, i.e. one vector-memory instruction for the whole wavefront — and each
    item then reads LDS, instead of NI divergent gathers per lane, which made vector-memory
    instruction issue the kernel's limit.  Runs wider than the 512-byte window, or rows outside
    the run (a non-monotone index), take the global gathers."""
    lo_terms = " ".join(f"if (pass{it} && (int)j{it} < mlo) mlo = (int)j{it};" for it in range(NI))
    hi_terms = " ".join(f"if (pass{it} && (int)j{it} > mhi) mhi = (int)j{it};" for it in range(NI))
    # the window starts at jlo rounded down to 8 bytes of the widest staged element: every staged
    # array holds STAGE_W elements (512 bytes of the widest, fewer bytes of narrower ones)
    esz = max(_SIZEOF[g1.raw_type(s)] for s in second)
    span = 512 // esz
    b += [f"{ind}int mlo = 0x7fffffff, mhi = -1; {lo_terms} {hi_terms}",
          f"{ind}const u64 anyp = __ballot(mhi >= 0);",
          f"{ind}int jlo = 0, jhi = -1;",
          f"{ind}if (anyp) {{ jlo = __builtin_amdgcn_readlane(mlo, __ffsll((long long)anyp) - 1);",
          f"{ind}  jhi = __builtin_amdgcn_readlane(mhi, 63 - __clzll((long long)anyp)); }}",
          f"{ind}const int jw0 = jlo & ~{8 // esz - 1 if esz < 8 else 0};",
          f"{ind}const bool inrun = " + " && ".join(
              f"(!pass{it} || ((int)j{it} >= jlo && (int)j{it} <= jhi))" for it in range(NI)) + ";",
          f"{ind}const bool staged = anyp != 0ull && jhi - jw0 < {span} && __ballot(!inrun) == 0ull;"]
    # phase-2 registers (S-prefixed here, renamed to x/n/q after the branch), filled from LDS
    # or by the global gathers
    outs = []
    for it in range(NI):
        for s in second:
            outs.append((f"x{s}_{it}", _CTYPE[cols[s][0]]))
            if cols[s][1]:
                outs.append((f"n{s}_{it}", "bool"))
            enc = cols[s][2]
            if enc:
                outs.append((f"r{s}_{it}", "int"))
            if enc and enc[1]:
                outs.append((f"q{s}_{it}", "i64"))
    b.append(f"{ind}" + " ".join(f"{ct} S{n};" for n, ct in outs))
    b.append(f"{ind}if (staged) {{")
    i2 = ind + "  "
    # lane l copies elements [jw0 + l*8/esz, +8/esz) of each column: 8 bytes of the widest,
    # fewer of narrower ones; lanes whose piece starts past jhi stay idle (no read past the run's
    # last 8-byte word, which lies inside the column's allocation)
    for s in second:
        es = _SIZEOF[g1.raw_type(s)]
        per = 8 // esz * 1    # elements of the widest type per lane
        b.append(f"{i2}if (jw0 + cln * {per} <= jhi) {{")
        b.append(f"{i2}  " + " ".join(f"st{s}_s[wv][cln * {per} + {k}] = {g1.ptr(s)}[jw0 + cln * {per} + {k}];"
                                      for k in range(per)) if es * per != 8 else
                 f"{i2}  *reinterpret_cast<uint2*>(&st{s}_s[wv][cln * {per}]) = "
                 f"*reinterpret_cast<const uint2*>({g1.ptr(s)} + jw0 + cln * {per});")
        if cols[s][1]:
            b.append(f"{i2}  " + " ".join(f"sn{s}_s[wv][cln * {per} + {k}] = {g1.vptr(s)}[jw0 + cln * {per} + {k}];"
                                          for k in range(per)))
        b.append(f"{i2}}}")
    b.append(f"{i2}{_wave_sync(True)}")
    for it in range(NI):
        b.append(f"{i2}const int sj{it} = pass{it} ? (int)j{it} - jw0 : 0;")
        for s in second:
            enc = cols[s][2]
            raw = f"st{s}_s[wv][sj{it}]"
            if enc:
                b.append(f"{i2}Sr{s}_{it} = (int){raw};")
            if enc and enc[1]:
                base = args.add("q", f"B{s}", "long long")
                b.append(f"{i2}Sq{s}_{it} = {base} + (i64){raw};")
            b.append(f"{i2}Sx{s}_{it} = {g1.decode(s, raw)};")
            if cols[s][1]:
                b.append(f"{i2}Sn{s}_{it} = sn{s}_s[wv][sj{it}] != 0;")
    b.append(f"{i2}{_wave_sync(True)}")
    b.append(f"{ind}}} else {{")
    gl: List[str] = []
    fallback(gl)
    b += [f"{i2}{line.strip()}" for line in gl]
    b.append(f"{i2}" + " ".join(f"S{n} = {n};" for n, _ in outs))
    b.append(f"{ind}}}")
    b.append(f"{ind}" + " ".join(f"const {ct} {n} = S{n};" for n, ct in outs))


def _stage_aligned(p: NL.JoinParams, compacts) -> bool:
    """LDS staging copies 8-byte words of the right predicate columns (and validity bytes)."""
    ptrs = []
    for s in _pred_slots([(k, p.preds[k]) for k in range(p.nlp, p.npreds)]):
        c = (compacts or {}).get(s)
        ptrs.append(c.codes.data_ptr() if c else p.cols[s].data)
        ptrs.append(p.cols[s].valid)
    return all(int(x) % 8 == 0 for x in ptrs if x)


def _vec_aligned(p: NL.JoinParams, compacts, jidx) -> bool:
    """Vector loads need 16-byte aligned bases for every streamed left column."""
    ptrs = [jidx.data_ptr()]
    for s in _pred_slots([(k, p.preds[k]) for k in range(p.nlp)]):
        c = (compacts or {}).get(s)
        ptrs.append(c.codes.data_ptr() if c else p.cols[s].data)
        ptrs.append(p.cols[s].valid)
    return _vec_aligned_ptrs(ptrs)


def join_index_agg(p: NL.JoinParams, rstart, rlen, jx, compacts=None, nrows: int = 0,
                   rnrows: int = 0):
    """Same outputs as ``join_agg``.  ``jx``: the join index from ``join_index.get_join_index``
    (``codes`` int32 rows, or uint8/uint16 block-coded with ``base`` / ``log_blk``);
    ``nrows`` = left table rows (vectorized loads stay inside the columns)."""
    from ..ops import kernels as K
    jw = jx.width
    jlog = jx.log_blk if jw < 4 else 0
    vec = JI_VEC if JI_VEC > 0 and _vec_aligned(p, compacts, jx.codes) else 0
    if vec and jw < 4 and (1 << jlog) % vec:
        vec = 0
    if vec:
        # tiles over the ranges widened down to a multiple of vec rows (the kernel masks them)
        tp = K.ranges_to_tiles(rlen + (rstart & (vec - 1)), BLOCK * vec)
    else:
        tp = K.ranges_to_tiles(rlen, BLOCK * JI_ITEMS)
    grid = SCAN_GRID or NL.lib().hs_scan_grid()
    GA = p.naggs * (p.num_groups if p.group_col >= 0 else 1)
    stage = bool(JI_STAGE and vec) and _stage_aligned(p, compacts)
    bitmap = bool(JI_BITMAP and JI_COMPACT and rnrows > 0 and p.npreds > p.nlp and
                  _right_only(p))
    k = kernel_for(join_index_agg_shape(p, compacts, vec, jw, jlog, stage, bitmap),
                   lambda: gen_join_index_agg(p, compacts, vec, jw, jlog, stage, bitmap))
    bm = pred_bitmap(p, compacts, rnrows, rstart.device) if "rbm" in k.args._index else None
    parts = _partials(grid, GA, rstart.device)
    v = {"rstart": rstart.data_ptr(), "rlen": rlen.data_ptr(), "tile_prefix": tp.data_ptr(),
         "jidx": jx.codes.data_ptr(), "jbase": jx.base.data_ptr() if jw < 4 else 0,
         "R": rstart.numel(), "nrows": nrows, "psum": parts[0].data_ptr(),
         "pcnt": parts[1].data_ptr(), "pmin": parts[2].data_ptr(), "pmax": parts[3].data_ptr(),
         "num_groups": p.num_groups, "group_base": p.group_base,
         "rbm": bm.data_ptr() if bm is not None else 0}
    _fill_common(v, p.cols, [(k_, p.preds[k_]) for k_ in range(p.npreds)],
                 [p.aggs[i] for i in range(p.naggs)], compacts)
    k.launch(grid, v, NL.stream_ptr(), GA * 32 if p.group_col >= 0 else 0)
    return _final(parts, grid, GA, rstart.device)


# ------------------------------------------------------------------------------------------------
# Shape cache
# ------------------------------------------------------------------------------------------------
_KERNELS: Dict[tuple, Kernel] = {}


def kernel_for(shape: tuple, make) -> Kernel:
    k = _KERNELS.get(shape)
    if k is None:
        k = make()
        _KERNELS[shape] = k
    return k


# ------------------------------------------------------------------------------------------------
# Entry points (same outputs as ops.kernels.scan_agg / join_agg)
# ------------------------------------------------------------------------------------------------
class _NullTensor:
    """Stand-in for the partials of a hash-mode launch (their kernel arguments are unused)."""

    @staticmethod
    def data_ptr() -> int:
        return 0


_NULLT = _NullTensor()


def _partials(grid: int, GA: int, dev):
    import torch
    return (torch.empty(grid * GA, dtype=torch.float64, device=dev),
            torch.empty(grid * GA, dtype=torch.int64, device=dev),
            torch.empty(grid * GA, dtype=torch.float64, device=dev),
            torch.empty(grid * GA, dtype=torch.float64, device=dev))


def _final(parts, grid: int, GA: int, dev):
    import torch
    from ..ops import kernels as K
    out = K.agg_outputs(GA, dev)
    NL.check(NL.lib().hs_agg_final(NL.ptr(parts[0]), NL.ptr(parts[1]), NL.ptr(parts[2]),
                                   NL.ptr(parts[3]), grid, GA, NL.ptr(out[0]), NL.ptr(out[1]),
                                   NL.ptr(out[2]), NL.ptr(out[3]), NL.stream_ptr()),
             "hs_agg_final")
    return out


def scan_vec(p: NL.ScanParams, compacts=None, nrows: int = 0) -> int:
    """Rows per thread of the vectorized scan kernel for this query (0 = strided kernel): the
    predicate columns must have 16-byte aligned bases."""
    if SCAN_VEC <= 0 or nrows <= 0:
        return 0
    ptrs = []
    for s in _pred_slots([(k, p.preds[k]) for k in range(p.npreds)]):
        c = (compacts or {}).get(s)
        ptrs.append(c.codes.data_ptr() if c else p.cols[s].data)
        ptrs.append(p.cols[s].valid)
    return SCAN_VEC if _vec_aligned_ptrs(ptrs) else 0


def scan_agg(p: NL.ScanParams, rstart, rlen, tile_prefix=None, compacts=None, nrows: int = 0,
             hk=None, htab=None):
    """``tile_prefix`` must use this kernel's tile (BLOCK * SCAN_ITEMS); None computes it.
    ``compacts``: slot -> ``encoding.Compact`` read instead of the full-width column.
    ``nrows``: rows of the scanned table (enables the vectorized kernel)."""
    from ..ops import kernels as K
    vec = scan_vec(p, compacts, nrows)
    if vec:
        tile_prefix = K.ranges_to_tiles(rlen + (rstart & (vec - 1)), BLOCK * vec)
    elif tile_prefix is None or BLOCK * SCAN_ITEMS != NL.lib().hs_scan_tile_rows():
        tile_prefix = K.ranges_to_tiles(rlen, BLOCK * SCAN_ITEMS)
    grid = SCAN_GRID or NL.lib().hs_scan_grid()
    GA = p.naggs * (p.num_groups if p.group_col >= 0 else 1)
    k = kernel_for(scan_agg_shape(p, compacts, vec, hk), lambda: gen_scan_agg(p, compacts, vec, hk))
    if hk is not None:
        v = scan_agg_values(p, rstart, rlen, tile_prefix, (_NULLT,) * 4, compacts)
        v["nrows"] = nrows
        v.update(htab.kernel_values())
        v.update(hk.values())
        k.launch(grid, v, NL.stream_ptr(), 0)
        return None
    parts = _partials(grid, GA, rstart.device)
    v = scan_agg_values(p, rstart, rlen, tile_prefix, parts, compacts)
    v["nrows"] = nrows
    k.launch(grid, v, NL.stream_ptr(), GA * 32 if p.group_col >= 0 else 0)
    return _final(parts, grid, GA, rstart.device)


def join_agg(p: NL.JoinParams, rstart, rlen, rbucket, roff, max_tiles: int, compacts=None,
             cache_spans: bool = False):
    """``max_tiles`` = ``ops.kernels.join_max_tiles`` (AOT tile); rescaled to this kernel's tile.
    ``cache_spans``: the row ranges are the left table's cached full ranges, so the tile span
    records (a function of the two key columns and the layouts only, not of the query's
    literals) are reused across queries instead of re-searched."""
    import torch
    from ..ops import kernels as K
    L = NL.lib()
    grid = JOIN_GRID or L.hs_scan_grid()
    GA = p.naggs * (p.num_groups if p.group_col >= 0 else 1)
    dev = rstart.device
    tile = JOIN_BLOCK * JOIN_ITEMS
    tp, spans = _jit_join._join_spans(p, rstart, rlen, rbucket, roff, max_tiles, tile, cache_spans)
    k = kernel_for(join_agg_shape(p, compacts), lambda: gen_join_agg(p, compacts))
    parts = _partials(grid, GA, dev)
    k.launch(grid, _jit_join.join_agg_values(p, tp, spans, parts, compacts), NL.stream_ptr(),
             GA * 32 if p.group_col >= 0 else 0)
    return _final(parts, grid, GA, dev)


# the hash-mode / run top-K emitters (imported last: jit_hash reads this module's helpers)
from . import jit_hash as JH  # noqa: E402

# the join generators (imported last: jit_join reads this module's helpers and tunables);
# their names stay importable from here
from . import jit_join as _jit_join  # noqa: E402
for _n in _jit_join.__all__:
    globals()[_n] = getattr(_jit_join, _n)
