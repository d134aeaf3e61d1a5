// Shared device definitions for the hyperspace_amd HIP kernels (gfx950 / MI355X, wave64).
//
// Columns are passed as ColDesc {data, valid, type}: fixed-width little-endian values plus an
// optional byte-per-row validity mask (1 = valid).  String columns reach the device either as
// dictionary codes (int32, dictionary sorted on the host so code order == string order) or, for
// hashing, as (offsets, chars).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HS_WAVE 64
#define HS_MAX_COLS 16
#define HS_MAX_PREDS 16
#define HS_MAX_AGGS 8
#define HS_MAX_TERMS 3

enum HsType : int32_t {
  HS_I8 = 0, HS_I16 = 1, HS_I32 = 2, HS_I64 = 3, HS_F32 = 4, HS_F64 = 5, HS_BOOL = 6,
  HS_U32 = 7, HS_U64 = 8
};

struct ColDesc {
  const void* data;
  const uint8_t* valid;  // nullptr => all valid
  int32_t type;
  int32_t pad;
};

__device__ __forceinline__ bool col_valid(const ColDesc& c, int64_t row) {
  return c.valid == nullptr || c.valid[row] != 0;
}

__device__ __forceinline__ int64_t load_i64(const ColDesc& c, int64_t row) {
  switch (c.type) {
    case HS_I8: return ((const int8_t*)c.data)[row];
    case HS_I16: return ((const int16_t*)c.data)[row];
    case HS_I32: return ((const int32_t*)c.data)[row];
    case HS_I64: return ((const int64_t*)c.data)[row];
    case HS_F32: return (int64_t)((const float*)c.data)[row];
    case HS_F64: return (int64_t)((const double*)c.data)[row];
    case HS_BOOL: return ((const uint8_t*)c.data)[row];
    case HS_U32: return ((const uint32_t*)c.data)[row];
    default: return (int64_t)((const uint64_t*)c.data)[row];
  }
}

__device__ __forceinline__ double load_f64(const ColDesc& c, int64_t row) {
  switch (c.type) {
    case HS_F64: return ((const double*)c.data)[row];
    case HS_F32: return ((const float*)c.data)[row];
    default: return (double)load_i64(c, row);
  }
}

// ---------------------------------------------------------------------------------------------
// Spark Murmur3_x86_32 (seed chaining, hashUnsafeBytes tail semantics).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t hs_rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t hs_mix_k1(uint32_t k1) {
  k1 *= 0xcc9e2d51u;
  k1 = hs_rotl(k1, 15);
  return k1 * 0x1b873593u;
}
__device__ __forceinline__ uint32_t hs_mix_h1(uint32_t h1, uint32_t k1) {
  h1 ^= k1;
  h1 = hs_rotl(h1, 13);
  return h1 * 5u + 0xe6546b64u;
}
__device__ __forceinline__ uint32_t hs_fmix(uint32_t h1, uint32_t len) {
  h1 ^= len;
  h1 ^= h1 >> 16;
  h1 *= 0x85ebca6bu;
  h1 ^= h1 >> 13;
  h1 *= 0xc2b2ae35u;
  h1 ^= h1 >> 16;
  return h1;
}
__device__ __forceinline__ uint32_t hs_hash_int(uint32_t v, uint32_t seed) {
  return hs_fmix(hs_mix_h1(seed, hs_mix_k1(v)), 4);
}
__device__ __forceinline__ uint32_t hs_hash_long(uint64_t v, uint32_t seed) {
  uint32_t h1 = hs_mix_h1(seed, hs_mix_k1((uint32_t)v));
  h1 = hs_mix_h1(h1, hs_mix_k1((uint32_t)(v >> 32)));
  return hs_fmix(h1, 8);
}

// Order-preserving unsigned image of a typed key (ascending).
__device__ __forceinline__ uint64_t hs_sortable(const ColDesc& c, int64_t row) {
  switch (c.type) {
    case HS_I8: return (uint64_t)(uint8_t)(((const int8_t*)c.data)[row] ^ (int8_t)0x80);
    case HS_I16: return (uint64_t)(uint16_t)(((const int16_t*)c.data)[row] ^ (int16_t)0x8000);
    case HS_I32: return (uint64_t)((uint32_t)((const int32_t*)c.data)[row] ^ 0x80000000u);
    case HS_I64: return (uint64_t)((const int64_t*)c.data)[row] ^ 0x8000000000000000ull;
    case HS_F32: {
      uint32_t b = ((const uint32_t*)c.data)[row];
      return (uint64_t)((b & 0x80000000u) ? ~b : (b | 0x80000000u));
    }
    case HS_F64: {
      uint64_t b = ((const uint64_t*)c.data)[row];
      return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
    }
    case HS_BOOL: return ((const uint8_t*)c.data)[row];
    case HS_U32: return ((const uint32_t*)c.data)[row];
    default: return ((const uint64_t*)c.data)[row];
  }
}

__device__ __forceinline__ uint64_t hs_lanemask_lt() {
  const int lane = threadIdx.x & 63;
  return lane == 0 ? 0ull : ((~0ull) >> (64 - lane));
}

template <typename T>
__device__ __forceinline__ T hs_wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

__device__ __forceinline__ double hs_wave_min(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmin(v, __shfl_xor(v, off, 64));
  return v;
}

__device__ __forceinline__ double hs_wave_max(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// XCD-aware remap: spread consecutive logical tiles across the 8 XCDs' L2s is the HW default;
// for tile loops that re-read neighbours (join right segments) keep neighbours on one XCD.
__device__ __forceinline__ int hs_xcd_remap(int bid, int nblocks) {
  const int xcd = bid & 7;
  const int q = nblocks >> 3, r = nblocks & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

#define HS_CHECK(x)                                          \
  do {                                                       \
    hipError_t _e = (x);                                     \
    if (_e != hipSuccess) return (int)_e;                    \
  } while (0)
