// Key-domain bitmap of a join's build side (exec/gpu.py GpuBackend._semi_join_agg).
//
// An inner equi-join whose aggregate reads only the probe side, and whose build side has unique
// keys, is a semi-join: each probe row matches at most one build row and contributes its own
// columns once.  The build keys (the materialized output of another join, a filtered dimension)
// are set as bits of a bitmap over their [lo, hi] domain - 1 bit per key value, 75 MB for
// TPC-H SF100 orderkeys, which stays in the 256 MB MALL - and the probe side runs as a plain
// index scan with one more predicate, bit_test(key - lo), fused into the generated scan kernel
// (PK_BITMAP).  This replaces the reference's Exchange + Sort of both sides before a
// SortMergeJoin (a join whose side is itself a join is not index-rewritable:
// JoinIndexRule.scala:100-105,149-150).
//
// hs_key_bitmap sets the bits with 64-bit atomic ORs and raises flags[0] when a bit was already
// set (a duplicate build key: the caller falls back to the general join).  hs_bitmap_popcount
// counts set bits (cross-rank uniqueness check after the ranks' bitmaps are OR-ed together).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hs_common.h"

namespace {

__global__ __launch_bounds__(256) void hs_key_bitmap_kernel(ColDesc c, int64_t n, int64_t base,
                                                            int64_t nbits,
                                                            unsigned long long* __restrict__ words,
                                                            int* __restrict__ flags) {
  int dup = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    if (!col_valid(c, i)) continue;
    const int64_t v = load_i64(c, i) - base;
    if (v < 0 || v >= nbits) {
      dup |= 2;   // outside the domain the caller computed: never expected
      continue;
    }
    const unsigned long long bit = 1ull << (v & 63);
    const unsigned long long old = atomicOr(&words[v >> 6], bit);
    dup |= (old & bit) ? 1 : 0;
  }
  if (__any(dup & 1) && (threadIdx.x & 63) == 0) atomicOr(&flags[0], 1);
  if (__any(dup & 2) && (threadIdx.x & 63) == 0) atomicOr(&flags[0], 2);
}

__global__ __launch_bounds__(256) void hs_bitmap_popcount_kernel(
    const unsigned long long* __restrict__ words, int64_t nwords,
    unsigned long long* __restrict__ out) {
  unsigned long long s = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nwords;
       i += (int64_t)gridDim.x * blockDim.x)
    s += __popcll(words[i]);
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

unsigned grid_for(int64_t n) {
  const int64_t g = (n + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace

extern "C" {

// words: zeroed, ceil(nbits / 64) entries; flags: one zeroed int (bit 0 duplicate, bit 1 out of
// domain).
int hs_key_bitmap(const ColDesc* c, int64_t n, int64_t base, int64_t nbits,
                  unsigned long long* words, int* flags, void* stream) {
  if (n > 0)
    hipLaunchKernelGGL(hs_key_bitmap_kernel, dim3(grid_for(n)), dim3(256), 0,
                       (hipStream_t)stream, *c, n, base, nbits, words, flags);
  return (int)hipGetLastError();
}

// out: one zeroed uint64.
int hs_bitmap_popcount(const unsigned long long* words, int64_t nwords, unsigned long long* out,
                       void* stream) {
  if (nwords > 0)
    hipLaunchKernelGGL(hs_bitmap_popcount_kernel, dim3(grid_for(nwords)), dim3(256), 0,
                       (hipStream_t)stream, words, nwords, out);
  return (int)hipGetLastError();
}

}  // extern "C"
