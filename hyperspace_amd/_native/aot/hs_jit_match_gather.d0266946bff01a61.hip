
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
struct Args {
  const int* MATCH;
  long long N;
  int* S8;
  const int* c8;
  short* S9;
  const short* c9;
};
extern "C" __global__ __launch_bounds__(256) void hs_jit_match_gather(Args a) {
  for (i64 i = (i64)blockIdx.x * 256 + threadIdx.x; i < a.N; i += (i64)gridDim.x * 256) {
    const int m_ = a.MATCH[i]; const int j_ = m_ >= 0 ? m_ : 0;
    a.S8[i] = a.c8[j_];
    a.S9[i] = a.c9[j_];
  }
}
