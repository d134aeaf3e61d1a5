
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
  const u64* HIT;
  unsigned* tags;
  long long NRUNS;
  const int* S8;
  const short* S9;
  long long B8;
  long long B9;
  long long CL4;
  long long CH4;
};
extern "C" __global__ __launch_bounds__(256) void hs_jit_run_tags2(Args a) {
  const int lane = (int)(threadIdx.x & 63);
  const i64 G = (a.NRUNS + 63) >> 6;
  const i64 nwv = (i64)gridDim.x * 4;
  const i64 wv = (i64)blockIdx.x * 4 + (i64)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const i64 per = (G + nwv - 1) / nwv;
  const i64 gbeg = wv * per;
  const i64 gend = G < gbeg + per ? G : gbeg + per;
  for (i64 gi = gbeg; gi < gend; gi += 4) {
    const bool in0 = gi + 0 < gend;
    const int r0 = in0 ? (int)(((gi + 0) << 6) + lane) : lane;
    const u64 hb0 = a.HIT[in0 ? gi + 0 : 0];
    const int w8_g0 = a.S8[r0];
    const short w9_g0 = a.S9[r0];
    const bool in1 = gi + 1 < gend;
    const int r1 = in1 ? (int)(((gi + 1) << 6) + lane) : lane;
    const u64 hb1 = a.HIT[in1 ? gi + 1 : 0];
    const int w8_g1 = a.S8[r1];
    const short w9_g1 = a.S9[r1];
    const bool in2 = gi + 2 < gend;
    const int r2 = in2 ? (int)(((gi + 2) << 6) + lane) : lane;
    const u64 hb2 = a.HIT[in2 ? gi + 2 : 0];
    const int w8_g2 = a.S8[r2];
    const short w9_g2 = a.S9[r2];
    const bool in3 = gi + 3 < gend;
    const int r3 = in3 ? (int)(((gi + 3) << 6) + lane) : lane;
    const u64 hb3 = a.HIT[in3 ? gi + 3 : 0];
    const int w8_g3 = a.S8[r3];
    const short w9_g3 = a.S9[r3];
    const bool hit0 = in0 && ((hb0 >> lane) & 1ull);
    const int r8_g0 = (int)w8_g0;
    const long long x8_g0 = (long long)(a.B8 + (i64)w8_g0);
    const int r9_g0 = (int)w9_g0;
    const int x9_g0 = (int)(a.B9 + (i64)w9_g0);
    const bool hit1 = in1 && ((hb1 >> lane) & 1ull);
    const int r8_g1 = (int)w8_g1;
    const long long x8_g1 = (long long)(a.B8 + (i64)w8_g1);
    const int r9_g1 = (int)w9_g1;
    const int x9_g1 = (int)(a.B9 + (i64)w9_g1);
    const bool hit2 = in2 && ((hb2 >> lane) & 1ull);
    const int r8_g2 = (int)w8_g2;
    const long long x8_g2 = (long long)(a.B8 + (i64)w8_g2);
    const int r9_g2 = (int)w9_g2;
    const int x9_g2 = (int)(a.B9 + (i64)w9_g2);
    const bool hit3 = in3 && ((hb3 >> lane) & 1ull);
    const int r8_g3 = (int)w8_g3;
    const long long x8_g3 = (long long)(a.B8 + (i64)w8_g3);
    const int r9_g3 = (int)w9_g3;
    const int x9_g3 = (int)(a.B9 + (i64)w9_g3);
    const unsigned tg0 = (hit0 && ((true)) && ((true)) && ((true && (r9_g0 >= (int)a.CL4 && r9_g0 <= (int)a.CH4)))) ? 1u : 0u;
    { const u64 bal_ = __ballot(tg0 != 0u);
      if (in0 && lane < 2) a.tags[((gi + 0) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
    const unsigned tg1 = (hit1 && ((true)) && ((true)) && ((true && (r9_g1 >= (int)a.CL4 && r9_g1 <= (int)a.CH4)))) ? 1u : 0u;
    { const u64 bal_ = __ballot(tg1 != 0u);
      if (in1 && lane < 2) a.tags[((gi + 1) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
    const unsigned tg2 = (hit2 && ((true)) && ((true)) && ((true && (r9_g2 >= (int)a.CL4 && r9_g2 <= (int)a.CH4)))) ? 1u : 0u;
    { const u64 bal_ = __ballot(tg2 != 0u);
      if (in2 && lane < 2) a.tags[((gi + 2) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
    const unsigned tg3 = (hit3 && ((true)) && ((true)) && ((true && (r9_g3 >= (int)a.CL4 && r9_g3 <= (int)a.CH4)))) ? 1u : 0u;
    { const u64 bal_ = __ballot(tg3 != 0u);
      if (in3 && lane < 2) a.tags[((gi + 3) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
  }
}
