
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
  const int* RK0;
  const long long* RNG;
  unsigned* tags;
  long long NRG;
  long long NRUNS;
  long long KLO;
  long long KSP;
  long long KOF;
  const int* c8;
  long long B8;
  const int* c9;
  long long B9;
  const short* c10;
  long long B10;
  long long CL4;
  long long CH4;
  const unsigned long long* S6;
  long long N6;
  long long L6;
};
extern "C" __global__ __launch_bounds__(256) void hs_jit_run_tags2(Args a) {
  auto IMG = [&](int row_) -> unsigned { return (false ? 0u : ({ const i64 __v_ = (i64)((long long)(a.B8 + (i64)a.c8[row_])); const i64 d_ = __v_ - a.KLO; (d_ < 0) ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); })); };
  auto IMGF = [&](int row_) -> unsigned { return (false ? 0u : ({ const i64 __v_ = (i64)((long long)(a.B8 + (i64)a.c8[row_])); const i64 d_ = __v_ - a.KLO; (d_ < 0) ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); })); };
  const int lane = (int)(threadIdx.x & 63);
  const i64 G = (a.NRUNS + 63) >> 6;
  const i64 nwv = (i64)gridDim.x * 4;
  const i64 wv = (i64)blockIdx.x * 4 + (i64)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const i64 per = (G + nwv - 1) / nwv;
  const i64 gbeg = wv * per;
  const i64 gend = G < gbeg + per ? G : gbeg + per;
  if (gbeg >= gend || a.NRG <= 0) return;
  const i64* RG = a.RNG;
  int rg = 0;
  { int lo = 0, hi = (int)a.NRG; const i64 r0 = gbeg << 6;
    while (hi - lo > 1) { const int m = (lo + hi) >> 1; if (RG[4 * m] <= r0) lo = m; else hi = m; }
    rg = lo; }
  int lr0 = (int)RG[4 * rg], lr1 = (int)RG[4 * rg + 1], s0 = (int)RG[4 * rg + 2], s1 = (int)RG[4 * rg + 3];
  i64 nxt0 = rg + 1 < a.NRG ? RG[4 * (rg + 1)] : 0x7fffffffffffffffll;
  int gbase = -1;   // right row of the next group's first run (-1: range-relative)
  for (i64 gi = gbeg; gi < gend; gi += 4) {
    while (nxt0 <= (gi << 6)) {
      ++rg; lr0 = (int)RG[4 * rg]; lr1 = (int)RG[4 * rg + 1]; s0 = (int)RG[4 * rg + 2];
      s1 = (int)RG[4 * rg + 3]; gbase = -1;
      nxt0 = rg + 1 < a.NRG ? RG[4 * (rg + 1)] : 0x7fffffffffffffffll; }
    if (((gi + 4) << 6) <= nxt0) {
      const int r0 = (int)(((gi + 0) << 6) + lane);
      const bool in0 = gi + 0 < gend;
      const int l0_0 = lr0, l1_0 = lr1, a0_0 = s0, a1_0 = s1; const bool own0 = true;
      const bool act0 = in0 && r0 < a.NRUNS && r0 >= l0_0 && r0 < l1_0 && a1_0 > a0_0;
      int j0 = (own0 && gbase >= 0) ? gbase + 0 + lane : a0_0 + (r0 - l0_0);
      j0 = act0 ? (j0 < a0_0 ? a0_0 : (j0 >= a1_0 ? a1_0 - 1 : j0)) : 0;
      const unsigned key0 = (unsigned)a.RK0[act0 ? r0 : 0] + (unsigned)a.KOF;
      const unsigned k0 = IMGF(j0);
      const int w9_g0 = a.c9[j0];
      const int r9_g0 = (int)w9_g0;
      const long long x9_g0 = (long long)(a.B9 + (i64)w9_g0);
      const short w10_g0 = a.c10[j0];
      const int r10_g0 = (int)w10_g0;
      const int x10_g0 = (int)(a.B10 + (i64)w10_g0);
      const int w8_g0 = a.c8[j0];
      const int r8_g0 = (int)w8_g0;
      const long long x8_g0 = (long long)(a.B8 + (i64)w8_g0);
      const int r1 = (int)(((gi + 1) << 6) + lane);
      const bool in1 = gi + 1 < gend;
      const int l0_1 = lr0, l1_1 = lr1, a0_1 = s0, a1_1 = s1; const bool own1 = true;
      const bool act1 = in1 && r1 < a.NRUNS && r1 >= l0_1 && r1 < l1_1 && a1_1 > a0_1;
      int j1 = (own1 && gbase >= 0) ? gbase + 64 + lane : a0_1 + (r1 - l0_1);
      j1 = act1 ? (j1 < a0_1 ? a0_1 : (j1 >= a1_1 ? a1_1 - 1 : j1)) : 0;
      const unsigned key1 = (unsigned)a.RK0[act1 ? r1 : 0] + (unsigned)a.KOF;
      const unsigned k1 = IMGF(j1);
      const int w9_g1 = a.c9[j1];
      const int r9_g1 = (int)w9_g1;
      const long long x9_g1 = (long long)(a.B9 + (i64)w9_g1);
      const short w10_g1 = a.c10[j1];
      const int r10_g1 = (int)w10_g1;
      const int x10_g1 = (int)(a.B10 + (i64)w10_g1);
      const int w8_g1 = a.c8[j1];
      const int r8_g1 = (int)w8_g1;
      const long long x8_g1 = (long long)(a.B8 + (i64)w8_g1);
      const int r2 = (int)(((gi + 2) << 6) + lane);
      const bool in2 = gi + 2 < gend;
      const int l0_2 = lr0, l1_2 = lr1, a0_2 = s0, a1_2 = s1; const bool own2 = true;
      const bool act2 = in2 && r2 < a.NRUNS && r2 >= l0_2 && r2 < l1_2 && a1_2 > a0_2;
      int j2 = (own2 && gbase >= 0) ? gbase + 128 + lane : a0_2 + (r2 - l0_2);
      j2 = act2 ? (j2 < a0_2 ? a0_2 : (j2 >= a1_2 ? a1_2 - 1 : j2)) : 0;
      const unsigned key2 = (unsigned)a.RK0[act2 ? r2 : 0] + (unsigned)a.KOF;
      const unsigned k2 = IMGF(j2);
      const int w9_g2 = a.c9[j2];
      const int r9_g2 = (int)w9_g2;
      const long long x9_g2 = (long long)(a.B9 + (i64)w9_g2);
      const short w10_g2 = a.c10[j2];
      const int r10_g2 = (int)w10_g2;
      const int x10_g2 = (int)(a.B10 + (i64)w10_g2);
      const int w8_g2 = a.c8[j2];
      const int r8_g2 = (int)w8_g2;
      const long long x8_g2 = (long long)(a.B8 + (i64)w8_g2);
      const int r3 = (int)(((gi + 3) << 6) + lane);
      const bool in3 = gi + 3 < gend;
      const int l0_3 = lr0, l1_3 = lr1, a0_3 = s0, a1_3 = s1; const bool own3 = true;
      const bool act3 = in3 && r3 < a.NRUNS && r3 >= l0_3 && r3 < l1_3 && a1_3 > a0_3;
      int j3 = (own3 && gbase >= 0) ? gbase + 192 + lane : a0_3 + (r3 - l0_3);
      j3 = act3 ? (j3 < a0_3 ? a0_3 : (j3 >= a1_3 ? a1_3 - 1 : j3)) : 0;
      const unsigned key3 = (unsigned)a.RK0[act3 ? r3 : 0] + (unsigned)a.KOF;
      const unsigned k3 = IMGF(j3);
      const int w9_g3 = a.c9[j3];
      const int r9_g3 = (int)w9_g3;
      const long long x9_g3 = (long long)(a.B9 + (i64)w9_g3);
      const short w10_g3 = a.c10[j3];
      const int r10_g3 = (int)w10_g3;
      const int x10_g3 = (int)(a.B10 + (i64)w10_g3);
      const int w8_g3 = a.c8[j3];
      const int r8_g3 = (int)w8_g3;
      const long long x8_g3 = (long long)(a.B8 + (i64)w8_g3);
      bool hit0 = act0 && k0 == key0;
      int m0 = j0;
      unsigned tg0 = ((hit0) && ((true)) && ((true)) && ((true && (r10_g0 >= (int)a.CL4 && r10_g0 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_g0 - a.L6))) ? 1u : 0u);
      if (act0 && !hit0) {
        const unsigned key_ = key0; int lo_, hi_;
        const unsigned kj_ = IMG(j0);
        if (kj_ == key_) { lo_ = j0; hi_ = j0; }
        else if (kj_ > key_) {
          hi_ = j0; int st_ = 1; lo_ = j0 - 1;
          while (lo_ > a0_0 && IMG(lo_) >= key_) { hi_ = lo_; st_ <<= 1; lo_ = hi_ - st_; }
          if (lo_ < a0_0) lo_ = a0_0;
        } else {
          lo_ = j0 + 1; int st_ = 1; hi_ = j0 + 1;
          while (hi_ < a1_0 && IMG(hi_) < key_) { lo_ = hi_ + 1; st_ <<= 1; hi_ = j0 + st_; }
          if (hi_ > a1_0) hi_ = a1_0;
        }
        while (lo_ < hi_) { const int md_ = (lo_ + hi_) >> 1; if (IMG(md_) < key_) lo_ = md_ + 1; else hi_ = md_; }
        m0 = lo_;
        hit0 = lo_ < a1_0 && IMG(lo_) == key_;
        const int jm0 = hit0 ? lo_ : 0;
        const int w9_h0 = a.c9[jm0];
        const int r9_h0 = (int)w9_h0;
        const long long x9_h0 = (long long)(a.B9 + (i64)w9_h0);
        const short w10_h0 = a.c10[jm0];
        const int r10_h0 = (int)w10_h0;
        const int x10_h0 = (int)(a.B10 + (i64)w10_h0);
        const int w8_h0 = a.c8[jm0];
        const int r8_h0 = (int)w8_h0;
        const long long x8_h0 = (long long)(a.B8 + (i64)w8_h0);
        tg0 = ((hit0) && ((true)) && ((true)) && ((true && (r10_h0 >= (int)a.CL4 && r10_h0 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_h0 - a.L6))) ? 1u : 0u);
      }
      { const u64 bal_ = __ballot(tg0 != 0u);
        if (in0 && lane < 2) a.tags[((gi + 0) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
      bool hit1 = act1 && k1 == key1;
      int m1 = j1;
      unsigned tg1 = ((hit1) && ((true)) && ((true)) && ((true && (r10_g1 >= (int)a.CL4 && r10_g1 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_g1 - a.L6))) ? 1u : 0u);
      if (act1 && !hit1) {
        const unsigned key_ = key1; int lo_, hi_;
        const unsigned kj_ = IMG(j1);
        if (kj_ == key_) { lo_ = j1; hi_ = j1; }
        else if (kj_ > key_) {
          hi_ = j1; int st_ = 1; lo_ = j1 - 1;
          while (lo_ > a0_1 && IMG(lo_) >= key_) { hi_ = lo_; st_ <<= 1; lo_ = hi_ - st_; }
          if (lo_ < a0_1) lo_ = a0_1;
        } else {
          lo_ = j1 + 1; int st_ = 1; hi_ = j1 + 1;
          while (hi_ < a1_1 && IMG(hi_) < key_) { lo_ = hi_ + 1; st_ <<= 1; hi_ = j1 + st_; }
          if (hi_ > a1_1) hi_ = a1_1;
        }
        while (lo_ < hi_) { const int md_ = (lo_ + hi_) >> 1; if (IMG(md_) < key_) lo_ = md_ + 1; else hi_ = md_; }
        m1 = lo_;
        hit1 = lo_ < a1_1 && IMG(lo_) == key_;
        const int jm1 = hit1 ? lo_ : 0;
        const int w9_h1 = a.c9[jm1];
        const int r9_h1 = (int)w9_h1;
        const long long x9_h1 = (long long)(a.B9 + (i64)w9_h1);
        const short w10_h1 = a.c10[jm1];
        const int r10_h1 = (int)w10_h1;
        const int x10_h1 = (int)(a.B10 + (i64)w10_h1);
        const int w8_h1 = a.c8[jm1];
        const int r8_h1 = (int)w8_h1;
        const long long x8_h1 = (long long)(a.B8 + (i64)w8_h1);
        tg1 = ((hit1) && ((true)) && ((true)) && ((true && (r10_h1 >= (int)a.CL4 && r10_h1 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_h1 - a.L6))) ? 1u : 0u);
      }
      { const u64 bal_ = __ballot(tg1 != 0u);
        if (in1 && lane < 2) a.tags[((gi + 1) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
      bool hit2 = act2 && k2 == key2;
      int m2 = j2;
      unsigned tg2 = ((hit2) && ((true)) && ((true)) && ((true && (r10_g2 >= (int)a.CL4 && r10_g2 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_g2 - a.L6))) ? 1u : 0u);
      if (act2 && !hit2) {
        const unsigned key_ = key2; int lo_, hi_;
        const unsigned kj_ = IMG(j2);
        if (kj_ == key_) { lo_ = j2; hi_ = j2; }
        else if (kj_ > key_) {
          hi_ = j2; int st_ = 1; lo_ = j2 - 1;
          while (lo_ > a0_2 && IMG(lo_) >= key_) { hi_ = lo_; st_ <<= 1; lo_ = hi_ - st_; }
          if (lo_ < a0_2) lo_ = a0_2;
        } else {
          lo_ = j2 + 1; int st_ = 1; hi_ = j2 + 1;
          while (hi_ < a1_2 && IMG(hi_) < key_) { lo_ = hi_ + 1; st_ <<= 1; hi_ = j2 + st_; }
          if (hi_ > a1_2) hi_ = a1_2;
        }
        while (lo_ < hi_) { const int md_ = (lo_ + hi_) >> 1; if (IMG(md_) < key_) lo_ = md_ + 1; else hi_ = md_; }
        m2 = lo_;
        hit2 = lo_ < a1_2 && IMG(lo_) == key_;
        const int jm2 = hit2 ? lo_ : 0;
        const int w9_h2 = a.c9[jm2];
        const int r9_h2 = (int)w9_h2;
        const long long x9_h2 = (long long)(a.B9 + (i64)w9_h2);
        const short w10_h2 = a.c10[jm2];
        const int r10_h2 = (int)w10_h2;
        const int x10_h2 = (int)(a.B10 + (i64)w10_h2);
        const int w8_h2 = a.c8[jm2];
        const int r8_h2 = (int)w8_h2;
        const long long x8_h2 = (long long)(a.B8 + (i64)w8_h2);
        tg2 = ((hit2) && ((true)) && ((true)) && ((true && (r10_h2 >= (int)a.CL4 && r10_h2 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_h2 - a.L6))) ? 1u : 0u);
      }
      { const u64 bal_ = __ballot(tg2 != 0u);
        if (in2 && lane < 2) a.tags[((gi + 2) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
      bool hit3 = act3 && k3 == key3;
      int m3 = j3;
      unsigned tg3 = ((hit3) && ((true)) && ((true)) && ((true && (r10_g3 >= (int)a.CL4 && r10_g3 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_g3 - a.L6))) ? 1u : 0u);
      if (act3 && !hit3) {
        const unsigned key_ = key3; int lo_, hi_;
        const unsigned kj_ = IMG(j3);
        if (kj_ == key_) { lo_ = j3; hi_ = j3; }
        else if (kj_ > key_) {
          hi_ = j3; int st_ = 1; lo_ = j3 - 1;
          while (lo_ > a0_3 && IMG(lo_) >= key_) { hi_ = lo_; st_ <<= 1; lo_ = hi_ - st_; }
          if (lo_ < a0_3) lo_ = a0_3;
        } else {
          lo_ = j3 + 1; int st_ = 1; hi_ = j3 + 1;
          while (hi_ < a1_3 && IMG(hi_) < key_) { lo_ = hi_ + 1; st_ <<= 1; hi_ = j3 + st_; }
          if (hi_ > a1_3) hi_ = a1_3;
        }
        while (lo_ < hi_) { const int md_ = (lo_ + hi_) >> 1; if (IMG(md_) < key_) lo_ = md_ + 1; else hi_ = md_; }
        m3 = lo_;
        hit3 = lo_ < a1_3 && IMG(lo_) == key_;
        const int jm3 = hit3 ? lo_ : 0;
        const int w9_h3 = a.c9[jm3];
        const int r9_h3 = (int)w9_h3;
        const long long x9_h3 = (long long)(a.B9 + (i64)w9_h3);
        const short w10_h3 = a.c10[jm3];
        const int r10_h3 = (int)w10_h3;
        const int x10_h3 = (int)(a.B10 + (i64)w10_h3);
        const int w8_h3 = a.c8[jm3];
        const int r8_h3 = (int)w8_h3;
        const long long x8_h3 = (long long)(a.B8 + (i64)w8_h3);
        tg3 = ((hit3) && ((true)) && ((true)) && ((true && (r10_h3 >= (int)a.CL4 && r10_h3 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_h3 - a.L6))) ? 1u : 0u);
      }
      { const u64 bal_ = __ballot(tg3 != 0u);
        if (in3 && lane < 2) a.tags[((gi + 3) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
      { const int nx_ = __shfl((hit3 && own3) ? m3 + 1 : (int)-1, 63, 64);
        gbase = nx_; }
    } else {   // a range starts inside this iteration's groups
      const int r0 = (int)(((gi + 0) << 6) + lane);
      const bool in0 = gi + 0 < gend;
      int l0_0 = lr0, l1_0 = lr1, a0_0 = s0, a1_0 = s1; bool own0 = true;
      if (r0 >= nxt0) { own0 = false; int q_ = rg;
        while (q_ + 1 < (int)a.NRG && RG[4 * (q_ + 1)] <= r0) ++q_;
        l0_0 = (int)RG[4 * q_]; l1_0 = (int)RG[4 * q_ + 1]; a0_0 = (int)RG[4 * q_ + 2]; a1_0 = (int)RG[4 * q_ + 3]; }
      const bool act0 = in0 && r0 < a.NRUNS && r0 >= l0_0 && r0 < l1_0 && a1_0 > a0_0;
      int j0 = (own0 && gbase >= 0) ? gbase + 0 + lane : a0_0 + (r0 - l0_0);
      j0 = act0 ? (j0 < a0_0 ? a0_0 : (j0 >= a1_0 ? a1_0 - 1 : j0)) : 0;
      const unsigned key0 = (unsigned)a.RK0[act0 ? r0 : 0] + (unsigned)a.KOF;
      const unsigned k0 = IMGF(j0);
      const int w9_g0 = a.c9[j0];
      const int r9_g0 = (int)w9_g0;
      const long long x9_g0 = (long long)(a.B9 + (i64)w9_g0);
      const short w10_g0 = a.c10[j0];
      const int r10_g0 = (int)w10_g0;
      const int x10_g0 = (int)(a.B10 + (i64)w10_g0);
      const int w8_g0 = a.c8[j0];
      const int r8_g0 = (int)w8_g0;
      const long long x8_g0 = (long long)(a.B8 + (i64)w8_g0);
      const int r1 = (int)(((gi + 1) << 6) + lane);
      const bool in1 = gi + 1 < gend;
      int l0_1 = lr0, l1_1 = lr1, a0_1 = s0, a1_1 = s1; bool own1 = true;
      if (r1 >= nxt0) { own1 = false; int q_ = rg;
        while (q_ + 1 < (int)a.NRG && RG[4 * (q_ + 1)] <= r1) ++q_;
        l0_1 = (int)RG[4 * q_]; l1_1 = (int)RG[4 * q_ + 1]; a0_1 = (int)RG[4 * q_ + 2]; a1_1 = (int)RG[4 * q_ + 3]; }
      const bool act1 = in1 && r1 < a.NRUNS && r1 >= l0_1 && r1 < l1_1 && a1_1 > a0_1;
      int j1 = (own1 && gbase >= 0) ? gbase + 64 + lane : a0_1 + (r1 - l0_1);
      j1 = act1 ? (j1 < a0_1 ? a0_1 : (j1 >= a1_1 ? a1_1 - 1 : j1)) : 0;
      const unsigned key1 = (unsigned)a.RK0[act1 ? r1 : 0] + (unsigned)a.KOF;
      const unsigned k1 = IMGF(j1);
      const int w9_g1 = a.c9[j1];
      const int r9_g1 = (int)w9_g1;
      const long long x9_g1 = (long long)(a.B9 + (i64)w9_g1);
      const short w10_g1 = a.c10[j1];
      const int r10_g1 = (int)w10_g1;
      const int x10_g1 = (int)(a.B10 + (i64)w10_g1);
      const int w8_g1 = a.c8[j1];
      const int r8_g1 = (int)w8_g1;
      const long long x8_g1 = (long long)(a.B8 + (i64)w8_g1);
      const int r2 = (int)(((gi + 2) << 6) + lane);
      const bool in2 = gi + 2 < gend;
      int l0_2 = lr0, l1_2 = lr1, a0_2 = s0, a1_2 = s1; bool own2 = true;
      if (r2 >= nxt0) { own2 = false; int q_ = rg;
        while (q_ + 1 < (int)a.NRG && RG[4 * (q_ + 1)] <= r2) ++q_;
        l0_2 = (int)RG[4 * q_]; l1_2 = (int)RG[4 * q_ + 1]; a0_2 = (int)RG[4 * q_ + 2]; a1_2 = (int)RG[4 * q_ + 3]; }
      const bool act2 = in2 && r2 < a.NRUNS && r2 >= l0_2 && r2 < l1_2 && a1_2 > a0_2;
      int j2 = (own2 && gbase >= 0) ? gbase + 128 + lane : a0_2 + (r2 - l0_2);
      j2 = act2 ? (j2 < a0_2 ? a0_2 : (j2 >= a1_2 ? a1_2 - 1 : j2)) : 0;
      const unsigned key2 = (unsigned)a.RK0[act2 ? r2 : 0] + (unsigned)a.KOF;
      const unsigned k2 = IMGF(j2);
      const int w9_g2 = a.c9[j2];
      const int r9_g2 = (int)w9_g2;
      const long long x9_g2 = (long long)(a.B9 + (i64)w9_g2);
      const short w10_g2 = a.c10[j2];
      const int r10_g2 = (int)w10_g2;
      const int x10_g2 = (int)(a.B10 + (i64)w10_g2);
      const int w8_g2 = a.c8[j2];
      const int r8_g2 = (int)w8_g2;
      const long long x8_g2 = (long long)(a.B8 + (i64)w8_g2);
      const int r3 = (int)(((gi + 3) << 6) + lane);
      const bool in3 = gi + 3 < gend;
      int l0_3 = lr0, l1_3 = lr1, a0_3 = s0, a1_3 = s1; bool own3 = true;
      if (r3 >= nxt0) { own3 = false; int q_ = rg;
        while (q_ + 1 < (int)a.NRG && RG[4 * (q_ + 1)] <= r3) ++q_;
        l0_3 = (int)RG[4 * q_]; l1_3 = (int)RG[4 * q_ + 1]; a0_3 = (int)RG[4 * q_ + 2]; a1_3 = (int)RG[4 * q_ + 3]; }
      const bool act3 = in3 && r3 < a.NRUNS && r3 >= l0_3 && r3 < l1_3 && a1_3 > a0_3;
      int j3 = (own3 && gbase >= 0) ? gbase + 192 + lane : a0_3 + (r3 - l0_3);
      j3 = act3 ? (j3 < a0_3 ? a0_3 : (j3 >= a1_3 ? a1_3 - 1 : j3)) : 0;
      const unsigned key3 = (unsigned)a.RK0[act3 ? r3 : 0] + (unsigned)a.KOF;
      const unsigned k3 = IMGF(j3);
      const int w9_g3 = a.c9[j3];
      const int r9_g3 = (int)w9_g3;
      const long long x9_g3 = (long long)(a.B9 + (i64)w9_g3);
      const short w10_g3 = a.c10[j3];
      const int r10_g3 = (int)w10_g3;
      const int x10_g3 = (int)(a.B10 + (i64)w10_g3);
      const int w8_g3 = a.c8[j3];
      const int r8_g3 = (int)w8_g3;
      const long long x8_g3 = (long long)(a.B8 + (i64)w8_g3);
      bool hit0 = act0 && k0 == key0;
      int m0 = j0;
      unsigned tg0 = ((hit0) && ((true)) && ((true)) && ((true && (r10_g0 >= (int)a.CL4 && r10_g0 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_g0 - a.L6))) ? 1u : 0u);
      if (act0 && !hit0) {
        const unsigned key_ = key0; int lo_, hi_;
        const unsigned kj_ = IMG(j0);
        if (kj_ == key_) { lo_ = j0; hi_ = j0; }
        else if (kj_ > key_) {
          hi_ = j0; int st_ = 1; lo_ = j0 - 1;
          while (lo_ > a0_0 && IMG(lo_) >= key_) { hi_ = lo_; st_ <<= 1; lo_ = hi_ - st_; }
          if (lo_ < a0_0) lo_ = a0_0;
        } else {
          lo_ = j0 + 1; int st_ = 1; hi_ = j0 + 1;
          while (hi_ < a1_0 && IMG(hi_) < key_) { lo_ = hi_ + 1; st_ <<= 1; hi_ = j0 + st_; }
          if (hi_ > a1_0) hi_ = a1_0;
        }
        while (lo_ < hi_) { const int md_ = (lo_ + hi_) >> 1; if (IMG(md_) < key_) lo_ = md_ + 1; else hi_ = md_; }
        m0 = lo_;
        hit0 = lo_ < a1_0 && IMG(lo_) == key_;
        const int jm0 = hit0 ? lo_ : 0;
        const int w9_h0 = a.c9[jm0];
        const int r9_h0 = (int)w9_h0;
        const long long x9_h0 = (long long)(a.B9 + (i64)w9_h0);
        const short w10_h0 = a.c10[jm0];
        const int r10_h0 = (int)w10_h0;
        const int x10_h0 = (int)(a.B10 + (i64)w10_h0);
        const int w8_h0 = a.c8[jm0];
        const int r8_h0 = (int)w8_h0;
        const long long x8_h0 = (long long)(a.B8 + (i64)w8_h0);
        tg0 = ((hit0) && ((true)) && ((true)) && ((true && (r10_h0 >= (int)a.CL4 && r10_h0 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_h0 - a.L6))) ? 1u : 0u);
      }
      { const u64 bal_ = __ballot(tg0 != 0u);
        if (in0 && lane < 2) a.tags[((gi + 0) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
      bool hit1 = act1 && k1 == key1;
      int m1 = j1;
      unsigned tg1 = ((hit1) && ((true)) && ((true)) && ((true && (r10_g1 >= (int)a.CL4 && r10_g1 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_g1 - a.L6))) ? 1u : 0u);
      if (act1 && !hit1) {
        const unsigned key_ = key1; int lo_, hi_;
        const unsigned kj_ = IMG(j1);
        if (kj_ == key_) { lo_ = j1; hi_ = j1; }
        else if (kj_ > key_) {
          hi_ = j1; int st_ = 1; lo_ = j1 - 1;
          while (lo_ > a0_1 && IMG(lo_) >= key_) { hi_ = lo_; st_ <<= 1; lo_ = hi_ - st_; }
          if (lo_ < a0_1) lo_ = a0_1;
        } else {
          lo_ = j1 + 1; int st_ = 1; hi_ = j1 + 1;
          while (hi_ < a1_1 && IMG(hi_) < key_) { lo_ = hi_ + 1; st_ <<= 1; hi_ = j1 + st_; }
          if (hi_ > a1_1) hi_ = a1_1;
        }
        while (lo_ < hi_) { const int md_ = (lo_ + hi_) >> 1; if (IMG(md_) < key_) lo_ = md_ + 1; else hi_ = md_; }
        m1 = lo_;
        hit1 = lo_ < a1_1 && IMG(lo_) == key_;
        const int jm1 = hit1 ? lo_ : 0;
        const int w9_h1 = a.c9[jm1];
        const int r9_h1 = (int)w9_h1;
        const long long x9_h1 = (long long)(a.B9 + (i64)w9_h1);
        const short w10_h1 = a.c10[jm1];
        const int r10_h1 = (int)w10_h1;
        const int x10_h1 = (int)(a.B10 + (i64)w10_h1);
        const int w8_h1 = a.c8[jm1];
        const int r8_h1 = (int)w8_h1;
        const long long x8_h1 = (long long)(a.B8 + (i64)w8_h1);
        tg1 = ((hit1) && ((true)) && ((true)) && ((true && (r10_h1 >= (int)a.CL4 && r10_h1 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_h1 - a.L6))) ? 1u : 0u);
      }
      { const u64 bal_ = __ballot(tg1 != 0u);
        if (in1 && lane < 2) a.tags[((gi + 1) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
      bool hit2 = act2 && k2 == key2;
      int m2 = j2;
      unsigned tg2 = ((hit2) && ((true)) && ((true)) && ((true && (r10_g2 >= (int)a.CL4 && r10_g2 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_g2 - a.L6))) ? 1u : 0u);
      if (act2 && !hit2) {
        const unsigned key_ = key2; int lo_, hi_;
        const unsigned kj_ = IMG(j2);
        if (kj_ == key_) { lo_ = j2; hi_ = j2; }
        else if (kj_ > key_) {
          hi_ = j2; int st_ = 1; lo_ = j2 - 1;
          while (lo_ > a0_2 && IMG(lo_) >= key_) { hi_ = lo_; st_ <<= 1; lo_ = hi_ - st_; }
          if (lo_ < a0_2) lo_ = a0_2;
        } else {
          lo_ = j2 + 1; int st_ = 1; hi_ = j2 + 1;
          while (hi_ < a1_2 && IMG(hi_) < key_) { lo_ = hi_ + 1; st_ <<= 1; hi_ = j2 + st_; }
          if (hi_ > a1_2) hi_ = a1_2;
        }
        while (lo_ < hi_) { const int md_ = (lo_ + hi_) >> 1; if (IMG(md_) < key_) lo_ = md_ + 1; else hi_ = md_; }
        m2 = lo_;
        hit2 = lo_ < a1_2 && IMG(lo_) == key_;
        const int jm2 = hit2 ? lo_ : 0;
        const int w9_h2 = a.c9[jm2];
        const int r9_h2 = (int)w9_h2;
        const long long x9_h2 = (long long)(a.B9 + (i64)w9_h2);
        const short w10_h2 = a.c10[jm2];
        const int r10_h2 = (int)w10_h2;
        const int x10_h2 = (int)(a.B10 + (i64)w10_h2);
        const int w8_h2 = a.c8[jm2];
        const int r8_h2 = (int)w8_h2;
        const long long x8_h2 = (long long)(a.B8 + (i64)w8_h2);
        tg2 = ((hit2) && ((true)) && ((true)) && ((true && (r10_h2 >= (int)a.CL4 && r10_h2 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_h2 - a.L6))) ? 1u : 0u);
      }
      { const u64 bal_ = __ballot(tg2 != 0u);
        if (in2 && lane < 2) a.tags[((gi + 2) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
      bool hit3 = act3 && k3 == key3;
      int m3 = j3;
      unsigned tg3 = ((hit3) && ((true)) && ((true)) && ((true && (r10_g3 >= (int)a.CL4 && r10_g3 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_g3 - a.L6))) ? 1u : 0u);
      if (act3 && !hit3) {
        const unsigned key_ = key3; int lo_, hi_;
        const unsigned kj_ = IMG(j3);
        if (kj_ == key_) { lo_ = j3; hi_ = j3; }
        else if (kj_ > key_) {
          hi_ = j3; int st_ = 1; lo_ = j3 - 1;
          while (lo_ > a0_3 && IMG(lo_) >= key_) { hi_ = lo_; st_ <<= 1; lo_ = hi_ - st_; }
          if (lo_ < a0_3) lo_ = a0_3;
        } else {
          lo_ = j3 + 1; int st_ = 1; hi_ = j3 + 1;
          while (hi_ < a1_3 && IMG(hi_) < key_) { lo_ = hi_ + 1; st_ <<= 1; hi_ = j3 + st_; }
          if (hi_ > a1_3) hi_ = a1_3;
        }
        while (lo_ < hi_) { const int md_ = (lo_ + hi_) >> 1; if (IMG(md_) < key_) lo_ = md_ + 1; else hi_ = md_; }
        m3 = lo_;
        hit3 = lo_ < a1_3 && IMG(lo_) == key_;
        const int jm3 = hit3 ? lo_ : 0;
        const int w9_h3 = a.c9[jm3];
        const int r9_h3 = (int)w9_h3;
        const long long x9_h3 = (long long)(a.B9 + (i64)w9_h3);
        const short w10_h3 = a.c10[jm3];
        const int r10_h3 = (int)w10_h3;
        const int x10_h3 = (int)(a.B10 + (i64)w10_h3);
        const int w8_h3 = a.c8[jm3];
        const int r8_h3 = (int)w8_h3;
        const long long x8_h3 = (long long)(a.B8 + (i64)w8_h3);
        tg3 = ((hit3) && ((true)) && ((true)) && ((true && (r10_h3 >= (int)a.CL4 && r10_h3 <= (int)a.CH4))) && ((true)) && ((true && bit_test(a.S6, a.N6 * 64, (i64)x9_h3 - a.L6))) ? 1u : 0u);
      }
      { const u64 bal_ = __ballot(tg3 != 0u);
        if (in3 && lane < 2) a.tags[((gi + 3) << 1) + lane] = (unsigned)(bal_ >> (32 * lane)); }
      { const int nx_ = __shfl((hit3 && own3) ? m3 + 1 : (int)-1, 63, 64);
        gbase = nx_; }
    }
  }
}
