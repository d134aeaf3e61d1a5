
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
  const long long* rstart;
  const long long* rlen;
  const long long* tile_prefix;
  const unsigned char* jidx;
  const int* jbase;
  long long R;
  double* psum;
  double* pmin;
  double* pmax;
  long long* pcnt;
  long long nrows;
  const short* c1;
  long long B1;
  long long CL1;
  long long CH1;
  const int* c8;
  long long B8;
  const short* c9;
  long long B9;
  long long CL4;
  long long CH4;
  const int* c2;
  long long B2;
  double R2;
  const signed char* c3;
  long long B3;
  double R3;
  double A0_0;
  double B0_0;
  double A0_1;
  double B0_1;
};
extern "C" __global__ __launch_bounds__(256) void hs_jit_join_index_agg(Args a) {
  typedef unsigned short crow_t; __shared__ crow_t crow_s[4][512]; __shared__ int cj_s[4][512];
  const int cln = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int NA = 3;
  double acc0 = 0.0; unsigned cnt0 = 0u;
  double acc1 = 0.0; unsigned cnt1 = 0u;
  double acc2 = 0.0; unsigned cnt2 = 0u;
  const i64 ntiles = a.tile_prefix[a.R];
  const i64 per = (ntiles + gridDim.x - 1) / gridDim.x;
  const i64 t0 = (i64)blockIdx.x * per;
  const i64 t1 = ntiles < t0 + per ? ntiles : t0 + per;
  int r = 0;
  if (t0 < t1) { int lo = 0, hi = (int)a.R;
    while (hi - lo > 1) { const int m = (lo + hi) >> 1; if (a.tile_prefix[m] <= t0) lo = m; else hi = m; }
    r = lo; }
  i64 rsP = 0, reP = 0, tb0P = 0, g0P = 0; bool fullP = false;
  unsigned char jrvP[8];
  short x1vP[8];
  int jbP = (int)0;
  i64 t = t0;
  if (t < t1) {
    while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= t) ++r;
    { const i64 off_ = (t - a.tile_prefix[r]) * 2048;
      rsP = a.rstart[r]; reP = rsP + a.rlen[r];
      tb0P = (rsP & ~(i64)7) + off_;
      g0P = tb0P + (i64)threadIdx.x * 8; }
    fullP = tb0P + 2048 <= a.nrows;
    if (fullP) {
      vload<unsigned char, 8>(a.jidx, g0P, jrvP);
      vload<short, 8>(a.c1, g0P, x1vP);
      jbP = a.jbase[g0P >> 7];
    }
  }
  for (; t < t1 && fullP; ++t) {
    const i64 rs = rsP, re = reP, tb0 = tb0P, g0 = g0P;
    unsigned char jrv[8]; jrv[0] = jrvP[0]; jrv[1] = jrvP[1]; jrv[2] = jrvP[2]; jrv[3] = jrvP[3]; jrv[4] = jrvP[4]; jrv[5] = jrvP[5]; jrv[6] = jrvP[6]; jrv[7] = jrvP[7];
    short x1v[8]; x1v[0] = x1vP[0]; x1v[1] = x1vP[1]; x1v[2] = x1vP[2]; x1v[3] = x1vP[3]; x1v[4] = x1vP[4]; x1v[5] = x1vP[5]; x1v[6] = x1vP[6]; x1v[7] = x1vP[7];
    const int jb = jbP;
    if (t + 1 < t1) {
      while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= (t + 1)) ++r;
      { const i64 off_ = ((t + 1) - a.tile_prefix[r]) * 2048;
        rsP = a.rstart[r]; reP = rsP + a.rlen[r];
        tb0P = (rsP & ~(i64)7) + off_;
        g0P = tb0P + (i64)threadIdx.x * 8; }
      fullP = tb0P + 2048 <= a.nrows;
      if (fullP) {
        vload<unsigned char, 8>(a.jidx, g0P, jrvP);
        vload<short, 8>(a.c1, g0P, x1vP);
        jbP = a.jbase[g0P >> 7];
      }
    } else fullP = false;
    const i64 dlo_ = rs - g0, dhi_ = re - g0;
    const int alo = dlo_ <= 0 ? 0 : (dlo_ >= 8 ? 8 : (int)dlo_);
    const int ahi = dhi_ <= 0 ? 0 : (dhi_ >= 8 ? 8 : (int)dhi_);
    const bool act0 = 0 >= alo && 0 < ahi;
    const i64 row0 = g0 + 0;
    const bool act1 = 1 >= alo && 1 < ahi;
    const i64 row1 = g0 + 1;
    const bool act2 = 2 >= alo && 2 < ahi;
    const i64 row2 = g0 + 2;
    const bool act3 = 3 >= alo && 3 < ahi;
    const i64 row3 = g0 + 3;
    const bool act4 = 4 >= alo && 4 < ahi;
    const i64 row4 = g0 + 4;
    const bool act5 = 5 >= alo && 5 < ahi;
    const i64 row5 = g0 + 5;
    const bool act6 = 6 >= alo && 6 < ahi;
    const i64 row6 = g0 + 6;
    const bool act7 = 7 >= alo && 7 < ahi;
    const i64 row7 = g0 + 7;
    const int r1_0 = (int)x1v[0];
    const int x1_0 = (int)(a.B1 + (i64)x1v[0]);
    const int r1_1 = (int)x1v[1];
    const int x1_1 = (int)(a.B1 + (i64)x1v[1]);
    const int r1_2 = (int)x1v[2];
    const int x1_2 = (int)(a.B1 + (i64)x1v[2]);
    const int r1_3 = (int)x1v[3];
    const int x1_3 = (int)(a.B1 + (i64)x1v[3]);
    const int r1_4 = (int)x1v[4];
    const int x1_4 = (int)(a.B1 + (i64)x1v[4]);
    const int r1_5 = (int)x1v[5];
    const int x1_5 = (int)(a.B1 + (i64)x1v[5]);
    const int r1_6 = (int)x1v[6];
    const int x1_6 = (int)(a.B1 + (i64)x1v[6]);
    const int r1_7 = (int)x1v[7];
    const int x1_7 = (int)(a.B1 + (i64)x1v[7]);
    const int jr0 = act0 && jrv[0] != 0xFF ? jb + (int)jrv[0] : -1;
    const int jr1 = act1 && jrv[1] != 0xFF ? jb + (int)jrv[1] : -1;
    const int jr2 = act2 && jrv[2] != 0xFF ? jb + (int)jrv[2] : -1;
    const int jr3 = act3 && jrv[3] != 0xFF ? jb + (int)jrv[3] : -1;
    const int jr4 = act4 && jrv[4] != 0xFF ? jb + (int)jrv[4] : -1;
    const int jr5 = act5 && jrv[5] != 0xFF ? jb + (int)jrv[5] : -1;
    const int jr6 = act6 && jrv[6] != 0xFF ? jb + (int)jrv[6] : -1;
    const int jr7 = act7 && jrv[7] != 0xFF ? jb + (int)jrv[7] : -1;
    bool pass0 = act0 && jr0 >= 0 && ((true)) && ((true && (r1_0 >= (int)a.CL1 && r1_0 <= (int)a.CH1)));
    const i64 j0 = pass0 ? (i64)jr0 : 0;
    bool pass1 = act1 && jr1 >= 0 && ((true)) && ((true && (r1_1 >= (int)a.CL1 && r1_1 <= (int)a.CH1)));
    const i64 j1 = pass1 ? (i64)jr1 : 0;
    bool pass2 = act2 && jr2 >= 0 && ((true)) && ((true && (r1_2 >= (int)a.CL1 && r1_2 <= (int)a.CH1)));
    const i64 j2 = pass2 ? (i64)jr2 : 0;
    bool pass3 = act3 && jr3 >= 0 && ((true)) && ((true && (r1_3 >= (int)a.CL1 && r1_3 <= (int)a.CH1)));
    const i64 j3 = pass3 ? (i64)jr3 : 0;
    bool pass4 = act4 && jr4 >= 0 && ((true)) && ((true && (r1_4 >= (int)a.CL1 && r1_4 <= (int)a.CH1)));
    const i64 j4 = pass4 ? (i64)jr4 : 0;
    bool pass5 = act5 && jr5 >= 0 && ((true)) && ((true && (r1_5 >= (int)a.CL1 && r1_5 <= (int)a.CH1)));
    const i64 j5 = pass5 ? (i64)jr5 : 0;
    bool pass6 = act6 && jr6 >= 0 && ((true)) && ((true && (r1_6 >= (int)a.CL1 && r1_6 <= (int)a.CH1)));
    const i64 j6 = pass6 ? (i64)jr6 : 0;
    bool pass7 = act7 && jr7 >= 0 && ((true)) && ((true && (r1_7 >= (int)a.CL1 && r1_7 <= (int)a.CH1)));
    const i64 j7 = pass7 ? (i64)jr7 : 0;
    const int w8_0 = a.c8[j0];
    const int r8_0 = (int)w8_0;
    const long long x8_0 = (long long)(a.B8 + (i64)w8_0);
    const short w9_0 = a.c9[j0];
    const int r9_0 = (int)w9_0;
    const int x9_0 = (int)(a.B9 + (i64)w9_0);
    const int w8_1 = a.c8[j1];
    const int r8_1 = (int)w8_1;
    const long long x8_1 = (long long)(a.B8 + (i64)w8_1);
    const short w9_1 = a.c9[j1];
    const int r9_1 = (int)w9_1;
    const int x9_1 = (int)(a.B9 + (i64)w9_1);
    const int w8_2 = a.c8[j2];
    const int r8_2 = (int)w8_2;
    const long long x8_2 = (long long)(a.B8 + (i64)w8_2);
    const short w9_2 = a.c9[j2];
    const int r9_2 = (int)w9_2;
    const int x9_2 = (int)(a.B9 + (i64)w9_2);
    const int w8_3 = a.c8[j3];
    const int r8_3 = (int)w8_3;
    const long long x8_3 = (long long)(a.B8 + (i64)w8_3);
    const short w9_3 = a.c9[j3];
    const int r9_3 = (int)w9_3;
    const int x9_3 = (int)(a.B9 + (i64)w9_3);
    const int w8_4 = a.c8[j4];
    const int r8_4 = (int)w8_4;
    const long long x8_4 = (long long)(a.B8 + (i64)w8_4);
    const short w9_4 = a.c9[j4];
    const int r9_4 = (int)w9_4;
    const int x9_4 = (int)(a.B9 + (i64)w9_4);
    const int w8_5 = a.c8[j5];
    const int r8_5 = (int)w8_5;
    const long long x8_5 = (long long)(a.B8 + (i64)w8_5);
    const short w9_5 = a.c9[j5];
    const int r9_5 = (int)w9_5;
    const int x9_5 = (int)(a.B9 + (i64)w9_5);
    const int w8_6 = a.c8[j6];
    const int r8_6 = (int)w8_6;
    const long long x8_6 = (long long)(a.B8 + (i64)w8_6);
    const short w9_6 = a.c9[j6];
    const int r9_6 = (int)w9_6;
    const int x9_6 = (int)(a.B9 + (i64)w9_6);
    const int w8_7 = a.c8[j7];
    const int r8_7 = (int)w8_7;
    const long long x8_7 = (long long)(a.B8 + (i64)w8_7);
    const short w9_7 = a.c9[j7];
    const int r9_7 = (int)w9_7;
    const int x9_7 = (int)(a.B9 + (i64)w9_7);
    pass0 = pass0 && ((true)) && ((true)) && ((true && (r9_0 >= (int)a.CL4 && r9_0 <= (int)a.CH4)));
    pass1 = pass1 && ((true)) && ((true)) && ((true && (r9_1 >= (int)a.CL4 && r9_1 <= (int)a.CH4)));
    pass2 = pass2 && ((true)) && ((true)) && ((true && (r9_2 >= (int)a.CL4 && r9_2 <= (int)a.CH4)));
    pass3 = pass3 && ((true)) && ((true)) && ((true && (r9_3 >= (int)a.CL4 && r9_3 <= (int)a.CH4)));
    pass4 = pass4 && ((true)) && ((true)) && ((true && (r9_4 >= (int)a.CL4 && r9_4 <= (int)a.CH4)));
    pass5 = pass5 && ((true)) && ((true)) && ((true && (r9_5 >= (int)a.CL4 && r9_5 <= (int)a.CH4)));
    pass6 = pass6 && ((true)) && ((true)) && ((true && (r9_6 >= (int)a.CL4 && r9_6 <= (int)a.CH4)));
    pass7 = pass7 && ((true)) && ((true)) && ((true && (r9_7 >= (int)a.CL4 && r9_7 <= (int)a.CH4)));
    int wtot = 0;
    { const bool pz = pass0; const u64 bm = __ballot(pz);
      const int pos0 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos0] = (crow_t)(row0 - tb0); cj_s[wv][pos0] = (int)(j0); }
      wtot += __popcll(bm); }
    { const bool pz = pass1; const u64 bm = __ballot(pz);
      const int pos1 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos1] = (crow_t)(row1 - tb0); cj_s[wv][pos1] = (int)(j1); }
      wtot += __popcll(bm); }
    { const bool pz = pass2; const u64 bm = __ballot(pz);
      const int pos2 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos2] = (crow_t)(row2 - tb0); cj_s[wv][pos2] = (int)(j2); }
      wtot += __popcll(bm); }
    { const bool pz = pass3; const u64 bm = __ballot(pz);
      const int pos3 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos3] = (crow_t)(row3 - tb0); cj_s[wv][pos3] = (int)(j3); }
      wtot += __popcll(bm); }
    { const bool pz = pass4; const u64 bm = __ballot(pz);
      const int pos4 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos4] = (crow_t)(row4 - tb0); cj_s[wv][pos4] = (int)(j4); }
      wtot += __popcll(bm); }
    { const bool pz = pass5; const u64 bm = __ballot(pz);
      const int pos5 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos5] = (crow_t)(row5 - tb0); cj_s[wv][pos5] = (int)(j5); }
      wtot += __popcll(bm); }
    { const bool pz = pass6; const u64 bm = __ballot(pz);
      const int pos6 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos6] = (crow_t)(row6 - tb0); cj_s[wv][pos6] = (int)(j6); }
      wtot += __popcll(bm); }
    { const bool pz = pass7; const u64 bm = __ballot(pz);
      const int pos7 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos7] = (crow_t)(row7 - tb0); cj_s[wv][pos7] = (int)(j7); }
      wtot += __popcll(bm); }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int cb = 0; cb < wtot; cb += 64) {
      const int ce = cb + cln;
      bool cok = ce < wtot;
      const i64 crow = tb0 + (cok ? crow_s[wv][ce] : 0);
      const i64 cj = cok ? (i64)cj_s[wv][ce] : 0;
      const int w2_c = a.c2[crow];
      const int r2_c = (int)w2_c;
      const i64 q2_c = a.B2 + (i64)w2_c;
      const double x2_c = (double)((double)(a.B2 + (i64)w2_c) * a.R2);
      const signed char w3_c = a.c3[crow];
      const int r3_c = (int)w3_c;
      const i64 q3_c = a.B3 + (i64)w3_c;
      const double x3_c = (double)((double)(a.B3 + (i64)w3_c) * a.R3);
      { const bool ok = cok && true; const double v = ok ? (a.A0_0 + a.B0_0 * (double)x2_c) * (a.A0_1 + a.B0_1 * (double)x3_c) : 0.0;
        acc0 += v; cnt0 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc1 += v; cnt1 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc2 += v; cnt2 += ok ? 1u : 0u; }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  for (; t < t1; ++t) {
    while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= t) ++r;
    const i64 off = (t - a.tile_prefix[r]) * 2048;
    const i64 rs = a.rstart[r], re = rs + a.rlen[r];
    const i64 tb0 = (rs & ~(i64)7) + off;
    const i64 g0 = tb0 + (i64)threadIdx.x * 8;
    const i64 dlo_ = rs - g0, dhi_ = re - g0;
    const int alo = dlo_ <= 0 ? 0 : (dlo_ >= 8 ? 8 : (int)dlo_);
    const int ahi = dhi_ <= 0 ? 0 : (dhi_ >= 8 ? 8 : (int)dhi_);
    const bool act0 = 0 >= alo && 0 < ahi;
    const i64 row0 = g0 + 0;
    const bool act1 = 1 >= alo && 1 < ahi;
    const i64 row1 = g0 + 1;
    const bool act2 = 2 >= alo && 2 < ahi;
    const i64 row2 = g0 + 2;
    const bool act3 = 3 >= alo && 3 < ahi;
    const i64 row3 = g0 + 3;
    const bool act4 = 4 >= alo && 4 < ahi;
    const i64 row4 = g0 + 4;
    const bool act5 = 5 >= alo && 5 < ahi;
    const i64 row5 = g0 + 5;
    const bool act6 = 6 >= alo && 6 < ahi;
    const i64 row6 = g0 + 6;
    const bool act7 = 7 >= alo && 7 < ahi;
    const i64 row7 = g0 + 7;
    unsigned char jrv[8];
    jrv[0] = act0 ? a.jidx[g0 + 0] : (unsigned char)0; jrv[1] = act1 ? a.jidx[g0 + 1] : (unsigned char)0; jrv[2] = act2 ? a.jidx[g0 + 2] : (unsigned char)0; jrv[3] = act3 ? a.jidx[g0 + 3] : (unsigned char)0; jrv[4] = act4 ? a.jidx[g0 + 4] : (unsigned char)0; jrv[5] = act5 ? a.jidx[g0 + 5] : (unsigned char)0; jrv[6] = act6 ? a.jidx[g0 + 6] : (unsigned char)0; jrv[7] = act7 ? a.jidx[g0 + 7] : (unsigned char)0;
    short x1v[8];
    x1v[0] = act0 ? a.c1[g0 + 0] : (short)0; x1v[1] = act1 ? a.c1[g0 + 1] : (short)0; x1v[2] = act2 ? a.c1[g0 + 2] : (short)0; x1v[3] = act3 ? a.c1[g0 + 3] : (short)0; x1v[4] = act4 ? a.c1[g0 + 4] : (short)0; x1v[5] = act5 ? a.c1[g0 + 5] : (short)0; x1v[6] = act6 ? a.c1[g0 + 6] : (short)0; x1v[7] = act7 ? a.c1[g0 + 7] : (short)0;
    const int jb = a.jbase[g0 >> 7];
    const int r1_0 = (int)x1v[0];
    const int x1_0 = (int)(a.B1 + (i64)x1v[0]);
    const int r1_1 = (int)x1v[1];
    const int x1_1 = (int)(a.B1 + (i64)x1v[1]);
    const int r1_2 = (int)x1v[2];
    const int x1_2 = (int)(a.B1 + (i64)x1v[2]);
    const int r1_3 = (int)x1v[3];
    const int x1_3 = (int)(a.B1 + (i64)x1v[3]);
    const int r1_4 = (int)x1v[4];
    const int x1_4 = (int)(a.B1 + (i64)x1v[4]);
    const int r1_5 = (int)x1v[5];
    const int x1_5 = (int)(a.B1 + (i64)x1v[5]);
    const int r1_6 = (int)x1v[6];
    const int x1_6 = (int)(a.B1 + (i64)x1v[6]);
    const int r1_7 = (int)x1v[7];
    const int x1_7 = (int)(a.B1 + (i64)x1v[7]);
    const int jr0 = act0 && jrv[0] != 0xFF ? jb + (int)jrv[0] : -1;
    const int jr1 = act1 && jrv[1] != 0xFF ? jb + (int)jrv[1] : -1;
    const int jr2 = act2 && jrv[2] != 0xFF ? jb + (int)jrv[2] : -1;
    const int jr3 = act3 && jrv[3] != 0xFF ? jb + (int)jrv[3] : -1;
    const int jr4 = act4 && jrv[4] != 0xFF ? jb + (int)jrv[4] : -1;
    const int jr5 = act5 && jrv[5] != 0xFF ? jb + (int)jrv[5] : -1;
    const int jr6 = act6 && jrv[6] != 0xFF ? jb + (int)jrv[6] : -1;
    const int jr7 = act7 && jrv[7] != 0xFF ? jb + (int)jrv[7] : -1;
    bool pass0 = act0 && jr0 >= 0 && ((true)) && ((true && (r1_0 >= (int)a.CL1 && r1_0 <= (int)a.CH1)));
    const i64 j0 = pass0 ? (i64)jr0 : 0;
    bool pass1 = act1 && jr1 >= 0 && ((true)) && ((true && (r1_1 >= (int)a.CL1 && r1_1 <= (int)a.CH1)));
    const i64 j1 = pass1 ? (i64)jr1 : 0;
    bool pass2 = act2 && jr2 >= 0 && ((true)) && ((true && (r1_2 >= (int)a.CL1 && r1_2 <= (int)a.CH1)));
    const i64 j2 = pass2 ? (i64)jr2 : 0;
    bool pass3 = act3 && jr3 >= 0 && ((true)) && ((true && (r1_3 >= (int)a.CL1 && r1_3 <= (int)a.CH1)));
    const i64 j3 = pass3 ? (i64)jr3 : 0;
    bool pass4 = act4 && jr4 >= 0 && ((true)) && ((true && (r1_4 >= (int)a.CL1 && r1_4 <= (int)a.CH1)));
    const i64 j4 = pass4 ? (i64)jr4 : 0;
    bool pass5 = act5 && jr5 >= 0 && ((true)) && ((true && (r1_5 >= (int)a.CL1 && r1_5 <= (int)a.CH1)));
    const i64 j5 = pass5 ? (i64)jr5 : 0;
    bool pass6 = act6 && jr6 >= 0 && ((true)) && ((true && (r1_6 >= (int)a.CL1 && r1_6 <= (int)a.CH1)));
    const i64 j6 = pass6 ? (i64)jr6 : 0;
    bool pass7 = act7 && jr7 >= 0 && ((true)) && ((true && (r1_7 >= (int)a.CL1 && r1_7 <= (int)a.CH1)));
    const i64 j7 = pass7 ? (i64)jr7 : 0;
    const int w8_0 = a.c8[j0];
    const int r8_0 = (int)w8_0;
    const long long x8_0 = (long long)(a.B8 + (i64)w8_0);
    const short w9_0 = a.c9[j0];
    const int r9_0 = (int)w9_0;
    const int x9_0 = (int)(a.B9 + (i64)w9_0);
    const int w8_1 = a.c8[j1];
    const int r8_1 = (int)w8_1;
    const long long x8_1 = (long long)(a.B8 + (i64)w8_1);
    const short w9_1 = a.c9[j1];
    const int r9_1 = (int)w9_1;
    const int x9_1 = (int)(a.B9 + (i64)w9_1);
    const int w8_2 = a.c8[j2];
    const int r8_2 = (int)w8_2;
    const long long x8_2 = (long long)(a.B8 + (i64)w8_2);
    const short w9_2 = a.c9[j2];
    const int r9_2 = (int)w9_2;
    const int x9_2 = (int)(a.B9 + (i64)w9_2);
    const int w8_3 = a.c8[j3];
    const int r8_3 = (int)w8_3;
    const long long x8_3 = (long long)(a.B8 + (i64)w8_3);
    const short w9_3 = a.c9[j3];
    const int r9_3 = (int)w9_3;
    const int x9_3 = (int)(a.B9 + (i64)w9_3);
    const int w8_4 = a.c8[j4];
    const int r8_4 = (int)w8_4;
    const long long x8_4 = (long long)(a.B8 + (i64)w8_4);
    const short w9_4 = a.c9[j4];
    const int r9_4 = (int)w9_4;
    const int x9_4 = (int)(a.B9 + (i64)w9_4);
    const int w8_5 = a.c8[j5];
    const int r8_5 = (int)w8_5;
    const long long x8_5 = (long long)(a.B8 + (i64)w8_5);
    const short w9_5 = a.c9[j5];
    const int r9_5 = (int)w9_5;
    const int x9_5 = (int)(a.B9 + (i64)w9_5);
    const int w8_6 = a.c8[j6];
    const int r8_6 = (int)w8_6;
    const long long x8_6 = (long long)(a.B8 + (i64)w8_6);
    const short w9_6 = a.c9[j6];
    const int r9_6 = (int)w9_6;
    const int x9_6 = (int)(a.B9 + (i64)w9_6);
    const int w8_7 = a.c8[j7];
    const int r8_7 = (int)w8_7;
    const long long x8_7 = (long long)(a.B8 + (i64)w8_7);
    const short w9_7 = a.c9[j7];
    const int r9_7 = (int)w9_7;
    const int x9_7 = (int)(a.B9 + (i64)w9_7);
    pass0 = pass0 && ((true)) && ((true)) && ((true && (r9_0 >= (int)a.CL4 && r9_0 <= (int)a.CH4)));
    pass1 = pass1 && ((true)) && ((true)) && ((true && (r9_1 >= (int)a.CL4 && r9_1 <= (int)a.CH4)));
    pass2 = pass2 && ((true)) && ((true)) && ((true && (r9_2 >= (int)a.CL4 && r9_2 <= (int)a.CH4)));
    pass3 = pass3 && ((true)) && ((true)) && ((true && (r9_3 >= (int)a.CL4 && r9_3 <= (int)a.CH4)));
    pass4 = pass4 && ((true)) && ((true)) && ((true && (r9_4 >= (int)a.CL4 && r9_4 <= (int)a.CH4)));
    pass5 = pass5 && ((true)) && ((true)) && ((true && (r9_5 >= (int)a.CL4 && r9_5 <= (int)a.CH4)));
    pass6 = pass6 && ((true)) && ((true)) && ((true && (r9_6 >= (int)a.CL4 && r9_6 <= (int)a.CH4)));
    pass7 = pass7 && ((true)) && ((true)) && ((true && (r9_7 >= (int)a.CL4 && r9_7 <= (int)a.CH4)));
    int wtot = 0;
    { const bool pz = pass0; const u64 bm = __ballot(pz);
      const int pos0 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos0] = (crow_t)(row0 - tb0); cj_s[wv][pos0] = (int)(j0); }
      wtot += __popcll(bm); }
    { const bool pz = pass1; const u64 bm = __ballot(pz);
      const int pos1 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos1] = (crow_t)(row1 - tb0); cj_s[wv][pos1] = (int)(j1); }
      wtot += __popcll(bm); }
    { const bool pz = pass2; const u64 bm = __ballot(pz);
      const int pos2 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos2] = (crow_t)(row2 - tb0); cj_s[wv][pos2] = (int)(j2); }
      wtot += __popcll(bm); }
    { const bool pz = pass3; const u64 bm = __ballot(pz);
      const int pos3 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos3] = (crow_t)(row3 - tb0); cj_s[wv][pos3] = (int)(j3); }
      wtot += __popcll(bm); }
    { const bool pz = pass4; const u64 bm = __ballot(pz);
      const int pos4 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos4] = (crow_t)(row4 - tb0); cj_s[wv][pos4] = (int)(j4); }
      wtot += __popcll(bm); }
    { const bool pz = pass5; const u64 bm = __ballot(pz);
      const int pos5 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos5] = (crow_t)(row5 - tb0); cj_s[wv][pos5] = (int)(j5); }
      wtot += __popcll(bm); }
    { const bool pz = pass6; const u64 bm = __ballot(pz);
      const int pos6 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos6] = (crow_t)(row6 - tb0); cj_s[wv][pos6] = (int)(j6); }
      wtot += __popcll(bm); }
    { const bool pz = pass7; const u64 bm = __ballot(pz);
      const int pos7 = wtot + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u));
      if (pz) { crow_s[wv][pos7] = (crow_t)(row7 - tb0); cj_s[wv][pos7] = (int)(j7); }
      wtot += __popcll(bm); }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int cb = 0; cb < wtot; cb += 64) {
      const int ce = cb + cln;
      bool cok = ce < wtot;
      const i64 crow = tb0 + (cok ? crow_s[wv][ce] : 0);
      const i64 cj = cok ? (i64)cj_s[wv][ce] : 0;
      const int w2_c = a.c2[crow];
      const int r2_c = (int)w2_c;
      const i64 q2_c = a.B2 + (i64)w2_c;
      const double x2_c = (double)((double)(a.B2 + (i64)w2_c) * a.R2);
      const signed char w3_c = a.c3[crow];
      const int r3_c = (int)w3_c;
      const i64 q3_c = a.B3 + (i64)w3_c;
      const double x3_c = (double)((double)(a.B3 + (i64)w3_c) * a.R3);
      { const bool ok = cok && true; const double v = ok ? (a.A0_0 + a.B0_0 * (double)x2_c) * (a.A0_1 + a.B0_1 * (double)x3_c) : 0.0;
        acc0 += v; cnt0 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc1 += v; cnt1 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc2 += v; cnt2 += ok ? 1u : 0u; }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  __shared__ double rv[4][NA]; __shared__ i64 rc[4][NA];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  { const double r = wsum(acc0); const i64 c = wsumi((i64)cnt0); if (lane == 0) { rv[w][0] = r; rc[w][0] = c; } }
  { const double r = wsum(acc1); const i64 c = wsumi((i64)cnt1); if (lane == 0) { rv[w][1] = r; rc[w][1] = c; } }
  { const double r = wsum(acc2); const i64 c = wsumi((i64)cnt2); if (lane == 0) { rv[w][2] = r; rc[w][2] = c; } }
  __syncthreads();
  if (threadIdx.x == 0) {
    { double t = 0.0; i64 c = 0;
      for (int k = 0; k < 4; ++k) { t = t + rv[k][0]; c += rc[k][0]; }
      const i64 o = (i64)blockIdx.x * NA + 0;
      a.psum[o] = t; a.pcnt[o] = c;
      a.pmin[o] = __builtin_inf(); a.pmax[o] = -__builtin_inf(); }
    { double t = 0.0; i64 c = 0;
      for (int k = 0; k < 4; ++k) { t = t + rv[k][1]; c += rc[k][1]; }
      const i64 o = (i64)blockIdx.x * NA + 1;
      a.psum[o] = t; a.pcnt[o] = c;
      a.pmin[o] = __builtin_inf(); a.pmax[o] = -__builtin_inf(); }
    { double t = 0.0; i64 c = 0;
      for (int k = 0; k < 4; ++k) { t = t + rv[k][2]; c += rc[k][2]; }
      const i64 o = (i64)blockIdx.x * NA + 2;
      a.psum[o] = t; a.pcnt[o] = c;
      a.pmin[o] = __builtin_inf(); a.pmax[o] = -__builtin_inf(); }
  }
}
