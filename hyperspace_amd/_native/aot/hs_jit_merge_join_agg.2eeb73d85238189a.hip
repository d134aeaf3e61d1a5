
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
  const long long* spans;
  long long R;
  long long nrows;
  long long rdup;
  double* psum;
  double* pmin;
  double* pmax;
  long long* pcnt;
  long long KLO;
  long long KSP;
  long long KOF;
  const int* c0;
  const short* c1;
  const int* c8;
  long long B8;
  const short* c9;
  long long B9;
  long long CL4;
  long long CH4;
  long long B0;
  long long B1;
  long long CL1;
  long long CH1;
  const int* c2;
  long long B2;
  double R2;
  const signed char* c3;
  long long B3;
  double R3;
  const signed char* c10;
  long long B10;
  unsigned long long* hkeys;
  double* hsum;
  long long* hcnt;
  long long HM;
  long long* hflag;
  long long HL0;
  long long HS0;
  long long HL1;
  long long HS1;
  long long HL2;
  long long HS2;
  double A0_0;
  double B0_0;
  double A0_1;
  double B0_1;
};
extern "C" __global__ __launch_bounds__(256) void hs_jit_merge_join_agg(Args a) {
  constexpr int NA = 2;
  double acc0 = 0.0; unsigned cnt0 = 0u;
  double acc1 = 0.0; unsigned cnt1 = 0u;
  __shared__ unsigned skeys_[1][2049]; __shared__ unsigned char spass_[1][2048];
  const int cln = threadIdx.x & 63, wv = threadIdx.x >> 6;
  constexpr int DUMP = 128;
  __shared__ int lrow_s[4][192]; __shared__ int lj_s[4][192];
  int wcnt = 0;   // wavefront-uniform length of this wavefront's (row, j) list
  const i64 ntiles = a.tile_prefix[a.R];
  const i64 per = (ntiles + gridDim.x - 1) / gridDim.x;
  const i64 t0 = (i64)blockIdx.x * per;
  const i64 t1 = ntiles < t0 + per ? ntiles : t0 + per;
  int r = 0;
  if (t0 < t1) { int lo = 0, hi = (int)a.R;
    while (hi - lo > 1) { const int m = (lo + hi) >> 1; if (a.tile_prefix[m] <= t0) lo = m; else hi = m; }
    r = lo; }
  for (i64 t = t0; t < t1; ++t) {
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
    if (tb0 + 2048 <= a.nrows) {
    int x0v[8];
    vload<int, 8>(a.c0, g0, x0v);
    short x1v[8];
    vload<short, 8>(a.c1, g0, x1v);
    const i64 ss = a.spans[4 * t + 2], se = a.spans[4 * t + 3];
    const int ns = (int)(se - ss);
    const bool staged = ns <= 2048;
    unsigned* const skeys = skeys_[0];
    unsigned char* const spass = spass_[0];
    if (staged) for (int sqb = 0; sqb < ns; sqb += 1024) {
      const int sq0 = sqb + 0 + (int)threadIdx.x;
      const bool sv0 = sq0 < ns;
      const i64 jr0 = ss + (sv0 ? sq0 : 0);
      const int sq1 = sqb + 256 + (int)threadIdx.x;
      const bool sv1 = sq1 < ns;
      const i64 jr1 = ss + (sv1 ? sq1 : 0);
      const int sq2 = sqb + 512 + (int)threadIdx.x;
      const bool sv2 = sq2 < ns;
      const i64 jr2 = ss + (sv2 ? sq2 : 0);
      const int sq3 = sqb + 768 + (int)threadIdx.x;
      const bool sv3 = sq3 < ns;
      const i64 jr3 = ss + (sv3 ? sq3 : 0);
      const int w8_s0 = a.c8[jr0];
      const int r8_s0 = (int)w8_s0;
      const long long x8_s0 = (long long)(a.B8 + (i64)w8_s0);
      const short w9_s0 = a.c9[jr0];
      const int r9_s0 = (int)w9_s0;
      const int x9_s0 = (int)(a.B9 + (i64)w9_s0);
      const int w8_s1 = a.c8[jr1];
      const int r8_s1 = (int)w8_s1;
      const long long x8_s1 = (long long)(a.B8 + (i64)w8_s1);
      const short w9_s1 = a.c9[jr1];
      const int r9_s1 = (int)w9_s1;
      const int x9_s1 = (int)(a.B9 + (i64)w9_s1);
      const int w8_s2 = a.c8[jr2];
      const int r8_s2 = (int)w8_s2;
      const long long x8_s2 = (long long)(a.B8 + (i64)w8_s2);
      const short w9_s2 = a.c9[jr2];
      const int r9_s2 = (int)w9_s2;
      const int x9_s2 = (int)(a.B9 + (i64)w9_s2);
      const int w8_s3 = a.c8[jr3];
      const int r8_s3 = (int)w8_s3;
      const long long x8_s3 = (long long)(a.B8 + (i64)w8_s3);
      const short w9_s3 = a.c9[jr3];
      const int r9_s3 = (int)w9_s3;
      const int x9_s3 = (int)(a.B9 + (i64)w9_s3);
      if (sv0) { const bool kv = true;
        skeys[sq0] = kv ? ({ const i64 d_ = (i64)(x8_s0) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) : (unsigned)0;
        spass[sq0] = (kv && ((true)) && ((true)) && ((true && (r9_s0 >= (int)a.CL4 && r9_s0 <= (int)a.CH4)))) ? 1 : 0;
      }
      if (sv1) { const bool kv = true;
        skeys[sq1] = kv ? ({ const i64 d_ = (i64)(x8_s1) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) : (unsigned)0;
        spass[sq1] = (kv && ((true)) && ((true)) && ((true && (r9_s1 >= (int)a.CL4 && r9_s1 <= (int)a.CH4)))) ? 1 : 0;
      }
      if (sv2) { const bool kv = true;
        skeys[sq2] = kv ? ({ const i64 d_ = (i64)(x8_s2) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) : (unsigned)0;
        spass[sq2] = (kv && ((true)) && ((true)) && ((true && (r9_s2 >= (int)a.CL4 && r9_s2 <= (int)a.CH4)))) ? 1 : 0;
      }
      if (sv3) { const bool kv = true;
        skeys[sq3] = kv ? ({ const i64 d_ = (i64)(x8_s3) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) : (unsigned)0;
        spass[sq3] = (kv && ((true)) && ((true)) && ((true && (r9_s3 >= (int)a.CL4 && r9_s3 <= (int)a.CH4)))) ? 1 : 0;
      }
    }
    if (staged && threadIdx.x == 0) skeys[ns] = 0xFFFFFFFFu;   // walk sentinel
    const int r0_0 = (int)x0v[0];
    const long long x0_0 = (long long)(a.B0 + (i64)x0v[0]);
    const int r1_0 = (int)x1v[0];
    const int x1_0 = (int)(a.B1 + (i64)x1v[0]);
    const int r0_1 = (int)x0v[1];
    const long long x0_1 = (long long)(a.B0 + (i64)x0v[1]);
    const int r1_1 = (int)x1v[1];
    const int x1_1 = (int)(a.B1 + (i64)x1v[1]);
    const int r0_2 = (int)x0v[2];
    const long long x0_2 = (long long)(a.B0 + (i64)x0v[2]);
    const int r1_2 = (int)x1v[2];
    const int x1_2 = (int)(a.B1 + (i64)x1v[2]);
    const int r0_3 = (int)x0v[3];
    const long long x0_3 = (long long)(a.B0 + (i64)x0v[3]);
    const int r1_3 = (int)x1v[3];
    const int x1_3 = (int)(a.B1 + (i64)x1v[3]);
    const int r0_4 = (int)x0v[4];
    const long long x0_4 = (long long)(a.B0 + (i64)x0v[4]);
    const int r1_4 = (int)x1v[4];
    const int x1_4 = (int)(a.B1 + (i64)x1v[4]);
    const int r0_5 = (int)x0v[5];
    const long long x0_5 = (long long)(a.B0 + (i64)x0v[5]);
    const int r1_5 = (int)x1v[5];
    const int x1_5 = (int)(a.B1 + (i64)x1v[5]);
    const int r0_6 = (int)x0v[6];
    const long long x0_6 = (long long)(a.B0 + (i64)x0v[6]);
    const int r1_6 = (int)x1v[6];
    const int x1_6 = (int)(a.B1 + (i64)x1v[6]);
    const int r0_7 = (int)x0v[7];
    const long long x0_7 = (long long)(a.B0 + (i64)x0v[7]);
    const int r1_7 = (int)x1v[7];
    const int x1_7 = (int)(a.B1 + (i64)x1v[7]);
    unsigned kvb = 0u, mb = 0u;
    { const bool kv = act0 && true; kvb |= kv ? 1u : 0u; mb |= (kv && ((true)) && ((true && (r1_0 >= (int)a.CL1 && r1_0 <= (int)a.CH1)))) ? 1u : 0u; }
    const unsigned k0 = ((unsigned)x0v[0] + (unsigned)a.KOF);
    { const bool kv = act1 && true; kvb |= kv ? 2u : 0u; mb |= (kv && ((true)) && ((true && (r1_1 >= (int)a.CL1 && r1_1 <= (int)a.CH1)))) ? 2u : 0u; }
    const unsigned k1 = ((unsigned)x0v[1] + (unsigned)a.KOF);
    { const bool kv = act2 && true; kvb |= kv ? 4u : 0u; mb |= (kv && ((true)) && ((true && (r1_2 >= (int)a.CL1 && r1_2 <= (int)a.CH1)))) ? 4u : 0u; }
    const unsigned k2 = ((unsigned)x0v[2] + (unsigned)a.KOF);
    { const bool kv = act3 && true; kvb |= kv ? 8u : 0u; mb |= (kv && ((true)) && ((true && (r1_3 >= (int)a.CL1 && r1_3 <= (int)a.CH1)))) ? 8u : 0u; }
    const unsigned k3 = ((unsigned)x0v[3] + (unsigned)a.KOF);
    { const bool kv = act4 && true; kvb |= kv ? 16u : 0u; mb |= (kv && ((true)) && ((true && (r1_4 >= (int)a.CL1 && r1_4 <= (int)a.CH1)))) ? 16u : 0u; }
    const unsigned k4 = ((unsigned)x0v[4] + (unsigned)a.KOF);
    { const bool kv = act5 && true; kvb |= kv ? 32u : 0u; mb |= (kv && ((true)) && ((true && (r1_5 >= (int)a.CL1 && r1_5 <= (int)a.CH1)))) ? 32u : 0u; }
    const unsigned k5 = ((unsigned)x0v[5] + (unsigned)a.KOF);
    { const bool kv = act6 && true; kvb |= kv ? 64u : 0u; mb |= (kv && ((true)) && ((true && (r1_6 >= (int)a.CL1 && r1_6 <= (int)a.CH1)))) ? 64u : 0u; }
    const unsigned k6 = ((unsigned)x0v[6] + (unsigned)a.KOF);
    { const bool kv = act7 && true; kvb |= kv ? 128u : 0u; mb |= (kv && ((true)) && ((true && (r1_7 >= (int)a.CL1 && r1_7 <= (int)a.CH1)))) ? 128u : 0u; }
    const unsigned k7 = ((unsigned)x0v[7] + (unsigned)a.KOF);
    __syncthreads();
    unsigned kf = 0xFFFFFFFFu;
    kf = ((mb >> 7) & 1u) ? k7 : kf;
    kf = ((mb >> 6) & 1u) ? k6 : kf;
    kf = ((mb >> 5) & 1u) ? k5 : kf;
    kf = ((mb >> 4) & 1u) ? k4 : kf;
    kf = ((mb >> 3) & 1u) ? k3 : kf;
    kf = ((mb >> 2) & 1u) ? k2 : kf;
    kf = ((mb >> 1) & 1u) ? k1 : kf;
    kf = ((mb >> 0) & 1u) ? k0 : kf;
    unsigned mtb = 0u;
    int jl0 = 0;
    int jl1 = 0;
    int jl2 = 0;
    int jl3 = 0;
    int jl4 = 0;
    int jl5 = 0;
    int jl6 = 0;
    int jl7 = 0;
    bool slow = !staged;
    int jw0 = 0;
    if (staged) {
      int lo = 0;
      for (int st = ns > 0 ? (1 << (31 - __builtin_clz(ns))) : 0; st > 0; st >>= 1) {
        const int c = lo + st; const unsigned sv = skeys[c <= ns ? c - 1 : ns];
        lo = (c <= ns && sv < kf) ? c : lo; }
      jw0 = lo; int jw = lo; unsigned v = skeys[jw];
      { const unsigned ke = ((kvb >> 0) & 1u) ? k0 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 0) & 1u) && v == ke && jw < ns) ? 1u : 0u; jl0 = jw; }
      { const unsigned ke = ((kvb >> 1) & 1u) ? k1 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 1) & 1u) && v == ke && jw < ns) ? 2u : 0u; jl1 = jw; }
      { const unsigned ke = ((kvb >> 2) & 1u) ? k2 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 2) & 1u) && v == ke && jw < ns) ? 4u : 0u; jl2 = jw; }
      { const unsigned ke = ((kvb >> 3) & 1u) ? k3 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 3) & 1u) && v == ke && jw < ns) ? 8u : 0u; jl3 = jw; }
      { const unsigned ke = ((kvb >> 4) & 1u) ? k4 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 4) & 1u) && v == ke && jw < ns) ? 16u : 0u; jl4 = jw; }
      { const unsigned ke = ((kvb >> 5) & 1u) ? k5 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 5) & 1u) && v == ke && jw < ns) ? 32u : 0u; jl5 = jw; }
      { const unsigned ke = ((kvb >> 6) & 1u) ? k6 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 6) & 1u) && v == ke && jw < ns) ? 64u : 0u; jl6 = jw; }
      { const unsigned ke = ((kvb >> 7) & 1u) ? k7 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 7) & 1u) && v == ke && jw < ns) ? 128u : 0u; jl7 = jw; }
    }
    if (__any(slow)) {
      if (slow) { int jw = jw0; mtb = 0u;
        if (((mb >> 0) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k0) ++jw;
            hit = jw < ns && skeys[jw] == k0; jl0 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k0) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k0; jl0 = (int)(lo - ss); }
          mtb |= hit ? 1u : 0u;
        }
        if (((mb >> 1) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k1) ++jw;
            hit = jw < ns && skeys[jw] == k1; jl1 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k1) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k1; jl1 = (int)(lo - ss); }
          mtb |= hit ? 2u : 0u;
        }
        if (((mb >> 2) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k2) ++jw;
            hit = jw < ns && skeys[jw] == k2; jl2 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k2) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k2; jl2 = (int)(lo - ss); }
          mtb |= hit ? 4u : 0u;
        }
        if (((mb >> 3) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k3) ++jw;
            hit = jw < ns && skeys[jw] == k3; jl3 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k3) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k3; jl3 = (int)(lo - ss); }
          mtb |= hit ? 8u : 0u;
        }
        if (((mb >> 4) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k4) ++jw;
            hit = jw < ns && skeys[jw] == k4; jl4 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k4) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k4; jl4 = (int)(lo - ss); }
          mtb |= hit ? 16u : 0u;
        }
        if (((mb >> 5) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k5) ++jw;
            hit = jw < ns && skeys[jw] == k5; jl5 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k5) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k5; jl5 = (int)(lo - ss); }
          mtb |= hit ? 32u : 0u;
        }
        if (((mb >> 6) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k6) ++jw;
            hit = jw < ns && skeys[jw] == k6; jl6 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k6) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k6; jl6 = (int)(lo - ss); }
          mtb |= hit ? 64u : 0u;
        }
        if (((mb >> 7) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k7) ++jw;
            hit = jw < ns && skeys[jw] == k7; jl7 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k7) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k7; jl7 = (int)(lo - ss); }
          mtb |= hit ? 128u : 0u;
        }
      }
    }
    { unsigned pb = mtb;
    if (staged) {
      pb &= spass[((mtb >> 0) & 1u) ? jl0 : 0] != 0 ? ~0u : ~1u;
      pb &= spass[((mtb >> 1) & 1u) ? jl1 : 0] != 0 ? ~0u : ~2u;
      pb &= spass[((mtb >> 2) & 1u) ? jl2 : 0] != 0 ? ~0u : ~4u;
      pb &= spass[((mtb >> 3) & 1u) ? jl3 : 0] != 0 ? ~0u : ~8u;
      pb &= spass[((mtb >> 4) & 1u) ? jl4 : 0] != 0 ? ~0u : ~16u;
      pb &= spass[((mtb >> 5) & 1u) ? jl5 : 0] != 0 ? ~0u : ~32u;
      pb &= spass[((mtb >> 6) & 1u) ? jl6 : 0] != 0 ? ~0u : ~64u;
      pb &= spass[((mtb >> 7) & 1u) ? jl7 : 0] != 0 ? ~0u : ~128u;
    } else {
      { const i64 jq0 = ss + (((mtb >> 0) & 1u) ? jl0 : 0);
        const int w8_0 = a.c8[jq0];
        const int r8_0 = (int)w8_0;
        const long long x8_0 = (long long)(a.B8 + (i64)w8_0);
        const short w9_0 = a.c9[jq0];
        const int r9_0 = (int)w9_0;
        const int x9_0 = (int)(a.B9 + (i64)w9_0);
        pb &= (((true)) && ((true)) && ((true && (r9_0 >= (int)a.CL4 && r9_0 <= (int)a.CH4)))) ? ~0u : ~1u; }
      { const i64 jq1 = ss + (((mtb >> 1) & 1u) ? jl1 : 0);
        const int w8_1 = a.c8[jq1];
        const int r8_1 = (int)w8_1;
        const long long x8_1 = (long long)(a.B8 + (i64)w8_1);
        const short w9_1 = a.c9[jq1];
        const int r9_1 = (int)w9_1;
        const int x9_1 = (int)(a.B9 + (i64)w9_1);
        pb &= (((true)) && ((true)) && ((true && (r9_1 >= (int)a.CL4 && r9_1 <= (int)a.CH4)))) ? ~0u : ~2u; }
      { const i64 jq2 = ss + (((mtb >> 2) & 1u) ? jl2 : 0);
        const int w8_2 = a.c8[jq2];
        const int r8_2 = (int)w8_2;
        const long long x8_2 = (long long)(a.B8 + (i64)w8_2);
        const short w9_2 = a.c9[jq2];
        const int r9_2 = (int)w9_2;
        const int x9_2 = (int)(a.B9 + (i64)w9_2);
        pb &= (((true)) && ((true)) && ((true && (r9_2 >= (int)a.CL4 && r9_2 <= (int)a.CH4)))) ? ~0u : ~4u; }
      { const i64 jq3 = ss + (((mtb >> 3) & 1u) ? jl3 : 0);
        const int w8_3 = a.c8[jq3];
        const int r8_3 = (int)w8_3;
        const long long x8_3 = (long long)(a.B8 + (i64)w8_3);
        const short w9_3 = a.c9[jq3];
        const int r9_3 = (int)w9_3;
        const int x9_3 = (int)(a.B9 + (i64)w9_3);
        pb &= (((true)) && ((true)) && ((true && (r9_3 >= (int)a.CL4 && r9_3 <= (int)a.CH4)))) ? ~0u : ~8u; }
      { const i64 jq4 = ss + (((mtb >> 4) & 1u) ? jl4 : 0);
        const int w8_4 = a.c8[jq4];
        const int r8_4 = (int)w8_4;
        const long long x8_4 = (long long)(a.B8 + (i64)w8_4);
        const short w9_4 = a.c9[jq4];
        const int r9_4 = (int)w9_4;
        const int x9_4 = (int)(a.B9 + (i64)w9_4);
        pb &= (((true)) && ((true)) && ((true && (r9_4 >= (int)a.CL4 && r9_4 <= (int)a.CH4)))) ? ~0u : ~16u; }
      { const i64 jq5 = ss + (((mtb >> 5) & 1u) ? jl5 : 0);
        const int w8_5 = a.c8[jq5];
        const int r8_5 = (int)w8_5;
        const long long x8_5 = (long long)(a.B8 + (i64)w8_5);
        const short w9_5 = a.c9[jq5];
        const int r9_5 = (int)w9_5;
        const int x9_5 = (int)(a.B9 + (i64)w9_5);
        pb &= (((true)) && ((true)) && ((true && (r9_5 >= (int)a.CL4 && r9_5 <= (int)a.CH4)))) ? ~0u : ~32u; }
      { const i64 jq6 = ss + (((mtb >> 6) & 1u) ? jl6 : 0);
        const int w8_6 = a.c8[jq6];
        const int r8_6 = (int)w8_6;
        const long long x8_6 = (long long)(a.B8 + (i64)w8_6);
        const short w9_6 = a.c9[jq6];
        const int r9_6 = (int)w9_6;
        const int x9_6 = (int)(a.B9 + (i64)w9_6);
        pb &= (((true)) && ((true)) && ((true && (r9_6 >= (int)a.CL4 && r9_6 <= (int)a.CH4)))) ? ~0u : ~64u; }
      { const i64 jq7 = ss + (((mtb >> 7) & 1u) ? jl7 : 0);
        const int w8_7 = a.c8[jq7];
        const int r8_7 = (int)w8_7;
        const long long x8_7 = (long long)(a.B8 + (i64)w8_7);
        const short w9_7 = a.c9[jq7];
        const int r9_7 = (int)w9_7;
        const int x9_7 = (int)(a.B9 + (i64)w9_7);
        pb &= (((true)) && ((true)) && ((true && (r9_7 >= (int)a.CL4 && r9_7 <= (int)a.CH4)))) ? ~0u : ~128u; }
    }
    { unsigned pend = pb;
      while (__any(pend != 0u)) {
        const bool has = pend != 0u;
        const int it = has ? __builtin_ctz(pend) : 0;
        pend &= pend - 1u;
        int jv = jl0;
        jv = it == 1 ? jl1 : jv;
        jv = it == 2 ? jl2 : jv;
        jv = it == 3 ? jl3 : jv;
        jv = it == 4 ? jl4 : jv;
        jv = it == 5 ? jl5 : jv;
        jv = it == 6 ? jl6 : jv;
        jv = it == 7 ? jl7 : jv;
        const u64 bm = __ballot(has);
        const int wp = has ? wcnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u)) : DUMP + cln;
        lrow_s[wv][wp] = (int)(g0 + it); lj_s[wv][wp] = (int)(ss + jv);
        wcnt += __popcll(bm);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        while (wcnt >= 64) {
          const int cb = wcnt > 64 ? wcnt - 64 : 0;
          const int ce = cb + cln;
          bool cok = ce < wcnt;
          const i64 crow = (i64)lrow_s[wv][cok ? ce : cb];
          const i64 cj = (i64)lj_s[wv][cok ? ce : cb];
          const int w2_c = a.c2[crow];
          const int r2_c = (int)w2_c;
          const i64 q2_c = a.B2 + (i64)w2_c;
          const double x2_c = (double)((double)(a.B2 + (i64)w2_c) * a.R2);
          const signed char w3_c = a.c3[crow];
          const int r3_c = (int)w3_c;
          const i64 q3_c = a.B3 + (i64)w3_c;
          const double x3_c = (double)((double)(a.B3 + (i64)w3_c) * a.R3);
          const int w0_c = a.c0[crow];
          const int r0_c = (int)w0_c;
          const long long x0_c = (long long)(a.B0 + (i64)w0_c);
          const short w9_c = a.c9[cj];
          const int r9_c = (int)w9_c;
          const int x9_c = (int)(a.B9 + (i64)w9_c);
          const signed char w10_c = a.c10[cj];
          const int r10_c = (int)w10_c;
          const int x10_c = (int)(a.B10 + (i64)w10_c);
          { const int hln = (int)(threadIdx.x & 63u); const bool hok = cok;
            u64 hk = 0ull; const bool hnul = false;
            hk |= (u64)((i64)x0_c - a.HL0) << (unsigned)a.HS0;
            hk |= (u64)((i64)x9_c - a.HL1) << (unsigned)a.HS1;
            hk |= (u64)((i64)x10_c - a.HL2) << (unsigned)a.HS2;
            const u64 hkp = __shfl_up(hk, 1u, 64);
            const int hfp = __shfl_up((hok ? 1 : 0) | (hnul ? 2 : 0), 1u, 64);
            const bool hsame = hln > 0 && hok && (hfp & 1) != 0 && ((hfp >> 1) & 1) == (hnul ? 1 : 0) && hkp == hk;
            const u64 hH = __ballot(!hsame);
            const int hss = 63 - __builtin_clzll(hH & ((2ull << hln) - 1ull));
            const bool htl = hok && (hln == 63 || ((hH >> ((hln + 1) & 63)) & 1ull) != 0ull);
            const bool hq0 = hok && true;
            double hv0 = hq0 ? (double)((a.A0_0 + a.B0_0 * (double)x2_c) * (a.A0_1 + a.B0_1 * (double)x3_c)) : 0.0;
            #pragma unroll
            for (int hd = 1; hd < 64; hd <<= 1) {
              const double u_hv0 = __shfl_up(hv0, (unsigned)hd, 64);
              if (hln - hd >= hss) {
                hv0 = hv0 + u_hv0;
              }
            }
            if (htl) {
              long long hs_ = -1;
              if (hnul) hs_ = a.HM + 1; else if (hk == ~0ull) hs_ = a.HM; else {
                u64 hh = hs_mix64(hk) & (u64)(a.HM - 1);
                for (int pr_ = 0; pr_ < 512; ++pr_) {
                  const u64 pv_ = atomicCAS(&a.hkeys[hh], ~0ull, hk);
                  if (pv_ == ~0ull || pv_ == hk) { hs_ = (long long)hh; break; }
                  hh = (hh + 1ull) & (u64)(a.HM - 1);
                }
                if (hs_ < 0) a.hflag[0] = 1;
              }
              if (hs_ >= 0) {
                const long long hst = a.HM + 2;   // SoA: aggregate i of slot s at i * (M + 2) + s
                const unsigned long long hrn = (unsigned long long)(hln - hss + 1);
                unsafeAtomicAdd(&a.hsum[0 * hst + hs_], hv0);
                if (hs_ >= a.HM) atomicAdd((unsigned long long*)&a.hcnt[1 * hst + hs_], hrn);
              }
            }
          }
          wcnt = cb;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
    }
    }
    if (a.rdup) while (true) {
      if (((mtb >> 0) & 1u)) { ++jl0;
        const bool more = jl0 < ns && (staged ? skeys[jl0] == k0 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl0)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k0));
        if (!more) mtb &= ~1u; }
      if (((mtb >> 1) & 1u)) { ++jl1;
        const bool more = jl1 < ns && (staged ? skeys[jl1] == k1 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl1)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k1));
        if (!more) mtb &= ~2u; }
      if (((mtb >> 2) & 1u)) { ++jl2;
        const bool more = jl2 < ns && (staged ? skeys[jl2] == k2 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl2)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k2));
        if (!more) mtb &= ~4u; }
      if (((mtb >> 3) & 1u)) { ++jl3;
        const bool more = jl3 < ns && (staged ? skeys[jl3] == k3 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl3)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k3));
        if (!more) mtb &= ~8u; }
      if (((mtb >> 4) & 1u)) { ++jl4;
        const bool more = jl4 < ns && (staged ? skeys[jl4] == k4 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl4)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k4));
        if (!more) mtb &= ~16u; }
      if (((mtb >> 5) & 1u)) { ++jl5;
        const bool more = jl5 < ns && (staged ? skeys[jl5] == k5 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl5)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k5));
        if (!more) mtb &= ~32u; }
      if (((mtb >> 6) & 1u)) { ++jl6;
        const bool more = jl6 < ns && (staged ? skeys[jl6] == k6 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl6)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k6));
        if (!more) mtb &= ~64u; }
      if (((mtb >> 7) & 1u)) { ++jl7;
        const bool more = jl7 < ns && (staged ? skeys[jl7] == k7 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl7)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k7));
        if (!more) mtb &= ~128u; }
      if (!__any(mtb != 0u)) break;
      { unsigned pb = mtb;
      if (staged) {
        pb &= spass[((mtb >> 0) & 1u) ? jl0 : 0] != 0 ? ~0u : ~1u;
        pb &= spass[((mtb >> 1) & 1u) ? jl1 : 0] != 0 ? ~0u : ~2u;
        pb &= spass[((mtb >> 2) & 1u) ? jl2 : 0] != 0 ? ~0u : ~4u;
        pb &= spass[((mtb >> 3) & 1u) ? jl3 : 0] != 0 ? ~0u : ~8u;
        pb &= spass[((mtb >> 4) & 1u) ? jl4 : 0] != 0 ? ~0u : ~16u;
        pb &= spass[((mtb >> 5) & 1u) ? jl5 : 0] != 0 ? ~0u : ~32u;
        pb &= spass[((mtb >> 6) & 1u) ? jl6 : 0] != 0 ? ~0u : ~64u;
        pb &= spass[((mtb >> 7) & 1u) ? jl7 : 0] != 0 ? ~0u : ~128u;
      } else {
        { const i64 jq0 = ss + (((mtb >> 0) & 1u) ? jl0 : 0);
          const int w8_0 = a.c8[jq0];
          const int r8_0 = (int)w8_0;
          const long long x8_0 = (long long)(a.B8 + (i64)w8_0);
          const short w9_0 = a.c9[jq0];
          const int r9_0 = (int)w9_0;
          const int x9_0 = (int)(a.B9 + (i64)w9_0);
          pb &= (((true)) && ((true)) && ((true && (r9_0 >= (int)a.CL4 && r9_0 <= (int)a.CH4)))) ? ~0u : ~1u; }
        { const i64 jq1 = ss + (((mtb >> 1) & 1u) ? jl1 : 0);
          const int w8_1 = a.c8[jq1];
          const int r8_1 = (int)w8_1;
          const long long x8_1 = (long long)(a.B8 + (i64)w8_1);
          const short w9_1 = a.c9[jq1];
          const int r9_1 = (int)w9_1;
          const int x9_1 = (int)(a.B9 + (i64)w9_1);
          pb &= (((true)) && ((true)) && ((true && (r9_1 >= (int)a.CL4 && r9_1 <= (int)a.CH4)))) ? ~0u : ~2u; }
        { const i64 jq2 = ss + (((mtb >> 2) & 1u) ? jl2 : 0);
          const int w8_2 = a.c8[jq2];
          const int r8_2 = (int)w8_2;
          const long long x8_2 = (long long)(a.B8 + (i64)w8_2);
          const short w9_2 = a.c9[jq2];
          const int r9_2 = (int)w9_2;
          const int x9_2 = (int)(a.B9 + (i64)w9_2);
          pb &= (((true)) && ((true)) && ((true && (r9_2 >= (int)a.CL4 && r9_2 <= (int)a.CH4)))) ? ~0u : ~4u; }
        { const i64 jq3 = ss + (((mtb >> 3) & 1u) ? jl3 : 0);
          const int w8_3 = a.c8[jq3];
          const int r8_3 = (int)w8_3;
          const long long x8_3 = (long long)(a.B8 + (i64)w8_3);
          const short w9_3 = a.c9[jq3];
          const int r9_3 = (int)w9_3;
          const int x9_3 = (int)(a.B9 + (i64)w9_3);
          pb &= (((true)) && ((true)) && ((true && (r9_3 >= (int)a.CL4 && r9_3 <= (int)a.CH4)))) ? ~0u : ~8u; }
        { const i64 jq4 = ss + (((mtb >> 4) & 1u) ? jl4 : 0);
          const int w8_4 = a.c8[jq4];
          const int r8_4 = (int)w8_4;
          const long long x8_4 = (long long)(a.B8 + (i64)w8_4);
          const short w9_4 = a.c9[jq4];
          const int r9_4 = (int)w9_4;
          const int x9_4 = (int)(a.B9 + (i64)w9_4);
          pb &= (((true)) && ((true)) && ((true && (r9_4 >= (int)a.CL4 && r9_4 <= (int)a.CH4)))) ? ~0u : ~16u; }
        { const i64 jq5 = ss + (((mtb >> 5) & 1u) ? jl5 : 0);
          const int w8_5 = a.c8[jq5];
          const int r8_5 = (int)w8_5;
          const long long x8_5 = (long long)(a.B8 + (i64)w8_5);
          const short w9_5 = a.c9[jq5];
          const int r9_5 = (int)w9_5;
          const int x9_5 = (int)(a.B9 + (i64)w9_5);
          pb &= (((true)) && ((true)) && ((true && (r9_5 >= (int)a.CL4 && r9_5 <= (int)a.CH4)))) ? ~0u : ~32u; }
        { const i64 jq6 = ss + (((mtb >> 6) & 1u) ? jl6 : 0);
          const int w8_6 = a.c8[jq6];
          const int r8_6 = (int)w8_6;
          const long long x8_6 = (long long)(a.B8 + (i64)w8_6);
          const short w9_6 = a.c9[jq6];
          const int r9_6 = (int)w9_6;
          const int x9_6 = (int)(a.B9 + (i64)w9_6);
          pb &= (((true)) && ((true)) && ((true && (r9_6 >= (int)a.CL4 && r9_6 <= (int)a.CH4)))) ? ~0u : ~64u; }
        { const i64 jq7 = ss + (((mtb >> 7) & 1u) ? jl7 : 0);
          const int w8_7 = a.c8[jq7];
          const int r8_7 = (int)w8_7;
          const long long x8_7 = (long long)(a.B8 + (i64)w8_7);
          const short w9_7 = a.c9[jq7];
          const int r9_7 = (int)w9_7;
          const int x9_7 = (int)(a.B9 + (i64)w9_7);
          pb &= (((true)) && ((true)) && ((true && (r9_7 >= (int)a.CL4 && r9_7 <= (int)a.CH4)))) ? ~0u : ~128u; }
      }
      { unsigned pend = pb;
        while (__any(pend != 0u)) {
          const bool has = pend != 0u;
          const int it = has ? __builtin_ctz(pend) : 0;
          pend &= pend - 1u;
          int jv = jl0;
          jv = it == 1 ? jl1 : jv;
          jv = it == 2 ? jl2 : jv;
          jv = it == 3 ? jl3 : jv;
          jv = it == 4 ? jl4 : jv;
          jv = it == 5 ? jl5 : jv;
          jv = it == 6 ? jl6 : jv;
          jv = it == 7 ? jl7 : jv;
          const u64 bm = __ballot(has);
          const int wp = has ? wcnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u)) : DUMP + cln;
          lrow_s[wv][wp] = (int)(g0 + it); lj_s[wv][wp] = (int)(ss + jv);
          wcnt += __popcll(bm);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          while (wcnt >= 64) {
            const int cb = wcnt > 64 ? wcnt - 64 : 0;
            const int ce = cb + cln;
            bool cok = ce < wcnt;
            const i64 crow = (i64)lrow_s[wv][cok ? ce : cb];
            const i64 cj = (i64)lj_s[wv][cok ? ce : cb];
            const int w2_c = a.c2[crow];
            const int r2_c = (int)w2_c;
            const i64 q2_c = a.B2 + (i64)w2_c;
            const double x2_c = (double)((double)(a.B2 + (i64)w2_c) * a.R2);
            const signed char w3_c = a.c3[crow];
            const int r3_c = (int)w3_c;
            const i64 q3_c = a.B3 + (i64)w3_c;
            const double x3_c = (double)((double)(a.B3 + (i64)w3_c) * a.R3);
            const int w0_c = a.c0[crow];
            const int r0_c = (int)w0_c;
            const long long x0_c = (long long)(a.B0 + (i64)w0_c);
            const short w9_c = a.c9[cj];
            const int r9_c = (int)w9_c;
            const int x9_c = (int)(a.B9 + (i64)w9_c);
            const signed char w10_c = a.c10[cj];
            const int r10_c = (int)w10_c;
            const int x10_c = (int)(a.B10 + (i64)w10_c);
            { const int hln = (int)(threadIdx.x & 63u); const bool hok = cok;
              u64 hk = 0ull; const bool hnul = false;
              hk |= (u64)((i64)x0_c - a.HL0) << (unsigned)a.HS0;
              hk |= (u64)((i64)x9_c - a.HL1) << (unsigned)a.HS1;
              hk |= (u64)((i64)x10_c - a.HL2) << (unsigned)a.HS2;
              const u64 hkp = __shfl_up(hk, 1u, 64);
              const int hfp = __shfl_up((hok ? 1 : 0) | (hnul ? 2 : 0), 1u, 64);
              const bool hsame = hln > 0 && hok && (hfp & 1) != 0 && ((hfp >> 1) & 1) == (hnul ? 1 : 0) && hkp == hk;
              const u64 hH = __ballot(!hsame);
              const int hss = 63 - __builtin_clzll(hH & ((2ull << hln) - 1ull));
              const bool htl = hok && (hln == 63 || ((hH >> ((hln + 1) & 63)) & 1ull) != 0ull);
              const bool hq0 = hok && true;
              double hv0 = hq0 ? (double)((a.A0_0 + a.B0_0 * (double)x2_c) * (a.A0_1 + a.B0_1 * (double)x3_c)) : 0.0;
              #pragma unroll
              for (int hd = 1; hd < 64; hd <<= 1) {
                const double u_hv0 = __shfl_up(hv0, (unsigned)hd, 64);
                if (hln - hd >= hss) {
                  hv0 = hv0 + u_hv0;
                }
              }
              if (htl) {
                long long hs_ = -1;
                if (hnul) hs_ = a.HM + 1; else if (hk == ~0ull) hs_ = a.HM; else {
                  u64 hh = hs_mix64(hk) & (u64)(a.HM - 1);
                  for (int pr_ = 0; pr_ < 512; ++pr_) {
                    const u64 pv_ = atomicCAS(&a.hkeys[hh], ~0ull, hk);
                    if (pv_ == ~0ull || pv_ == hk) { hs_ = (long long)hh; break; }
                    hh = (hh + 1ull) & (u64)(a.HM - 1);
                  }
                  if (hs_ < 0) a.hflag[0] = 1;
                }
                if (hs_ >= 0) {
                  const long long hst = a.HM + 2;   // SoA: aggregate i of slot s at i * (M + 2) + s
                  const unsigned long long hrn = (unsigned long long)(hln - hss + 1);
                  unsafeAtomicAdd(&a.hsum[0 * hst + hs_], hv0);
                  if (hs_ >= a.HM) atomicAdd((unsigned long long*)&a.hcnt[1 * hst + hs_], hrn);
                }
              }
            }
            wcnt = cb;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          }
        }
      }
      }
    }
    __syncthreads();
    } else {
    int x0v[8];
    x0v[0] = act0 ? a.c0[g0 + 0] : (int)0; x0v[1] = act1 ? a.c0[g0 + 1] : (int)0; x0v[2] = act2 ? a.c0[g0 + 2] : (int)0; x0v[3] = act3 ? a.c0[g0 + 3] : (int)0; x0v[4] = act4 ? a.c0[g0 + 4] : (int)0; x0v[5] = act5 ? a.c0[g0 + 5] : (int)0; x0v[6] = act6 ? a.c0[g0 + 6] : (int)0; x0v[7] = act7 ? a.c0[g0 + 7] : (int)0;
    short x1v[8];
    x1v[0] = act0 ? a.c1[g0 + 0] : (short)0; x1v[1] = act1 ? a.c1[g0 + 1] : (short)0; x1v[2] = act2 ? a.c1[g0 + 2] : (short)0; x1v[3] = act3 ? a.c1[g0 + 3] : (short)0; x1v[4] = act4 ? a.c1[g0 + 4] : (short)0; x1v[5] = act5 ? a.c1[g0 + 5] : (short)0; x1v[6] = act6 ? a.c1[g0 + 6] : (short)0; x1v[7] = act7 ? a.c1[g0 + 7] : (short)0;
    const i64 ss = a.spans[4 * t + 2], se = a.spans[4 * t + 3];
    const int ns = (int)(se - ss);
    const bool staged = ns <= 2048;
    unsigned* const skeys = skeys_[0];
    unsigned char* const spass = spass_[0];
    if (staged) for (int sqb = 0; sqb < ns; sqb += 1024) {
      const int sq0 = sqb + 0 + (int)threadIdx.x;
      const bool sv0 = sq0 < ns;
      const i64 jr0 = ss + (sv0 ? sq0 : 0);
      const int sq1 = sqb + 256 + (int)threadIdx.x;
      const bool sv1 = sq1 < ns;
      const i64 jr1 = ss + (sv1 ? sq1 : 0);
      const int sq2 = sqb + 512 + (int)threadIdx.x;
      const bool sv2 = sq2 < ns;
      const i64 jr2 = ss + (sv2 ? sq2 : 0);
      const int sq3 = sqb + 768 + (int)threadIdx.x;
      const bool sv3 = sq3 < ns;
      const i64 jr3 = ss + (sv3 ? sq3 : 0);
      const int w8_s0 = a.c8[jr0];
      const int r8_s0 = (int)w8_s0;
      const long long x8_s0 = (long long)(a.B8 + (i64)w8_s0);
      const short w9_s0 = a.c9[jr0];
      const int r9_s0 = (int)w9_s0;
      const int x9_s0 = (int)(a.B9 + (i64)w9_s0);
      const int w8_s1 = a.c8[jr1];
      const int r8_s1 = (int)w8_s1;
      const long long x8_s1 = (long long)(a.B8 + (i64)w8_s1);
      const short w9_s1 = a.c9[jr1];
      const int r9_s1 = (int)w9_s1;
      const int x9_s1 = (int)(a.B9 + (i64)w9_s1);
      const int w8_s2 = a.c8[jr2];
      const int r8_s2 = (int)w8_s2;
      const long long x8_s2 = (long long)(a.B8 + (i64)w8_s2);
      const short w9_s2 = a.c9[jr2];
      const int r9_s2 = (int)w9_s2;
      const int x9_s2 = (int)(a.B9 + (i64)w9_s2);
      const int w8_s3 = a.c8[jr3];
      const int r8_s3 = (int)w8_s3;
      const long long x8_s3 = (long long)(a.B8 + (i64)w8_s3);
      const short w9_s3 = a.c9[jr3];
      const int r9_s3 = (int)w9_s3;
      const int x9_s3 = (int)(a.B9 + (i64)w9_s3);
      if (sv0) { const bool kv = true;
        skeys[sq0] = kv ? ({ const i64 d_ = (i64)(x8_s0) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) : (unsigned)0;
        spass[sq0] = (kv && ((true)) && ((true)) && ((true && (r9_s0 >= (int)a.CL4 && r9_s0 <= (int)a.CH4)))) ? 1 : 0;
      }
      if (sv1) { const bool kv = true;
        skeys[sq1] = kv ? ({ const i64 d_ = (i64)(x8_s1) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) : (unsigned)0;
        spass[sq1] = (kv && ((true)) && ((true)) && ((true && (r9_s1 >= (int)a.CL4 && r9_s1 <= (int)a.CH4)))) ? 1 : 0;
      }
      if (sv2) { const bool kv = true;
        skeys[sq2] = kv ? ({ const i64 d_ = (i64)(x8_s2) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) : (unsigned)0;
        spass[sq2] = (kv && ((true)) && ((true)) && ((true && (r9_s2 >= (int)a.CL4 && r9_s2 <= (int)a.CH4)))) ? 1 : 0;
      }
      if (sv3) { const bool kv = true;
        skeys[sq3] = kv ? ({ const i64 d_ = (i64)(x8_s3) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) : (unsigned)0;
        spass[sq3] = (kv && ((true)) && ((true)) && ((true && (r9_s3 >= (int)a.CL4 && r9_s3 <= (int)a.CH4)))) ? 1 : 0;
      }
    }
    if (staged && threadIdx.x == 0) skeys[ns] = 0xFFFFFFFFu;   // walk sentinel
    const int r0_0 = (int)x0v[0];
    const long long x0_0 = (long long)(a.B0 + (i64)x0v[0]);
    const int r1_0 = (int)x1v[0];
    const int x1_0 = (int)(a.B1 + (i64)x1v[0]);
    const int r0_1 = (int)x0v[1];
    const long long x0_1 = (long long)(a.B0 + (i64)x0v[1]);
    const int r1_1 = (int)x1v[1];
    const int x1_1 = (int)(a.B1 + (i64)x1v[1]);
    const int r0_2 = (int)x0v[2];
    const long long x0_2 = (long long)(a.B0 + (i64)x0v[2]);
    const int r1_2 = (int)x1v[2];
    const int x1_2 = (int)(a.B1 + (i64)x1v[2]);
    const int r0_3 = (int)x0v[3];
    const long long x0_3 = (long long)(a.B0 + (i64)x0v[3]);
    const int r1_3 = (int)x1v[3];
    const int x1_3 = (int)(a.B1 + (i64)x1v[3]);
    const int r0_4 = (int)x0v[4];
    const long long x0_4 = (long long)(a.B0 + (i64)x0v[4]);
    const int r1_4 = (int)x1v[4];
    const int x1_4 = (int)(a.B1 + (i64)x1v[4]);
    const int r0_5 = (int)x0v[5];
    const long long x0_5 = (long long)(a.B0 + (i64)x0v[5]);
    const int r1_5 = (int)x1v[5];
    const int x1_5 = (int)(a.B1 + (i64)x1v[5]);
    const int r0_6 = (int)x0v[6];
    const long long x0_6 = (long long)(a.B0 + (i64)x0v[6]);
    const int r1_6 = (int)x1v[6];
    const int x1_6 = (int)(a.B1 + (i64)x1v[6]);
    const int r0_7 = (int)x0v[7];
    const long long x0_7 = (long long)(a.B0 + (i64)x0v[7]);
    const int r1_7 = (int)x1v[7];
    const int x1_7 = (int)(a.B1 + (i64)x1v[7]);
    unsigned kvb = 0u, mb = 0u;
    { const bool kv = act0 && true; kvb |= kv ? 1u : 0u; mb |= (kv && ((true)) && ((true && (r1_0 >= (int)a.CL1 && r1_0 <= (int)a.CH1)))) ? 1u : 0u; }
    const unsigned k0 = ((unsigned)x0v[0] + (unsigned)a.KOF);
    { const bool kv = act1 && true; kvb |= kv ? 2u : 0u; mb |= (kv && ((true)) && ((true && (r1_1 >= (int)a.CL1 && r1_1 <= (int)a.CH1)))) ? 2u : 0u; }
    const unsigned k1 = ((unsigned)x0v[1] + (unsigned)a.KOF);
    { const bool kv = act2 && true; kvb |= kv ? 4u : 0u; mb |= (kv && ((true)) && ((true && (r1_2 >= (int)a.CL1 && r1_2 <= (int)a.CH1)))) ? 4u : 0u; }
    const unsigned k2 = ((unsigned)x0v[2] + (unsigned)a.KOF);
    { const bool kv = act3 && true; kvb |= kv ? 8u : 0u; mb |= (kv && ((true)) && ((true && (r1_3 >= (int)a.CL1 && r1_3 <= (int)a.CH1)))) ? 8u : 0u; }
    const unsigned k3 = ((unsigned)x0v[3] + (unsigned)a.KOF);
    { const bool kv = act4 && true; kvb |= kv ? 16u : 0u; mb |= (kv && ((true)) && ((true && (r1_4 >= (int)a.CL1 && r1_4 <= (int)a.CH1)))) ? 16u : 0u; }
    const unsigned k4 = ((unsigned)x0v[4] + (unsigned)a.KOF);
    { const bool kv = act5 && true; kvb |= kv ? 32u : 0u; mb |= (kv && ((true)) && ((true && (r1_5 >= (int)a.CL1 && r1_5 <= (int)a.CH1)))) ? 32u : 0u; }
    const unsigned k5 = ((unsigned)x0v[5] + (unsigned)a.KOF);
    { const bool kv = act6 && true; kvb |= kv ? 64u : 0u; mb |= (kv && ((true)) && ((true && (r1_6 >= (int)a.CL1 && r1_6 <= (int)a.CH1)))) ? 64u : 0u; }
    const unsigned k6 = ((unsigned)x0v[6] + (unsigned)a.KOF);
    { const bool kv = act7 && true; kvb |= kv ? 128u : 0u; mb |= (kv && ((true)) && ((true && (r1_7 >= (int)a.CL1 && r1_7 <= (int)a.CH1)))) ? 128u : 0u; }
    const unsigned k7 = ((unsigned)x0v[7] + (unsigned)a.KOF);
    __syncthreads();
    unsigned kf = 0xFFFFFFFFu;
    kf = ((mb >> 7) & 1u) ? k7 : kf;
    kf = ((mb >> 6) & 1u) ? k6 : kf;
    kf = ((mb >> 5) & 1u) ? k5 : kf;
    kf = ((mb >> 4) & 1u) ? k4 : kf;
    kf = ((mb >> 3) & 1u) ? k3 : kf;
    kf = ((mb >> 2) & 1u) ? k2 : kf;
    kf = ((mb >> 1) & 1u) ? k1 : kf;
    kf = ((mb >> 0) & 1u) ? k0 : kf;
    unsigned mtb = 0u;
    int jl0 = 0;
    int jl1 = 0;
    int jl2 = 0;
    int jl3 = 0;
    int jl4 = 0;
    int jl5 = 0;
    int jl6 = 0;
    int jl7 = 0;
    bool slow = !staged;
    int jw0 = 0;
    if (staged) {
      int lo = 0;
      for (int st = ns > 0 ? (1 << (31 - __builtin_clz(ns))) : 0; st > 0; st >>= 1) {
        const int c = lo + st; const unsigned sv = skeys[c <= ns ? c - 1 : ns];
        lo = (c <= ns && sv < kf) ? c : lo; }
      jw0 = lo; int jw = lo; unsigned v = skeys[jw];
      { const unsigned ke = ((kvb >> 0) & 1u) ? k0 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 0) & 1u) && v == ke && jw < ns) ? 1u : 0u; jl0 = jw; }
      { const unsigned ke = ((kvb >> 1) & 1u) ? k1 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 1) & 1u) && v == ke && jw < ns) ? 2u : 0u; jl1 = jw; }
      { const unsigned ke = ((kvb >> 2) & 1u) ? k2 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 2) & 1u) && v == ke && jw < ns) ? 4u : 0u; jl2 = jw; }
      { const unsigned ke = ((kvb >> 3) & 1u) ? k3 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 3) & 1u) && v == ke && jw < ns) ? 8u : 0u; jl3 = jw; }
      { const unsigned ke = ((kvb >> 4) & 1u) ? k4 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 4) & 1u) && v == ke && jw < ns) ? 16u : 0u; jl4 = jw; }
      { const unsigned ke = ((kvb >> 5) & 1u) ? k5 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 5) & 1u) && v == ke && jw < ns) ? 32u : 0u; jl5 = jw; }
      { const unsigned ke = ((kvb >> 6) & 1u) ? k6 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 6) & 1u) && v == ke && jw < ns) ? 64u : 0u; jl6 = jw; }
      { const unsigned ke = ((kvb >> 7) & 1u) ? k7 : (unsigned)0;
        { const bool c = v < ke; jw += c ? 1 : 0; v = skeys[jw]; }
        slow = slow || v < ke;
        mtb |= (((mb >> 7) & 1u) && v == ke && jw < ns) ? 128u : 0u; jl7 = jw; }
    }
    if (__any(slow)) {
      if (slow) { int jw = jw0; mtb = 0u;
        if (((mb >> 0) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k0) ++jw;
            hit = jw < ns && skeys[jw] == k0; jl0 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k0) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k0; jl0 = (int)(lo - ss); }
          mtb |= hit ? 1u : 0u;
        }
        if (((mb >> 1) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k1) ++jw;
            hit = jw < ns && skeys[jw] == k1; jl1 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k1) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k1; jl1 = (int)(lo - ss); }
          mtb |= hit ? 2u : 0u;
        }
        if (((mb >> 2) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k2) ++jw;
            hit = jw < ns && skeys[jw] == k2; jl2 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k2) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k2; jl2 = (int)(lo - ss); }
          mtb |= hit ? 4u : 0u;
        }
        if (((mb >> 3) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k3) ++jw;
            hit = jw < ns && skeys[jw] == k3; jl3 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k3) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k3; jl3 = (int)(lo - ss); }
          mtb |= hit ? 8u : 0u;
        }
        if (((mb >> 4) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k4) ++jw;
            hit = jw < ns && skeys[jw] == k4; jl4 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k4) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k4; jl4 = (int)(lo - ss); }
          mtb |= hit ? 16u : 0u;
        }
        if (((mb >> 5) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k5) ++jw;
            hit = jw < ns && skeys[jw] == k5; jl5 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k5) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k5; jl5 = (int)(lo - ss); }
          mtb |= hit ? 32u : 0u;
        }
        if (((mb >> 6) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k6) ++jw;
            hit = jw < ns && skeys[jw] == k6; jl6 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k6) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k6; jl6 = (int)(lo - ss); }
          mtb |= hit ? 64u : 0u;
        }
        if (((mb >> 7) & 1u)) { bool hit;
          if (staged) { while (jw < ns && skeys[jw] < k7) ++jw;
            hit = jw < ns && skeys[jw] == k7; jl7 = jw; }
          else { i64 lo = ss, hi = se;
            while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < k7) lo = md + 1; else hi = md; }
            hit = lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k7; jl7 = (int)(lo - ss); }
          mtb |= hit ? 128u : 0u;
        }
      }
    }
    { unsigned pb = mtb;
    if (staged) {
      pb &= spass[((mtb >> 0) & 1u) ? jl0 : 0] != 0 ? ~0u : ~1u;
      pb &= spass[((mtb >> 1) & 1u) ? jl1 : 0] != 0 ? ~0u : ~2u;
      pb &= spass[((mtb >> 2) & 1u) ? jl2 : 0] != 0 ? ~0u : ~4u;
      pb &= spass[((mtb >> 3) & 1u) ? jl3 : 0] != 0 ? ~0u : ~8u;
      pb &= spass[((mtb >> 4) & 1u) ? jl4 : 0] != 0 ? ~0u : ~16u;
      pb &= spass[((mtb >> 5) & 1u) ? jl5 : 0] != 0 ? ~0u : ~32u;
      pb &= spass[((mtb >> 6) & 1u) ? jl6 : 0] != 0 ? ~0u : ~64u;
      pb &= spass[((mtb >> 7) & 1u) ? jl7 : 0] != 0 ? ~0u : ~128u;
    } else {
      { const i64 jq0 = ss + (((mtb >> 0) & 1u) ? jl0 : 0);
        const int w8_0 = a.c8[jq0];
        const int r8_0 = (int)w8_0;
        const long long x8_0 = (long long)(a.B8 + (i64)w8_0);
        const short w9_0 = a.c9[jq0];
        const int r9_0 = (int)w9_0;
        const int x9_0 = (int)(a.B9 + (i64)w9_0);
        pb &= (((true)) && ((true)) && ((true && (r9_0 >= (int)a.CL4 && r9_0 <= (int)a.CH4)))) ? ~0u : ~1u; }
      { const i64 jq1 = ss + (((mtb >> 1) & 1u) ? jl1 : 0);
        const int w8_1 = a.c8[jq1];
        const int r8_1 = (int)w8_1;
        const long long x8_1 = (long long)(a.B8 + (i64)w8_1);
        const short w9_1 = a.c9[jq1];
        const int r9_1 = (int)w9_1;
        const int x9_1 = (int)(a.B9 + (i64)w9_1);
        pb &= (((true)) && ((true)) && ((true && (r9_1 >= (int)a.CL4 && r9_1 <= (int)a.CH4)))) ? ~0u : ~2u; }
      { const i64 jq2 = ss + (((mtb >> 2) & 1u) ? jl2 : 0);
        const int w8_2 = a.c8[jq2];
        const int r8_2 = (int)w8_2;
        const long long x8_2 = (long long)(a.B8 + (i64)w8_2);
        const short w9_2 = a.c9[jq2];
        const int r9_2 = (int)w9_2;
        const int x9_2 = (int)(a.B9 + (i64)w9_2);
        pb &= (((true)) && ((true)) && ((true && (r9_2 >= (int)a.CL4 && r9_2 <= (int)a.CH4)))) ? ~0u : ~4u; }
      { const i64 jq3 = ss + (((mtb >> 3) & 1u) ? jl3 : 0);
        const int w8_3 = a.c8[jq3];
        const int r8_3 = (int)w8_3;
        const long long x8_3 = (long long)(a.B8 + (i64)w8_3);
        const short w9_3 = a.c9[jq3];
        const int r9_3 = (int)w9_3;
        const int x9_3 = (int)(a.B9 + (i64)w9_3);
        pb &= (((true)) && ((true)) && ((true && (r9_3 >= (int)a.CL4 && r9_3 <= (int)a.CH4)))) ? ~0u : ~8u; }
      { const i64 jq4 = ss + (((mtb >> 4) & 1u) ? jl4 : 0);
        const int w8_4 = a.c8[jq4];
        const int r8_4 = (int)w8_4;
        const long long x8_4 = (long long)(a.B8 + (i64)w8_4);
        const short w9_4 = a.c9[jq4];
        const int r9_4 = (int)w9_4;
        const int x9_4 = (int)(a.B9 + (i64)w9_4);
        pb &= (((true)) && ((true)) && ((true && (r9_4 >= (int)a.CL4 && r9_4 <= (int)a.CH4)))) ? ~0u : ~16u; }
      { const i64 jq5 = ss + (((mtb >> 5) & 1u) ? jl5 : 0);
        const int w8_5 = a.c8[jq5];
        const int r8_5 = (int)w8_5;
        const long long x8_5 = (long long)(a.B8 + (i64)w8_5);
        const short w9_5 = a.c9[jq5];
        const int r9_5 = (int)w9_5;
        const int x9_5 = (int)(a.B9 + (i64)w9_5);
        pb &= (((true)) && ((true)) && ((true && (r9_5 >= (int)a.CL4 && r9_5 <= (int)a.CH4)))) ? ~0u : ~32u; }
      { const i64 jq6 = ss + (((mtb >> 6) & 1u) ? jl6 : 0);
        const int w8_6 = a.c8[jq6];
        const int r8_6 = (int)w8_6;
        const long long x8_6 = (long long)(a.B8 + (i64)w8_6);
        const short w9_6 = a.c9[jq6];
        const int r9_6 = (int)w9_6;
        const int x9_6 = (int)(a.B9 + (i64)w9_6);
        pb &= (((true)) && ((true)) && ((true && (r9_6 >= (int)a.CL4 && r9_6 <= (int)a.CH4)))) ? ~0u : ~64u; }
      { const i64 jq7 = ss + (((mtb >> 7) & 1u) ? jl7 : 0);
        const int w8_7 = a.c8[jq7];
        const int r8_7 = (int)w8_7;
        const long long x8_7 = (long long)(a.B8 + (i64)w8_7);
        const short w9_7 = a.c9[jq7];
        const int r9_7 = (int)w9_7;
        const int x9_7 = (int)(a.B9 + (i64)w9_7);
        pb &= (((true)) && ((true)) && ((true && (r9_7 >= (int)a.CL4 && r9_7 <= (int)a.CH4)))) ? ~0u : ~128u; }
    }
    { unsigned pend = pb;
      while (__any(pend != 0u)) {
        const bool has = pend != 0u;
        const int it = has ? __builtin_ctz(pend) : 0;
        pend &= pend - 1u;
        int jv = jl0;
        jv = it == 1 ? jl1 : jv;
        jv = it == 2 ? jl2 : jv;
        jv = it == 3 ? jl3 : jv;
        jv = it == 4 ? jl4 : jv;
        jv = it == 5 ? jl5 : jv;
        jv = it == 6 ? jl6 : jv;
        jv = it == 7 ? jl7 : jv;
        const u64 bm = __ballot(has);
        const int wp = has ? wcnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u)) : DUMP + cln;
        lrow_s[wv][wp] = (int)(g0 + it); lj_s[wv][wp] = (int)(ss + jv);
        wcnt += __popcll(bm);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        while (wcnt >= 64) {
          const int cb = wcnt > 64 ? wcnt - 64 : 0;
          const int ce = cb + cln;
          bool cok = ce < wcnt;
          const i64 crow = (i64)lrow_s[wv][cok ? ce : cb];
          const i64 cj = (i64)lj_s[wv][cok ? ce : cb];
          const int w2_c = a.c2[crow];
          const int r2_c = (int)w2_c;
          const i64 q2_c = a.B2 + (i64)w2_c;
          const double x2_c = (double)((double)(a.B2 + (i64)w2_c) * a.R2);
          const signed char w3_c = a.c3[crow];
          const int r3_c = (int)w3_c;
          const i64 q3_c = a.B3 + (i64)w3_c;
          const double x3_c = (double)((double)(a.B3 + (i64)w3_c) * a.R3);
          const int w0_c = a.c0[crow];
          const int r0_c = (int)w0_c;
          const long long x0_c = (long long)(a.B0 + (i64)w0_c);
          const short w9_c = a.c9[cj];
          const int r9_c = (int)w9_c;
          const int x9_c = (int)(a.B9 + (i64)w9_c);
          const signed char w10_c = a.c10[cj];
          const int r10_c = (int)w10_c;
          const int x10_c = (int)(a.B10 + (i64)w10_c);
          { const int hln = (int)(threadIdx.x & 63u); const bool hok = cok;
            u64 hk = 0ull; const bool hnul = false;
            hk |= (u64)((i64)x0_c - a.HL0) << (unsigned)a.HS0;
            hk |= (u64)((i64)x9_c - a.HL1) << (unsigned)a.HS1;
            hk |= (u64)((i64)x10_c - a.HL2) << (unsigned)a.HS2;
            const u64 hkp = __shfl_up(hk, 1u, 64);
            const int hfp = __shfl_up((hok ? 1 : 0) | (hnul ? 2 : 0), 1u, 64);
            const bool hsame = hln > 0 && hok && (hfp & 1) != 0 && ((hfp >> 1) & 1) == (hnul ? 1 : 0) && hkp == hk;
            const u64 hH = __ballot(!hsame);
            const int hss = 63 - __builtin_clzll(hH & ((2ull << hln) - 1ull));
            const bool htl = hok && (hln == 63 || ((hH >> ((hln + 1) & 63)) & 1ull) != 0ull);
            const bool hq0 = hok && true;
            double hv0 = hq0 ? (double)((a.A0_0 + a.B0_0 * (double)x2_c) * (a.A0_1 + a.B0_1 * (double)x3_c)) : 0.0;
            #pragma unroll
            for (int hd = 1; hd < 64; hd <<= 1) {
              const double u_hv0 = __shfl_up(hv0, (unsigned)hd, 64);
              if (hln - hd >= hss) {
                hv0 = hv0 + u_hv0;
              }
            }
            if (htl) {
              long long hs_ = -1;
              if (hnul) hs_ = a.HM + 1; else if (hk == ~0ull) hs_ = a.HM; else {
                u64 hh = hs_mix64(hk) & (u64)(a.HM - 1);
                for (int pr_ = 0; pr_ < 512; ++pr_) {
                  const u64 pv_ = atomicCAS(&a.hkeys[hh], ~0ull, hk);
                  if (pv_ == ~0ull || pv_ == hk) { hs_ = (long long)hh; break; }
                  hh = (hh + 1ull) & (u64)(a.HM - 1);
                }
                if (hs_ < 0) a.hflag[0] = 1;
              }
              if (hs_ >= 0) {
                const long long hst = a.HM + 2;   // SoA: aggregate i of slot s at i * (M + 2) + s
                const unsigned long long hrn = (unsigned long long)(hln - hss + 1);
                unsafeAtomicAdd(&a.hsum[0 * hst + hs_], hv0);
                if (hs_ >= a.HM) atomicAdd((unsigned long long*)&a.hcnt[1 * hst + hs_], hrn);
              }
            }
          }
          wcnt = cb;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        }
      }
    }
    }
    if (a.rdup) while (true) {
      if (((mtb >> 0) & 1u)) { ++jl0;
        const bool more = jl0 < ns && (staged ? skeys[jl0] == k0 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl0)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k0));
        if (!more) mtb &= ~1u; }
      if (((mtb >> 1) & 1u)) { ++jl1;
        const bool more = jl1 < ns && (staged ? skeys[jl1] == k1 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl1)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k1));
        if (!more) mtb &= ~2u; }
      if (((mtb >> 2) & 1u)) { ++jl2;
        const bool more = jl2 < ns && (staged ? skeys[jl2] == k2 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl2)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k2));
        if (!more) mtb &= ~4u; }
      if (((mtb >> 3) & 1u)) { ++jl3;
        const bool more = jl3 < ns && (staged ? skeys[jl3] == k3 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl3)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k3));
        if (!more) mtb &= ~8u; }
      if (((mtb >> 4) & 1u)) { ++jl4;
        const bool more = jl4 < ns && (staged ? skeys[jl4] == k4 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl4)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k4));
        if (!more) mtb &= ~16u; }
      if (((mtb >> 5) & 1u)) { ++jl5;
        const bool more = jl5 < ns && (staged ? skeys[jl5] == k5 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl5)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k5));
        if (!more) mtb &= ~32u; }
      if (((mtb >> 6) & 1u)) { ++jl6;
        const bool more = jl6 < ns && (staged ? skeys[jl6] == k6 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl6)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k6));
        if (!more) mtb &= ~64u; }
      if (((mtb >> 7) & 1u)) { ++jl7;
        const bool more = jl7 < ns && (staged ? skeys[jl7] == k7 : (!(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[(ss + jl7)])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == k7));
        if (!more) mtb &= ~128u; }
      if (!__any(mtb != 0u)) break;
      { unsigned pb = mtb;
      if (staged) {
        pb &= spass[((mtb >> 0) & 1u) ? jl0 : 0] != 0 ? ~0u : ~1u;
        pb &= spass[((mtb >> 1) & 1u) ? jl1 : 0] != 0 ? ~0u : ~2u;
        pb &= spass[((mtb >> 2) & 1u) ? jl2 : 0] != 0 ? ~0u : ~4u;
        pb &= spass[((mtb >> 3) & 1u) ? jl3 : 0] != 0 ? ~0u : ~8u;
        pb &= spass[((mtb >> 4) & 1u) ? jl4 : 0] != 0 ? ~0u : ~16u;
        pb &= spass[((mtb >> 5) & 1u) ? jl5 : 0] != 0 ? ~0u : ~32u;
        pb &= spass[((mtb >> 6) & 1u) ? jl6 : 0] != 0 ? ~0u : ~64u;
        pb &= spass[((mtb >> 7) & 1u) ? jl7 : 0] != 0 ? ~0u : ~128u;
      } else {
        { const i64 jq0 = ss + (((mtb >> 0) & 1u) ? jl0 : 0);
          const int w8_0 = a.c8[jq0];
          const int r8_0 = (int)w8_0;
          const long long x8_0 = (long long)(a.B8 + (i64)w8_0);
          const short w9_0 = a.c9[jq0];
          const int r9_0 = (int)w9_0;
          const int x9_0 = (int)(a.B9 + (i64)w9_0);
          pb &= (((true)) && ((true)) && ((true && (r9_0 >= (int)a.CL4 && r9_0 <= (int)a.CH4)))) ? ~0u : ~1u; }
        { const i64 jq1 = ss + (((mtb >> 1) & 1u) ? jl1 : 0);
          const int w8_1 = a.c8[jq1];
          const int r8_1 = (int)w8_1;
          const long long x8_1 = (long long)(a.B8 + (i64)w8_1);
          const short w9_1 = a.c9[jq1];
          const int r9_1 = (int)w9_1;
          const int x9_1 = (int)(a.B9 + (i64)w9_1);
          pb &= (((true)) && ((true)) && ((true && (r9_1 >= (int)a.CL4 && r9_1 <= (int)a.CH4)))) ? ~0u : ~2u; }
        { const i64 jq2 = ss + (((mtb >> 2) & 1u) ? jl2 : 0);
          const int w8_2 = a.c8[jq2];
          const int r8_2 = (int)w8_2;
          const long long x8_2 = (long long)(a.B8 + (i64)w8_2);
          const short w9_2 = a.c9[jq2];
          const int r9_2 = (int)w9_2;
          const int x9_2 = (int)(a.B9 + (i64)w9_2);
          pb &= (((true)) && ((true)) && ((true && (r9_2 >= (int)a.CL4 && r9_2 <= (int)a.CH4)))) ? ~0u : ~4u; }
        { const i64 jq3 = ss + (((mtb >> 3) & 1u) ? jl3 : 0);
          const int w8_3 = a.c8[jq3];
          const int r8_3 = (int)w8_3;
          const long long x8_3 = (long long)(a.B8 + (i64)w8_3);
          const short w9_3 = a.c9[jq3];
          const int r9_3 = (int)w9_3;
          const int x9_3 = (int)(a.B9 + (i64)w9_3);
          pb &= (((true)) && ((true)) && ((true && (r9_3 >= (int)a.CL4 && r9_3 <= (int)a.CH4)))) ? ~0u : ~8u; }
        { const i64 jq4 = ss + (((mtb >> 4) & 1u) ? jl4 : 0);
          const int w8_4 = a.c8[jq4];
          const int r8_4 = (int)w8_4;
          const long long x8_4 = (long long)(a.B8 + (i64)w8_4);
          const short w9_4 = a.c9[jq4];
          const int r9_4 = (int)w9_4;
          const int x9_4 = (int)(a.B9 + (i64)w9_4);
          pb &= (((true)) && ((true)) && ((true && (r9_4 >= (int)a.CL4 && r9_4 <= (int)a.CH4)))) ? ~0u : ~16u; }
        { const i64 jq5 = ss + (((mtb >> 5) & 1u) ? jl5 : 0);
          const int w8_5 = a.c8[jq5];
          const int r8_5 = (int)w8_5;
          const long long x8_5 = (long long)(a.B8 + (i64)w8_5);
          const short w9_5 = a.c9[jq5];
          const int r9_5 = (int)w9_5;
          const int x9_5 = (int)(a.B9 + (i64)w9_5);
          pb &= (((true)) && ((true)) && ((true && (r9_5 >= (int)a.CL4 && r9_5 <= (int)a.CH4)))) ? ~0u : ~32u; }
        { const i64 jq6 = ss + (((mtb >> 6) & 1u) ? jl6 : 0);
          const int w8_6 = a.c8[jq6];
          const int r8_6 = (int)w8_6;
          const long long x8_6 = (long long)(a.B8 + (i64)w8_6);
          const short w9_6 = a.c9[jq6];
          const int r9_6 = (int)w9_6;
          const int x9_6 = (int)(a.B9 + (i64)w9_6);
          pb &= (((true)) && ((true)) && ((true && (r9_6 >= (int)a.CL4 && r9_6 <= (int)a.CH4)))) ? ~0u : ~64u; }
        { const i64 jq7 = ss + (((mtb >> 7) & 1u) ? jl7 : 0);
          const int w8_7 = a.c8[jq7];
          const int r8_7 = (int)w8_7;
          const long long x8_7 = (long long)(a.B8 + (i64)w8_7);
          const short w9_7 = a.c9[jq7];
          const int r9_7 = (int)w9_7;
          const int x9_7 = (int)(a.B9 + (i64)w9_7);
          pb &= (((true)) && ((true)) && ((true && (r9_7 >= (int)a.CL4 && r9_7 <= (int)a.CH4)))) ? ~0u : ~128u; }
      }
      { unsigned pend = pb;
        while (__any(pend != 0u)) {
          const bool has = pend != 0u;
          const int it = has ? __builtin_ctz(pend) : 0;
          pend &= pend - 1u;
          int jv = jl0;
          jv = it == 1 ? jl1 : jv;
          jv = it == 2 ? jl2 : jv;
          jv = it == 3 ? jl3 : jv;
          jv = it == 4 ? jl4 : jv;
          jv = it == 5 ? jl5 : jv;
          jv = it == 6 ? jl6 : jv;
          jv = it == 7 ? jl7 : jv;
          const u64 bm = __ballot(has);
          const int wp = has ? wcnt + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bm >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bm, 0u)) : DUMP + cln;
          lrow_s[wv][wp] = (int)(g0 + it); lj_s[wv][wp] = (int)(ss + jv);
          wcnt += __popcll(bm);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          while (wcnt >= 64) {
            const int cb = wcnt > 64 ? wcnt - 64 : 0;
            const int ce = cb + cln;
            bool cok = ce < wcnt;
            const i64 crow = (i64)lrow_s[wv][cok ? ce : cb];
            const i64 cj = (i64)lj_s[wv][cok ? ce : cb];
            const int w2_c = a.c2[crow];
            const int r2_c = (int)w2_c;
            const i64 q2_c = a.B2 + (i64)w2_c;
            const double x2_c = (double)((double)(a.B2 + (i64)w2_c) * a.R2);
            const signed char w3_c = a.c3[crow];
            const int r3_c = (int)w3_c;
            const i64 q3_c = a.B3 + (i64)w3_c;
            const double x3_c = (double)((double)(a.B3 + (i64)w3_c) * a.R3);
            const int w0_c = a.c0[crow];
            const int r0_c = (int)w0_c;
            const long long x0_c = (long long)(a.B0 + (i64)w0_c);
            const short w9_c = a.c9[cj];
            const int r9_c = (int)w9_c;
            const int x9_c = (int)(a.B9 + (i64)w9_c);
            const signed char w10_c = a.c10[cj];
            const int r10_c = (int)w10_c;
            const int x10_c = (int)(a.B10 + (i64)w10_c);
            { const int hln = (int)(threadIdx.x & 63u); const bool hok = cok;
              u64 hk = 0ull; const bool hnul = false;
              hk |= (u64)((i64)x0_c - a.HL0) << (unsigned)a.HS0;
              hk |= (u64)((i64)x9_c - a.HL1) << (unsigned)a.HS1;
              hk |= (u64)((i64)x10_c - a.HL2) << (unsigned)a.HS2;
              const u64 hkp = __shfl_up(hk, 1u, 64);
              const int hfp = __shfl_up((hok ? 1 : 0) | (hnul ? 2 : 0), 1u, 64);
              const bool hsame = hln > 0 && hok && (hfp & 1) != 0 && ((hfp >> 1) & 1) == (hnul ? 1 : 0) && hkp == hk;
              const u64 hH = __ballot(!hsame);
              const int hss = 63 - __builtin_clzll(hH & ((2ull << hln) - 1ull));
              const bool htl = hok && (hln == 63 || ((hH >> ((hln + 1) & 63)) & 1ull) != 0ull);
              const bool hq0 = hok && true;
              double hv0 = hq0 ? (double)((a.A0_0 + a.B0_0 * (double)x2_c) * (a.A0_1 + a.B0_1 * (double)x3_c)) : 0.0;
              #pragma unroll
              for (int hd = 1; hd < 64; hd <<= 1) {
                const double u_hv0 = __shfl_up(hv0, (unsigned)hd, 64);
                if (hln - hd >= hss) {
                  hv0 = hv0 + u_hv0;
                }
              }
              if (htl) {
                long long hs_ = -1;
                if (hnul) hs_ = a.HM + 1; else if (hk == ~0ull) hs_ = a.HM; else {
                  u64 hh = hs_mix64(hk) & (u64)(a.HM - 1);
                  for (int pr_ = 0; pr_ < 512; ++pr_) {
                    const u64 pv_ = atomicCAS(&a.hkeys[hh], ~0ull, hk);
                    if (pv_ == ~0ull || pv_ == hk) { hs_ = (long long)hh; break; }
                    hh = (hh + 1ull) & (u64)(a.HM - 1);
                  }
                  if (hs_ < 0) a.hflag[0] = 1;
                }
                if (hs_ >= 0) {
                  const long long hst = a.HM + 2;   // SoA: aggregate i of slot s at i * (M + 2) + s
                  const unsigned long long hrn = (unsigned long long)(hln - hss + 1);
                  unsafeAtomicAdd(&a.hsum[0 * hst + hs_], hv0);
                  if (hs_ >= a.HM) atomicAdd((unsigned long long*)&a.hcnt[1 * hst + hs_], hrn);
                }
              }
            }
            wcnt = cb;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
          }
        }
      }
      }
    }
    __syncthreads();
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  while (wcnt > 0) {
    const int cb = wcnt > 64 ? wcnt - 64 : 0;
    const int ce = cb + cln;
    bool cok = ce < wcnt;
    const i64 crow = (i64)lrow_s[wv][cok ? ce : cb];
    const i64 cj = (i64)lj_s[wv][cok ? ce : cb];
    const int w2_c = a.c2[crow];
    const int r2_c = (int)w2_c;
    const i64 q2_c = a.B2 + (i64)w2_c;
    const double x2_c = (double)((double)(a.B2 + (i64)w2_c) * a.R2);
    const signed char w3_c = a.c3[crow];
    const int r3_c = (int)w3_c;
    const i64 q3_c = a.B3 + (i64)w3_c;
    const double x3_c = (double)((double)(a.B3 + (i64)w3_c) * a.R3);
    const int w0_c = a.c0[crow];
    const int r0_c = (int)w0_c;
    const long long x0_c = (long long)(a.B0 + (i64)w0_c);
    const short w9_c = a.c9[cj];
    const int r9_c = (int)w9_c;
    const int x9_c = (int)(a.B9 + (i64)w9_c);
    const signed char w10_c = a.c10[cj];
    const int r10_c = (int)w10_c;
    const int x10_c = (int)(a.B10 + (i64)w10_c);
    { const int hln = (int)(threadIdx.x & 63u); const bool hok = cok;
      u64 hk = 0ull; const bool hnul = false;
      hk |= (u64)((i64)x0_c - a.HL0) << (unsigned)a.HS0;
      hk |= (u64)((i64)x9_c - a.HL1) << (unsigned)a.HS1;
      hk |= (u64)((i64)x10_c - a.HL2) << (unsigned)a.HS2;
      const u64 hkp = __shfl_up(hk, 1u, 64);
      const int hfp = __shfl_up((hok ? 1 : 0) | (hnul ? 2 : 0), 1u, 64);
      const bool hsame = hln > 0 && hok && (hfp & 1) != 0 && ((hfp >> 1) & 1) == (hnul ? 1 : 0) && hkp == hk;
      const u64 hH = __ballot(!hsame);
      const int hss = 63 - __builtin_clzll(hH & ((2ull << hln) - 1ull));
      const bool htl = hok && (hln == 63 || ((hH >> ((hln + 1) & 63)) & 1ull) != 0ull);
      const bool hq0 = hok && true;
      double hv0 = hq0 ? (double)((a.A0_0 + a.B0_0 * (double)x2_c) * (a.A0_1 + a.B0_1 * (double)x3_c)) : 0.0;
      #pragma unroll
      for (int hd = 1; hd < 64; hd <<= 1) {
        const double u_hv0 = __shfl_up(hv0, (unsigned)hd, 64);
        if (hln - hd >= hss) {
          hv0 = hv0 + u_hv0;
        }
      }
      if (htl) {
        long long hs_ = -1;
        if (hnul) hs_ = a.HM + 1; else if (hk == ~0ull) hs_ = a.HM; else {
          u64 hh = hs_mix64(hk) & (u64)(a.HM - 1);
          for (int pr_ = 0; pr_ < 512; ++pr_) {
            const u64 pv_ = atomicCAS(&a.hkeys[hh], ~0ull, hk);
            if (pv_ == ~0ull || pv_ == hk) { hs_ = (long long)hh; break; }
            hh = (hh + 1ull) & (u64)(a.HM - 1);
          }
          if (hs_ < 0) a.hflag[0] = 1;
        }
        if (hs_ >= 0) {
          const long long hst = a.HM + 2;   // SoA: aggregate i of slot s at i * (M + 2) + s
          const unsigned long long hrn = (unsigned long long)(hln - hss + 1);
          unsafeAtomicAdd(&a.hsum[0 * hst + hs_], hv0);
          if (hs_ >= a.HM) atomicAdd((unsigned long long*)&a.hcnt[1 * hst + hs_], hrn);
        }
      }
    }
    wcnt = cb;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}
