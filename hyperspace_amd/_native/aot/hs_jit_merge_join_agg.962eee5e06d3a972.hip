
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
  const int* TR;
  const int* RK0;
  const unsigned long long* GM0;
  const int* GR0;
  const short* c1;
  const int* c8;
  long long B8;
  const short* c9;
  long long B9;
  long long CL4;
  long long CH4;
  long long B1;
  long long CL1;
  long long CH1;
  const int* c2;
  long long B2;
  double R2;
  const signed char* c3;
  long long B3;
  double R3;
  const int* c0;
  long long B0;
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
  __shared__ unsigned lrk_[4096];
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
    const i64 off = (t - a.tile_prefix[r]) * 4096;
    const i64 rs = a.rstart[r], re = rs + a.rlen[r];
    const i64 tb0 = (rs & ~(i64)15) + off;
    const i64 g0 = tb0 + (i64)threadIdx.x * 16;
    const i64 dlo_ = rs - g0, dhi_ = re - g0;
    const int alo = dlo_ <= 0 ? 0 : (dlo_ >= 16 ? 16 : (int)dlo_);
    const int ahi = dhi_ <= 0 ? 0 : (dhi_ >= 16 ? 16 : (int)dhi_);
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
    const bool act8 = 8 >= alo && 8 < ahi;
    const i64 row8 = g0 + 8;
    const bool act9 = 9 >= alo && 9 < ahi;
    const i64 row9 = g0 + 9;
    const bool act10 = 10 >= alo && 10 < ahi;
    const i64 row10 = g0 + 10;
    const bool act11 = 11 >= alo && 11 < ahi;
    const i64 row11 = g0 + 11;
    const bool act12 = 12 >= alo && 12 < ahi;
    const i64 row12 = g0 + 12;
    const bool act13 = 13 >= alo && 13 < ahi;
    const i64 row13 = g0 + 13;
    const bool act14 = 14 >= alo && 14 < ahi;
    const i64 row14 = g0 + 14;
    const bool act15 = 15 >= alo && 15 < ahi;
    const i64 row15 = g0 + 15;
    if (tb0 + 4096 <= a.nrows) {
    short x1v[16];
    vload<short, 16>(a.c1, g0, x1v);
    const i64 ss = a.spans[4 * t + 2], se = a.spans[4 * t + 3];
    const int ra_ = a.TR[2 * t], nl_ = a.TR[2 * t + 1];
    const i64 gi_ = (g0 < a.nrows ? g0 : a.nrows - 1) >> 6;
    const unsigned long long gm_ = a.GM0[gi_];
    const int gr_ = a.GR0[gi_];
    for (int q_ = (int)threadIdx.x; q_ < nl_; q_ += 256) lrk_[q_] = (unsigned)a.RK0[ra_ + q_] + (unsigned)a.KOF;
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
    const int r1_8 = (int)x1v[8];
    const int x1_8 = (int)(a.B1 + (i64)x1v[8]);
    const int r1_9 = (int)x1v[9];
    const int x1_9 = (int)(a.B1 + (i64)x1v[9]);
    const int r1_10 = (int)x1v[10];
    const int x1_10 = (int)(a.B1 + (i64)x1v[10]);
    const int r1_11 = (int)x1v[11];
    const int x1_11 = (int)(a.B1 + (i64)x1v[11]);
    const int r1_12 = (int)x1v[12];
    const int x1_12 = (int)(a.B1 + (i64)x1v[12]);
    const int r1_13 = (int)x1v[13];
    const int x1_13 = (int)(a.B1 + (i64)x1v[13]);
    const int r1_14 = (int)x1v[14];
    const int x1_14 = (int)(a.B1 + (i64)x1v[14]);
    const int r1_15 = (int)x1v[15];
    const int x1_15 = (int)(a.B1 + (i64)x1v[15]);
    unsigned kvb = 0u, mb = 0u;
    { const bool kv = act0 && true; kvb |= kv ? 1u : 0u; mb |= (kv && ((true)) && ((true && (r1_0 >= (int)a.CL1 && r1_0 <= (int)a.CH1)))) ? 1u : 0u; }
    { const bool kv = act1 && true; kvb |= kv ? 2u : 0u; mb |= (kv && ((true)) && ((true && (r1_1 >= (int)a.CL1 && r1_1 <= (int)a.CH1)))) ? 2u : 0u; }
    { const bool kv = act2 && true; kvb |= kv ? 4u : 0u; mb |= (kv && ((true)) && ((true && (r1_2 >= (int)a.CL1 && r1_2 <= (int)a.CH1)))) ? 4u : 0u; }
    { const bool kv = act3 && true; kvb |= kv ? 8u : 0u; mb |= (kv && ((true)) && ((true && (r1_3 >= (int)a.CL1 && r1_3 <= (int)a.CH1)))) ? 8u : 0u; }
    { const bool kv = act4 && true; kvb |= kv ? 16u : 0u; mb |= (kv && ((true)) && ((true && (r1_4 >= (int)a.CL1 && r1_4 <= (int)a.CH1)))) ? 16u : 0u; }
    { const bool kv = act5 && true; kvb |= kv ? 32u : 0u; mb |= (kv && ((true)) && ((true && (r1_5 >= (int)a.CL1 && r1_5 <= (int)a.CH1)))) ? 32u : 0u; }
    { const bool kv = act6 && true; kvb |= kv ? 64u : 0u; mb |= (kv && ((true)) && ((true && (r1_6 >= (int)a.CL1 && r1_6 <= (int)a.CH1)))) ? 64u : 0u; }
    { const bool kv = act7 && true; kvb |= kv ? 128u : 0u; mb |= (kv && ((true)) && ((true && (r1_7 >= (int)a.CL1 && r1_7 <= (int)a.CH1)))) ? 128u : 0u; }
    { const bool kv = act8 && true; kvb |= kv ? 256u : 0u; mb |= (kv && ((true)) && ((true && (r1_8 >= (int)a.CL1 && r1_8 <= (int)a.CH1)))) ? 256u : 0u; }
    { const bool kv = act9 && true; kvb |= kv ? 512u : 0u; mb |= (kv && ((true)) && ((true && (r1_9 >= (int)a.CL1 && r1_9 <= (int)a.CH1)))) ? 512u : 0u; }
    { const bool kv = act10 && true; kvb |= kv ? 1024u : 0u; mb |= (kv && ((true)) && ((true && (r1_10 >= (int)a.CL1 && r1_10 <= (int)a.CH1)))) ? 1024u : 0u; }
    { const bool kv = act11 && true; kvb |= kv ? 2048u : 0u; mb |= (kv && ((true)) && ((true && (r1_11 >= (int)a.CL1 && r1_11 <= (int)a.CH1)))) ? 2048u : 0u; }
    { const bool kv = act12 && true; kvb |= kv ? 4096u : 0u; mb |= (kv && ((true)) && ((true && (r1_12 >= (int)a.CL1 && r1_12 <= (int)a.CH1)))) ? 4096u : 0u; }
    { const bool kv = act13 && true; kvb |= kv ? 8192u : 0u; mb |= (kv && ((true)) && ((true && (r1_13 >= (int)a.CL1 && r1_13 <= (int)a.CH1)))) ? 8192u : 0u; }
    { const bool kv = act14 && true; kvb |= kv ? 16384u : 0u; mb |= (kv && ((true)) && ((true && (r1_14 >= (int)a.CL1 && r1_14 <= (int)a.CH1)))) ? 16384u : 0u; }
    { const bool kv = act15 && true; kvb |= kv ? 32768u : 0u; mb |= (kv && ((true)) && ((true && (r1_15 >= (int)a.CL1 && r1_15 <= (int)a.CH1)))) ? 32768u : 0u; }
    __syncthreads();
    { const int c_ = (nl_ + 255) / 256;
      const int q0_ = (int)threadIdx.x * c_;
      const int q1_ = q0_ + c_ < nl_ ? q0_ + c_ : nl_;
      if (staged) {
        int j_ = 0;
        if (q0_ < q1_) { const unsigned key_ = lrk_[q0_]; int lo = 0;
          for (int st = ns > 0 ? (1 << (31 - __builtin_clz(ns))) : 0; st > 0; st >>= 1) {
            const int c = lo + st; lo = (c <= ns && skeys[c - 1] < key_) ? c : lo; }
          j_ = lo; }
        for (int q = q0_; q < q1_; ++q) {
          const unsigned key_ = lrk_[q];
          if (skeys[j_] < key_) { ++j_;
            if (skeys[j_] < key_) { int lo = j_ + 1, hi = ns;
              while (lo < hi) { const int m = (lo + hi) >> 1; if (skeys[m] < key_) lo = m + 1; else hi = m; }
              j_ = lo; } }
          lrk_[q] = (j_ < ns && skeys[j_] == key_ && spass[j_]) ? (unsigned)j_ : 0xFFFFFFFFu;
        }
      } else {
        for (int q = q0_; q < q1_; ++q) { const unsigned key_ = lrk_[q]; i64 lo = ss, hi = se;
          while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < key_) lo = md + 1; else hi = md; }
          lrk_[q] = (lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == key_) ? (unsigned)(lo - ss) : 0xFFFFFFFFu; }
      }
    }
    __syncthreads();
    unsigned mtb = 0u;
    int jl0 = 0;
    int jl1 = 0;
    int jl2 = 0;
    int jl3 = 0;
    int jl4 = 0;
    int jl5 = 0;
    int jl6 = 0;
    int jl7 = 0;
    int jl8 = 0;
    int jl9 = 0;
    int jl10 = 0;
    int jl11 = 0;
    int jl12 = 0;
    int jl13 = 0;
    int jl14 = 0;
    int jl15 = 0;
    { const int sh_ = (int)(g0 & 63);
      const int rq0_ = gr_ + (int)__popcll(gm_ & ((2ull << sh_) - 2ull)) - ra_;
      const unsigned gl_ = (unsigned)(gm_ >> sh_);
      const int rmax_ = nl_ > 0 ? nl_ - 1 : 0;
      { const int ri_ = min(max(rq0_, 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 0) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 1u : 0u; jl0 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 2u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 1) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 2u : 0u; jl1 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 6u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 2) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 4u : 0u; jl2 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 14u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 3) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 8u : 0u; jl3 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 30u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 4) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 16u : 0u; jl4 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 62u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 5) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 32u : 0u; jl5 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 126u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 6) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 64u : 0u; jl6 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 254u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 7) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 128u : 0u; jl7 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 510u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 8) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 256u : 0u; jl8 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 1022u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 9) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 512u : 0u; jl9 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 2046u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 10) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 1024u : 0u; jl10 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 4094u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 11) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 2048u : 0u; jl11 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 8190u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 12) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 4096u : 0u; jl12 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 16382u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 13) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 8192u : 0u; jl13 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 32766u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 14) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 16384u : 0u; jl14 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 65534u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 15) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 32768u : 0u; jl15 = h_ ? (int)jm_ : 0; }
    }
    { unsigned pb = mtb;
    if (false) {
      pb &= spass[((mtb >> 0) & 1u) ? jl0 : 0] != 0 ? ~0u : ~1u;
      pb &= spass[((mtb >> 1) & 1u) ? jl1 : 0] != 0 ? ~0u : ~2u;
      pb &= spass[((mtb >> 2) & 1u) ? jl2 : 0] != 0 ? ~0u : ~4u;
      pb &= spass[((mtb >> 3) & 1u) ? jl3 : 0] != 0 ? ~0u : ~8u;
      pb &= spass[((mtb >> 4) & 1u) ? jl4 : 0] != 0 ? ~0u : ~16u;
      pb &= spass[((mtb >> 5) & 1u) ? jl5 : 0] != 0 ? ~0u : ~32u;
      pb &= spass[((mtb >> 6) & 1u) ? jl6 : 0] != 0 ? ~0u : ~64u;
      pb &= spass[((mtb >> 7) & 1u) ? jl7 : 0] != 0 ? ~0u : ~128u;
      pb &= spass[((mtb >> 8) & 1u) ? jl8 : 0] != 0 ? ~0u : ~256u;
      pb &= spass[((mtb >> 9) & 1u) ? jl9 : 0] != 0 ? ~0u : ~512u;
      pb &= spass[((mtb >> 10) & 1u) ? jl10 : 0] != 0 ? ~0u : ~1024u;
      pb &= spass[((mtb >> 11) & 1u) ? jl11 : 0] != 0 ? ~0u : ~2048u;
      pb &= spass[((mtb >> 12) & 1u) ? jl12 : 0] != 0 ? ~0u : ~4096u;
      pb &= spass[((mtb >> 13) & 1u) ? jl13 : 0] != 0 ? ~0u : ~8192u;
      pb &= spass[((mtb >> 14) & 1u) ? jl14 : 0] != 0 ? ~0u : ~16384u;
      pb &= spass[((mtb >> 15) & 1u) ? jl15 : 0] != 0 ? ~0u : ~32768u;
    } else if (!staged) {
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
      { const i64 jq8 = ss + (((mtb >> 8) & 1u) ? jl8 : 0);
        const int w8_8 = a.c8[jq8];
        const int r8_8 = (int)w8_8;
        const long long x8_8 = (long long)(a.B8 + (i64)w8_8);
        const short w9_8 = a.c9[jq8];
        const int r9_8 = (int)w9_8;
        const int x9_8 = (int)(a.B9 + (i64)w9_8);
        pb &= (((true)) && ((true)) && ((true && (r9_8 >= (int)a.CL4 && r9_8 <= (int)a.CH4)))) ? ~0u : ~256u; }
      { const i64 jq9 = ss + (((mtb >> 9) & 1u) ? jl9 : 0);
        const int w8_9 = a.c8[jq9];
        const int r8_9 = (int)w8_9;
        const long long x8_9 = (long long)(a.B8 + (i64)w8_9);
        const short w9_9 = a.c9[jq9];
        const int r9_9 = (int)w9_9;
        const int x9_9 = (int)(a.B9 + (i64)w9_9);
        pb &= (((true)) && ((true)) && ((true && (r9_9 >= (int)a.CL4 && r9_9 <= (int)a.CH4)))) ? ~0u : ~512u; }
      { const i64 jq10 = ss + (((mtb >> 10) & 1u) ? jl10 : 0);
        const int w8_10 = a.c8[jq10];
        const int r8_10 = (int)w8_10;
        const long long x8_10 = (long long)(a.B8 + (i64)w8_10);
        const short w9_10 = a.c9[jq10];
        const int r9_10 = (int)w9_10;
        const int x9_10 = (int)(a.B9 + (i64)w9_10);
        pb &= (((true)) && ((true)) && ((true && (r9_10 >= (int)a.CL4 && r9_10 <= (int)a.CH4)))) ? ~0u : ~1024u; }
      { const i64 jq11 = ss + (((mtb >> 11) & 1u) ? jl11 : 0);
        const int w8_11 = a.c8[jq11];
        const int r8_11 = (int)w8_11;
        const long long x8_11 = (long long)(a.B8 + (i64)w8_11);
        const short w9_11 = a.c9[jq11];
        const int r9_11 = (int)w9_11;
        const int x9_11 = (int)(a.B9 + (i64)w9_11);
        pb &= (((true)) && ((true)) && ((true && (r9_11 >= (int)a.CL4 && r9_11 <= (int)a.CH4)))) ? ~0u : ~2048u; }
      { const i64 jq12 = ss + (((mtb >> 12) & 1u) ? jl12 : 0);
        const int w8_12 = a.c8[jq12];
        const int r8_12 = (int)w8_12;
        const long long x8_12 = (long long)(a.B8 + (i64)w8_12);
        const short w9_12 = a.c9[jq12];
        const int r9_12 = (int)w9_12;
        const int x9_12 = (int)(a.B9 + (i64)w9_12);
        pb &= (((true)) && ((true)) && ((true && (r9_12 >= (int)a.CL4 && r9_12 <= (int)a.CH4)))) ? ~0u : ~4096u; }
      { const i64 jq13 = ss + (((mtb >> 13) & 1u) ? jl13 : 0);
        const int w8_13 = a.c8[jq13];
        const int r8_13 = (int)w8_13;
        const long long x8_13 = (long long)(a.B8 + (i64)w8_13);
        const short w9_13 = a.c9[jq13];
        const int r9_13 = (int)w9_13;
        const int x9_13 = (int)(a.B9 + (i64)w9_13);
        pb &= (((true)) && ((true)) && ((true && (r9_13 >= (int)a.CL4 && r9_13 <= (int)a.CH4)))) ? ~0u : ~8192u; }
      { const i64 jq14 = ss + (((mtb >> 14) & 1u) ? jl14 : 0);
        const int w8_14 = a.c8[jq14];
        const int r8_14 = (int)w8_14;
        const long long x8_14 = (long long)(a.B8 + (i64)w8_14);
        const short w9_14 = a.c9[jq14];
        const int r9_14 = (int)w9_14;
        const int x9_14 = (int)(a.B9 + (i64)w9_14);
        pb &= (((true)) && ((true)) && ((true && (r9_14 >= (int)a.CL4 && r9_14 <= (int)a.CH4)))) ? ~0u : ~16384u; }
      { const i64 jq15 = ss + (((mtb >> 15) & 1u) ? jl15 : 0);
        const int w8_15 = a.c8[jq15];
        const int r8_15 = (int)w8_15;
        const long long x8_15 = (long long)(a.B8 + (i64)w8_15);
        const short w9_15 = a.c9[jq15];
        const int r9_15 = (int)w9_15;
        const int x9_15 = (int)(a.B9 + (i64)w9_15);
        pb &= (((true)) && ((true)) && ((true && (r9_15 >= (int)a.CL4 && r9_15 <= (int)a.CH4)))) ? ~0u : ~32768u; }
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
        jv = it == 8 ? jl8 : jv;
        jv = it == 9 ? jl9 : jv;
        jv = it == 10 ? jl10 : jv;
        jv = it == 11 ? jl11 : jv;
        jv = it == 12 ? jl12 : jv;
        jv = it == 13 ? jl13 : jv;
        jv = it == 14 ? jl14 : jv;
        jv = it == 15 ? jl15 : jv;
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
    __syncthreads();
    } else {
    short x1v[16];
    x1v[0] = act0 ? a.c1[g0 + 0] : (short)0; x1v[1] = act1 ? a.c1[g0 + 1] : (short)0; x1v[2] = act2 ? a.c1[g0 + 2] : (short)0; x1v[3] = act3 ? a.c1[g0 + 3] : (short)0; x1v[4] = act4 ? a.c1[g0 + 4] : (short)0; x1v[5] = act5 ? a.c1[g0 + 5] : (short)0; x1v[6] = act6 ? a.c1[g0 + 6] : (short)0; x1v[7] = act7 ? a.c1[g0 + 7] : (short)0; x1v[8] = act8 ? a.c1[g0 + 8] : (short)0; x1v[9] = act9 ? a.c1[g0 + 9] : (short)0; x1v[10] = act10 ? a.c1[g0 + 10] : (short)0; x1v[11] = act11 ? a.c1[g0 + 11] : (short)0; x1v[12] = act12 ? a.c1[g0 + 12] : (short)0; x1v[13] = act13 ? a.c1[g0 + 13] : (short)0; x1v[14] = act14 ? a.c1[g0 + 14] : (short)0; x1v[15] = act15 ? a.c1[g0 + 15] : (short)0;
    const i64 ss = a.spans[4 * t + 2], se = a.spans[4 * t + 3];
    const int ra_ = a.TR[2 * t], nl_ = a.TR[2 * t + 1];
    const i64 gi_ = (g0 < a.nrows ? g0 : a.nrows - 1) >> 6;
    const unsigned long long gm_ = a.GM0[gi_];
    const int gr_ = a.GR0[gi_];
    for (int q_ = (int)threadIdx.x; q_ < nl_; q_ += 256) lrk_[q_] = (unsigned)a.RK0[ra_ + q_] + (unsigned)a.KOF;
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
    const int r1_8 = (int)x1v[8];
    const int x1_8 = (int)(a.B1 + (i64)x1v[8]);
    const int r1_9 = (int)x1v[9];
    const int x1_9 = (int)(a.B1 + (i64)x1v[9]);
    const int r1_10 = (int)x1v[10];
    const int x1_10 = (int)(a.B1 + (i64)x1v[10]);
    const int r1_11 = (int)x1v[11];
    const int x1_11 = (int)(a.B1 + (i64)x1v[11]);
    const int r1_12 = (int)x1v[12];
    const int x1_12 = (int)(a.B1 + (i64)x1v[12]);
    const int r1_13 = (int)x1v[13];
    const int x1_13 = (int)(a.B1 + (i64)x1v[13]);
    const int r1_14 = (int)x1v[14];
    const int x1_14 = (int)(a.B1 + (i64)x1v[14]);
    const int r1_15 = (int)x1v[15];
    const int x1_15 = (int)(a.B1 + (i64)x1v[15]);
    unsigned kvb = 0u, mb = 0u;
    { const bool kv = act0 && true; kvb |= kv ? 1u : 0u; mb |= (kv && ((true)) && ((true && (r1_0 >= (int)a.CL1 && r1_0 <= (int)a.CH1)))) ? 1u : 0u; }
    { const bool kv = act1 && true; kvb |= kv ? 2u : 0u; mb |= (kv && ((true)) && ((true && (r1_1 >= (int)a.CL1 && r1_1 <= (int)a.CH1)))) ? 2u : 0u; }
    { const bool kv = act2 && true; kvb |= kv ? 4u : 0u; mb |= (kv && ((true)) && ((true && (r1_2 >= (int)a.CL1 && r1_2 <= (int)a.CH1)))) ? 4u : 0u; }
    { const bool kv = act3 && true; kvb |= kv ? 8u : 0u; mb |= (kv && ((true)) && ((true && (r1_3 >= (int)a.CL1 && r1_3 <= (int)a.CH1)))) ? 8u : 0u; }
    { const bool kv = act4 && true; kvb |= kv ? 16u : 0u; mb |= (kv && ((true)) && ((true && (r1_4 >= (int)a.CL1 && r1_4 <= (int)a.CH1)))) ? 16u : 0u; }
    { const bool kv = act5 && true; kvb |= kv ? 32u : 0u; mb |= (kv && ((true)) && ((true && (r1_5 >= (int)a.CL1 && r1_5 <= (int)a.CH1)))) ? 32u : 0u; }
    { const bool kv = act6 && true; kvb |= kv ? 64u : 0u; mb |= (kv && ((true)) && ((true && (r1_6 >= (int)a.CL1 && r1_6 <= (int)a.CH1)))) ? 64u : 0u; }
    { const bool kv = act7 && true; kvb |= kv ? 128u : 0u; mb |= (kv && ((true)) && ((true && (r1_7 >= (int)a.CL1 && r1_7 <= (int)a.CH1)))) ? 128u : 0u; }
    { const bool kv = act8 && true; kvb |= kv ? 256u : 0u; mb |= (kv && ((true)) && ((true && (r1_8 >= (int)a.CL1 && r1_8 <= (int)a.CH1)))) ? 256u : 0u; }
    { const bool kv = act9 && true; kvb |= kv ? 512u : 0u; mb |= (kv && ((true)) && ((true && (r1_9 >= (int)a.CL1 && r1_9 <= (int)a.CH1)))) ? 512u : 0u; }
    { const bool kv = act10 && true; kvb |= kv ? 1024u : 0u; mb |= (kv && ((true)) && ((true && (r1_10 >= (int)a.CL1 && r1_10 <= (int)a.CH1)))) ? 1024u : 0u; }
    { const bool kv = act11 && true; kvb |= kv ? 2048u : 0u; mb |= (kv && ((true)) && ((true && (r1_11 >= (int)a.CL1 && r1_11 <= (int)a.CH1)))) ? 2048u : 0u; }
    { const bool kv = act12 && true; kvb |= kv ? 4096u : 0u; mb |= (kv && ((true)) && ((true && (r1_12 >= (int)a.CL1 && r1_12 <= (int)a.CH1)))) ? 4096u : 0u; }
    { const bool kv = act13 && true; kvb |= kv ? 8192u : 0u; mb |= (kv && ((true)) && ((true && (r1_13 >= (int)a.CL1 && r1_13 <= (int)a.CH1)))) ? 8192u : 0u; }
    { const bool kv = act14 && true; kvb |= kv ? 16384u : 0u; mb |= (kv && ((true)) && ((true && (r1_14 >= (int)a.CL1 && r1_14 <= (int)a.CH1)))) ? 16384u : 0u; }
    { const bool kv = act15 && true; kvb |= kv ? 32768u : 0u; mb |= (kv && ((true)) && ((true && (r1_15 >= (int)a.CL1 && r1_15 <= (int)a.CH1)))) ? 32768u : 0u; }
    __syncthreads();
    { const int c_ = (nl_ + 255) / 256;
      const int q0_ = (int)threadIdx.x * c_;
      const int q1_ = q0_ + c_ < nl_ ? q0_ + c_ : nl_;
      if (staged) {
        int j_ = 0;
        if (q0_ < q1_) { const unsigned key_ = lrk_[q0_]; int lo = 0;
          for (int st = ns > 0 ? (1 << (31 - __builtin_clz(ns))) : 0; st > 0; st >>= 1) {
            const int c = lo + st; lo = (c <= ns && skeys[c - 1] < key_) ? c : lo; }
          j_ = lo; }
        for (int q = q0_; q < q1_; ++q) {
          const unsigned key_ = lrk_[q];
          if (skeys[j_] < key_) { ++j_;
            if (skeys[j_] < key_) { int lo = j_ + 1, hi = ns;
              while (lo < hi) { const int m = (lo + hi) >> 1; if (skeys[m] < key_) lo = m + 1; else hi = m; }
              j_ = lo; } }
          lrk_[q] = (j_ < ns && skeys[j_] == key_ && spass[j_]) ? (unsigned)j_ : 0xFFFFFFFFu;
        }
      } else {
        for (int q = q0_; q < q1_; ++q) { const unsigned key_ = lrk_[q]; i64 lo = ss, hi = se;
          while (lo < hi) { const i64 md = (lo + hi) >> 1; const bool nv = false; if (nv || ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[md])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) < key_) lo = md + 1; else hi = md; }
          lrk_[q] = (lo < se && !(false) && ({ const i64 d_ = (i64)((long long)(a.B8 + (i64)a.c8[lo])) - a.KLO; d_ < 0 ? 0u : (d_ > a.KSP ? 0xFFFFFFFFu : (unsigned)(d_ + 1)); }) == key_) ? (unsigned)(lo - ss) : 0xFFFFFFFFu; }
      }
    }
    __syncthreads();
    unsigned mtb = 0u;
    int jl0 = 0;
    int jl1 = 0;
    int jl2 = 0;
    int jl3 = 0;
    int jl4 = 0;
    int jl5 = 0;
    int jl6 = 0;
    int jl7 = 0;
    int jl8 = 0;
    int jl9 = 0;
    int jl10 = 0;
    int jl11 = 0;
    int jl12 = 0;
    int jl13 = 0;
    int jl14 = 0;
    int jl15 = 0;
    { const int sh_ = (int)(g0 & 63);
      const int rq0_ = gr_ + (int)__popcll(gm_ & ((2ull << sh_) - 2ull)) - ra_;
      const unsigned gl_ = (unsigned)(gm_ >> sh_);
      const int rmax_ = nl_ > 0 ? nl_ - 1 : 0;
      { const int ri_ = min(max(rq0_, 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 0) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 1u : 0u; jl0 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 2u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 1) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 2u : 0u; jl1 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 6u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 2) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 4u : 0u; jl2 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 14u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 3) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 8u : 0u; jl3 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 30u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 4) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 16u : 0u; jl4 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 62u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 5) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 32u : 0u; jl5 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 126u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 6) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 64u : 0u; jl6 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 254u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 7) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 128u : 0u; jl7 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 510u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 8) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 256u : 0u; jl8 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 1022u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 9) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 512u : 0u; jl9 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 2046u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 10) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 1024u : 0u; jl10 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 4094u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 11) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 2048u : 0u; jl11 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 8190u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 12) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 4096u : 0u; jl12 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 16382u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 13) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 8192u : 0u; jl13 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 32766u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 14) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 16384u : 0u; jl14 = h_ ? (int)jm_ : 0; }
      { const int ri_ = min(max((rq0_ + (int)__popc(gl_ & 65534u)), 0), rmax_);
        const unsigned jm_ = lrk_[ri_];
        const bool h_ = ((mb >> 15) & 1u) && jm_ != 0xFFFFFFFFu;
        mtb |= h_ ? 32768u : 0u; jl15 = h_ ? (int)jm_ : 0; }
    }
    { unsigned pb = mtb;
    if (false) {
      pb &= spass[((mtb >> 0) & 1u) ? jl0 : 0] != 0 ? ~0u : ~1u;
      pb &= spass[((mtb >> 1) & 1u) ? jl1 : 0] != 0 ? ~0u : ~2u;
      pb &= spass[((mtb >> 2) & 1u) ? jl2 : 0] != 0 ? ~0u : ~4u;
      pb &= spass[((mtb >> 3) & 1u) ? jl3 : 0] != 0 ? ~0u : ~8u;
      pb &= spass[((mtb >> 4) & 1u) ? jl4 : 0] != 0 ? ~0u : ~16u;
      pb &= spass[((mtb >> 5) & 1u) ? jl5 : 0] != 0 ? ~0u : ~32u;
      pb &= spass[((mtb >> 6) & 1u) ? jl6 : 0] != 0 ? ~0u : ~64u;
      pb &= spass[((mtb >> 7) & 1u) ? jl7 : 0] != 0 ? ~0u : ~128u;
      pb &= spass[((mtb >> 8) & 1u) ? jl8 : 0] != 0 ? ~0u : ~256u;
      pb &= spass[((mtb >> 9) & 1u) ? jl9 : 0] != 0 ? ~0u : ~512u;
      pb &= spass[((mtb >> 10) & 1u) ? jl10 : 0] != 0 ? ~0u : ~1024u;
      pb &= spass[((mtb >> 11) & 1u) ? jl11 : 0] != 0 ? ~0u : ~2048u;
      pb &= spass[((mtb >> 12) & 1u) ? jl12 : 0] != 0 ? ~0u : ~4096u;
      pb &= spass[((mtb >> 13) & 1u) ? jl13 : 0] != 0 ? ~0u : ~8192u;
      pb &= spass[((mtb >> 14) & 1u) ? jl14 : 0] != 0 ? ~0u : ~16384u;
      pb &= spass[((mtb >> 15) & 1u) ? jl15 : 0] != 0 ? ~0u : ~32768u;
    } else if (!staged) {
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
      { const i64 jq8 = ss + (((mtb >> 8) & 1u) ? jl8 : 0);
        const int w8_8 = a.c8[jq8];
        const int r8_8 = (int)w8_8;
        const long long x8_8 = (long long)(a.B8 + (i64)w8_8);
        const short w9_8 = a.c9[jq8];
        const int r9_8 = (int)w9_8;
        const int x9_8 = (int)(a.B9 + (i64)w9_8);
        pb &= (((true)) && ((true)) && ((true && (r9_8 >= (int)a.CL4 && r9_8 <= (int)a.CH4)))) ? ~0u : ~256u; }
      { const i64 jq9 = ss + (((mtb >> 9) & 1u) ? jl9 : 0);
        const int w8_9 = a.c8[jq9];
        const int r8_9 = (int)w8_9;
        const long long x8_9 = (long long)(a.B8 + (i64)w8_9);
        const short w9_9 = a.c9[jq9];
        const int r9_9 = (int)w9_9;
        const int x9_9 = (int)(a.B9 + (i64)w9_9);
        pb &= (((true)) && ((true)) && ((true && (r9_9 >= (int)a.CL4 && r9_9 <= (int)a.CH4)))) ? ~0u : ~512u; }
      { const i64 jq10 = ss + (((mtb >> 10) & 1u) ? jl10 : 0);
        const int w8_10 = a.c8[jq10];
        const int r8_10 = (int)w8_10;
        const long long x8_10 = (long long)(a.B8 + (i64)w8_10);
        const short w9_10 = a.c9[jq10];
        const int r9_10 = (int)w9_10;
        const int x9_10 = (int)(a.B9 + (i64)w9_10);
        pb &= (((true)) && ((true)) && ((true && (r9_10 >= (int)a.CL4 && r9_10 <= (int)a.CH4)))) ? ~0u : ~1024u; }
      { const i64 jq11 = ss + (((mtb >> 11) & 1u) ? jl11 : 0);
        const int w8_11 = a.c8[jq11];
        const int r8_11 = (int)w8_11;
        const long long x8_11 = (long long)(a.B8 + (i64)w8_11);
        const short w9_11 = a.c9[jq11];
        const int r9_11 = (int)w9_11;
        const int x9_11 = (int)(a.B9 + (i64)w9_11);
        pb &= (((true)) && ((true)) && ((true && (r9_11 >= (int)a.CL4 && r9_11 <= (int)a.CH4)))) ? ~0u : ~2048u; }
      { const i64 jq12 = ss + (((mtb >> 12) & 1u) ? jl12 : 0);
        const int w8_12 = a.c8[jq12];
        const int r8_12 = (int)w8_12;
        const long long x8_12 = (long long)(a.B8 + (i64)w8_12);
        const short w9_12 = a.c9[jq12];
        const int r9_12 = (int)w9_12;
        const int x9_12 = (int)(a.B9 + (i64)w9_12);
        pb &= (((true)) && ((true)) && ((true && (r9_12 >= (int)a.CL4 && r9_12 <= (int)a.CH4)))) ? ~0u : ~4096u; }
      { const i64 jq13 = ss + (((mtb >> 13) & 1u) ? jl13 : 0);
        const int w8_13 = a.c8[jq13];
        const int r8_13 = (int)w8_13;
        const long long x8_13 = (long long)(a.B8 + (i64)w8_13);
        const short w9_13 = a.c9[jq13];
        const int r9_13 = (int)w9_13;
        const int x9_13 = (int)(a.B9 + (i64)w9_13);
        pb &= (((true)) && ((true)) && ((true && (r9_13 >= (int)a.CL4 && r9_13 <= (int)a.CH4)))) ? ~0u : ~8192u; }
      { const i64 jq14 = ss + (((mtb >> 14) & 1u) ? jl14 : 0);
        const int w8_14 = a.c8[jq14];
        const int r8_14 = (int)w8_14;
        const long long x8_14 = (long long)(a.B8 + (i64)w8_14);
        const short w9_14 = a.c9[jq14];
        const int r9_14 = (int)w9_14;
        const int x9_14 = (int)(a.B9 + (i64)w9_14);
        pb &= (((true)) && ((true)) && ((true && (r9_14 >= (int)a.CL4 && r9_14 <= (int)a.CH4)))) ? ~0u : ~16384u; }
      { const i64 jq15 = ss + (((mtb >> 15) & 1u) ? jl15 : 0);
        const int w8_15 = a.c8[jq15];
        const int r8_15 = (int)w8_15;
        const long long x8_15 = (long long)(a.B8 + (i64)w8_15);
        const short w9_15 = a.c9[jq15];
        const int r9_15 = (int)w9_15;
        const int x9_15 = (int)(a.B9 + (i64)w9_15);
        pb &= (((true)) && ((true)) && ((true && (r9_15 >= (int)a.CL4 && r9_15 <= (int)a.CH4)))) ? ~0u : ~32768u; }
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
        jv = it == 8 ? jl8 : jv;
        jv = it == 9 ? jl9 : jv;
        jv = it == 10 ? jl10 : jv;
        jv = it == 11 ? jl11 : jv;
        jv = it == 12 ? jl12 : jv;
        jv = it == 13 ? jl13 : jv;
        jv = it == 14 ? jl14 : jv;
        jv = it == 15 ? jl15 : jv;
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
