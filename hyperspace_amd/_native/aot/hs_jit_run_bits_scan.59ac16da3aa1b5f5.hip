
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
  const unsigned long long* GM0;
  const int* GR0;
  const unsigned* tags;
  long long R;
  long long nrows;
  double* psum;
  double* pmin;
  double* pmax;
  long long* pcnt;
  const short* c1;
  long long CL1;
  long long CH1;
  long long B1;
  const unsigned long long* PK;
  long long B2;
  double R2;
  long long B3;
  double R3;
  double A0_0;
  double B0_0;
  double A0_1;
  double B0_1;
};
extern "C" __global__ __launch_bounds__(256) void hs_jit_run_bits_scan(Args a) {
  constexpr int NA = 3;
  double acc0 = 0.0; unsigned cnt0 = 0u;
  double acc1 = 0.0; unsigned cnt1 = 0u;
  double acc2 = 0.0; unsigned cnt2 = 0u;
  __shared__ unsigned short lst_[4][1024];
  const int ln = (int)(threadIdx.x & 63);
  const int wq = (int)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const i64 ntiles = a.tile_prefix[a.R];
  const i64 nwv = (i64)gridDim.x * 4;
  const i64 wid = (i64)blockIdx.x * 4 + wq;
  const i64 per = (ntiles + nwv - 1) / nwv;
  const i64 t0 = wid * per;
  const i64 t1 = ntiles < t0 + per ? ntiles : t0 + per;
  int r = 0;
  if (t0 < t1) { int lo = 0, hi = (int)a.R;
    while (hi - lo > 1) { const int m = (lo + hi) >> 1; if (a.tile_prefix[m] <= t0) lo = m; else hi = m; }
    r = lo; }
  i64 rsN = 0, reN = 0, tbN = 0; u64 gmN = 0ull; i64 grN = 0;
  if (t0 < t1) {
    while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= t0) ++r;
    rsN = a.rstart[r]; reN = rsN + a.rlen[r];
    tbN = (rsN & ~(i64)63) + (t0 - a.tile_prefix[r]) * 4096;
    { const i64 r0_ = tbN + 64 * ln; const i64 g_ = (r0_ < a.nrows ? r0_ : a.nrows - 1) >> 6;
      gmN = a.GM0[g_] | 1ull; grN = a.GR0[g_]; }
  }
  for (i64 t = t0; t < t1; ++t) {
    const i64 rs = rsN, re = reN, tb0 = tbN; const u64 m_ = gmN; const i64 q0 = grN;
    const i64 row0 = tb0 + 64 * ln;
    const i64 lo_ = rs - row0, hi_ = re - row0;
    const int alo = lo_ <= 0 ? 0 : (lo_ >= 64 ? 64 : (int)lo_);
    const int ahi = hi_ <= 0 ? 0 : (hi_ >= 64 ? 64 : (int)hi_);
    const u64 am = alo >= ahi ? 0ull : ((ahi == 64 ? ~0ull : ((1ull << ahi) - 1ull)) & ~((1ull << alo) - 1ull));
    const i64 w_ = q0 >> 5; const unsigned sh_ = (unsigned)(q0 & 31);
    const u64 lw_ = (u64)a.tags[w_] | ((u64)a.tags[w_ + 1] << 32);
    const u64 hw_ = (u64)a.tags[w_ + 2];
    const bool vok_ = row0 + 64 <= a.nrows;
    unsigned x1w[32];
    if (vok_) { vload<unsigned, 32>((const unsigned*)a.c1, row0 * 2 / 4, x1w); } else { for (int k_ = 0; k_ < 32; ++k_) x1w[k_] = 0u; for (int k_ = 0; k_ < 64 && row0 + k_ < a.nrows; ++k_) { const unsigned u_ = (unsigned)(unsigned short)a.c1[row0 + k_]; x1w[k_ / 2] |= u_ << (16 * (k_ % 2)); } }
    if (t + 1 < t1) {
      while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= (t + 1)) ++r;
      rsN = a.rstart[r]; reN = rsN + a.rlen[r];
      tbN = (rsN & ~(i64)63) + ((t + 1) - a.tile_prefix[r]) * 4096;
      { const i64 r0_ = tbN + 64 * ln; const i64 g_ = (r0_ < a.nrows ? r0_ : a.nrows - 1) >> 6;
        gmN = a.GM0[g_] | 1ull; grN = a.GR0[g_]; }
    }
    const u64 T_ = sh_ ? ((lw_ >> sh_) | (hw_ << (64 - sh_))) : lw_;
    const int nr_ = __popcll(m_);
    const u64 Tm_ = nr_ >= 64 ? T_ : (T_ & ((1ull << nr_) - 1ull));
    u64 c_ = T_ ^ (T_ << 1), d_ = 0ull, mm_ = (am && Tm_) ? m_ : 0ull;
    while (mm_) { const u64 lb_ = mm_ & (0ull - mm_); if (c_ & 1ull) d_ |= lb_; c_ >>= 1; mm_ ^= lb_; }
    d_ ^= d_ << 1; d_ ^= d_ << 2; d_ ^= d_ << 4; d_ ^= d_ << 8; d_ ^= d_ << 16; d_ ^= d_ << 32;
    d_ &= am;
    unsigned plo_ = 0u, phi_ = 0u;
    #pragma unroll
    for (int k_ = 0; k_ < 32; ++k_) {
      const auto xr1_k = ((short)(x1w[(0 + k_) / 2] >> (16 * ((0 + k_) % 2))));
      const int r1_k = (int)xr1_k;
      const int x1_k = (int)(a.B1 + (i64)xr1_k);
      plo_ |= (((true)) && ((true && (r1_k >= (int)a.CL1 && r1_k <= (int)a.CH1))) ? 1u : 0u) << k_;
    }
    #pragma unroll
    for (int k_ = 0; k_ < 32; ++k_) {
      const auto xr1_k = ((short)(x1w[(32 + k_) / 2] >> (16 * ((32 + k_) % 2))));
      const int r1_k = (int)xr1_k;
      const int x1_k = (int)(a.B1 + (i64)xr1_k);
      phi_ |= (((true)) && ((true && (r1_k >= (int)a.CL1 && r1_k <= (int)a.CH1))) ? 1u : 0u) << k_;
    }
    d_ &= ((u64)phi_ << 32) | (u64)plo_;
    const int cn_ = __popcll(d_);
    int inc_ = cn_;
    for (int o_ = 1; o_ < 64; o_ <<= 1) { const int y_ = __shfl_up(inc_, o_, 64); if (ln >= o_) inc_ += y_; }
    const int tot_ = __shfl(inc_, 63, 64);
    for (int wb_ = 0; wb_ < tot_; wb_ += 1024) {
    const int wn_ = tot_ - wb_ < 1024 ? tot_ - wb_ : 1024;
    { int pos_ = inc_ - cn_ - wb_; u64 e_ = d_;
      while (e_) { const int bq_ = __builtin_ctzll(e_); if (pos_ >= 0 && pos_ < 1024) { lst_[wq][pos_] = (unsigned short)(64 * ln + bq_); } ++pos_; e_ &= e_ - 1ull; } }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int cb = 0; cb < wn_; cb += 256) {
      const int ce0 = cb + 0 + ln;
      const bool cok0 = ce0 < wn_;
      const i64 crow0 = tb0 + (cok0 ? (i64)lst_[wq][ce0] : 0);
      const int ce1 = cb + 64 + ln;
      const bool cok1 = ce1 < wn_;
      const i64 crow1 = tb0 + (cok1 ? (i64)lst_[wq][ce1] : 0);
      const int ce2 = cb + 128 + ln;
      const bool cok2 = ce2 < wn_;
      const i64 crow2 = tb0 + (cok2 ? (i64)lst_[wq][ce2] : 0);
      const int ce3 = cb + 192 + ln;
      const bool cok3 = ce3 < wn_;
      const i64 crow3 = tb0 + (cok3 ? (i64)lst_[wq][ce3] : 0);
      const u64 pk0_ = a.PK[crow0];
      const int r2_c0 = (int)((int)(unsigned)(pk0_ >> 0));
      const i64 q2_c0 = a.B2 + (i64)((int)(unsigned)(pk0_ >> 0));
      const double x2_c0 = (double)((double)(a.B2 + (i64)((int)(unsigned)(pk0_ >> 0))) * a.R2);
      const int r3_c0 = (int)((signed char)(unsigned char)(pk0_ >> 32));
      const i64 q3_c0 = a.B3 + (i64)((signed char)(unsigned char)(pk0_ >> 32));
      const double x3_c0 = (double)((double)(a.B3 + (i64)((signed char)(unsigned char)(pk0_ >> 32))) * a.R3);
      const u64 pk1_ = a.PK[crow1];
      const int r2_c1 = (int)((int)(unsigned)(pk1_ >> 0));
      const i64 q2_c1 = a.B2 + (i64)((int)(unsigned)(pk1_ >> 0));
      const double x2_c1 = (double)((double)(a.B2 + (i64)((int)(unsigned)(pk1_ >> 0))) * a.R2);
      const int r3_c1 = (int)((signed char)(unsigned char)(pk1_ >> 32));
      const i64 q3_c1 = a.B3 + (i64)((signed char)(unsigned char)(pk1_ >> 32));
      const double x3_c1 = (double)((double)(a.B3 + (i64)((signed char)(unsigned char)(pk1_ >> 32))) * a.R3);
      const u64 pk2_ = a.PK[crow2];
      const int r2_c2 = (int)((int)(unsigned)(pk2_ >> 0));
      const i64 q2_c2 = a.B2 + (i64)((int)(unsigned)(pk2_ >> 0));
      const double x2_c2 = (double)((double)(a.B2 + (i64)((int)(unsigned)(pk2_ >> 0))) * a.R2);
      const int r3_c2 = (int)((signed char)(unsigned char)(pk2_ >> 32));
      const i64 q3_c2 = a.B3 + (i64)((signed char)(unsigned char)(pk2_ >> 32));
      const double x3_c2 = (double)((double)(a.B3 + (i64)((signed char)(unsigned char)(pk2_ >> 32))) * a.R3);
      const u64 pk3_ = a.PK[crow3];
      const int r2_c3 = (int)((int)(unsigned)(pk3_ >> 0));
      const i64 q2_c3 = a.B2 + (i64)((int)(unsigned)(pk3_ >> 0));
      const double x2_c3 = (double)((double)(a.B2 + (i64)((int)(unsigned)(pk3_ >> 0))) * a.R2);
      const int r3_c3 = (int)((signed char)(unsigned char)(pk3_ >> 32));
      const i64 q3_c3 = a.B3 + (i64)((signed char)(unsigned char)(pk3_ >> 32));
      const double x3_c3 = (double)((double)(a.B3 + (i64)((signed char)(unsigned char)(pk3_ >> 32))) * a.R3);
      { bool cok = cok0;
      { const bool ok = cok && true; const double v = ok ? (a.A0_0 + a.B0_0 * (double)x2_c0) * (a.A0_1 + a.B0_1 * (double)x3_c0) : 0.0;
        acc0 += v; cnt0 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc1 += v; cnt1 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc2 += v; cnt2 += ok ? 1u : 0u; }
      }
      { bool cok = cok1;
      { const bool ok = cok && true; const double v = ok ? (a.A0_0 + a.B0_0 * (double)x2_c1) * (a.A0_1 + a.B0_1 * (double)x3_c1) : 0.0;
        acc0 += v; cnt0 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc1 += v; cnt1 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc2 += v; cnt2 += ok ? 1u : 0u; }
      }
      { bool cok = cok2;
      { const bool ok = cok && true; const double v = ok ? (a.A0_0 + a.B0_0 * (double)x2_c2) * (a.A0_1 + a.B0_1 * (double)x3_c2) : 0.0;
        acc0 += v; cnt0 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc1 += v; cnt1 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc2 += v; cnt2 += ok ? 1u : 0u; }
      }
      { bool cok = cok3;
      { const bool ok = cok && true; const double v = ok ? (a.A0_0 + a.B0_0 * (double)x2_c3) * (a.A0_1 + a.B0_1 * (double)x3_c3) : 0.0;
        acc0 += v; cnt0 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc1 += v; cnt1 += ok ? 1u : 0u; }
      { const bool ok = cok && true; const double v = ok ? 1.0 : 0.0;
        acc2 += v; cnt2 += ok ? 1u : 0u; }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); __builtin_amdgcn_wave_barrier(); __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
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
