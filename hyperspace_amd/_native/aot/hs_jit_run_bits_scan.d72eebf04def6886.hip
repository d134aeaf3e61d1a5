
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
  const unsigned long long* GM0;
  const int* GR0;
  const unsigned* tags;
  long long R;
  long long nrows;
  double* psum;
  double* pmin;
  double* pmax;
  long long* pcnt;
  const unsigned* P12_1;
  long long P12O_1;
  long long CL1;
  long long CH1;
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
  __shared__ unsigned char dlut_[512];
  for (int e_ = (int)threadIdx.x; e_ < 512; e_ += 256) {
    unsigned k_ = 0u, o_ = 0u;
    for (int j_ = 0; j_ < 4; ++j_) { k_ += (e_ >> j_) & 1; o_ |= (((unsigned)e_ >> (4u + k_)) & 1u) << j_; }
    dlut_[e_] = (unsigned char)o_; }
  __syncthreads();
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
  i64 rsC = 0, reC = 0, tbC = 0; u64 gmC = 0ull; int grC = 0;
  i64 rsN = 0, reN = 0, tbN = 0; u64 gmN = 0ull; int grN = 0;
  unsigned tw0A_ = 0u, tw1A_ = 0u, tw2A_ = 0u, tw0B_ = 0u, tw1B_ = 0u, tw2B_ = 0u;
  unsigned x1qA[24], x1qB[24];
  if (t0 < t1) {
    while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= t0) ++r;
    rsN = a.rstart[r]; reN = rsN + a.rlen[r];
    tbN = (rsN & ~(i64)63) + (t0 - a.tile_prefix[r]) * 4096;
    { const i64 r0_ = tbN + 64 * ln; const i64 g_ = (r0_ < a.nrows ? r0_ : a.nrows - 1) >> 6;
      gmN = a.GM0[g_]; grN = a.GR0[g_]; }
  }
  for (i64 t = t0; t < t1; ++t) {
   {
    rsC = rsN; reC = reN; tbC = tbN; gmC = gmN; grC = grN;
    { const i64 w_ = (i64)grC >> 5; tw0A_ = a.tags[w_]; tw1A_ = a.tags[w_ + 1]; tw2A_ = a.tags[w_ + 2]; }
    bload<24>(hs_rsrc((const char*)a.P12_1 + (tbC >> 6) * 96, ((a.nrows + 63 - tbC) >> 6) * 96), (unsigned)(ln * 96), x1qA);
    if (t + 1 < t1) {
      while (r + 1 < (int)a.R && a.tile_prefix[r + 1] <= (t + 1)) ++r;
      rsN = a.rstart[r]; reN = rsN + a.rlen[r];
      tbN = (rsN & ~(i64)63) + ((t + 1) - a.tile_prefix[r]) * 4096;
      { const i64 r0_ = tbN + 64 * ln; const i64 g_ = (r0_ < a.nrows ? r0_ : a.nrows - 1) >> 6;
        gmN = a.GM0[g_]; grN = a.GR0[g_]; }
    }
    const i64 rs = rsC, re = reC, tb0 = tbC; const u64 m_ = gmC | 1ull; const i64 q0 = (i64)grC;
    const i64 row0 = tb0 + 64 * ln;
    const i64 lo_ = rs - row0, hi_ = re - row0;
    const int alo = lo_ <= 0 ? 0 : (lo_ >= 64 ? 64 : (int)lo_);
    const int ahi = hi_ <= 0 ? 0 : (hi_ >= 64 ? 64 : (int)hi_);
    const u64 am = alo >= ahi ? 0ull : ((ahi == 64 ? ~0ull : ((1ull << ahi) - 1ull)) & ~((1ull << alo) - 1ull));
    const unsigned sh_ = (unsigned)(q0 & 31);
    const u64 lw_ = (u64)tw0A_ | ((u64)tw1A_ << 32);
    const u64 hw_ = (u64)tw2A_;
    const u64 T_ = sh_ ? ((lw_ >> sh_) | (hw_ << (64 - sh_))) : lw_;
    u64 d_ = (u64)dlut_[((unsigned)m_ & 15u) | ((((unsigned)T_ << 1) & 31u) << 4)];
    unsigned P_ = (unsigned)__popc((unsigned)m_ & 15u);
    #pragma unroll
    for (int i_ = 1; i_ < 16; ++i_) {
      const unsigned mn_ = (unsigned)(m_ >> (4 * i_)) & 15u;
      const unsigned ix_ = mn_ | (((unsigned)(T_ >> (P_ - 1u)) & 31u) << 4);
      d_ |= (u64)dlut_[ix_] << (4 * i_);
      P_ += (unsigned)__popc(mn_);
    }
    d_ &= am;
    unsigned plo_ = 0u, phi_ = 0u;
    {
      const unsigned a1_ = x1qA[0], b1_ = x1qA[1], c1_ = x1qA[2];
      const unsigned v1_0 = a1_ & 0xFFFu, v1_1 = (a1_ >> 12) & 0xFFFu, v1_2 = ((a1_ >> 24) | (b1_ << 8)) & 0xFFFu, v1_3 = (b1_ >> 4) & 0xFFFu;
      const unsigned v1_4 = (b1_ >> 16) & 0xFFFu, v1_5 = ((b1_ >> 28) | (c1_ << 4)) & 0xFFFu, v1_6 = (c1_ >> 8) & 0xFFFu, v1_7 = c1_ >> 20;
      {
        const unsigned pw1_ = v1_0 | (v1_1 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 15) & 65537u;
      }
      {
        const unsigned pw1_ = v1_2 | (v1_3 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 14) & 131074u;
      }
      {
        const unsigned pw1_ = v1_4 | (v1_5 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 13) & 262148u;
      }
      {
        const unsigned pw1_ = v1_6 | (v1_7 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 12) & 524296u;
      }
    }
    {
      const unsigned a1_ = x1qA[3], b1_ = x1qA[4], c1_ = x1qA[5];
      const unsigned v1_0 = a1_ & 0xFFFu, v1_1 = (a1_ >> 12) & 0xFFFu, v1_2 = ((a1_ >> 24) | (b1_ << 8)) & 0xFFFu, v1_3 = (b1_ >> 4) & 0xFFFu;
      const unsigned v1_4 = (b1_ >> 16) & 0xFFFu, v1_5 = ((b1_ >> 28) | (c1_ << 4)) & 0xFFFu, v1_6 = (c1_ >> 8) & 0xFFFu, v1_7 = c1_ >> 20;
      {
        const unsigned pw1_ = v1_0 | (v1_1 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 11) & 1048592u;
      }
      {
        const unsigned pw1_ = v1_2 | (v1_3 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 10) & 2097184u;
      }
      {
        const unsigned pw1_ = v1_4 | (v1_5 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 9) & 4194368u;
      }
      {
        const unsigned pw1_ = v1_6 | (v1_7 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 8) & 8388736u;
      }
    }
    {
      const unsigned a1_ = x1qA[6], b1_ = x1qA[7], c1_ = x1qA[8];
      const unsigned v1_0 = a1_ & 0xFFFu, v1_1 = (a1_ >> 12) & 0xFFFu, v1_2 = ((a1_ >> 24) | (b1_ << 8)) & 0xFFFu, v1_3 = (b1_ >> 4) & 0xFFFu;
      const unsigned v1_4 = (b1_ >> 16) & 0xFFFu, v1_5 = ((b1_ >> 28) | (c1_ << 4)) & 0xFFFu, v1_6 = (c1_ >> 8) & 0xFFFu, v1_7 = c1_ >> 20;
      {
        const unsigned pw1_ = v1_0 | (v1_1 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 7) & 16777472u;
      }
      {
        const unsigned pw1_ = v1_2 | (v1_3 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 6) & 33554944u;
      }
      {
        const unsigned pw1_ = v1_4 | (v1_5 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 5) & 67109888u;
      }
      {
        const unsigned pw1_ = v1_6 | (v1_7 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 4) & 134219776u;
      }
    }
    {
      const unsigned a1_ = x1qA[9], b1_ = x1qA[10], c1_ = x1qA[11];
      const unsigned v1_0 = a1_ & 0xFFFu, v1_1 = (a1_ >> 12) & 0xFFFu, v1_2 = ((a1_ >> 24) | (b1_ << 8)) & 0xFFFu, v1_3 = (b1_ >> 4) & 0xFFFu;
      const unsigned v1_4 = (b1_ >> 16) & 0xFFFu, v1_5 = ((b1_ >> 28) | (c1_ << 4)) & 0xFFFu, v1_6 = (c1_ >> 8) & 0xFFFu, v1_7 = c1_ >> 20;
      {
        const unsigned pw1_ = v1_0 | (v1_1 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 3) & 268439552u;
      }
      {
        const unsigned pw1_ = v1_2 | (v1_3 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 2) & 536879104u;
      }
      {
        const unsigned pw1_ = v1_4 | (v1_5 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 1) & 1073758208u;
      }
      {
        const unsigned pw1_ = v1_6 | (v1_7 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        plo_ |= (s2_ >> 0) & 2147516416u;
      }
    }
    {
      const unsigned a1_ = x1qA[12], b1_ = x1qA[13], c1_ = x1qA[14];
      const unsigned v1_0 = a1_ & 0xFFFu, v1_1 = (a1_ >> 12) & 0xFFFu, v1_2 = ((a1_ >> 24) | (b1_ << 8)) & 0xFFFu, v1_3 = (b1_ >> 4) & 0xFFFu;
      const unsigned v1_4 = (b1_ >> 16) & 0xFFFu, v1_5 = ((b1_ >> 28) | (c1_ << 4)) & 0xFFFu, v1_6 = (c1_ >> 8) & 0xFFFu, v1_7 = c1_ >> 20;
      {
        const unsigned pw1_ = v1_0 | (v1_1 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 15) & 65537u;
      }
      {
        const unsigned pw1_ = v1_2 | (v1_3 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 14) & 131074u;
      }
      {
        const unsigned pw1_ = v1_4 | (v1_5 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 13) & 262148u;
      }
      {
        const unsigned pw1_ = v1_6 | (v1_7 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 12) & 524296u;
      }
    }
    {
      const unsigned a1_ = x1qA[15], b1_ = x1qA[16], c1_ = x1qA[17];
      const unsigned v1_0 = a1_ & 0xFFFu, v1_1 = (a1_ >> 12) & 0xFFFu, v1_2 = ((a1_ >> 24) | (b1_ << 8)) & 0xFFFu, v1_3 = (b1_ >> 4) & 0xFFFu;
      const unsigned v1_4 = (b1_ >> 16) & 0xFFFu, v1_5 = ((b1_ >> 28) | (c1_ << 4)) & 0xFFFu, v1_6 = (c1_ >> 8) & 0xFFFu, v1_7 = c1_ >> 20;
      {
        const unsigned pw1_ = v1_0 | (v1_1 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 11) & 1048592u;
      }
      {
        const unsigned pw1_ = v1_2 | (v1_3 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 10) & 2097184u;
      }
      {
        const unsigned pw1_ = v1_4 | (v1_5 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 9) & 4194368u;
      }
      {
        const unsigned pw1_ = v1_6 | (v1_7 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 8) & 8388736u;
      }
    }
    {
      const unsigned a1_ = x1qA[18], b1_ = x1qA[19], c1_ = x1qA[20];
      const unsigned v1_0 = a1_ & 0xFFFu, v1_1 = (a1_ >> 12) & 0xFFFu, v1_2 = ((a1_ >> 24) | (b1_ << 8)) & 0xFFFu, v1_3 = (b1_ >> 4) & 0xFFFu;
      const unsigned v1_4 = (b1_ >> 16) & 0xFFFu, v1_5 = ((b1_ >> 28) | (c1_ << 4)) & 0xFFFu, v1_6 = (c1_ >> 8) & 0xFFFu, v1_7 = c1_ >> 20;
      {
        const unsigned pw1_ = v1_0 | (v1_1 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 7) & 16777472u;
      }
      {
        const unsigned pw1_ = v1_2 | (v1_3 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 6) & 33554944u;
      }
      {
        const unsigned pw1_ = v1_4 | (v1_5 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 5) & 67109888u;
      }
      {
        const unsigned pw1_ = v1_6 | (v1_7 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 4) & 134219776u;
      }
    }
    {
      const unsigned a1_ = x1qA[21], b1_ = x1qA[22], c1_ = x1qA[23];
      const unsigned v1_0 = a1_ & 0xFFFu, v1_1 = (a1_ >> 12) & 0xFFFu, v1_2 = ((a1_ >> 24) | (b1_ << 8)) & 0xFFFu, v1_3 = (b1_ >> 4) & 0xFFFu;
      const unsigned v1_4 = (b1_ >> 16) & 0xFFFu, v1_5 = ((b1_ >> 28) | (c1_ << 4)) & 0xFFFu, v1_6 = (c1_ >> 8) & 0xFFFu, v1_7 = c1_ >> 20;
      {
        const unsigned pw1_ = v1_0 | (v1_1 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 3) & 268439552u;
      }
      {
        const unsigned pw1_ = v1_2 | (v1_3 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 2) & 536879104u;
      }
      {
        const unsigned pw1_ = v1_4 | (v1_5 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 1) & 1073758208u;
      }
      {
        const unsigned pw1_ = v1_6 | (v1_7 << 16);
        const unsigned s2_ = ((0u) | (hs_rng2(pw1_, hs_c16lo((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)), hs_c16hi((a.CL1 - a.P12O_1), (a.CH1 - a.P12O_1)))));
        phi_ |= (s2_ >> 0) & 2147516416u;
      }
    }
    plo_ = hs_unzip16(plo_);
    phi_ = hs_unzip16(phi_);
    d_ &= ~(((u64)phi_ << 32) | (u64)plo_);
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
      const u64* PKt_ = a.PK + tb0;
      const int ce0 = cb + 0 + ln;
      const bool cok0 = ce0 < wn_;
      const int cof0 = cok0 ? (int)lst_[wq][ce0] : 0;
      const i64 crow0 = tb0 + (i64)cof0;
      const int ce1 = cb + 64 + ln;
      const bool cok1 = ce1 < wn_;
      const int cof1 = cok1 ? (int)lst_[wq][ce1] : 0;
      const i64 crow1 = tb0 + (i64)cof1;
      const int ce2 = cb + 128 + ln;
      const bool cok2 = ce2 < wn_;
      const int cof2 = cok2 ? (int)lst_[wq][ce2] : 0;
      const i64 crow2 = tb0 + (i64)cof2;
      const int ce3 = cb + 192 + ln;
      const bool cok3 = ce3 < wn_;
      const int cof3 = cok3 ? (int)lst_[wq][ce3] : 0;
      const i64 crow3 = tb0 + (i64)cof3;
      const u64 pk0_ = PKt_[cof0];
      const int r2_c0 = (int)((int)(unsigned)(pk0_ >> 0));
      const i64 q2_c0 = a.B2 + (i64)((int)(unsigned)(pk0_ >> 0));
      const double x2_c0 = (double)((double)(a.B2 + (i64)((int)(unsigned)(pk0_ >> 0))) * a.R2);
      const int r3_c0 = (int)((signed char)(unsigned char)(pk0_ >> 32));
      const i64 q3_c0 = a.B3 + (i64)((signed char)(unsigned char)(pk0_ >> 32));
      const double x3_c0 = (double)((double)(a.B3 + (i64)((signed char)(unsigned char)(pk0_ >> 32))) * a.R3);
      const u64 pk1_ = PKt_[cof1];
      const int r2_c1 = (int)((int)(unsigned)(pk1_ >> 0));
      const i64 q2_c1 = a.B2 + (i64)((int)(unsigned)(pk1_ >> 0));
      const double x2_c1 = (double)((double)(a.B2 + (i64)((int)(unsigned)(pk1_ >> 0))) * a.R2);
      const int r3_c1 = (int)((signed char)(unsigned char)(pk1_ >> 32));
      const i64 q3_c1 = a.B3 + (i64)((signed char)(unsigned char)(pk1_ >> 32));
      const double x3_c1 = (double)((double)(a.B3 + (i64)((signed char)(unsigned char)(pk1_ >> 32))) * a.R3);
      const u64 pk2_ = PKt_[cof2];
      const int r2_c2 = (int)((int)(unsigned)(pk2_ >> 0));
      const i64 q2_c2 = a.B2 + (i64)((int)(unsigned)(pk2_ >> 0));
      const double x2_c2 = (double)((double)(a.B2 + (i64)((int)(unsigned)(pk2_ >> 0))) * a.R2);
      const int r3_c2 = (int)((signed char)(unsigned char)(pk2_ >> 32));
      const i64 q3_c2 = a.B3 + (i64)((signed char)(unsigned char)(pk2_ >> 32));
      const double x3_c2 = (double)((double)(a.B3 + (i64)((signed char)(unsigned char)(pk2_ >> 32))) * a.R3);
      const u64 pk3_ = PKt_[cof3];
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
