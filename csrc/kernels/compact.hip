// Lossless HBM column compaction (exec/encoding.py): one probe pass + one encode pass.
//
// hs_compact_probe reads a column once and reduces everything the encoder decides on:
//   integers: min/max over valid rows;
//   float64:  any non-finite value, any -0.0, and for every decimal scale k = 0..4 whether
//             q = rint(x * 10^k) reproduces x bit for bit under the IEEE division the generated
//             kernels decode with (q / 10^k), whether |q| reaches 2^52, and min/max of q.
// Per-wave reductions go through DPP/shuffles, then one atomic per wave into a small int64
// result block.  This replaces the chain of PyTorch elementwise/reduce launches (mul, round,
// div, abs, compare, all, aminmax per scale) and their host round trips with one launch and one
// 256-byte readback.
//
// hs_compact_encode writes the narrow codes: code = value - base (value = q for a decimal
// scale), invalid rows get the code of `fill`.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

namespace {

enum : int { T_I8 = 0, T_I16, T_I32, T_I64, T_F32, T_F64, T_BOOL, T_U32, T_U64 };
constexpr int kMaxK = 4;
// result block layout (int64)
enum : int {
  R_ANY = 0, R_NONFINITE = 1, R_NEGZERO = 2, R_IMIN = 3, R_IMAX = 4,
  R_K = 5,           // + 4*k: inexact, overflow, qmin, qmax
  R_SIZE = R_K + 4 * (kMaxK + 1)
};

__device__ inline int64_t load_int(const void* d, int t, int64_t i) {
  switch (t) {
    case T_I8: return ((const int8_t*)d)[i];
    case T_I16: return ((const int16_t*)d)[i];
    case T_I32: return ((const int32_t*)d)[i];
    case T_U32: return (int64_t)((const uint32_t*)d)[i];
    case T_BOOL: return ((const uint8_t*)d)[i];
    default: return ((const int64_t*)d)[i];
  }
}

__device__ inline int64_t wave_min(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t w = __shfl_xor(v, o);
    v = w < v ? w : v;
  }
  return v;
}

__device__ inline int64_t wave_max(int64_t v) {
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t w = __shfl_xor(v, o);
    v = w > v ? w : v;
  }
  return v;
}

__constant__ double kPow10[kMaxK + 1] = {1.0, 10.0, 100.0, 1000.0, 10000.0};

__global__ __launch_bounds__(256) void hs_compact_probe_kernel(const void* __restrict__ data,
                                                               const uint8_t* __restrict__ valid,
                                                               int64_t n, int type, int maxk,
                                                               long long* __restrict__ res) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int lane = threadIdx.x & 63;
  int any = 0;
  if (type != T_F64) {
    int64_t mn = LLONG_MAX, mx = LLONG_MIN;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      if (valid && !valid[i]) continue;
      const int64_t v = load_int(data, type, i);
      mn = v < mn ? v : mn;
      mx = v > mx ? v : mx;
      any = 1;
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    const bool a = __any(any);
    if (lane == 0 && a) {
      atomicMin(&res[R_IMIN], (long long)mn);
      atomicMax(&res[R_IMAX], (long long)mx);
      atomicOr((unsigned long long*)&res[R_ANY], 1ull);
    }
    return;
  }
  const double* x = (const double*)data;
  int nonfinite = 0, negzero = 0;
  int inexact[kMaxK + 1] = {0}, over[kMaxK + 1] = {0};
  int64_t qmin[kMaxK + 1], qmax[kMaxK + 1];
#pragma unroll
  for (int k = 0; k <= kMaxK; ++k) {
    qmin[k] = LLONG_MAX;
    qmax[k] = LLONG_MIN;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (valid && !valid[i]) continue;
    const double v = x[i];
    any = 1;
    if (!isfinite(v)) {
      nonfinite = 1;
      continue;
    }
    if (v == 0.0 && signbit(v)) negzero = 1;
#pragma unroll
    for (int k = 0; k <= kMaxK; ++k) {
      if (k > maxk) break;
      const double q = rint(v * kPow10[k]);
      if (fabs(q) >= 4503599627370496.0) {   // 2^52
        over[k] = 1;
        continue;
      }
      const double back = q / kPow10[k];   // IEEE division, as the kernels decode
      if (__double_as_longlong(back) != __double_as_longlong(v)) inexact[k] = 1;
      const int64_t qi = (int64_t)q;
      qmin[k] = qi < qmin[k] ? qi : qmin[k];
      qmax[k] = qi > qmax[k] ? qi : qmax[k];
    }
  }
  const bool a = __any(any), nf = __any(nonfinite), nz = __any(negzero);
  if (lane == 0 && a) atomicOr((unsigned long long*)&res[R_ANY], 1ull);
  if (lane == 0 && nf) atomicOr((unsigned long long*)&res[R_NONFINITE], 1ull);
  if (lane == 0 && nz) atomicOr((unsigned long long*)&res[R_NEGZERO], 1ull);
#pragma unroll
  for (int k = 0; k <= kMaxK; ++k) {
    if (k > maxk) break;
    const bool ie = __any(inexact[k]), ov = __any(over[k]);
    const int64_t mn = wave_min(qmin[k]), mx = wave_max(qmax[k]);
    if (lane == 0) {
      if (ie) atomicOr((unsigned long long*)&res[R_K + 4 * k], 1ull);
      if (ov) atomicOr((unsigned long long*)&res[R_K + 4 * k + 1], 1ull);
      if (mn != LLONG_MAX) atomicMin(&res[R_K + 4 * k + 2], (long long)mn);
      if (mx != LLONG_MIN) atomicMax(&res[R_K + 4 * k + 3], (long long)mx);
    }
  }
}

template <typename C>
__global__ __launch_bounds__(256) void hs_compact_encode_kernel(const void* __restrict__ data,
                                                                const uint8_t* __restrict__ valid,
                                                                int64_t n, int type, int k,
                                                                int64_t base, int64_t fill,
                                                                C* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t v;
    if (valid && !valid[i]) {
      v = fill;
    } else if (type == T_F64) {
      v = (int64_t)rint(((const double*)data)[i] * kPow10[k]);
    } else {
      v = load_int(data, type, i);
    }
    out[i] = (C)(v - base);
  }
}

inline unsigned grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 4096 ? (b < 1 ? 1 : b) : 4096);
}

}  // namespace

extern "C" {

int hs_compact_result_size() { return R_SIZE; }

// res: R_SIZE int64s, initialised by the caller (mins INT64_MAX, maxes INT64_MIN, flags 0)
int hs_compact_probe(const void* data, const uint8_t* valid, int64_t n, int type, int maxk,
                     int64_t* res, void* stream) {
  if (n <= 0) return 0;
  if (maxk < 0 || maxk > kMaxK) return -1;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hs_compact_probe_kernel, dim3(grid_for(n)), dim3(256), 0,
                     (hipStream_t)stream, data, valid, n, type, maxk, (long long*)res);
  return (int)hipGetLastError();
}

// width 1/2/4 bytes; k = decimal scale digits for float64 columns (ignored for integers)
int hs_compact_encode(const void* data, const uint8_t* valid, int64_t n, int type, int k,
                      int64_t base, int64_t fill, int width, void* out, void* stream) {
  if (n <= 0) return 0;
  if (k < 0 || k > kMaxK) return -1;
  (void)hipGetLastError();
  const dim3 g(grid_for(n)), b(256);
  hipStream_t s = (hipStream_t)stream;
  if (width == 1)
    hipLaunchKernelGGL(hs_compact_encode_kernel<int8_t>, g, b, 0, s, data, valid, n, type, k,
                       base, fill, (int8_t*)out);
  else if (width == 2)
    hipLaunchKernelGGL(hs_compact_encode_kernel<int16_t>, g, b, 0, s, data, valid, n, type, k,
                       base, fill, (int16_t*)out);
  else if (width == 4)
    hipLaunchKernelGGL(hs_compact_encode_kernel<int32_t>, g, b, 0, s, data, valid, n, type, k,
                       base, fill, (int32_t*)out);
  else
    return -1;
  return (int)hipGetLastError();
}

}  // extern "C"
