// Lossless HBM column compaction (exec/encoding.py): one probe pass + one encode pass.
//
// hs_compact_probe reads a column once and reduces everything the encoder decides on:
//   integers: min/max over valid rows;
//   float64:  any non-finite value, any -0.0, and for every decimal scale k = 0..4 whether
//             q = rint(x * 10^k) reproduces x bit for bit under the IEEE division the generated
//             kernels decode with (q / 10^k), whether |q| reaches 2^52, and min/max of q.
// Per-wave reductions go through shuffles, per-block ones through LDS; each block writes one
// partial record and a one-block pass folds them (no global atomics).  This replaces the chain of PyTorch elementwise/reduce launches (mul, round,
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
constexpr int kProbeBlocks = 1024;   // stage-1 blocks (grid-stride over the column)
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

__constant__ double kPow10[kMaxK + 1] = {1.0, 10.0, 100.0, 1000.0, 10000.0};

// per-field combine of the result block: 0 = or, 1 = min, 2 = max
__host__ __device__ inline int field_kind(int f) {
  if (f == R_IMIN) return 1;
  if (f == R_IMAX) return 2;
  if (f >= R_K) {
    const int j = (f - R_K) & 3;
    return j == 2 ? 1 : (j == 3 ? 2 : 0);
  }
  return 0;
}

__device__ inline int64_t field_init(int f) {
  const int k = field_kind(f);
  return k == 1 ? LLONG_MAX : (k == 2 ? LLONG_MIN : 0);
}

__device__ inline int64_t combine(int kind, int64_t a, int64_t b) {
  return kind == 1 ? (a < b ? a : b) : (kind == 2 ? (a > b ? a : b) : (a | b));
}

// Stage 1: every block reduces its grid-stride share to one partial result record (wave
// shuffles, then the block's waves through LDS) -- no global atomics: with thousands of waves
// hammering one int64 the atomics serialised (~0.5 ms even for an 864K-row column).
__global__ __launch_bounds__(256) void hs_compact_probe_kernel(const void* __restrict__ data,
                                                               const uint8_t* __restrict__ valid,
                                                               int64_t n, int type, int maxk,
                                                               long long* __restrict__ partials) {
  __shared__ int64_t red[4][R_SIZE];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t r[R_SIZE];
#pragma unroll
  for (int f = 0; f < R_SIZE; ++f) r[f] = field_init(f);
  if (type != T_F64) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      if (valid && !valid[i]) continue;
      const int64_t v = load_int(data, type, i);
      r[R_IMIN] = v < r[R_IMIN] ? v : r[R_IMIN];
      r[R_IMAX] = v > r[R_IMAX] ? v : r[R_IMAX];
      r[R_ANY] = 1;
    }
  } else {
    const double* x = (const double*)data;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
      if (valid && !valid[i]) continue;
      const double v = x[i];
      r[R_ANY] = 1;
      if (!isfinite(v)) {
        r[R_NONFINITE] = 1;
        continue;
      }
      if (v == 0.0 && signbit(v)) r[R_NEGZERO] = 1;
#pragma unroll
      for (int k = 0; k <= kMaxK; ++k) {
        if (k > maxk) break;
        const double q = rint(v * kPow10[k]);
        if (fabs(q) >= 4503599627370496.0) {   // 2^52
          r[R_K + 4 * k + 1] = 1;
          continue;
        }
        const double back = q / kPow10[k];   // IEEE division, as the kernels decode
        if (__double_as_longlong(back) != __double_as_longlong(v)) r[R_K + 4 * k] = 1;
        const int64_t qi = (int64_t)q;
        r[R_K + 4 * k + 2] = qi < r[R_K + 4 * k + 2] ? qi : r[R_K + 4 * k + 2];
        r[R_K + 4 * k + 3] = qi > r[R_K + 4 * k + 3] ? qi : r[R_K + 4 * k + 3];
      }
    }
  }
#pragma unroll
  for (int f = 0; f < R_SIZE; ++f) {
    const int kind = field_kind(f);
    int64_t v = r[f];
    for (int o = 32; o > 0; o >>= 1) v = combine(kind, v, __shfl_xor(v, o));
    if (lane == 0) red[w][f] = v;
  }
  __syncthreads();
  if (threadIdx.x < R_SIZE) {
    const int f = threadIdx.x, kind = field_kind(f);
    int64_t v = red[0][f];
    for (int ww = 1; ww < (int)(blockDim.x >> 6); ++ww) v = combine(kind, v, red[ww][f]);
    partials[(int64_t)blockIdx.x * R_SIZE + f] = v;
  }
}

// Stage 2: one thread per field folds the blocks' partial records into the result block.
__global__ __launch_bounds__(64) void hs_compact_probe_final_kernel(
    const long long* __restrict__ partials, int nblocks, long long* __restrict__ res) {
  const int f = threadIdx.x;
  if (f >= R_SIZE) return;
  const int kind = field_kind(f);
  int64_t v = field_init(f);
  for (int b = 0; b < nblocks; ++b) v = combine(kind, v, partials[(int64_t)b * R_SIZE + f]);
  res[f] = v;
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

// partial records of stage 1 (int64 elements of the caller's workspace)
int64_t hs_compact_probe_ws_elems() { return (int64_t)kProbeBlocks * R_SIZE; }

// res: R_SIZE int64s (written entirely); ws: hs_compact_probe_ws_elems() int64s
int hs_compact_probe(const void* data, const uint8_t* valid, int64_t n, int type, int maxk,
                     int64_t* res, int64_t* ws, void* stream) {
  if (maxk < 0 || maxk > kMaxK) return -1;
  (void)hipGetLastError();
  int64_t b = (n + 255) / 256;
  const int nb = (int)(b < 1 ? 1 : (b > kProbeBlocks ? kProbeBlocks : b));
  hipLaunchKernelGGL(hs_compact_probe_kernel, dim3(nb), dim3(256), 0, (hipStream_t)stream, data,
                     valid, n, type, maxk, (long long*)ws);
  hipLaunchKernelGGL(hs_compact_probe_final_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream,
                     (const long long*)ws, nb, (long long*)res);
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
