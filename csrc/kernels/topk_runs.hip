// Run top-K candidates (exec/hash_agg.py TopKPlan, generated walk exec/jit_runs.py): every
// wavefront of the key-run walk leaves its best K entries in K fixed slots (keys, order-value
// images, per-aggregate sums / counts; empty slots carry the image of -inf), its K-th best value
// (WTH) and the largest value it dropped (DMX), all as order-preserving signed 64-bit images.
// Two small kernels finish the selection on the device, with no atomics in the walk itself:
//
//   hs_topk_runs_threshold: ctl[0] = max WTH (a value below it has K > k better ones: it can not
//                           reach the top k), ctl[2] = max DMX;
//   hs_topk_runs_compact:   the slots at or above ctl[0] appended to dense output arrays
//                           (wavefront-aggregated counter ctl[1]; at most ocap kept).
//
// C ABI, launched by the Python executor on the query stream.
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ long long wave_max(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const long long u = __shfl_xor(v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}

__global__ __launch_bounds__(kBlock) void topk_runs_threshold_kernel(
    const long long* __restrict__ wth, const long long* __restrict__ dmx, long long n,
    long long* __restrict__ ctl) {
  long long a = LLONG_MIN, b = LLONG_MIN;
  const long long stride = (long long)gridDim.x * kBlock;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    a = wth[i] > a ? wth[i] : a;
    b = dmx[i] > b ? dmx[i] : b;
  }
  a = wave_max(a);
  b = wave_max(b);
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&ctl[0], a);
    atomicMax(&ctl[2], b);
  }
}

__global__ __launch_bounds__(kBlock) void topk_runs_compact_kernel(
    const unsigned long long* __restrict__ keys, const long long* __restrict__ vimg,
    const double* __restrict__ sums, const long long* __restrict__ cnts, int NA, long long cap,
    long long* __restrict__ ctl, long long ocap, unsigned long long* __restrict__ okeys,
    double* __restrict__ osums, long long* __restrict__ ocnts) {
  const long long thr = ctl[0];
  const int lane = threadIdx.x & 63;
  const long long stride = (long long)gridDim.x * kBlock;
  for (long long base = (long long)blockIdx.x * kBlock; base < cap; base += stride) {
    const long long i = base + threadIdx.x;
    const bool live = i < cap && keys[i] != ~0ull && vimg[i] >= thr;
    const unsigned long long m = __ballot(live);
    if (m == 0ull) continue;
    long long at = 0;
    if (lane == 0) at = (long long)atomicAdd((unsigned long long*)&ctl[1], (unsigned long long)__popcll(m));
    at = __shfl(at, 0, 64) + __popcll(m & ((1ull << lane) - 1ull));
    if (live && at < ocap) {
      okeys[at] = keys[i];
      for (int a = 0; a < NA; ++a) {
        osums[(long long)a * ocap + at] = sums[(long long)a * cap + i];
        ocnts[(long long)a * ocap + at] = cnts[(long long)a * cap + i];
      }
    }
  }
}

int grid_for(long long n) {
  long long g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return (int)g;
}

}  // namespace

extern "C" {

int hs_topk_runs_threshold(const long long* wth, const long long* dmx, long long n, long long* ctl,
                           void* stream) {
  if (n <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(topk_runs_threshold_kernel, dim3(grid_for(n)), dim3(kBlock), 0,
                     (hipStream_t)stream, wth, dmx, n, ctl);
  return (int)hipGetLastError();
}

int hs_topk_runs_compact(const unsigned long long* keys, const long long* vimg, const double* sums,
                         const long long* cnts, int NA, long long cap, long long* ctl,
                         long long ocap, unsigned long long* okeys, double* osums,
                         long long* ocnts, void* stream) {
  if (cap <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(topk_runs_compact_kernel, dim3(grid_for(cap)), dim3(kBlock), 0,
                     (hipStream_t)stream, keys, vimg, sums, cnts, NA, cap, ctl, ocap, okeys, osums,
                     ocnts);
  return (int)hipGetLastError();
}

}  // extern "C"
