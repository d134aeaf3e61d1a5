// Run top-K threshold (exec/hash_agg.py TopKPlan, generated walk exec/jit_runs.py): every
// wavefront of the key-run walk leaves its best K entries in K fixed slots (keys, unsigned
// smallest-first order images, per-aggregate sums / counts), its K-th best value (WTH) and the
// largest value it dropped (DMX), both as order-preserving signed 64-bit images.  One small
// kernel reduces those over wavefronts, with no atomics in the walk itself:
//
//   hs_topk_runs_threshold: ctl[0] = max WTH, ctl[2] = max DMX - every value the slots do not
//                           hold is at most max(ctl[0], ctl[2]).
//
// The slots' top k are then picked by the radix select of hash_agg.hip (hs_topk_select) over
// the slot images, and the host checks that bound against the k-th best value.
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

}  // extern "C"
