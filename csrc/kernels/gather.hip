// Column gather by row ids (the permutation apply of K4 and the output materialization of
// K7/K8), one launch for all columns of a table: a 2-D grid (row blocks x columns) so every
// column streams its writes coalesced while the random reads spread over the whole chip.
#include "hs_common.h"

#define GA_MAX_COLS 32

struct GatherCol {
  const void* src;
  void* dst;
  const uint8_t* src_valid;  // nullable
  uint8_t* dst_valid;        // nullable
  int32_t elem_bytes;        // 1, 2, 4, 8
  int32_t pad;
};

struct GatherParams {
  GatherCol cols[GA_MAX_COLS];
  int32_t ncols;
  int32_t idx_is_u32;
};

__global__ __launch_bounds__(256) void hs_gather_kernel(GatherParams p, const void* __restrict__ idx,
                                                        int64_t n) {
  const GatherCol& c = p.cols[blockIdx.y];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t r = p.idx_is_u32 ? (int64_t)((const uint32_t*)idx)[i] : ((const int64_t*)idx)[i];
    switch (c.elem_bytes) {
      case 1: ((uint8_t*)c.dst)[i] = ((const uint8_t*)c.src)[r]; break;
      case 2: ((uint16_t*)c.dst)[i] = ((const uint16_t*)c.src)[r]; break;
      case 4: ((uint32_t*)c.dst)[i] = ((const uint32_t*)c.src)[r]; break;
      default: ((uint64_t*)c.dst)[i] = ((const uint64_t*)c.src)[r]; break;
    }
    if (c.dst_valid) c.dst_valid[i] = c.src_valid ? c.src_valid[r] : (uint8_t)1;
  }
}

// Bucket offsets from sorted bucket ids: off[b] = first i with bucket[i] >= b  (b in [0, B]).
__global__ void hs_bucket_offsets_kernel(const int32_t* __restrict__ sorted_bucket, int64_t n,
                                         int B, int64_t* __restrict__ off) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b > B) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (sorted_bucket[mid] < b) lo = mid + 1; else hi = mid;
  }
  off[b] = lo;
}

extern "C" {

int hs_gather_params_size() { return (int)sizeof(GatherParams); }

int hs_gather(const GatherParams* p, const void* idx, int64_t n, void* stream) {
  if (n == 0 || p->ncols == 0) return 0;
  int64_t gx = (n + 255) / 256;
  if (gx > 2048) gx = 2048;
  hipLaunchKernelGGL(hs_gather_kernel, dim3((unsigned)gx, p->ncols), dim3(256), 0,
                     (hipStream_t)stream, *p, idx, n);
  return (int)hipGetLastError();
}

int hs_bucket_offsets(const int32_t* sorted_bucket, int64_t n, int B, int64_t* off, void* stream) {
  hipLaunchKernelGGL(hs_bucket_offsets_kernel, dim3((B + 1 + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, sorted_bucket, n, B, off);
  return (int)hipGetLastError();
}

}  // extern "C"
