// Packed row exchange for the multi-GPU index build (SURVEY §2.3 K3 "all-to-all", §5.8).
//
// The Spark hash-partition shuffle becomes ONE uneven all-to-all of a byte buffer per batch of
// rows, not one collective per column.  Rows go to rank dest = bucket % world.  The send buffer
// holds one contiguous segment per destination; inside a segment every column is a dense run of
// that destination's values (16-byte aligned), in source row order (stable):
//
//   segment d = [col 0: cnt_d values][pad][col 1: cnt_d values][pad] ... [col C-1 ...][pad]
//
// Kernels:
//   hs_xch_count   per 4096-row tile, rows per destination (LDS counters)      -> tile_cnt[T][W]
//   hs_xch_scan    one block: tile counts -> tile bases (exclusive over tiles), per-destination
//                  totals and the byte layout of every segment                 -> meta
//   hs_xch_pack    per tile: stable in-tile rank of each row among rows with the same destination
//                  (wave ballots + per-wave LDS prefix), then every column value is written to
//                  its slot — all columns in one launch
//   hs_xch_unpack  receiver: a table of (src, dst, count, elem bytes) copies — every (batch,
//                  source rank, column) run of the received buffers into the final columns —
//                  in one launch
//
// meta (int64) layout, written by hs_xch_scan: [0, W) rows per destination; [W, 2W) left for the
// counts all-to-all to land in; [2W, 2W + W*(C+1)) byte offset of (segment d, column c) from the
// buffer start, with entry C = end of segment d.  Host code reads it with one D2H copy.
#include "hs_common.h"

#define XCH_MAX_COLS 32
#define XCH_MAX_DEST 64
#define XCH_TILE 4096
#define XCH_BLOCK 256

struct XchParams {
  const void* src[XCH_MAX_COLS];
  int32_t elem_bytes[XCH_MAX_COLS];  // 1, 2, 4 or 8
  int32_t ncols;
  int32_t world;
};

struct XchCopy {
  const void* src;
  void* dst;
  int64_t count;       // elements
  int32_t elem_bytes;  // 1, 2, 4 or 8
  int32_t pad;
};

__device__ __forceinline__ int xch_dest(const int32_t* bucket, int64_t row, int world) {
  return bucket[row] % world;  // bucket ids are non-negative (pmod)
}

__global__ __launch_bounds__(XCH_BLOCK) void hs_xch_count_kernel(const int32_t* __restrict__ bucket,
                                                                 int64_t n, int world,
                                                                 int64_t* __restrict__ tile_cnt) {
  __shared__ int32_t cnt[XCH_MAX_DEST];
  for (int d = threadIdx.x; d < world; d += blockDim.x) cnt[d] = 0;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * XCH_TILE;
  const int64_t hi = min(lo + (int64_t)XCH_TILE, n);
  for (int64_t r = lo + threadIdx.x; r < hi; r += blockDim.x) atomicAdd(&cnt[xch_dest(bucket, r, world)], 1);
  __syncthreads();
  for (int d = threadIdx.x; d < world; d += blockDim.x)
    tile_cnt[(int64_t)blockIdx.x * world + d] = cnt[d];
}

// One block of 256: exclusive scan of every destination's tile counts (in place) + layout.
__global__ __launch_bounds__(XCH_BLOCK) void hs_xch_scan_kernel(int64_t* __restrict__ tile_cnt,
                                                                int64_t ntiles, XchParams p,
                                                                int64_t* __restrict__ meta) {
  __shared__ int64_t part[XCH_BLOCK];
  __shared__ int64_t total[XCH_MAX_DEST];
  const int W = p.world;
  for (int d = 0; d < W; ++d) {
    int64_t carry = 0;
    for (int64_t base = 0; base < ntiles; base += XCH_BLOCK) {
      const int64_t t = base + threadIdx.x;
      const int64_t v = t < ntiles ? tile_cnt[t * W + d] : 0;
      part[threadIdx.x] = v;
      __syncthreads();
      // Hillis-Steele inclusive scan over 256 entries (8 steps; tiny next to the pack pass)
      for (int off = 1; off < XCH_BLOCK; off <<= 1) {
        const int64_t add = threadIdx.x >= off ? part[threadIdx.x - off] : 0;
        __syncthreads();
        part[threadIdx.x] += add;
        __syncthreads();
      }
      if (t < ntiles) tile_cnt[t * W + d] = carry + part[threadIdx.x] - v;
      carry += part[XCH_BLOCK - 1];
      __syncthreads();
    }
    if (threadIdx.x == 0) total[d] = carry;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    int64_t off = 0;
    int64_t* lay = meta + 2 * W;
    for (int d = 0; d < W; ++d) {
      meta[d] = total[d];
      for (int c = 0; c < p.ncols; ++c) {
        lay[d * (p.ncols + 1) + c] = off;
        off += (total[d] * p.elem_bytes[c] + 15) & ~(int64_t)15;
      }
      lay[d * (p.ncols + 1) + p.ncols] = off;
    }
  }
}

__device__ __forceinline__ void xch_copy_elem(const void* src, int64_t si, void* dst, int64_t di,
                                              int eb) {
  switch (eb) {
    case 1: ((uint8_t*)dst)[di] = ((const uint8_t*)src)[si]; break;
    case 2: ((uint16_t*)dst)[di] = ((const uint16_t*)src)[si]; break;
    case 4: ((uint32_t*)dst)[di] = ((const uint32_t*)src)[si]; break;
    default: ((uint64_t*)dst)[di] = ((const uint64_t*)src)[si]; break;
  }
}

__global__ __launch_bounds__(XCH_BLOCK) void hs_xch_pack_kernel(XchParams p,
                                                                const int32_t* __restrict__ bucket,
                                                                int64_t n,
                                                                const int64_t* __restrict__ tile_base,
                                                                const int64_t* __restrict__ meta,
                                                                uint8_t* __restrict__ send) {
  constexpr int NW = XCH_BLOCK / HS_WAVE;
  __shared__ int64_t running[XCH_MAX_DEST];
  __shared__ int32_t wave_cnt[NW][XCH_MAX_DEST];
  const int W = p.world;
  const int wave = threadIdx.x / HS_WAVE;
  const int lane = threadIdx.x & (HS_WAVE - 1);
  const int64_t tile = blockIdx.x;
  for (int d = threadIdx.x; d < W; d += blockDim.x) running[d] = tile_base[tile * W + d];
  const int64_t* lay = meta + 2 * W;
  const int64_t lo = tile * XCH_TILE;
  const int64_t hi = min(lo + (int64_t)XCH_TILE, n);
  const uint64_t lt = hs_lanemask_lt();
  __syncthreads();
  for (int64_t r0 = lo; r0 < hi; r0 += XCH_BLOCK) {
    const int64_t row = r0 + threadIdx.x;
    const bool live = row < hi;
    const int d = live ? xch_dest(bucket, row, W) : -1;
    int rank = 0;
    for (int dd = 0; dd < W; ++dd) {
      const uint64_t m = __ballot(d == dd);
      if (d == dd) rank = __popcll(m & lt);
      if (lane == 0) wave_cnt[wave][dd] = __popcll(m);
    }
    __syncthreads();
    if (live) {
      int64_t pos = running[d] + rank;
      for (int w = 0; w < wave; ++w) pos += wave_cnt[w][d];
      const int64_t* seg = lay + (int64_t)d * (p.ncols + 1);
      for (int c = 0; c < p.ncols; ++c)
        xch_copy_elem(p.src[c], row, send + seg[c], pos, p.elem_bytes[c]);
    }
    __syncthreads();
    for (int dd = threadIdx.x; dd < W; dd += blockDim.x) {
      int64_t s = 0;
      for (int w = 0; w < NW; ++w) s += wave_cnt[w][dd];
      running[dd] += s;
    }
    __syncthreads();
  }
}

template <typename T>
__device__ __forceinline__ void xch_copy_run(const T* __restrict__ s, T* __restrict__ d, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) d[i] = s[i];
}

__global__ __launch_bounds__(XCH_BLOCK) void hs_xch_unpack_kernel(const XchCopy* __restrict__ tab) {
  const XchCopy c = tab[blockIdx.y];
  switch (c.elem_bytes) {
    case 1: xch_copy_run((const uint8_t*)c.src, (uint8_t*)c.dst, c.count); break;
    case 2: xch_copy_run((const uint16_t*)c.src, (uint16_t*)c.dst, c.count); break;
    case 4: xch_copy_run((const uint32_t*)c.src, (uint32_t*)c.dst, c.count); break;
    default: xch_copy_run((const uint64_t*)c.src, (uint64_t*)c.dst, c.count); break;
  }
}

// Row counts per bucket id in [0, B) (LDS-privatised; B <= 16384), counts zeroed by the caller.
__global__ __launch_bounds__(XCH_BLOCK) void hs_histogram_kernel(const int32_t* __restrict__ ids,
                                                                 int64_t n, int B,
                                                                 int64_t* __restrict__ counts) {
  extern __shared__ __attribute__((aligned(16))) int32_t h[];
  for (int i = threadIdx.x; i < B; i += blockDim.x) h[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int32_t b = ids[i];
    if (b >= 0 && b < B) atomicAdd(&h[b], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < B; i += blockDim.x)
    if (h[i]) atomicAdd((unsigned long long*)&counts[i], (unsigned long long)h[i]);
}

extern "C" {

int hs_histogram(const int32_t* ids, int64_t n, int B, int64_t* counts, void* stream) {
  if (B <= 0 || B > 16384) return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  HS_CHECK(hipMemsetAsync(counts, 0, (size_t)B * sizeof(int64_t), s));
  if (n == 0) return 0;
  int64_t g = (n + XCH_BLOCK - 1) / XCH_BLOCK;
  if (g > 1024) g = 1024;
  hipLaunchKernelGGL(hs_histogram_kernel, dim3((unsigned)g), dim3(XCH_BLOCK),
                     (size_t)B * sizeof(int32_t), s, ids, n, B, counts);
  return (int)hipGetLastError();
}

int hs_xch_params_size() { return (int)sizeof(XchParams); }
int hs_xch_copy_size() { return (int)sizeof(XchCopy); }
int hs_xch_tile_rows() { return XCH_TILE; }

// tile_cnt: int64 [ceil(n / XCH_TILE) * world] scratch; meta: int64 [2W + W*(C+1)].
// send must hold meta's last layout entry bytes (<= n * row_bytes + 16 * W * C).
int hs_xch_pack(const XchParams* p, const int32_t* bucket, int64_t n, int64_t* tile_cnt,
                int64_t* meta, uint8_t* send, void* stream) {
  if (p->world < 1 || p->world > XCH_MAX_DEST || p->ncols < 0 || p->ncols > XCH_MAX_COLS)
    return (int)hipErrorInvalidValue;
  hipStream_t s = (hipStream_t)stream;
  const int64_t ntiles = (n + XCH_TILE - 1) / XCH_TILE;
  if (ntiles > 0)
    hipLaunchKernelGGL(hs_xch_count_kernel, dim3((unsigned)ntiles), dim3(XCH_BLOCK), 0, s, bucket,
                       n, p->world, tile_cnt);
  hipLaunchKernelGGL(hs_xch_scan_kernel, dim3(1), dim3(XCH_BLOCK), 0, s, tile_cnt, ntiles, *p,
                     meta);
  if (ntiles > 0)
    hipLaunchKernelGGL(hs_xch_pack_kernel, dim3((unsigned)ntiles), dim3(XCH_BLOCK), 0, s, *p,
                       bucket, n, tile_cnt, meta, send);
  return (int)hipGetLastError();
}

// tab: device array of ncopies XchCopy; max_count = the largest count (sizes the grid).
int hs_xch_unpack(const XchCopy* tab, int ncopies, int64_t max_count, void* stream) {
  if (ncopies <= 0 || max_count <= 0) return 0;
  if (ncopies > 65535) return (int)hipErrorInvalidValue;
  int64_t gx = (max_count + XCH_BLOCK - 1) / XCH_BLOCK;
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(hs_xch_unpack_kernel, dim3((unsigned)gx, (unsigned)ncopies), dim3(XCH_BLOCK),
                     0, (hipStream_t)stream, tab);
  return (int)hipGetLastError();
}

}  // extern "C"
