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
    if (r < 0) {   // outer-join padding row: NULL (int64 indices only)
      switch (c.elem_bytes) {
        case 1: ((uint8_t*)c.dst)[i] = 0; break;
        case 2: ((uint16_t*)c.dst)[i] = 0; break;
        case 4: ((uint32_t*)c.dst)[i] = 0; break;
        default: ((uint64_t*)c.dst)[i] = 0; break;
      }
      if (c.dst_valid) c.dst_valid[i] = 0;
      continue;
    }
    switch (c.elem_bytes) {
      case 1: ((uint8_t*)c.dst)[i] = ((const uint8_t*)c.src)[r]; break;
      case 2: ((uint16_t*)c.dst)[i] = ((const uint16_t*)c.src)[r]; break;
      case 4: ((uint32_t*)c.dst)[i] = ((const uint32_t*)c.src)[r]; break;
      default: ((uint64_t*)c.dst)[i] = ((const uint64_t*)c.src)[r]; break;
    }
    if (c.dst_valid) c.dst_valid[i] = c.src_valid ? c.src_valid[r] : (uint8_t)1;
  }
}

// Packed-row gather for permutations of whole tables (K4's permutation apply).  A random row
// read of one column fetches a whole memory sector for a few bytes, once per column; packing
// each row's fields (and validity bytes) into one `row_bytes` record first makes the random
// phase one sector per row: all fields of a record share it, so the per-column reads after the
// first hit the cache.  Field byte offsets within a record: GatherCol.pad (values), and
// `vbase` + column index (validity bytes).
__global__ __launch_bounds__(256) void hs_pack_rows_kernel(GatherParams p, int row_bytes,
                                                           int vbase, int64_t n,
                                                           uint8_t* __restrict__ rows) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint8_t* rec = rows + i * row_bytes;
    for (int c = 0; c < p.ncols; ++c) {
      const GatherCol& g = p.cols[c];
      uint8_t* f = rec + g.pad;
      switch (g.elem_bytes) {
        case 1: *f = ((const uint8_t*)g.src)[i]; break;
        case 2: *(uint16_t*)f = ((const uint16_t*)g.src)[i]; break;
        case 4: *(uint32_t*)f = ((const uint32_t*)g.src)[i]; break;
        default: *(uint64_t*)f = ((const uint64_t*)g.src)[i]; break;
      }
      if (g.dst_valid) rec[vbase + c] = g.src_valid ? g.src_valid[i] : (uint8_t)1;
    }
  }
}

__global__ __launch_bounds__(256) void hs_gather_rows_kernel(GatherParams p, int row_bytes,
                                                             int vbase,
                                                             const uint8_t* __restrict__ rows,
                                                             const void* __restrict__ idx,
                                                             int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t r = p.idx_is_u32 ? (int64_t)((const uint32_t*)idx)[i] : ((const int64_t*)idx)[i];
    const uint8_t* rec = rows + r * row_bytes;
    for (int c = 0; c < p.ncols; ++c) {
      const GatherCol& g = p.cols[c];
      const uint8_t* f = rec + g.pad;
      switch (g.elem_bytes) {
        case 1: ((uint8_t*)g.dst)[i] = *f; break;
        case 2: ((uint16_t*)g.dst)[i] = *(const uint16_t*)f; break;
        case 4: ((uint32_t*)g.dst)[i] = *(const uint32_t*)f; break;
        default: ((uint64_t*)g.dst)[i] = *(const uint64_t*)f; break;
      }
      if (g.dst_valid) g.dst_valid[i] = rec[vbase + c];
    }
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

// Outer / semi / anti joins: mark[idx[i]] = 1 for every matched row id (duplicate ids store the
// same byte, so the races are benign).
__global__ __launch_bounds__(256) void hs_mark_rows_kernel(const int64_t* __restrict__ idx, int64_t n,
                                                           uint8_t* __restrict__ mark) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t r = idx[i];
    if (r >= 0) mark[r] = 1;
  }
}

// Order-preserving selection of the row ids in `rows` whose mark equals `want`: per-block
// counts, an exclusive scan, then the stable write (3 launches, no atomics).
constexpr int kSelItems = 8;
constexpr int kSelChunk = 256 * kSelItems;

__global__ __launch_bounds__(256) void hs_select_marked_count(const int64_t* __restrict__ rows,
                                                              int64_t n,
                                                              const uint8_t* __restrict__ mark,
                                                              int want, int64_t* __restrict__ bc) {
  const int64_t i0 = (int64_t)blockIdx.x * kSelChunk + (int64_t)threadIdx.x * kSelItems;
  int c = 0;
#pragma unroll
  for (int k = 0; k < kSelItems; ++k) {
    const int64_t i = i0 + k;
    c += (i < n && (int)mark[rows[i]] == want) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  __shared__ int ws[4];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) bc[blockIdx.x] = (int64_t)ws[0] + ws[1] + ws[2] + ws[3];
}

__global__ __launch_bounds__(1024) void hs_select_marked_scan(int64_t* __restrict__ v, int64_t nb,
                                                              int64_t* __restrict__ total) {
  __shared__ int64_t part[1024];
  const int64_t per = (nb + blockDim.x - 1) / blockDim.x;
  const int64_t b = (int64_t)threadIdx.x * per;
  const int64_t e = b + per < nb ? b + per : nb;
  int64_t s = 0;
  for (int64_t i = b; i < e; ++i) s += v[i];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t run = 0;
    for (int i = 0; i < (int)blockDim.x; ++i) { const int64_t x = part[i]; part[i] = run; run += x; }
    *total = run;
  }
  __syncthreads();
  int64_t run = part[threadIdx.x];
  for (int64_t i = b; i < e; ++i) { const int64_t x = v[i]; v[i] = run; run += x; }
}

__global__ __launch_bounds__(256) void hs_select_marked_write(const int64_t* __restrict__ rows,
                                                              int64_t n,
                                                              const uint8_t* __restrict__ mark,
                                                              int want,
                                                              const int64_t* __restrict__ boff,
                                                              int64_t* __restrict__ out) {
  const int64_t i0 = (int64_t)blockIdx.x * kSelChunk + (int64_t)threadIdx.x * kSelItems;
  unsigned sel = 0u;
#pragma unroll
  for (int k = 0; k < kSelItems; ++k) {
    const int64_t i = i0 + k;
    sel |= (i < n && (int)mark[rows[i]] == want) ? (1u << k) : 0u;
  }
  const int c = __popc(sel);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int u = __shfl_up(inc, d, 64);
    if (lane >= d) inc += u;
  }
  __shared__ int wt[4];
  if (lane == 63) wt[w] = inc;
  __syncthreads();
  int base = 0;
  for (int k = 0; k < w; ++k) base += wt[k];
  int64_t pos = boff[blockIdx.x] + base + inc - c;
  for (int k = 0; k < kSelItems; ++k)
    if ((sel >> k) & 1u) out[pos++] = rows[i0 + k];
}

extern "C" {

int hs_mark_rows(const int64_t* idx, int64_t n, uint8_t* mark, void* stream) {
  if (n <= 0) return 0;
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(hs_mark_rows_kernel, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream,
                     idx, n, mark);
  return (int)hipGetLastError();
}

int64_t hs_select_marked_blocks(int64_t n) { return (n + kSelChunk - 1) / kSelChunk; }

// out: capacity n; ws: hs_select_marked_blocks(n) int64s; total: 1 int64 (selected count)
int hs_select_marked(const int64_t* rows, int64_t n, const uint8_t* mark, int want, int64_t* ws,
                     int64_t* total, int64_t* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n <= 0) {
    (void)hipMemsetAsync(total, 0, sizeof(int64_t), s);
    return (int)hipGetLastError();
  }
  const int64_t nb = hs_select_marked_blocks(n);
  hipLaunchKernelGGL(hs_select_marked_count, dim3((unsigned)nb), dim3(256), 0, s, rows, n, mark,
                     want, ws);
  hipLaunchKernelGGL(hs_select_marked_scan, dim3(1), dim3(1024), 0, s, ws, nb, total);
  hipLaunchKernelGGL(hs_select_marked_write, dim3((unsigned)nb), dim3(256), 0, s, rows, n, mark,
                     want, (const int64_t*)ws, out);
  return (int)hipGetLastError();
}

int hs_gather_params_size() { return (int)sizeof(GatherParams); }

int hs_gather(const GatherParams* p, const void* idx, int64_t n, void* stream) {
  if (n == 0 || p->ncols == 0) return 0;
  int64_t gx = (n + 255) / 256;
  if (gx > 2048) gx = 2048;
  hipLaunchKernelGGL(hs_gather_kernel, dim3((unsigned)gx, p->ncols), dim3(256), 0,
                     (hipStream_t)stream, *p, idx, n);
  return (int)hipGetLastError();
}

// Packed-row gather (no padding rows): pack every column into `rows` (n_src records of
// `row_bytes`, 16-byte multiple), then gather the records by `idx` into the destinations.
int hs_gather_packed(const GatherParams* p, int row_bytes, int vbase, int64_t n_src,
                     uint8_t* rows, const void* idx, int64_t n, void* stream) {
  if (n == 0 || p->ncols == 0) return 0;
  if (row_bytes <= 0 || row_bytes % 16 != 0) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int64_t gp = (n_src + 255) / 256 < 8192 ? (n_src + 255) / 256 : 8192;
  if (n_src > 0)
    hipLaunchKernelGGL(hs_pack_rows_kernel, dim3((unsigned)gp), dim3(256), 0, s, *p, row_bytes,
                       vbase, n_src, rows);
  const int64_t gg = (n + 255) / 256 < 8192 ? (n + 255) / 256 : 8192;
  hipLaunchKernelGGL(hs_gather_rows_kernel, dim3((unsigned)gg), dim3(256), 0, s, *p, row_bytes,
                     vbase, (const uint8_t*)rows, idx, n);
  return (int)hipGetLastError();
}

int hs_bucket_offsets(const int32_t* sorted_bucket, int64_t n, int B, int64_t* off, void* stream) {
  hipLaunchKernelGGL(hs_bucket_offsets_kernel, dim3((B + 1 + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, sorted_bucket, n, B, off);
  return (int)hipGetLastError();
}

}  // extern "C"
