// K4: LSD radix sort producing a stable row permutation.
//
// Sorting (bucket, k1, k2, ...) ascending is done column by column, least significant first:
// each column is gathered through the current permutation into an order-preserving unsigned key
// (minus its minimum, so only its significant bits are sorted), then sorted with 8-bit digit
// passes.  A pass = per-tile digit histogram -> exclusive scan (digit-major) -> stable scatter.
//
// Stable in-tile ranking without atomics: every wave owns a contiguous 1024-element slice of
// the 4096-element tile and walks it 64 elements at a time; lanes with equal digits are found
// with 8 ballots (wave64 match), ranked with popcount(mask & lanemask_lt) and a per-wave running
// count in LDS.  After the sweep the 4 per-wave digit totals are prefix-summed so element order
// == (wave, iteration, lane) == input order.
#include "hs_common.h"

#define RS_BLOCK 256
#define RS_WAVES (RS_BLOCK / 64)
#define RS_ITEMS 16
#define RS_TILE (RS_BLOCK * RS_ITEMS)
#define RS_BINS 256
static_assert(RS_BINS == RS_BLOCK, "rs_scatter scans one digit per thread");
#define SCAN_BLOCK 256
#define SCAN_ITEMS 8
#define SCAN_TILE (SCAN_BLOCK * SCAN_ITEMS)

// ------------------------------------------------------------------------------------------------
// Key construction: keys[i] = sortable(col[perm[i]]) - kmin ; nulls -> 0 (NULLS FIRST) unless
// null_last.  Optional bucket column path: keys[i] = bucket[perm[i]].
// ------------------------------------------------------------------------------------------------
template <typename KeyT>
__global__ __launch_bounds__(256) void rs_make_keys(ColDesc col, const uint32_t* __restrict__ perm,
                                                    int64_t n, uint64_t kmin, KeyT* __restrict__ keys) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t row = perm ? (int64_t)perm[i] : i;
    KeyT k = 0;
    if (col_valid(col, row)) k = (KeyT)(hs_sortable(col, row) - kmin);
    keys[i] = k;
  }
}

// validity flag as a 1-bit key (0 = null sorts first)
__global__ __launch_bounds__(256) void rs_make_valid_keys(const uint8_t* __restrict__ valid,
                                                          const uint32_t* __restrict__ perm,
                                                          int64_t n, uint32_t* __restrict__ keys) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t row = perm ? (int64_t)perm[i] : i;
    keys[i] = valid[row] ? 1u : 0u;
  }
}

__global__ __launch_bounds__(256) void rs_iota(uint32_t* __restrict__ perm, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    perm[i] = (uint32_t)i;
}

// ------------------------------------------------------------------------------------------------
// Pass kernels
// ------------------------------------------------------------------------------------------------
template <typename KeyT>
__global__ __launch_bounds__(RS_BLOCK) void rs_hist(const KeyT* __restrict__ keys, int64_t n,
                                                    int shift, int64_t ntiles,
                                                    uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[RS_BINS];
  for (int i = threadIdx.x; i < RS_BINS; i += RS_BLOCK) h[i] = 0;
  __syncthreads();
  const int64_t tile = blockIdx.x;
  const int64_t base = tile * RS_TILE;
#pragma unroll
  for (int it = 0; it < RS_ITEMS; ++it) {
    const int64_t i = base + (int64_t)it * RS_BLOCK + threadIdx.x;
    if (i < n) atomicAdd(&h[(uint32_t)(keys[i] >> shift) & 0xFF], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < RS_BINS; d += RS_BLOCK) hist[(int64_t)d * ntiles + tile] = h[d];
}

// Stable scatter of one 4096-element tile.  Ranking: see the file comment.  Writing: instead of
// storing every element straight to keys_out[global position] (256 digit runs per tile, each a
// scattered partial line), the tile is first reordered in LDS by its local digit-major position
// (tile digit start + per-wave prefix + rank), then threads walk the reordered tile in order and
// element i goes to g_off[digit] + (i - tile_start[digit]): consecutive lanes write consecutive
// addresses of one digit run, so global stores coalesce.
template <typename KeyT>
__global__ __launch_bounds__(RS_BLOCK) void rs_scatter(const KeyT* __restrict__ keys_in,
                                                       const uint32_t* __restrict__ vals_in,
                                                       KeyT* __restrict__ keys_out,
                                                       uint32_t* __restrict__ vals_out, int64_t n,
                                                       int shift, int64_t ntiles,
                                                       const uint32_t* __restrict__ offsets) {
  __shared__ uint32_t wave_cnt[RS_WAVES][RS_BINS];
  __shared__ uint32_t g_off[RS_BINS];
  __shared__ uint32_t t_start[RS_BINS];
  __shared__ uint32_t scan_tmp[RS_WAVES];
  __shared__ KeyT s_keys[RS_TILE];
  __shared__ uint32_t s_vals[RS_TILE];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int64_t tile = blockIdx.x;
  for (int i = threadIdx.x; i < RS_WAVES * RS_BINS; i += RS_BLOCK) (&wave_cnt[0][0])[i] = 0;
  for (int d = threadIdx.x; d < RS_BINS; d += RS_BLOCK) g_off[d] = offsets[(int64_t)d * ntiles + tile];
  __syncthreads();

  KeyT k[RS_ITEMS];
  uint32_t v[RS_ITEMS];
  uint32_t rank[RS_ITEMS];
  const int64_t wbase = tile * RS_TILE + (int64_t)w * (RS_ITEMS * 64);
  const uint64_t lt = hs_lanemask_lt();
#pragma unroll
  for (int it = 0; it < RS_ITEMS; ++it) {
    const int64_t i = wbase + it * 64 + lane;
    const bool active = i < n;
    k[it] = active ? keys_in[i] : (KeyT)0;
    v[it] = active ? vals_in[i] : 0u;
    const uint32_t d = (uint32_t)(k[it] >> shift) & 0xFF;
    uint64_t mask = __ballot(active);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const bool bit = (d >> b) & 1;
      const uint64_t bb = __ballot(bit);
      mask &= bit ? bb : ~bb;
    }
    const uint32_t before = (uint32_t)__popcll(mask & lt);
    const uint32_t cnt = (uint32_t)__popcll(mask);
    const bool leader = active && before == 0;
    uint32_t pre = active ? wave_cnt[w][d] : 0u;
    __builtin_amdgcn_wave_barrier();
    if (leader) wave_cnt[w][d] = pre + cnt;
    __builtin_amdgcn_wave_barrier();
    rank[it] = pre + before;
  }
  __syncthreads();
  // per digit (one per thread: RS_BINS == RS_BLOCK): exclusive prefix of the per-wave totals
  // across waves, and the digit's tile total
  const int dd = threadIdx.x;
  uint32_t total = 0;
#pragma unroll
  for (int ww = 0; ww < RS_WAVES; ++ww) {
    const uint32_t t = wave_cnt[ww][dd];
    wave_cnt[ww][dd] = total;
    total += t;
  }
  // exclusive scan of the tile totals over digits -> digit start inside the reordered tile
  uint32_t x = total;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) scan_tmp[w] = x;
  __syncthreads();
  uint32_t wpre = 0;
  for (int ww = 0; ww < w; ++ww) wpre += scan_tmp[ww];
  t_start[dd] = wpre + x - total;
  __syncthreads();
#pragma unroll
  for (int it = 0; it < RS_ITEMS; ++it) {
    const int64_t i = wbase + it * 64 + lane;
    if (i < n) {
      const uint32_t d = (uint32_t)(k[it] >> shift) & 0xFF;
      const uint32_t lp = t_start[d] + wave_cnt[w][d] + rank[it];
      s_keys[lp] = k[it];
      s_vals[lp] = v[it];
    }
  }
  __syncthreads();
  const int64_t rem = n - tile * RS_TILE;
  const int cnt_tile = rem < RS_TILE ? (int)rem : RS_TILE;
  for (int i = threadIdx.x; i < cnt_tile; i += RS_BLOCK) {
    const KeyT kk = s_keys[i];
    const uint32_t d = (uint32_t)(kk >> shift) & 0xFF;
    const uint32_t pos = g_off[d] + (uint32_t)i - t_start[d];
    keys_out[pos] = kk;
    vals_out[pos] = s_vals[i];
  }
}

// ------------------------------------------------------------------------------------------------
// Exclusive scan (uint32 / int64), reduce-then-scan.
// ------------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* lds_wave, T& total) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    T y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) lds_wave[w] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      T t = lds_wave[i];
      lds_wave[i] = run;
      run += t;
    }
    lds_wave[16] = run;
  }
  __syncthreads();
  total = lds_wave[16];
  T r = x - v + lds_wave[w];
  __syncthreads();
  return r;
}

template <typename T>
__global__ __launch_bounds__(SCAN_BLOCK) void scan_reduce(const T* __restrict__ in, int64_t n,
                                                          T* __restrict__ block_sums) {
  __shared__ T red[SCAN_BLOCK / 64];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  T s = 0;
#pragma unroll
  for (int it = 0; it < SCAN_ITEMS; ++it) {
    const int64_t i = base + (int64_t)it * SCAN_BLOCK + threadIdx.x;
    if (i < n) s += in[i];
  }
  s = hs_wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    T t = 0;
    for (int i = 0; i < SCAN_BLOCK / 64; ++i) t += red[i];
    block_sums[blockIdx.x] = t;
  }
}

template <typename T>
__global__ __launch_bounds__(SCAN_BLOCK) void scan_apply(const T* __restrict__ in, int64_t n,
                                                         const T* __restrict__ block_offsets,
                                                         T* __restrict__ out) {
  __shared__ T lds[17];
  const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
  // each thread owns SCAN_ITEMS consecutive elements
  T vals[SCAN_ITEMS];
  T local = 0;
#pragma unroll
  for (int it = 0; it < SCAN_ITEMS; ++it) {
    const int64_t i = base + (int64_t)threadIdx.x * SCAN_ITEMS + it;
    vals[it] = i < n ? in[i] : (T)0;
    local += vals[it];
  }
  T total;
  T pre = block_exclusive_scan<T>(local, lds, total);
  T run = pre + (block_offsets ? block_offsets[blockIdx.x] : (T)0);
#pragma unroll
  for (int it = 0; it < SCAN_ITEMS; ++it) {
    const int64_t i = base + (int64_t)threadIdx.x * SCAN_ITEMS + it;
    if (i < n) out[i] = run;
    run += vals[it];
  }
}

template <typename T>
static int exclusive_scan_impl(const T* in, T* out, int64_t n, T* tmp, int64_t tmp_elems,
                               hipStream_t s) {
  if (n <= 0) return 0;
  const int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb == 1) {
    hipLaunchKernelGGL(scan_apply<T>, dim3(1), dim3(SCAN_BLOCK), 0, s, in, n, (const T*)nullptr, out);
    return (int)hipGetLastError();
  }
  if (tmp_elems < nb) return -1;
  T* sums = tmp;
  hipLaunchKernelGGL(scan_reduce<T>, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, s, in, n, sums);
  int rc = exclusive_scan_impl<T>(sums, sums, nb, tmp + nb, tmp_elems - nb, s);
  if (rc) return rc;
  hipLaunchKernelGGL(scan_apply<T>, dim3((unsigned)nb), dim3(SCAN_BLOCK), 0, s, in, n,
                     (const T*)sums, out);
  return (int)hipGetLastError();
}

static int64_t scan_tmp_elems(int64_t n) {
  int64_t total = 0;
  while (true) {
    const int64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (nb <= 1) break;
    total += nb;
    n = nb;
  }
  return total + 16;
}

static int grid_for(int64_t n) {
  int64_t g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" {

int64_t hs_scan_tmp_elems(int64_t n) { return scan_tmp_elems(n); }

int hs_exclusive_scan_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* tmp,
                          int64_t tmp_elems, void* stream) {
  return exclusive_scan_impl<uint32_t>(in, out, n, tmp, tmp_elems, (hipStream_t)stream);
}

int hs_exclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, int64_t* tmp,
                          int64_t tmp_elems, void* stream) {
  return exclusive_scan_impl<int64_t>(in, out, n, tmp, tmp_elems, (hipStream_t)stream);
}

// Workspace (bytes) needed by hs_sort_columns for n rows.
int64_t hs_sort_workspace_bytes(int64_t n) {
  const int64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  const int64_t hist = (int64_t)RS_BINS * ntiles;
  int64_t b = 0;
  b += 2 * n * 8;                 // keys ping/pong (u64)
  b += n * 4;                     // perm pong
  b += 2 * hist * 4;              // hist + offsets
  b += scan_tmp_elems(hist) * 4;  // scan temps
  return b + 4096;
}

struct SortKeySpec {
  ColDesc col;
  uint64_t kmin;    // min sortable image
  int32_t bits;     // significant bits of (sortable - kmin)
  int32_t has_nulls;
};

// Produce perm (n uint32) such that rows are ordered by keys[0], keys[1], ... ascending with
// NULLS FIRST, stable w.r.t. the input row order (or the given initial perm when init_perm!=0).
int hs_sort_columns(const SortKeySpec* specs, int nkeys, int64_t n, uint32_t* perm,
                    int init_perm, void* workspace, int64_t ws_bytes, void* stream) {
  if (n == 0) return 0;
  if (n > 0xFFFFFFFFll) return -2;
  if (ws_bytes < hs_sort_workspace_bytes(n)) return -3;
  hipStream_t s = (hipStream_t)stream;
  const int64_t ntiles = (n + RS_TILE - 1) / RS_TILE;
  const int64_t hist_n = (int64_t)RS_BINS * ntiles;
  char* w = (char*)workspace;
  uint64_t* keys_a = (uint64_t*)w; w += n * 8;
  uint64_t* keys_b = (uint64_t*)w; w += n * 8;
  uint32_t* perm_b = (uint32_t*)w; w += n * 4;
  uint32_t* hist = (uint32_t*)w; w += hist_n * 4;
  uint32_t* offs = (uint32_t*)w; w += hist_n * 4;
  uint32_t* stmp = (uint32_t*)w;
  const int64_t stmp_elems = scan_tmp_elems(hist_n);
  if (!init_perm) hipLaunchKernelGGL(rs_iota, dim3(grid_for(n)), dim3(256), 0, s, perm, n);

  uint32_t* cur_perm = perm;
  uint32_t* alt_perm = perm_b;
  auto run_passes32 = [&](uint32_t* ka, uint32_t* kb, int bits) -> int {
    for (int shift = 0; shift < bits; shift += 8) {
      hipLaunchKernelGGL(rs_hist<uint32_t>, dim3((unsigned)ntiles), dim3(RS_BLOCK), 0, s, ka, n,
                         shift, ntiles, hist);
      int rc = exclusive_scan_impl<uint32_t>(hist, offs, hist_n, stmp, stmp_elems, s);
      if (rc) return rc;
      hipLaunchKernelGGL(rs_scatter<uint32_t>, dim3((unsigned)ntiles), dim3(RS_BLOCK), 0, s, ka,
                         cur_perm, kb, alt_perm, n, shift, ntiles, offs);
      uint32_t* t = ka; ka = kb; kb = t;
      uint32_t* tp = cur_perm; cur_perm = alt_perm; alt_perm = tp;
    }
    return 0;
  };
  auto run_passes64 = [&](uint64_t* ka, uint64_t* kb, int bits) -> int {
    for (int shift = 0; shift < bits; shift += 8) {
      hipLaunchKernelGGL(rs_hist<uint64_t>, dim3((unsigned)ntiles), dim3(RS_BLOCK), 0, s, ka, n,
                         shift, ntiles, hist);
      int rc = exclusive_scan_impl<uint32_t>(hist, offs, hist_n, stmp, stmp_elems, s);
      if (rc) return rc;
      hipLaunchKernelGGL(rs_scatter<uint64_t>, dim3((unsigned)ntiles), dim3(RS_BLOCK), 0, s, ka,
                         cur_perm, kb, alt_perm, n, shift, ntiles, offs);
      uint64_t* t = ka; ka = kb; kb = t;
      uint32_t* tp = cur_perm; cur_perm = alt_perm; alt_perm = tp;
    }
    return 0;
  };
  for (int k = nkeys - 1; k >= 0; --k) {
    const SortKeySpec& sp = specs[k];
    if (sp.bits > 0) {
      if (sp.bits <= 32) {
        hipLaunchKernelGGL(rs_make_keys<uint32_t>, dim3(grid_for(n)), dim3(256), 0, s, sp.col,
                           cur_perm, n, sp.kmin, (uint32_t*)keys_a);
        int rc = run_passes32((uint32_t*)keys_a, (uint32_t*)keys_b, sp.bits);
        if (rc) return rc;
      } else {
        hipLaunchKernelGGL(rs_make_keys<uint64_t>, dim3(grid_for(n)), dim3(256), 0, s, sp.col,
                           cur_perm, n, sp.kmin, keys_a);
        int rc = run_passes64(keys_a, keys_b, sp.bits);
        if (rc) return rc;
      }
    }
    if (sp.has_nulls && sp.col.valid != nullptr) {
      hipLaunchKernelGGL(rs_make_valid_keys, dim3(grid_for(n)), dim3(256), 0, s, sp.col.valid,
                         cur_perm, n, (uint32_t*)keys_a);
      int rc = run_passes32((uint32_t*)keys_a, (uint32_t*)keys_b, 1);
      if (rc) return rc;
    }
  }
  if (cur_perm != perm) hipMemcpyAsync(perm, cur_perm, n * 4, hipMemcpyDeviceToDevice, s);
  return (int)hipGetLastError();
}

int hs_sort_key_spec_size() { return (int)sizeof(SortKeySpec); }

}  // extern "C"
