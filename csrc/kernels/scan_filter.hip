// K7 / K10: index scan -> predicate -> aggregate / compaction.
//
// The scan works on *row ranges* of the device-resident index table: the index is sorted by its
// indexed column inside each bucket, so a range predicate on that column becomes one binary search
// per bucket (hs_range_search) — row-level zone pruning that is strictly finer than Parquet
// row-group stats.  An equality predicate on all bucket columns additionally prunes to a single
// bucket (the literal is Murmur3-hashed on the host).  Ranges are cut into 2048-row tiles; a
// fixed grid walks the tile list (its length lives in device memory, so no host round trip and
// the launch sequence is hipGraph-capturable).
#include "hs_scan.h"

#define SF_BLOCK 256
#define SF_ITEMS 8
#define SF_TILE (SF_BLOCK * SF_ITEMS)
#define SF_GRID 2048

struct ScanParams {
  ColDesc cols[HS_MAX_COLS];
  Pred preds[HS_MAX_PREDS];
  AggSpec aggs[HS_MAX_AGGS];
  int32_t npreds;
  int32_t naggs;
  int32_t group_col;   // -1: global aggregate
  int32_t num_groups;
  int64_t group_base;
};

// ------------------------------------------------------------------------------------------------
// Range search: for each selected bucket, [lower, upper) of the sorted key within the bucket.
// bounds are sortable images (hs_sortable) of the literal; nulls sort first and never match.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t lb_sorted(const ColDesc& c, int64_t lo, int64_t hi, uint64_t key,
                                             bool upper) {
  // first index in [lo,hi) whose (valid, sortable) > key (upper) or >= key (lower); null < all.
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    bool less;
    if (!col_valid(c, mid)) {
      less = true;
    } else {
      const uint64_t v = hs_sortable(c, mid);
      less = upper ? (v <= key) : (v < key);
    }
    if (less) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ void hs_range_search_kernel(ColDesc key, const int64_t* __restrict__ bucket_off,
                                       const int32_t* __restrict__ buckets, int nb, int has_lo,
                                       uint64_t lo_key, int lo_incl, int has_hi, uint64_t hi_key,
                                       int hi_incl, int64_t* __restrict__ rstart,
                                       int64_t* __restrict__ rlen, int32_t* __restrict__ rbucket) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  const int b = buckets ? buckets[i] : i;
  const int64_t s = bucket_off[b], e = bucket_off[b + 1];
  // skip nulls (NULLS FIRST): first valid row
  int64_t first_valid = s;
  if (key.valid != nullptr) {
    int64_t lo = s, hi = e;
    while (lo < hi) {
      const int64_t mid = lo + ((hi - lo) >> 1);
      if (!col_valid(key, mid)) lo = mid + 1; else hi = mid;
    }
    first_valid = lo;
  }
  int64_t a = first_valid, z = e;
  if (has_lo) a = lb_sorted(key, first_valid, e, lo_key, !lo_incl);
  if (has_hi) z = lb_sorted(key, first_valid, e, hi_key, hi_incl);
  if (z < a) z = a;
  rstart[i] = a;
  rlen[i] = z - a;
  if (rbucket) rbucket[i] = b;
}

// ranges -> tile prefix (single block, R arbitrary): tile_prefix[R] = total tiles.
__global__ __launch_bounds__(1024) void hs_ranges_to_tiles_kernel(const int64_t* __restrict__ rlen,
                                                                  int R, int tile_rows,
                                                                  int64_t* __restrict__ tile_prefix) {
  __shared__ int64_t wsum[16];
  __shared__ int64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < R; base += blockDim.x) {
    const int i = base + threadIdx.x;
    const int64_t t = i < R ? (rlen[i] + tile_rows - 1) / tile_rows : 0;
    // block inclusive scan
    int64_t x = t;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int off = 1; off < 64; off <<= 1) {
      int64_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t run = 0;
      for (int k = 0; k < (int)(blockDim.x >> 6); ++k) {
        int64_t v = wsum[k];
        wsum[k] = run;
        run += v;
      }
    }
    __syncthreads();
    const int64_t incl = x + wsum[w] + carry;
    if (i < R) tile_prefix[i] = incl - t;
    __syncthreads();
    if (threadIdx.x == blockDim.x - 1) carry = incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) tile_prefix[R] = carry;
}

__device__ __forceinline__ int find_range(const int64_t* tile_prefix, int R, int64_t t) {
  int lo = 0, hi = R;  // largest r with tile_prefix[r] <= t
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (tile_prefix[mid] <= t) lo = mid; else hi = mid;
  }
  return lo;
}

// ------------------------------------------------------------------------------------------------
// Fused filter + aggregate.
// ------------------------------------------------------------------------------------------------
template <bool GROUPED>
__global__ __launch_bounds__(SF_BLOCK) void hs_scan_agg_kernel(
    ScanParams p, const int64_t* __restrict__ rstart, const int64_t* __restrict__ rlen, int R,
    const int64_t* __restrict__ tile_prefix, double* __restrict__ psum, int64_t* __restrict__ pcnt,
    double* __restrict__ pmin, double* __restrict__ pmax) {
  extern __shared__ __attribute__((aligned(16))) double lds[];
  const int A = p.naggs;
  const int GA = GROUPED ? p.num_groups * A : A;
  double* g_sum = lds;
  double* g_min = lds + GA;
  double* g_max = lds + 2 * GA;
  unsigned long long* g_cnt = (unsigned long long*)(lds + 3 * GA);
  if (GROUPED) {
    for (int i = threadIdx.x; i < GA; i += SF_BLOCK) {
      g_sum[i] = 0.0;
      g_min[i] = __builtin_inf();
      g_max[i] = -__builtin_inf();
      g_cnt[i] = 0ull;
    }
    __syncthreads();
  }
  double s[HS_MAX_AGGS], mn[HS_MAX_AGGS], mx[HS_MAX_AGGS];
  int64_t c[HS_MAX_AGGS];
#pragma unroll
  for (int a = 0; a < HS_MAX_AGGS; ++a) {
    s[a] = 0.0;
    c[a] = 0;
    mn[a] = __builtin_inf();
    mx[a] = -__builtin_inf();
  }
  const int64_t ntiles = tile_prefix[R];
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int r = find_range(tile_prefix, R, t);
    const int64_t off = (t - tile_prefix[r]) * SF_TILE;
    const int64_t row0 = rstart[r] + off;
    const int64_t rows = min((int64_t)SF_TILE, rlen[r] - off);
#pragma unroll 2
    for (int it = 0; it < SF_ITEMS; ++it) {
      const int64_t k = (int64_t)it * SF_BLOCK + threadIdx.x;
      if (k >= rows) break;
      const int64_t row = row0 + k;
      RowRef rr{row, row};
      if (!hs_eval_cnf(p.preds, 0, p.npreds, p.cols, HS_MAX_COLS, rr)) continue;
      int gidx = 0;
      if (GROUPED) {
        const ColDesc& gc = p.cols[p.group_col];
        if (!col_valid(gc, row)) continue;  // null group handled on host (not supported here)
        gidx = (int)(load_i64(gc, row) - p.group_base);
        if (gidx < 0 || gidx >= p.num_groups) continue;
      }
#pragma unroll
      for (int a = 0; a < HS_MAX_AGGS; ++a) {
        if (a >= A) break;
        const AggSpec& ag = p.aggs[a];
        double v = 0.0;
        bool ok = true;
        if (ag.kind != AK_COUNT_STAR) ok = hs_agg_value(ag, p.cols, HS_MAX_COLS, rr, v);
        if (!ok) continue;
        if (GROUPED) {
          const int slot = gidx * A + a;
          if (ag.kind == AK_SUM) atomicAdd(&g_sum[slot], v);
          else if (ag.kind == AK_MIN) hs_lds_atomic_min(&g_min[slot], v);
          else if (ag.kind == AK_MAX) hs_lds_atomic_max(&g_max[slot], v);
          atomicAdd(&g_cnt[slot], 1ull);
        } else {
          s[a] += v;
          c[a] += 1;
          mn[a] = fmin(mn[a], v);
          mx[a] = fmax(mx[a], v);
        }
      }
    }
  }
  if (GROUPED) {
    __syncthreads();
    for (int i = threadIdx.x; i < GA; i += SF_BLOCK) {
      const int64_t o = (int64_t)blockIdx.x * GA + i;
      psum[o] = g_sum[i];
      pcnt[o] = (int64_t)g_cnt[i];
      pmin[o] = g_min[i];
      pmax[o] = g_max[i];
    }
    return;
  }
  // global aggregate: deterministic wave + block reduction
  __shared__ double r_s[SF_BLOCK / 64][HS_MAX_AGGS], r_mn[SF_BLOCK / 64][HS_MAX_AGGS],
      r_mx[SF_BLOCK / 64][HS_MAX_AGGS];
  __shared__ int64_t r_c[SF_BLOCK / 64][HS_MAX_AGGS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < HS_MAX_AGGS; ++a) {
    if (a >= A) break;
    const double ws = hs_wave_sum(s[a]);
    const int64_t wc = hs_wave_sum(c[a]);
    const double wmn = hs_wave_min(mn[a]);
    const double wmx = hs_wave_max(mx[a]);
    if (lane == 0) {
      r_s[w][a] = ws;
      r_c[w][a] = wc;
      r_mn[w][a] = wmn;
      r_mx[w][a] = wmx;
    }
  }
  __syncthreads();
  if (threadIdx.x < A) {
    const int a = threadIdx.x;
    double ts = 0.0, tmn = __builtin_inf(), tmx = -__builtin_inf();
    int64_t tc = 0;
    for (int ww = 0; ww < SF_BLOCK / 64; ++ww) {
      ts += r_s[ww][a];
      tc += r_c[ww][a];
      tmn = fmin(tmn, r_mn[ww][a]);
      tmx = fmax(tmx, r_mx[ww][a]);
    }
    const int64_t o = (int64_t)blockIdx.x * A + a;
    psum[o] = ts;
    pcnt[o] = tc;
    pmin[o] = tmn;
    pmax[o] = tmx;
  }
}

__global__ void hs_agg_final_kernel(const double* __restrict__ psum, const int64_t* __restrict__ pcnt,
                                    const double* __restrict__ pmin, const double* __restrict__ pmax,
                                    int nblk, int GA, double* __restrict__ osum,
                                    int64_t* __restrict__ ocnt, double* __restrict__ omin,
                                    double* __restrict__ omax) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= GA) return;
  double s = 0.0, mn = __builtin_inf(), mx = -__builtin_inf();
  int64_t c = 0;
  for (int b = 0; b < nblk; ++b) {
    const int64_t o = (int64_t)b * GA + i;
    s += psum[o];
    c += pcnt[o];
    mn = fmin(mn, pmin[o]);
    mx = fmax(mx, pmax[o]);
  }
  osum[i] = s;
  ocnt[i] = c;
  omin[i] = mn;
  omax[i] = mx;
}

// ------------------------------------------------------------------------------------------------
// Filter -> stable compaction of row ids.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(SF_BLOCK) void hs_scan_count_kernel(
    ScanParams p, const int64_t* __restrict__ rstart, const int64_t* __restrict__ rlen, int R,
    const int64_t* __restrict__ tile_prefix, int64_t* __restrict__ tile_counts) {
  __shared__ int64_t red[SF_BLOCK / 64];
  const int64_t ntiles = tile_prefix[R];
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int r = find_range(tile_prefix, R, t);
    const int64_t off = (t - tile_prefix[r]) * SF_TILE;
    const int64_t row0 = rstart[r] + off;
    const int64_t rows = min((int64_t)SF_TILE, rlen[r] - off);
    int64_t cnt = 0;
    for (int it = 0; it < SF_ITEMS; ++it) {
      const int64_t k = (int64_t)it * SF_BLOCK + threadIdx.x;
      if (k < rows) {
        RowRef rr{row0 + k, row0 + k};
        cnt += hs_eval_cnf(p.preds, 0, p.npreds, p.cols, HS_MAX_COLS, rr) ? 1 : 0;
      }
    }
    cnt = hs_wave_sum(cnt);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
      int64_t tot = 0;
      for (int w = 0; w < SF_BLOCK / 64; ++w) tot += red[w];
      tile_counts[t] = tot;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(SF_BLOCK) void hs_scan_select_kernel(
    ScanParams p, const int64_t* __restrict__ rstart, const int64_t* __restrict__ rlen, int R,
    const int64_t* __restrict__ tile_prefix, const int64_t* __restrict__ tile_offsets,
    int64_t* __restrict__ out_rows) {
  __shared__ int64_t wbase[SF_BLOCK / 64];
  __shared__ int64_t run;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = hs_lanemask_lt();
  const int64_t ntiles = tile_prefix[R];
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int r = find_range(tile_prefix, R, t);
    const int64_t off = (t - tile_prefix[r]) * SF_TILE;
    const int64_t row0 = rstart[r] + off;
    const int64_t rows = min((int64_t)SF_TILE, rlen[r] - off);
    if (threadIdx.x == 0) run = tile_offsets[t];
    __syncthreads();
    for (int it = 0; it < SF_ITEMS; ++it) {
      const int64_t k = (int64_t)it * SF_BLOCK + threadIdx.x;
      bool pass = false;
      if (k < rows) {
        RowRef rr{row0 + k, row0 + k};
        pass = hs_eval_cnf(p.preds, 0, p.npreds, p.cols, HS_MAX_COLS, rr);
      }
      const uint64_t m = __ballot(pass);
      if (lane == 0) wbase[w] = (int64_t)__popcll(m);
      __syncthreads();
      if (threadIdx.x == 0) {
        int64_t acc = run;
        for (int ww = 0; ww < SF_BLOCK / 64; ++ww) {
          const int64_t c = wbase[ww];
          wbase[ww] = acc;
          acc += c;
        }
        run = acc;
      }
      __syncthreads();
      if (pass) out_rows[wbase[w] + __popcll(m & lt)] = row0 + k;
      __syncthreads();
    }
  }
}

extern "C" {

int hs_scan_params_size() { return (int)sizeof(ScanParams); }
int hs_scan_tile_rows() { return SF_TILE; }
int hs_scan_grid() { return SF_GRID; }

int hs_range_search(const ColDesc* key, const int64_t* bucket_off, const int32_t* buckets, int nb,
                    int has_lo, uint64_t lo_key, int lo_incl, int has_hi, uint64_t hi_key,
                    int hi_incl, int64_t* rstart, int64_t* rlen, int32_t* rbucket, void* stream) {
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(hs_range_search_kernel, dim3((nb + 255) / 256), dim3(256), 0,
                     (hipStream_t)stream, *key, bucket_off, buckets, nb, has_lo, lo_key, lo_incl,
                     has_hi, hi_key, hi_incl, rstart, rlen, rbucket);
  return (int)hipGetLastError();
}

int hs_ranges_to_tiles(const int64_t* rlen, int R, int64_t* tile_prefix, void* stream) {
  hipLaunchKernelGGL(hs_ranges_to_tiles_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, rlen,
                     R, SF_TILE, tile_prefix);
  return (int)hipGetLastError();
}

// Partials: 4 arrays of grid*GA. Outputs: 4 arrays of GA.
int hs_scan_agg(const ScanParams* p, const int64_t* rstart, const int64_t* rlen, int R,
                const int64_t* tile_prefix, int grid, double* psum, int64_t* pcnt, double* pmin,
                double* pmax, double* osum, int64_t* ocnt, double* omin, double* omax,
                void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const bool grouped = p->group_col >= 0;
  const int GA = grouped ? p->num_groups * p->naggs : p->naggs;
  if (GA <= 0) return 0;
  if (grouped) {
    const size_t lds = (size_t)GA * 32;
    if (lds > 120 * 1024) return -5;
    hipLaunchKernelGGL(hs_scan_agg_kernel<true>, dim3(grid), dim3(SF_BLOCK), lds, s, *p, rstart,
                       rlen, R, tile_prefix, psum, pcnt, pmin, pmax);
  } else {
    hipLaunchKernelGGL(hs_scan_agg_kernel<false>, dim3(grid), dim3(SF_BLOCK), 0, s, *p, rstart,
                       rlen, R, tile_prefix, psum, pcnt, pmin, pmax);
  }
  hipLaunchKernelGGL(hs_agg_final_kernel, dim3((GA + 255) / 256), dim3(256), 0, s, psum, pcnt, pmin,
                     pmax, grid, GA, osum, ocnt, omin, omax);
  return (int)hipGetLastError();
}

int hs_scan_count(const ScanParams* p, const int64_t* rstart, const int64_t* rlen, int R,
                  const int64_t* tile_prefix, int grid, int64_t* tile_counts, void* stream) {
  hipLaunchKernelGGL(hs_scan_count_kernel, dim3(grid), dim3(SF_BLOCK), 0, (hipStream_t)stream, *p,
                     rstart, rlen, R, tile_prefix, tile_counts);
  return (int)hipGetLastError();
}

int hs_scan_select(const ScanParams* p, const int64_t* rstart, const int64_t* rlen, int R,
                   const int64_t* tile_prefix, const int64_t* tile_offsets, int grid,
                   int64_t* out_rows, void* stream) {
  hipLaunchKernelGGL(hs_scan_select_kernel, dim3(grid), dim3(SF_BLOCK), 0, (hipStream_t)stream, *p,
                     rstart, rlen, R, tile_prefix, tile_offsets, out_rows);
  return (int)hipGetLastError();
}

}  // extern "C"
