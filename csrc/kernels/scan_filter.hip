// K7 / K10: index scan -> predicate -> aggregate / compaction.
//
// The scan works on *row ranges* of the device-resident index table: the index is sorted by its
// indexed column inside each bucket, so a range predicate on that column becomes one binary search
// per bucket (hs_range_search) — row-level zone pruning that is strictly finer than Parquet
// row-group stats.  An equality predicate on all bucket columns additionally prunes to a single
// bucket (the literal is Murmur3-hashed on the host).  Ranges are cut into 2048-row tiles; each
// block of a fixed grid takes a contiguous chunk of the tile list (its length lives in device
// memory, so no host round trip and the launch sequence is hipGraph-capturable).
//
// Inside a tile every lane owns SF_ITEMS rows (stride SF_BLOCK, so each wave load is one
// coalesced 64-row segment) and evaluates them predicate-major (hs_vec.h): SF_ITEMS independent
// loads in flight per lane per column.
#include "hs_vec.h"

#define SF_BLOCK 256
#define SF_ITEMS 8
#define SF_TILE (SF_BLOCK * SF_ITEMS)
#define SF_GRID 2048
#define FIN_BLOCK 256   // final reduction: 4 waves (each lane sums grid/256 partials) - a block
                        // needing 16 free wave slots on one CU waited behind a concurrent
                        // join's waves (~110 us per final in the SF100 step timeline, r6)

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
// One wavefront per range: lanes 0-31 search the lower bound and lanes 32-63 the upper bound,
// each half with a 32-ary search (32 pivots per step, one ballot): log32(bucket rows) steps of
// one coalesced load each instead of ~2 x log2 dependent loads of a thread-per-bucket search
// (a 3M-row bucket: 5 round trips instead of 44).
#define RANGE_WAVES 4

// first index in [lo, hi] whose row is NOT "less": less = null (nulls sort first) or, for a
// valid row, sortable < key (upper: <= key); key_mode 2 = only the null prefix
__device__ __forceinline__ bool range_less(const ColDesc& c, int64_t r, uint64_t key, int mode) {
  if (!col_valid(c, r)) return true;
  if (mode == 2) return false;
  const uint64_t v = hs_sortable(c, r);
  return mode == 1 ? (v <= key) : (v < key);
}

__device__ __forceinline__ int64_t kary_bound(const ColDesc& c, int64_t lo, int64_t hi,
                                              uint64_t key, int mode, int gl, int half) {
  while (hi - lo > 32) {
    const int64_t span = hi - lo;
    const bool less = range_less(c, lo + span * (gl + 1) / 33, key, mode);
    const int cnt = __popc((uint32_t)(__ballot(less) >> (half * 32)));
    const int64_t nlo = cnt == 0 ? lo : lo + span * cnt / 33 + 1;
    const int64_t nhi = cnt == 32 ? hi : lo + span * (cnt + 1) / 33;
    lo = nlo;
    hi = nhi;
  }
  const bool less = lo + gl < hi && range_less(c, lo + gl, key, mode);
  return lo + __popc((uint32_t)(__ballot(less) >> (half * 32)));
}

__device__ __forceinline__ void range_one(const ColDesc& key, const int64_t* __restrict__ bucket_off,
                                          const int32_t* __restrict__ buckets, int i, int has_lo,
                                          uint64_t lo_key, int lo_incl, int has_hi,
                                          uint64_t hi_key, int hi_incl, int64_t* __restrict__ rstart,
                                          int64_t* __restrict__ rlen, int32_t* __restrict__ rbucket) {
  const int lane = threadIdx.x & 63, half = lane >> 5, gl = lane & 31;
  const int b = buckets ? buckets[i] : i;
  const int64_t s = bucket_off[b], e = bucket_off[b + 1];
  const int64_t first_valid = key.valid != nullptr ? kary_bound(key, s, e, 0, 2, gl, half) : s;
  int64_t r;
  if (half == 0) r = has_lo ? kary_bound(key, first_valid, e, lo_key, lo_incl ? 0 : 1, gl, 0)
                            : first_valid;
  else r = has_hi ? kary_bound(key, first_valid, e, hi_key, hi_incl ? 1 : 0, gl, 1) : e;
  const int64_t a = __shfl(r, 0, 64);
  int64_t z = __shfl(r, 32, 64);
  if (z < a) z = a;
  if (lane == 0) {
    rstart[i] = a;
    rlen[i] = z - a;
    if (rbucket) rbucket[i] = b;
  }
}

__global__ __launch_bounds__(64 * RANGE_WAVES) void hs_range_search_kernel(
    ColDesc key, const int64_t* __restrict__ bucket_off, const int32_t* __restrict__ buckets,
    int nb, int has_lo, uint64_t lo_key, int lo_incl, int has_hi, uint64_t hi_key, int hi_incl,
    int64_t* __restrict__ rstart, int64_t* __restrict__ rlen, int32_t* __restrict__ rbucket) {
  const int i = blockIdx.x * RANGE_WAVES + (threadIdx.x >> 6);
  if (i >= nb) return;   // wave-uniform
  range_one(key, bucket_off, buckets, i, has_lo, lo_key, lo_incl, has_hi, hi_key, hi_incl, rstart,
            rlen, rbucket);
}

// Key probes: for probe i, the rows of bucket pbucket[i] whose sorted key equals the sortable
// image pkey[i] (one bound pair per probe).  Drives a join from a small, filtered side
// into a large index sorted by the join key: only the matching key runs are scanned.
__global__ __launch_bounds__(64 * RANGE_WAVES) void hs_probe_ranges_kernel(
    ColDesc key, const int64_t* __restrict__ bucket_off, const int32_t* __restrict__ pbucket,
    const uint64_t* __restrict__ pkey, int np, int64_t* __restrict__ rstart,
    int64_t* __restrict__ rlen, int32_t* __restrict__ rbucket) {
  const int i = blockIdx.x * RANGE_WAVES + (threadIdx.x >> 6);
  if (i >= np) return;
  range_one(key, bucket_off, pbucket, i, 1, pkey[i], 1, 1, pkey[i], 1, rstart, rlen, rbucket);
}

// Bounds read from device memory (int64 x6: has_lo, lo, lo_incl, has_hi, hi, hi_incl), so a
// captured hipGraph replays with new literals after one H2D of the parameter block.
__global__ __launch_bounds__(64 * RANGE_WAVES) void hs_range_search_dev_kernel(
    ColDesc key, const int64_t* __restrict__ bucket_off, const int32_t* __restrict__ buckets,
    int nb, const int64_t* __restrict__ bp, int64_t* __restrict__ rstart,
    int64_t* __restrict__ rlen, int32_t* __restrict__ rbucket) {
  const int i = blockIdx.x * RANGE_WAVES + (threadIdx.x >> 6);
  if (i >= nb) return;
  range_one(key, bucket_off, buckets, i, (int)bp[0], (uint64_t)bp[1], (int)bp[2], (int)bp[3],
            (uint64_t)bp[4], (int)bp[5], rstart, rlen, rbucket);
}

// ranges -> tile prefix (ONE wavefront, R arbitrary): tile_prefix[R] = total tiles.
// rstart != nullptr: each range is widened down to a multiple of `align` rows first (the tiling of
// the vectorized generated kernels, which load `align` consecutive rows per thread).
// A single wavefront, no LDS and no barriers: this kernel sits in the middle of the scan
// pipeline's graph, and while a concurrent join's waves fill the device a 1024-thread block had to
// wait for 16 free wave slots on one CU (~185 us in the SF100 step timeline, r6) - one wave slot
// frees up at once.
__global__ __launch_bounds__(64) void hs_ranges_to_tiles_kernel(const int64_t* __restrict__ rlen,
                                                                int R, int tile_rows,
                                                                int64_t* __restrict__ tile_prefix,
                                                                const int64_t* __restrict__ rstart,
                                                                int64_t align) {
  const int lane = threadIdx.x & 63;
  int64_t carry = 0;
  for (int base = 0; base < R; base += 64) {
    const int i = base + lane;
    const int64_t len = i < R ? rlen[i] + (rstart != nullptr ? (rstart[i] & (align - 1)) : 0) : 0;
    const int64_t t = (len + tile_rows - 1) / tile_rows;
    int64_t x = t;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (i < R) tile_prefix[i] = carry + x - t;
    carry += __shfl(x, 63, 64);
  }
  if (lane == 0) tile_prefix[R] = carry;
}

// Walks a block's contiguous tile chunk, yielding (row0, rows) per tile.
struct TileWalker {
  const int64_t* tile_prefix;
  const int64_t* rstart;
  const int64_t* rlen;
  int R;
  int r;
  __device__ __forceinline__ void init(int64_t t0) { r = tile_range_of(tile_prefix, R, t0); }
  __device__ __forceinline__ void at(int64_t t, int64_t& row0, int64_t& rows) {
    while (r + 1 < R && tile_prefix[r + 1] <= t) ++r;
    const int64_t off = (t - tile_prefix[r]) * SF_TILE;
    row0 = rstart[r] + off;
    rows = min((int64_t)SF_TILE, rlen[r] - off);
  }
};

__device__ __forceinline__ void tile_rows(int64_t row0, int64_t rows, int64_t (&r)[SF_ITEMS],
                                          bool (&act)[SF_ITEMS]) {
#pragma unroll
  for (int i = 0; i < SF_ITEMS; ++i) {
    const int64_t k = (int64_t)i * SF_BLOCK + threadIdx.x;
    act[i] = k < rows;
    r[i] = act[i] ? row0 + k : row0;
  }
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
  GroupLds gl = group_lds(lds, GROUPED ? GA : 0);
  if (GROUPED) {
    group_lds_init(gl, GA, SF_BLOCK);
    __syncthreads();
  }
  AggAcc acc;
  acc_init(acc, p.aggs, A);
  int64_t t0, t1;
  block_tile_chunk(tile_prefix[R], t0, t1);
  if (t0 < t1) {
    TileWalker tw{tile_prefix, rstart, rlen, R, 0};
    tw.init(t0);
    for (int64_t t = t0; t < t1; ++t) {
      int64_t row0, rows;
      tw.at(t, row0, rows);
      int64_t r[SF_ITEMS];
      bool act[SF_ITEMS], pass[SF_ITEMS];
      tile_rows(row0, rows, r, act);
      veval_cnf(p.preds, 0, p.npreds, p.cols, HS_MAX_COLS, r, r, act, pass);
      int g[SF_ITEMS];
#pragma unroll
      for (int i = 0; i < SF_ITEMS; ++i) g[i] = 0;
      if (GROUPED)
        vgroup(p.cols, p.group_col, HS_MAX_COLS, p.group_base, p.num_groups, r, r, pass, g);
      vaccumulate<GROUPED, SF_ITEMS>(acc, p.aggs, A, p.cols, HS_MAX_COLS, r, r, pass, g, gl);
    }
  }
  acc_flush<GROUPED, SF_BLOCK>(acc, p.aggs, A, GA, gl, psum, pcnt, pmin, pmax);
}

// Deterministic final reduction: one workgroup per output slot, fixed-order tree.
__global__ __launch_bounds__(FIN_BLOCK) void hs_agg_final_kernel(
    const double* __restrict__ psum, const int64_t* __restrict__ pcnt,
    const double* __restrict__ pmin, const double* __restrict__ pmax, int nblk, int GA,
    double* __restrict__ osum, int64_t* __restrict__ ocnt, double* __restrict__ omin,
    double* __restrict__ omax) {
  __shared__ double rs[FIN_BLOCK / 64], rmn[FIN_BLOCK / 64], rmx[FIN_BLOCK / 64];
  __shared__ int64_t rc[FIN_BLOCK / 64];
  const int i = blockIdx.x;
  double s = 0.0, mn = __builtin_inf(), mx = -__builtin_inf();
  int64_t c = 0;
#pragma unroll 4
  for (int b = threadIdx.x; b < nblk; b += FIN_BLOCK) {
    const int64_t o = (int64_t)b * GA + i;
    s += psum[o];
    c += pcnt[o];
    mn = fmin(mn, pmin[o]);
    mx = fmax(mx, pmax[o]);
  }
  s = hs_wave_sum(s);
  c = hs_wave_sum(c);
  mn = hs_wave_min(mn);
  mx = hs_wave_max(mx);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    rs[w] = s;
    rc[w] = c;
    rmn[w] = mn;
    rmx[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double ts = 0.0, tmn = __builtin_inf(), tmx = -__builtin_inf();
    int64_t tc = 0;
    for (int k = 0; k < FIN_BLOCK / 64; ++k) {
      ts += rs[k];
      tc += rc[k];
      tmn = fmin(tmn, rmn[k]);
      tmx = fmax(tmx, rmx[k]);
    }
    osum[i] = ts;
    ocnt[i] = tc;
    omin[i] = tmn;
    omax[i] = tmx;
  }
}

// ------------------------------------------------------------------------------------------------
// Filter -> stable compaction of row ids (count pass, then emit pass at the scanned offsets).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(SF_BLOCK) void hs_scan_count_kernel(
    ScanParams p, const int64_t* __restrict__ rstart, const int64_t* __restrict__ rlen, int R,
    const int64_t* __restrict__ tile_prefix, int64_t* __restrict__ tile_counts) {
  __shared__ int64_t red[SF_BLOCK / 64];
  int64_t t0, t1;
  block_tile_chunk(tile_prefix[R], t0, t1);
  if (t0 >= t1) return;
  TileWalker tw{tile_prefix, rstart, rlen, R, 0};
  tw.init(t0);
  for (int64_t t = t0; t < t1; ++t) {
    int64_t row0, rows;
    tw.at(t, row0, rows);
    int64_t r[SF_ITEMS];
    bool act[SF_ITEMS], pass[SF_ITEMS];
    tile_rows(row0, rows, r, act);
    veval_cnf(p.preds, 0, p.npreds, p.cols, HS_MAX_COLS, r, r, act, pass);
    int64_t cnt = 0;
#pragma unroll
    for (int i = 0; i < SF_ITEMS; ++i) cnt += pass[i] ? 1 : 0;
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
  __shared__ int64_t wcnt[SF_ITEMS][SF_BLOCK / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t lt = hs_lanemask_lt();
  int64_t t0, t1;
  block_tile_chunk(tile_prefix[R], t0, t1);
  if (t0 >= t1) return;
  TileWalker tw{tile_prefix, rstart, rlen, R, 0};
  tw.init(t0);
  for (int64_t t = t0; t < t1; ++t) {
    int64_t row0, rows;
    tw.at(t, row0, rows);
    int64_t r[SF_ITEMS];
    bool act[SF_ITEMS], pass[SF_ITEMS];
    tile_rows(row0, rows, r, act);
    veval_cnf(p.preds, 0, p.npreds, p.cols, HS_MAX_COLS, r, r, act, pass);
    uint64_t m[SF_ITEMS];
#pragma unroll
    for (int i = 0; i < SF_ITEMS; ++i) {
      m[i] = __ballot(pass[i]);
      if (lane == 0) wcnt[i][w] = (int64_t)__popcll(m[i]);
    }
    __syncthreads();
    // output order = row order = (item, wave, lane)
    int64_t base = tile_offsets[t];
#pragma unroll
    for (int i = 0; i < SF_ITEMS; ++i) {
      int64_t mine = base;
      for (int ww = 0; ww < SF_BLOCK / 64; ++ww) {
        if (ww < w) mine += wcnt[i][ww];
        base += wcnt[i][ww];
      }
      if (pass[i]) out_rows[mine + __popcll(m[i] & lt)] = r[i];
    }
    __syncthreads();
  }
}

// Filter -> key bitmap: bit (key - base) of the key column ``key_slot`` for every row that
// passes the predicate.  A semi-join's build side (TPC-H Q3's customers of one market segment)
// goes from its filtered scan straight into the bitmap the probe tests: no row-id compaction,
// so no selected-row count has to reach the host to size a buffer, and the query submits
// without a synchronization.  Keys outside [base, base + nbits) and null keys set no bit.
__global__ __launch_bounds__(SF_BLOCK) void hs_scan_bitmap_kernel(
    ScanParams p, const int64_t* __restrict__ rstart, const int64_t* __restrict__ rlen, int R,
    const int64_t* __restrict__ tile_prefix, int key_slot, int64_t base, int64_t nbits,
    unsigned long long* __restrict__ words) {
  int64_t t0, t1;
  block_tile_chunk(tile_prefix[R], t0, t1);
  if (t0 >= t1) return;
  const ColDesc kc = p.cols[key_slot];
  TileWalker tw{tile_prefix, rstart, rlen, R, 0};
  tw.init(t0);
  for (int64_t t = t0; t < t1; ++t) {
    int64_t row0, rows;
    tw.at(t, row0, rows);
    int64_t r[SF_ITEMS];
    bool act[SF_ITEMS], pass[SF_ITEMS];
    tile_rows(row0, rows, r, act);
    veval_cnf(p.preds, 0, p.npreds, p.cols, HS_MAX_COLS, r, r, act, pass);
#pragma unroll
    for (int i = 0; i < SF_ITEMS; ++i) {
      if (!pass[i] || !col_valid(kc, r[i])) continue;
      const int64_t v = load_i64(kc, r[i]) - base;
      if (v < 0 || v >= nbits) continue;
      atomicOr(&words[v >> 6], 1ull << (v & 63));
    }
  }
}

extern "C" {

int hs_scan_params_size() { return (int)sizeof(ScanParams); }
int hs_scan_tile_rows() { return SF_TILE; }
int hs_scan_grid() { return SF_GRID; }

int hs_range_search_dev(const ColDesc* key, const int64_t* bucket_off, const int32_t* buckets,
                        int nb, const int64_t* dparams, int64_t* rstart, int64_t* rlen,
                        int32_t* rbucket, void* stream) {
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(hs_range_search_dev_kernel, dim3((nb + RANGE_WAVES - 1) / RANGE_WAVES),
                     dim3(64 * RANGE_WAVES), 0,
                     (hipStream_t)stream, *key, bucket_off, buckets, nb, dparams, rstart, rlen,
                     rbucket);
  return (int)hipGetLastError();
}

int hs_range_search(const ColDesc* key, const int64_t* bucket_off, const int32_t* buckets, int nb,
                    int has_lo, uint64_t lo_key, int lo_incl, int has_hi, uint64_t hi_key,
                    int hi_incl, int64_t* rstart, int64_t* rlen, int32_t* rbucket, void* stream) {
  if (nb <= 0) return 0;
  hipLaunchKernelGGL(hs_range_search_kernel, dim3((nb + RANGE_WAVES - 1) / RANGE_WAVES),
                     dim3(64 * RANGE_WAVES), 0,
                     (hipStream_t)stream, *key, bucket_off, buckets, nb, has_lo, lo_key, lo_incl,
                     has_hi, hi_key, hi_incl, rstart, rlen, rbucket);
  return (int)hipGetLastError();
}

int hs_probe_ranges(const ColDesc* key, const int64_t* bucket_off, const int32_t* pbucket,
                    const uint64_t* pkey, int np, int64_t* rstart, int64_t* rlen, int32_t* rbucket,
                    void* stream) {
  if (np <= 0) return 0;
  hipLaunchKernelGGL(hs_probe_ranges_kernel, dim3((np + RANGE_WAVES - 1) / RANGE_WAVES),
                     dim3(64 * RANGE_WAVES), 0,
                     (hipStream_t)stream, *key, bucket_off, pbucket, pkey, np, rstart, rlen,
                     rbucket);
  return (int)hipGetLastError();
}

int hs_ranges_to_tiles(const int64_t* rlen, int R, int tile_rows, int64_t* tile_prefix,
                       void* stream) {
  hipLaunchKernelGGL(hs_ranges_to_tiles_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, rlen,
                     R, tile_rows, tile_prefix, (const int64_t*)nullptr, (int64_t)1);
  return (int)hipGetLastError();
}

int hs_ranges_to_tiles_aligned(const int64_t* rstart, const int64_t* rlen, int R, int tile_rows,
                               int64_t align, int64_t* tile_prefix, void* stream) {
  hipLaunchKernelGGL(hs_ranges_to_tiles_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, rlen,
                     R, tile_rows, tile_prefix, rstart, align);
  return (int)hipGetLastError();
}

int hs_agg_final(const double* psum, const int64_t* pcnt, const double* pmin, const double* pmax,
                 int nblk, int GA, double* osum, int64_t* ocnt, double* omin, double* omax,
                 void* stream) {
  if (GA <= 0) return 0;
  hipLaunchKernelGGL(hs_agg_final_kernel, dim3(GA), dim3(FIN_BLOCK), 0, (hipStream_t)stream, psum,
                     pcnt, pmin, pmax, nblk, GA, osum, ocnt, omin, omax);
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
  return hs_agg_final(psum, pcnt, pmin, pmax, grid, GA, osum, ocnt, omin, omax, stream);
}

int hs_scan_count(const ScanParams* p, const int64_t* rstart, const int64_t* rlen, int R,
                  const int64_t* tile_prefix, int grid, int64_t* tile_counts, void* stream) {
  hipLaunchKernelGGL(hs_scan_count_kernel, dim3(grid), dim3(SF_BLOCK), 0, (hipStream_t)stream, *p,
                     rstart, rlen, R, tile_prefix, tile_counts);
  return (int)hipGetLastError();
}

int hs_scan_bitmap(const ScanParams* p, const int64_t* rstart, const int64_t* rlen, int R,
                   const int64_t* tile_prefix, int grid, int key_slot, int64_t base, int64_t nbits,
                   unsigned long long* words, void* stream) {
  if (key_slot < 0 || key_slot >= HS_MAX_COLS) return -1;
  hipLaunchKernelGGL(hs_scan_bitmap_kernel, dim3(grid), dim3(SF_BLOCK), 0, (hipStream_t)stream, *p,
                     rstart, rlen, R, tile_prefix, key_slot, base, nbits, words);
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
