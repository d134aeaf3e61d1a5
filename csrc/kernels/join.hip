// K8: co-located per-bucket sort-merge join of two bucketed covering indexes.
//
// Both sides are sorted by the join key inside every bucket and bucket b of the left index joins
// only bucket b of the right one (equal numBuckets => zero inter-GPU traffic).  A workgroup takes
// a 2048-row tile of one left bucket range; lane 0 binary-searches the right bucket for the
// tile's [first key, last key] span, the whole span of right keys is staged in LDS, and every
// lane then binary-searches its key in LDS (falls back to the global bucket when the span does
// not fit).  Modes: fused aggregate (filters on both sides + product-of-affine aggregates, the
// TPC-H Q3-style hot path) or count/emit of (left_row, right_row) pairs for general joins.
#include "hs_scan.h"

#define JN_BLOCK 256
#define JN_ITEMS 8
#define JN_TILE (JN_BLOCK * JN_ITEMS)
#define JN_LDS_KEYS 4096
#define JN_SPLIT 8   // column slots < 8: left side, >= 8: right side

struct JoinParams {
  ColDesc cols[HS_MAX_COLS];   // 0..7 left, 8..15 right
  Pred preds[HS_MAX_PREDS];    // [0, nlp): left-only, [nlp, npreds): per match
  AggSpec aggs[HS_MAX_AGGS];
  int32_t npreds;
  int32_t nlp;
  int32_t naggs;
  int32_t lkey;                // slot of left key
  int32_t rkey;                // slot of right key
  int32_t group_col;           // -1 or slot (either side)
  int32_t num_groups;
  int32_t key_is_float;
  int64_t group_base;
};

__device__ __forceinline__ uint64_t join_key(const ColDesc& c, int64_t row, bool is_float) {
  if (is_float) {
    double d = load_f64(c, row);
    if (d == 0.0) d = 0.0;
    uint64_t b = (uint64_t)__double_as_longlong(d);
    return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
  }
  return (uint64_t)load_i64(c, row) ^ 0x8000000000000000ull;
}

__device__ __forceinline__ int64_t find_range_j(const int64_t* tile_prefix, int R, int64_t t) {
  int lo = 0, hi = R;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (tile_prefix[mid] <= t) lo = mid; else hi = mid;
  }
  return lo;
}

// global lower/upper bound over [lo,hi) of the right key column (nulls first, never equal)
__device__ __forceinline__ int64_t rkey_bound(const ColDesc& c, int64_t lo, int64_t hi, uint64_t k,
                                              bool upper, bool is_float) {
  while (lo < hi) {
    const int64_t mid = lo + ((hi - lo) >> 1);
    bool less;
    if (!col_valid(c, mid)) less = true;
    else {
      const uint64_t v = join_key(c, mid, is_float);
      less = upper ? (v <= k) : (v < k);
    }
    if (less) lo = mid + 1; else hi = mid;
  }
  return lo;
}

struct TileCtx {
  int64_t row0, rows, rs, re;
  bool staged;
};

// Sets up the tile: left row span and the right key span [rs, re) staged into LDS when it fits.
__device__ __forceinline__ TileCtx join_tile_setup(const JoinParams& p, const int64_t* rstart,
                                                   const int64_t* rlen, const int32_t* rbucket,
                                                   const int64_t* roff, int R,
                                                   const int64_t* tile_prefix, int64_t t,
                                                   uint64_t* skeys, int64_t* sh) {
  const int r = (int)find_range_j(tile_prefix, R, t);
  const int64_t off = (t - tile_prefix[r]) * JN_TILE;
  TileCtx ctx;
  ctx.row0 = rstart[r] + off;
  ctx.rows = min((int64_t)JN_TILE, rlen[r] - off);
  const bool fl = p.key_is_float != 0;
  if (threadIdx.x == 0) {
    const int b = rbucket[r];
    const int64_t bs = roff[b], be = roff[b + 1];
    // first / last valid left key of the tile (left is sorted, nulls first)
    const ColDesc& lk = p.cols[p.lkey];
    int64_t f = ctx.row0, l = ctx.row0 + ctx.rows - 1;
    while (f <= l && !col_valid(lk, f)) ++f;
    int64_t rs = bs, re = bs;
    if (f <= l && col_valid(lk, l)) {
      const uint64_t kmin = join_key(lk, f, fl), kmax = join_key(lk, l, fl);
      rs = rkey_bound(p.cols[p.rkey], bs, be, kmin, false, fl);
      re = rkey_bound(p.cols[p.rkey], rs, be, kmax, true, fl);
    }
    sh[0] = rs;
    sh[1] = re;
  }
  __syncthreads();
  ctx.rs = sh[0];
  ctx.re = sh[1];
  ctx.staged = (ctx.re - ctx.rs) <= JN_LDS_KEYS;
  if (ctx.staged) {
    for (int64_t j = threadIdx.x; j < ctx.re - ctx.rs; j += JN_BLOCK)
      skeys[j] = join_key(p.cols[p.rkey], ctx.rs + j, fl);  // right keys in span are non-null
  }
  __syncthreads();
  return ctx;
}

__device__ __forceinline__ int64_t span_lower(const TileCtx& ctx, const uint64_t* skeys,
                                              const JoinParams& p, uint64_t k) {
  if (ctx.staged) {
    int64_t lo = 0, hi = ctx.re - ctx.rs;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (skeys[mid] < k) lo = mid + 1; else hi = mid;
    }
    return ctx.rs + lo;
  }
  return rkey_bound(p.cols[p.rkey], ctx.rs, ctx.re, k, false, p.key_is_float != 0);
}

__device__ __forceinline__ uint64_t span_key(const TileCtx& ctx, const uint64_t* skeys,
                                             const JoinParams& p, int64_t j) {
  return ctx.staged ? skeys[j - ctx.rs] : join_key(p.cols[p.rkey], j, p.key_is_float != 0);
}

// ------------------------------------------------------------------------------------------------
// Fused join + aggregate
// ------------------------------------------------------------------------------------------------
template <bool GROUPED>
__global__ __launch_bounds__(JN_BLOCK) void hs_join_agg_kernel(
    JoinParams p, const int64_t* __restrict__ rstart, const int64_t* __restrict__ rlen,
    const int32_t* __restrict__ rbucket, const int64_t* __restrict__ roff, int R,
    const int64_t* __restrict__ tile_prefix, double* __restrict__ psum, int64_t* __restrict__ pcnt,
    double* __restrict__ pmin, double* __restrict__ pmax) {
  __shared__ uint64_t skeys[JN_LDS_KEYS];
  __shared__ int64_t sh[2];
  extern __shared__ __attribute__((aligned(16))) double glds[];
  const int A = p.naggs;
  const int GA = GROUPED ? p.num_groups * A : A;
  GroupLds gl = group_lds(glds, GROUPED ? GA : 0);
  if (GROUPED) group_lds_init(gl, GA, JN_BLOCK);  // visible after the tile setup barrier
  AggAcc acc;
  acc_init(acc);
  const bool fl = p.key_is_float != 0;
  const ColDesc& lk = p.cols[p.lkey];
  const int64_t ntiles = tile_prefix[R];
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    TileCtx ctx = join_tile_setup(p, rstart, rlen, rbucket, roff, R, tile_prefix, t, skeys, sh);
    for (int it = 0; it < JN_ITEMS; ++it) {
      const int64_t k = (int64_t)it * JN_BLOCK + threadIdx.x;
      const int64_t lrow = ctx.row0 + k;
      RowRef rr{lrow, 0};
      bool lok = k < ctx.rows && col_valid(lk, lrow) &&
                 hs_eval_cnf(p.preds, 0, p.nlp, p.cols, JN_SPLIT, rr);
      uint64_t key = 0;
      int64_t j = 0;
      if (lok) {
        key = join_key(lk, lrow, fl);
        j = span_lower(ctx, skeys, p, key);
        lok = j < ctx.re && span_key(ctx, skeys, p, j) == key;
      }
      // one match per lane per round; rounds are wave-uniform so acc_row sees a converged wave
      while (__any(lok)) {
        bool pass = false;
        int gidx = 0;
        if (lok) {
          rr.r1 = j;
          pass = hs_eval_cnf(p.preds, p.nlp, p.npreds, p.cols, JN_SPLIT, rr);
          if (GROUPED && pass) {
            const ColDesc& gc = p.cols[p.group_col];
            const int64_t grow = p.group_col >= JN_SPLIT ? j : lrow;
            if (!col_valid(gc, grow)) {
              pass = false;
            } else {
              gidx = (int)(load_i64(gc, grow) - p.group_base);
              if (gidx < 0 || gidx >= p.num_groups) pass = false;
            }
          }
        }
        acc_row<GROUPED>(acc, p.aggs, A, pass, gidx, p.cols, JN_SPLIT, rr, gl);
        if (lok) {
          ++j;
          lok = j < ctx.re && span_key(ctx, skeys, p, j) == key;
        }
      }
    }
    __syncthreads();  // skeys reuse
  }
  acc_flush<GROUPED, JN_BLOCK>(acc, A, GA, gl, psum, pcnt, pmin, pmax);
}

// ------------------------------------------------------------------------------------------------
// Pair count / emit (general inner join)
// ------------------------------------------------------------------------------------------------
template <bool EMIT>
__global__ __launch_bounds__(JN_BLOCK) void hs_join_pairs_kernel(
    JoinParams p, const int64_t* __restrict__ rstart, const int64_t* __restrict__ rlen,
    const int32_t* __restrict__ rbucket, const int64_t* __restrict__ roff, int R,
    const int64_t* __restrict__ tile_prefix, int64_t* __restrict__ tile_counts,
    const int64_t* __restrict__ tile_offsets, int64_t* __restrict__ out_l,
    int64_t* __restrict__ out_r) {
  __shared__ uint64_t skeys[JN_LDS_KEYS];
  __shared__ int64_t sh[2];
  __shared__ int64_t wtot[JN_BLOCK / 64];
  __shared__ int64_t run;
  const bool fl = p.key_is_float != 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t ntiles = tile_prefix[R];
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    TileCtx ctx = join_tile_setup(p, rstart, rlen, rbucket, roff, R, tile_prefix, t, skeys, sh);
    if (EMIT && threadIdx.x == 0) run = tile_offsets[t];
    int64_t total = 0;
    for (int it = 0; it < JN_ITEMS; ++it) {
      const int64_t k = (int64_t)it * JN_BLOCK + threadIdx.x;
      int64_t cnt = 0, first = 0;
      uint64_t key = 0;
      int64_t lrow = 0;
      bool ok = false;
      if (k < ctx.rows) {
        lrow = ctx.row0 + k;
        const ColDesc& lk = p.cols[p.lkey];
        RowRef rr{lrow, 0};
        if (col_valid(lk, lrow) && hs_eval_cnf(p.preds, 0, p.nlp, p.cols, JN_SPLIT, rr)) {
          ok = true;
          key = join_key(lk, lrow, fl);
          first = span_lower(ctx, skeys, p, key);
          for (int64_t j = first; j < ctx.re && span_key(ctx, skeys, p, j) == key; ++j) {
            rr.r1 = j;
            if (hs_eval_cnf(p.preds, p.nlp, p.npreds, p.cols, JN_SPLIT, rr)) ++cnt;
          }
        }
      }
      if (!EMIT) {
        total += cnt;
        continue;
      }
      // stable exclusive prefix of cnt across the block (wave scan + wave totals)
      int64_t x = cnt;
      for (int off = 1; off < 64; off <<= 1) {
        int64_t y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      if (lane == 63) wtot[w] = x;
      __syncthreads();
      if (threadIdx.x == 0) {
        int64_t acc = run;
        for (int ww = 0; ww < JN_BLOCK / 64; ++ww) {
          const int64_t v = wtot[ww];
          wtot[ww] = acc;
          acc += v;
        }
        run = acc;
      }
      __syncthreads();
      int64_t pos = wtot[w] + x - cnt;
      if (ok && cnt) {
        RowRef rr{lrow, 0};
        for (int64_t j = first; j < ctx.re && span_key(ctx, skeys, p, j) == key; ++j) {
          rr.r1 = j;
          if (hs_eval_cnf(p.preds, p.nlp, p.npreds, p.cols, JN_SPLIT, rr)) {
            out_l[pos] = lrow;
            out_r[pos] = j;
            ++pos;
          }
        }
      }
      __syncthreads();
    }
    if (!EMIT) {
      total = hs_wave_sum(total);
      if (lane == 0) wtot[w] = total;
      __syncthreads();
      if (threadIdx.x == 0) {
        int64_t tt = 0;
        for (int ww = 0; ww < JN_BLOCK / 64; ++ww) tt += wtot[ww];
        tile_counts[t] = tt;
      }
    }
    __syncthreads();
  }
}

extern "C" {

int hs_join_params_size() { return (int)sizeof(JoinParams); }
int hs_join_tile_rows() { return JN_TILE; }

int hs_agg_final(const double* psum, const int64_t* pcnt, const double* pmin, const double* pmax,
                 int nblk, int GA, double* osum, int64_t* ocnt, double* omin, double* omax,
                 void* stream);

int hs_join_agg(const JoinParams* p, const int64_t* rstart, const int64_t* rlen,
                const int32_t* rbucket, const int64_t* roff, int R, const int64_t* tile_prefix,
                int grid, double* psum, int64_t* pcnt, double* pmin, double* pmax, double* osum,
                int64_t* ocnt, double* omin, double* omax, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const bool grouped = p->group_col >= 0;
  if (grouped) {
    const int GA = p->num_groups * p->naggs;
    const size_t lds = (size_t)GA * 32;
    if (lds > 96 * 1024) return -5;
    hipLaunchKernelGGL(hs_join_agg_kernel<true>, dim3(grid), dim3(JN_BLOCK), lds, s, *p, rstart,
                       rlen, rbucket, roff, R, tile_prefix, psum, pcnt, pmin, pmax);
  } else {
    hipLaunchKernelGGL(hs_join_agg_kernel<false>, dim3(grid), dim3(JN_BLOCK), 0, s, *p, rstart,
                       rlen, rbucket, roff, R, tile_prefix, psum, pcnt, pmin, pmax);
  }
  const int GA = grouped ? p->num_groups * p->naggs : p->naggs;
  return hs_agg_final(psum, pcnt, pmin, pmax, grid, GA, osum, ocnt, omin, omax, stream);
}

int hs_join_count(const JoinParams* p, const int64_t* rstart, const int64_t* rlen,
                  const int32_t* rbucket, const int64_t* roff, int R, const int64_t* tile_prefix,
                  int grid, int64_t* tile_counts, void* stream) {
  hipLaunchKernelGGL(hs_join_pairs_kernel<false>, dim3(grid), dim3(JN_BLOCK), 0,
                     (hipStream_t)stream, *p, rstart, rlen, rbucket, roff, R, tile_prefix,
                     tile_counts, (const int64_t*)nullptr, (int64_t*)nullptr, (int64_t*)nullptr);
  return (int)hipGetLastError();
}

int hs_join_emit(const JoinParams* p, const int64_t* rstart, const int64_t* rlen,
                 const int32_t* rbucket, const int64_t* roff, int R, const int64_t* tile_prefix,
                 int grid, const int64_t* tile_offsets, int64_t* out_l, int64_t* out_r,
                 void* stream) {
  hipLaunchKernelGGL(hs_join_pairs_kernel<true>, dim3(grid), dim3(JN_BLOCK), 0,
                     (hipStream_t)stream, *p, rstart, rlen, rbucket, roff, R, tile_prefix,
                     (int64_t*)nullptr, tile_offsets, out_l, out_r);
  return (int)hipGetLastError();
}

}  // extern "C"
