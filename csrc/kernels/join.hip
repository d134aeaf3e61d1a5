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
#define JN_LDS_KEYS 6144
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
  double* g_sum = glds;
  double* g_min = glds + GA;
  double* g_max = glds + 2 * GA;
  unsigned long long* g_cnt = (unsigned long long*)(glds + 3 * GA);
  if (GROUPED) {
    for (int i = threadIdx.x; i < GA; i += JN_BLOCK) {
      g_sum[i] = 0.0;
      g_min[i] = __builtin_inf();
      g_max[i] = -__builtin_inf();
      g_cnt[i] = 0ull;
    }
  }
  double s[HS_MAX_AGGS], mn[HS_MAX_AGGS], mx[HS_MAX_AGGS];
  int64_t c[HS_MAX_AGGS];
#pragma unroll
  for (int a = 0; a < HS_MAX_AGGS; ++a) {
    s[a] = 0.0; c[a] = 0; mn[a] = __builtin_inf(); mx[a] = -__builtin_inf();
  }
  const bool fl = p.key_is_float != 0;
  const int64_t ntiles = tile_prefix[R];
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    TileCtx ctx = join_tile_setup(p, rstart, rlen, rbucket, roff, R, tile_prefix, t, skeys, sh);
    for (int it = 0; it < JN_ITEMS; ++it) {
      const int64_t k = (int64_t)it * JN_BLOCK + threadIdx.x;
      if (k >= ctx.rows) break;
      const int64_t lrow = ctx.row0 + k;
      const ColDesc& lk = p.cols[p.lkey];
      if (!col_valid(lk, lrow)) continue;
      RowRef rr{lrow, 0};
      if (!hs_eval_cnf(p.preds, 0, p.nlp, p.cols, JN_SPLIT, rr)) continue;
      const uint64_t key = join_key(lk, lrow, fl);
      for (int64_t j = span_lower(ctx, skeys, p, key); j < ctx.re && span_key(ctx, skeys, p, j) == key; ++j) {
        rr.r1 = j;
        if (!hs_eval_cnf(p.preds, p.nlp, p.npreds, p.cols, JN_SPLIT, rr)) continue;
        int gidx = 0;
        if (GROUPED) {
          const ColDesc& gc = p.cols[p.group_col];
          const int64_t grow = p.group_col >= JN_SPLIT ? j : lrow;
          if (!col_valid(gc, grow)) continue;
          gidx = (int)(load_i64(gc, grow) - p.group_base);
          if (gidx < 0 || gidx >= p.num_groups) continue;
        }
#pragma unroll
        for (int a = 0; a < HS_MAX_AGGS; ++a) {
          if (a >= A) break;
          const AggSpec& ag = p.aggs[a];
          double v = 0.0;
          if (ag.kind != AK_COUNT_STAR && !hs_agg_value(ag, p.cols, JN_SPLIT, rr, v)) continue;
          if (GROUPED) {
            const int slot = gidx * A + a;
            if (ag.kind == AK_SUM) atomicAdd(&g_sum[slot], v);
            else if (ag.kind == AK_MIN) hs_lds_atomic_min(&g_min[slot], v);
            else if (ag.kind == AK_MAX) hs_lds_atomic_max(&g_max[slot], v);
            atomicAdd(&g_cnt[slot], 1ull);
          } else {
            s[a] += v; c[a] += 1; mn[a] = fmin(mn[a], v); mx[a] = fmax(mx[a], v);
          }
        }
      }
    }
    __syncthreads();  // skeys reuse
  }
  if (GROUPED) {
    __syncthreads();
    for (int i = threadIdx.x; i < GA; i += JN_BLOCK) {
      const int64_t o = (int64_t)blockIdx.x * GA + i;
      psum[o] = g_sum[i]; pcnt[o] = (int64_t)g_cnt[i]; pmin[o] = g_min[i]; pmax[o] = g_max[i];
    }
    return;
  }
  __shared__ double r_s[JN_BLOCK / 64][HS_MAX_AGGS], r_mn[JN_BLOCK / 64][HS_MAX_AGGS],
      r_mx[JN_BLOCK / 64][HS_MAX_AGGS];
  __shared__ int64_t r_c[JN_BLOCK / 64][HS_MAX_AGGS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < HS_MAX_AGGS; ++a) {
    if (a >= A) break;
    const double ws = hs_wave_sum(s[a]);
    const int64_t wc = hs_wave_sum(c[a]);
    const double wmn = hs_wave_min(mn[a]);
    const double wmx = hs_wave_max(mx[a]);
    if (lane == 0) { r_s[w][a] = ws; r_c[w][a] = wc; r_mn[w][a] = wmn; r_mx[w][a] = wmx; }
  }
  __syncthreads();
  if (threadIdx.x < A) {
    const int a = threadIdx.x;
    double ts = 0.0, tmn = __builtin_inf(), tmx = -__builtin_inf();
    int64_t tc = 0;
    for (int ww = 0; ww < JN_BLOCK / 64; ++ww) {
      ts += r_s[ww][a]; tc += r_c[ww][a]; tmn = fmin(tmn, r_mn[ww][a]); tmx = fmax(tmx, r_mx[ww][a]);
    }
    const int64_t o = (int64_t)blockIdx.x * A + a;
    psum[o] = ts; pcnt[o] = tc; pmin[o] = tmn; pmax[o] = tmx;
  }
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

int hs_join_agg(const JoinParams* p, const int64_t* rstart, const int64_t* rlen,
                const int32_t* rbucket, const int64_t* roff, int R, const int64_t* tile_prefix,
                int grid, double* psum, int64_t* pcnt, double* pmin, double* pmax, void* stream) {
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
  return (int)hipGetLastError();
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
