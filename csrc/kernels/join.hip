// K8: co-located per-bucket sort-merge join of two bucketed covering indexes.
//
// Both sides are sorted by the join key inside every bucket and bucket b of the left index joins
// only bucket b of the right one (equal numBuckets => zero inter-GPU traffic).
//
//  1. hs_join_spans_kernel — one *thread* per 2048-row left tile binary-searches the right
//     bucket for the tile's [first key, last key] span.  All tiles search concurrently, so the
//     ~40 dependent HBM round trips of a search are paid once for the whole join instead of once
//     per tile on a block's critical path.
//  2. the join kernels — each block takes a contiguous chunk of tiles, stages the tile's right
//     key span in LDS (coalesced), and every lane looks its SF_ITEMS left keys up in LDS; the
//     match rounds evaluate right-side predicates / aggregates predicate-major (hs_vec.h).
//
// Modes: fused aggregate (filters on both sides + product-of-affine aggregates, the TPC-H
// Q3-style hot path) or count/emit of (left_row, right_row) pairs for general joins.
#include "hs_vec.h"

#define JN_BLOCK 256
#define JN_ITEMS 4
#define JN_TILE (JN_BLOCK * JN_ITEMS)
#define JN_LDS_KEYS 2048
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

// Per tile: left rows [row0, row0+rows) and the right key span [rs, re).
__global__ __launch_bounds__(256) void hs_join_spans_kernel(
    JoinParams p, const int64_t* __restrict__ rstart, const int64_t* __restrict__ rlen,
    const int32_t* __restrict__ rbucket, const int64_t* __restrict__ roff, int R,
    const int64_t* __restrict__ tile_prefix, int64_t* __restrict__ spans, int tile_rows) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= tile_prefix[R]) return;
  const int r = tile_range_of(tile_prefix, R, t);
  const int64_t off = (t - tile_prefix[r]) * tile_rows;
  const int64_t row0 = rstart[r] + off;
  const int64_t rows = min((int64_t)tile_rows, rlen[r] - off);
  const bool fl = p.key_is_float != 0;
  const int b = rbucket[r];
  const int64_t bs = roff[b], be = roff[b + 1];
  const ColDesc& lk = p.cols[p.lkey];
  // first valid left key of the tile (left is sorted, nulls first) -> binary search
  int64_t f = row0, l = row0 + rows - 1;
  if (lk.valid != nullptr) {
    int64_t lo = row0, hi = row0 + rows;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (!col_valid(lk, mid)) lo = mid + 1; else hi = mid;
    }
    f = lo;
  }
  int64_t rs = bs, re = bs;
  if (f <= l) {
    const uint64_t kmin = join_key(lk, f, fl), kmax = join_key(lk, l, fl);
    rs = rkey_bound(p.cols[p.rkey], bs, be, kmin, false, fl);
    re = rkey_bound(p.cols[p.rkey], rs, be, kmax, true, fl);
  }
  spans[4 * t + 0] = row0;
  spans[4 * t + 1] = rows;
  spans[4 * t + 2] = rs;
  spans[4 * t + 3] = re;
}

// ---- sampled span search (generated-kernel path) ------------------------------------------
// A sparse index over the right side — every JN_SAMPLE-th key of each bucket, built per join in
// one strided pass (~1/64 of the right keys) — is small enough to stay in L2 / Infinity Cache.
// A tile's span start is then a search of the cached samples plus one <=64-key window in HBM,
// and the span end gallops forward from the start (spans are short for FK joins): ~9 HBM
// transactions per tile instead of ~40 dependent random reads for two full binary searches.
#define JN_SAMPLE 64

__global__ __launch_bounds__(256) void hs_join_sample_kernel(
    ColDesc rk, const int64_t* __restrict__ roff, const int64_t* __restrict__ soff, int B,
    int64_t nsamples, uint64_t* __restrict__ samples, int is_float) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsamples || i >= soff[B]) return;  // nsamples: host-side bound of soff[B]
  int lo = 0, hi = B;  // bucket b with soff[b] <= i < soff[b+1]
  while (hi - lo > 1) {
    const int md = (lo + hi) >> 1;
    if (soff[md] <= i) lo = md; else hi = md;
  }
  const int64_t row = roff[lo] + (i - soff[lo]) * JN_SAMPLE;
  // nulls sort first and never match: the minimum image keeps the samples ordered
  samples[i] = col_valid(rk, row) ? join_key(rk, row, is_float != 0) : 0ull;
}

// first row in [bs, be) whose key is >= k (nulls count as smaller), via the bucket's samples
__device__ __forceinline__ int64_t sampled_lower(const ColDesc& c, const uint64_t* smp, int64_t ns,
                                                 int64_t bs, int64_t be, uint64_t k, bool fl) {
  int64_t lo = 0, hi = ns;  // first sample >= k
  while (lo < hi) {
    const int64_t md = (lo + hi) >> 1;
    if (smp[md] < k) lo = md + 1; else hi = md;
  }
  const int64_t wlo = lo == 0 ? bs : bs + (lo - 1) * JN_SAMPLE + 1;
  const int64_t whi = lo == ns ? be : min(be, bs + lo * JN_SAMPLE);
  return rkey_bound(c, wlo, whi, k, false, fl);
}

// first row in [from, be) whose key is > k, galloping forward from `from`
__device__ __forceinline__ int64_t gallop_upper(const ColDesc& c, int64_t from, int64_t be,
                                                uint64_t k, bool fl) {
  int64_t lo = from, step = 1;
  while (lo < be) {
    const int64_t probe = min(be - 1, lo + step - 1);
    const bool le = !col_valid(c, probe) || join_key(c, probe, fl) <= k;
    if (!le) return rkey_bound(c, lo, probe, k, true, fl);
    lo = probe + 1;
    step <<= 1;
  }
  return be;
}

__global__ __launch_bounds__(256) void hs_join_spans_sampled_kernel(
    JoinParams p, const int64_t* __restrict__ rstart, const int64_t* __restrict__ rlen,
    const int32_t* __restrict__ rbucket, const int64_t* __restrict__ roff,
    const int64_t* __restrict__ soff, const uint64_t* __restrict__ samples, int R,
    const int64_t* __restrict__ tile_prefix, int64_t* __restrict__ spans, int tile_rows,
    int align) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= tile_prefix[R]) return;
  const int r = tile_range_of(tile_prefix, R, t);
  const int64_t off = (t - tile_prefix[r]) * tile_rows;
  // align > 1: tiles of range r start at rstart[r] rounded down to a multiple of `align` (the
  // vectorized merge join loads each thread's rows as aligned vectors); the tile's own rows are
  // its intersection with the range
  const int64_t a0 = (rstart[r] & ~(int64_t)(align - 1)) + off;
  const int64_t row0 = max(a0, rstart[r]);
  const int64_t rows = min(a0 + (int64_t)tile_rows, rstart[r] + rlen[r]) - row0;
  const bool fl = p.key_is_float != 0;
  const int b = rbucket[r];
  const int64_t bs = roff[b], be = roff[b + 1];
  const ColDesc& lk = p.cols[p.lkey];
  int64_t f = row0;
  const int64_t l = row0 + rows - 1;
  if (lk.valid != nullptr) {
    int64_t lo = row0, hi = row0 + rows;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (!col_valid(lk, mid)) lo = mid + 1; else hi = mid;
    }
    f = lo;
  }
  int64_t rs = bs, re = bs;
  if (f <= l) {
    const uint64_t kmin = join_key(lk, f, fl), kmax = join_key(lk, l, fl);
    const ColDesc& rk = p.cols[p.rkey];
    rs = sampled_lower(rk, samples + soff[b], soff[b + 1] - soff[b], bs, be, kmin, fl);
    re = gallop_upper(rk, rs, be, kmax, fl);
  }
  spans[4 * t + 0] = row0;
  spans[4 * t + 1] = rows;
  spans[4 * t + 2] = rs;
  spans[4 * t + 3] = re;
}

struct JTile {
  int64_t row0, rows, rs, re;
  bool staged;
};

__device__ __forceinline__ JTile jtile_load(const JoinParams& p, const int64_t* spans, int64_t t,
                                            uint64_t* skeys) {
  JTile c;
  c.row0 = spans[4 * t + 0];
  c.rows = spans[4 * t + 1];
  c.rs = spans[4 * t + 2];
  c.re = spans[4 * t + 3];
  c.staged = (c.re - c.rs) <= JN_LDS_KEYS;
  if (c.staged) {
    const bool fl = p.key_is_float != 0;
    for (int64_t j = threadIdx.x; j < c.re - c.rs; j += JN_BLOCK)
      skeys[j] = join_key(p.cols[p.rkey], c.rs + j, fl);  // right keys in span are non-null
  }
  __syncthreads();
  return c;
}

__device__ __forceinline__ int64_t span_lower(const JTile& c, const uint64_t* skeys,
                                              const JoinParams& p, uint64_t k) {
  if (c.staged) {
    int64_t lo = 0, hi = c.re - c.rs;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (skeys[mid] < k) lo = mid + 1; else hi = mid;
    }
    return c.rs + lo;
  }
  return rkey_bound(p.cols[p.rkey], c.rs, c.re, k, false, p.key_is_float != 0);
}

__device__ __forceinline__ uint64_t span_key(const JTile& c, const uint64_t* skeys,
                                             const JoinParams& p, int64_t j) {
  return c.staged ? skeys[j - c.rs] : join_key(p.cols[p.rkey], j, p.key_is_float != 0);
}

// Left batch of a tile: rows, left predicates, key lookup.  m[i]: row i has a first match at j[i].
__device__ __forceinline__ void jbatch_probe(const JoinParams& p, const JTile& c,
                                             const uint64_t* skeys, int64_t (&r0)[JN_ITEMS],
                                             uint64_t (&key)[JN_ITEMS], int64_t (&j)[JN_ITEMS],
                                             bool (&m)[JN_ITEMS]) {
  bool act[JN_ITEMS];
#pragma unroll
  for (int i = 0; i < JN_ITEMS; ++i) {
    const int64_t k = (int64_t)i * JN_BLOCK + threadIdx.x;
    act[i] = k < c.rows;
    r0[i] = act[i] ? c.row0 + k : c.row0;
  }
  const ColDesc& lk = p.cols[p.lkey];
  bool lv[JN_ITEMS];
  vvalid(lk, r0, act, lv);
  veval_cnf(p.preds, 0, p.nlp, p.cols, JN_SPLIT, r0, r0, lv, m);
  const bool fl = p.key_is_float != 0;
  if (fl) {
    double x[JN_ITEMS];
    vload_f64(lk, r0, m, x);
#pragma unroll
    for (int i = 0; i < JN_ITEMS; ++i) {
      double d = x[i] == 0.0 ? 0.0 : x[i];
      const uint64_t b = (uint64_t)__double_as_longlong(d);
      key[i] = (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
    }
  } else {
    int64_t x[JN_ITEMS];
    vload_i64(lk, r0, m, x);
#pragma unroll
    for (int i = 0; i < JN_ITEMS; ++i) key[i] = (uint64_t)x[i] ^ 0x8000000000000000ull;
  }
#pragma unroll
  for (int i = 0; i < JN_ITEMS; ++i) {
    j[i] = c.rs;
    if (m[i]) {
      j[i] = span_lower(c, skeys, p, key[i]);
      m[i] = j[i] < c.re && span_key(c, skeys, p, j[i]) == key[i];
    }
  }
}

__device__ __forceinline__ bool any_of(const bool (&m)[JN_ITEMS]) {
  bool a = false;
#pragma unroll
  for (int i = 0; i < JN_ITEMS; ++i) a = a || m[i];
  return a;
}

// ------------------------------------------------------------------------------------------------
// Fused join + aggregate
// ------------------------------------------------------------------------------------------------
template <bool GROUPED>
__global__ __launch_bounds__(JN_BLOCK) void hs_join_agg_kernel(
    JoinParams p, const int64_t* __restrict__ tile_prefix, int R,
    const int64_t* __restrict__ spans, double* __restrict__ psum, int64_t* __restrict__ pcnt,
    double* __restrict__ pmin, double* __restrict__ pmax) {
  __shared__ uint64_t skeys[JN_LDS_KEYS];
  extern __shared__ __attribute__((aligned(16))) double glds[];
  const int A = p.naggs;
  const int GA = GROUPED ? p.num_groups * A : A;
  GroupLds gl = group_lds(glds, GROUPED ? GA : 0);
  if (GROUPED) group_lds_init(gl, GA, JN_BLOCK);  // visible after the first tile barrier
  AggAcc acc;
  acc_init(acc, p.aggs, A);
  int64_t t0, t1;
  block_tile_chunk(tile_prefix[R], t0, t1);
  if (GROUPED) __syncthreads();
  for (int64_t t = t0; t < t1; ++t) {
    const JTile c = jtile_load(p, spans, t, skeys);
    int64_t r0[JN_ITEMS], j[JN_ITEMS];
    uint64_t key[JN_ITEMS];
    bool m[JN_ITEMS];
    jbatch_probe(p, c, skeys, r0, key, j, m);
    // match rounds: every row advances one right match per round (wave-uniform trip count)
    while (__any(any_of(m))) {
      bool pass[JN_ITEMS];
      veval_cnf(p.preds, p.nlp, p.npreds, p.cols, JN_SPLIT, r0, j, m, pass);
      int g[JN_ITEMS];
#pragma unroll
      for (int i = 0; i < JN_ITEMS; ++i) g[i] = 0;
      if (GROUPED)
        vgroup(p.cols, p.group_col, JN_SPLIT, p.group_base, p.num_groups, r0, j, pass, g);
      vaccumulate<GROUPED, JN_ITEMS>(acc, p.aggs, A, p.cols, JN_SPLIT, r0, j, pass, g, gl);
#pragma unroll
      for (int i = 0; i < JN_ITEMS; ++i) {
        if (m[i]) {
          ++j[i];
          m[i] = j[i] < c.re && span_key(c, skeys, p, j[i]) == key[i];
        }
      }
    }
    __syncthreads();  // skeys reuse
  }
  acc_flush<GROUPED, JN_BLOCK>(acc, p.aggs, A, GA, gl, psum, pcnt, pmin, pmax);
}

// ------------------------------------------------------------------------------------------------
// Pair count / emit (general inner join).  Output order: tile, then left row, then right row.
// ------------------------------------------------------------------------------------------------
template <bool EMIT>
__global__ __launch_bounds__(JN_BLOCK) void hs_join_pairs_kernel(
    JoinParams p, const int64_t* __restrict__ tile_prefix, int R,
    const int64_t* __restrict__ spans, int64_t* __restrict__ tile_counts,
    const int64_t* __restrict__ tile_offsets, int64_t* __restrict__ out_l,
    int64_t* __restrict__ out_r) {
  __shared__ uint64_t skeys[JN_LDS_KEYS];
  __shared__ int64_t wtot[JN_ITEMS][JN_BLOCK / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t t0, t1;
  block_tile_chunk(tile_prefix[R], t0, t1);
  for (int64_t t = t0; t < t1; ++t) {
    const JTile c = jtile_load(p, spans, t, skeys);
    int64_t r0[JN_ITEMS], j0[JN_ITEMS];
    uint64_t key[JN_ITEMS];
    bool m0[JN_ITEMS];
    jbatch_probe(p, c, skeys, r0, key, j0, m0);
    // count matches per row (right predicates evaluated per match round)
    int64_t cnt[JN_ITEMS], j[JN_ITEMS];
    bool m[JN_ITEMS];
#pragma unroll
    for (int i = 0; i < JN_ITEMS; ++i) {
      cnt[i] = 0;
      j[i] = j0[i];
      m[i] = m0[i];
    }
    while (__any(any_of(m))) {
      bool pass[JN_ITEMS];
      veval_cnf(p.preds, p.nlp, p.npreds, p.cols, JN_SPLIT, r0, j, m, pass);
#pragma unroll
      for (int i = 0; i < JN_ITEMS; ++i) {
        cnt[i] += pass[i] ? 1 : 0;
        if (m[i]) {
          ++j[i];
          m[i] = j[i] < c.re && span_key(c, skeys, p, j[i]) == key[i];
        }
      }
    }
    if (!EMIT) {
      int64_t tot = 0;
#pragma unroll
      for (int i = 0; i < JN_ITEMS; ++i) tot += cnt[i];
      tot = hs_wave_sum(tot);
      if (lane == 0) wtot[0][w] = tot;
      __syncthreads();
      if (threadIdx.x == 0) {
        int64_t tt = 0;
        for (int ww = 0; ww < JN_BLOCK / 64; ++ww) tt += wtot[0][ww];
        tile_counts[t] = tt;
      }
      __syncthreads();
      continue;
    }
    // exclusive position of each row's run: order (item, wave, lane) == left row order
    int64_t x[JN_ITEMS];
#pragma unroll
    for (int i = 0; i < JN_ITEMS; ++i) {
      int64_t v = cnt[i];
      for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(v, off, 64);
        if (lane >= off) v += y;
      }
      x[i] = v - cnt[i];
      if (lane == 63) wtot[i][w] = v;
    }
    __syncthreads();
    int64_t base = tile_offsets[t];
#pragma unroll
    for (int i = 0; i < JN_ITEMS; ++i) {
      int64_t mine = base;
      for (int ww = 0; ww < JN_BLOCK / 64; ++ww) {
        if (ww < w) mine += wtot[i][ww];
        base += wtot[i][ww];
      }
      x[i] += mine;
    }
    // emit rounds
#pragma unroll
    for (int i = 0; i < JN_ITEMS; ++i) {
      j[i] = j0[i];
      m[i] = m0[i];
    }
    while (__any(any_of(m))) {
      bool pass[JN_ITEMS];
      veval_cnf(p.preds, p.nlp, p.npreds, p.cols, JN_SPLIT, r0, j, m, pass);
#pragma unroll
      for (int i = 0; i < JN_ITEMS; ++i) {
        if (pass[i]) {
          out_l[x[i]] = r0[i];
          out_r[x[i]] = j[i];
          ++x[i];
        }
        if (m[i]) {
          ++j[i];
          m[i] = j[i] < c.re && span_key(c, skeys, p, j[i]) == key[i];
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------------------------
// Join index (exec/join_index.py): the first matching right row of every left row (-1 = none) for
// a pair of device-resident index tables.  Built ONCE per table pair with the same span + LDS
// search the join kernels use; the tables are immutable, so every later join of the pair is a
// streaming scan of the left table plus a gather of the right columns (exec/jit.py
// gen_join_index_agg) — no span search, no LDS staging, no binary search per query.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(JN_BLOCK) void hs_join_index_kernel(
    JoinParams p, const int64_t* __restrict__ tile_prefix, int R,
    const int64_t* __restrict__ spans, int32_t* __restrict__ jidx) {
  __shared__ uint64_t skeys[JN_LDS_KEYS];
  int64_t t0, t1;
  block_tile_chunk(tile_prefix[R], t0, t1);
  for (int64_t t = t0; t < t1; ++t) {
    const JTile c = jtile_load(p, spans, t, skeys);
    int64_t r0[JN_ITEMS], j0[JN_ITEMS];
    uint64_t key[JN_ITEMS];
    bool m0[JN_ITEMS];
    jbatch_probe(p, c, skeys, r0, key, j0, m0);  // p.nlp == 0: key validity only
#pragma unroll
    for (int i = 0; i < JN_ITEMS; ++i) {
      const int64_t k = (int64_t)i * JN_BLOCK + threadIdx.x;
      if (k < c.rows) jidx[r0[i]] = m0[i] ? (int32_t)j0[i] : -1;
    }
    __syncthreads();  // skeys is restaged by the next tile
  }
}

static int launch_spans(const JoinParams* p, const int64_t* rstart, const int64_t* rlen,
                        const int32_t* rbucket, const int64_t* roff, int R,
                        const int64_t* tile_prefix, int64_t max_tiles, int64_t* spans,
                        hipStream_t s, int tile_rows = JN_TILE) {
  if (max_tiles <= 0) return 0;
  const int64_t blocks = (max_tiles + 255) / 256;
  hipLaunchKernelGGL(hs_join_spans_kernel, dim3((unsigned)blocks), dim3(256), 0, s, *p, rstart,
                     rlen, rbucket, roff, R, tile_prefix, spans, tile_rows);
  return (int)hipGetLastError();
}

extern "C" {

// Per-tile (row0, rows, rs, re) only — consumed by the generated join kernels (exec/jit.py),
// whose tile size is a codegen parameter (tile_prefix must be built with the same tile_rows).
int hs_join_spans(const JoinParams* p, const int64_t* rstart, const int64_t* rlen,
                  const int32_t* rbucket, const int64_t* roff, int R, const int64_t* tile_prefix,
                  int64_t max_tiles, int64_t* spans, int tile_rows, void* stream) {
  return launch_spans(p, rstart, rlen, rbucket, roff, R, tile_prefix, max_tiles, spans,
                      (hipStream_t)stream, tile_rows);
}

// Sampled variant: soff (B+1, device) = per-bucket sample offsets, soff[b+1]-soff[b] =
// ceil(rows_b / JN_SAMPLE); samples = scratch of nsamples >= soff[B] uint64 (filled here).
// align: 1, or the power-of-two row alignment of the tiles (tile_prefix built from
// rlen + (rstart & (align - 1)))
int hs_join_spans_sampled(const JoinParams* p, const int64_t* rstart, const int64_t* rlen,
                          const int32_t* rbucket, const int64_t* roff, const int64_t* soff, int B,
                          int64_t nsamples, uint64_t* samples, int R, const int64_t* tile_prefix,
                          int64_t max_tiles, int64_t* spans, int tile_rows, int align,
                          void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (align < 1 || (align & (align - 1)) != 0) return (int)hipErrorInvalidValue;
  if (nsamples > 0)
    hipLaunchKernelGGL(hs_join_sample_kernel, dim3((unsigned)((nsamples + 255) / 256)), dim3(256),
                       0, s, p->cols[p->rkey], roff, soff, B, nsamples, samples, p->key_is_float);
  if (max_tiles > 0)
    hipLaunchKernelGGL(hs_join_spans_sampled_kernel, dim3((unsigned)((max_tiles + 255) / 256)),
                       dim3(256), 0, s, *p, rstart, rlen, rbucket, roff, soff, samples, R,
                       tile_prefix, spans, tile_rows, align);
  return (int)hipGetLastError();
}

// spans: per-tile records from hs_join_spans_sampled built with tile_rows = JN_TILE;
// jidx: one int32 per left row (rows outside the ranges are left untouched).
int hs_join_index(const JoinParams* p, int R, const int64_t* tile_prefix, const int64_t* spans,
                  int grid, int32_t* jidx, void* stream) {
  JoinParams q = *p;
  q.npreds = 0;
  q.nlp = 0;
  hipLaunchKernelGGL(hs_join_index_kernel, dim3(grid), dim3(JN_BLOCK), 0, (hipStream_t)stream, q,
                     tile_prefix, R, spans, jidx);
  return (int)hipGetLastError();
}

int hs_join_sample_stride() { return JN_SAMPLE; }

int hs_join_params_size() { return (int)sizeof(JoinParams); }
int hs_join_tile_rows() { return JN_TILE; }

int hs_agg_final(const double* psum, const int64_t* pcnt, const double* pmin, const double* pmax,
                 int nblk, int GA, double* osum, int64_t* ocnt, double* omin, double* omax,
                 void* stream);

// spans: scratch of 4 * max_tiles int64 (max_tiles >= tile_prefix[R]).
int hs_join_agg(const JoinParams* p, const int64_t* rstart, const int64_t* rlen,
                const int32_t* rbucket, const int64_t* roff, int R, const int64_t* tile_prefix,
                int64_t max_tiles, int64_t* spans, int grid, double* psum, int64_t* pcnt,
                double* pmin, double* pmax, double* osum, int64_t* ocnt, double* omin,
                double* omax, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  HS_CHECK((hipError_t)launch_spans(p, rstart, rlen, rbucket, roff, R, tile_prefix, max_tiles,
                                    spans, s));
  const bool grouped = p->group_col >= 0;
  if (grouped) {
    const int GA = p->num_groups * p->naggs;
    const size_t lds = (size_t)GA * 32;
    if (lds > 96 * 1024) return -5;
    hipLaunchKernelGGL(hs_join_agg_kernel<true>, dim3(grid), dim3(JN_BLOCK), lds, s, *p,
                       tile_prefix, R, spans, psum, pcnt, pmin, pmax);
  } else {
    hipLaunchKernelGGL(hs_join_agg_kernel<false>, dim3(grid), dim3(JN_BLOCK), 0, s, *p,
                       tile_prefix, R, spans, psum, pcnt, pmin, pmax);
  }
  const int GA = grouped ? p->num_groups * p->naggs : p->naggs;
  return hs_agg_final(psum, pcnt, pmin, pmax, grid, GA, osum, ocnt, omin, omax, stream);
}

int hs_join_count(const JoinParams* p, const int64_t* rstart, const int64_t* rlen,
                  const int32_t* rbucket, const int64_t* roff, int R, const int64_t* tile_prefix,
                  int64_t max_tiles, int64_t* spans, int grid, int64_t* tile_counts,
                  void* stream) {
  hipStream_t s = (hipStream_t)stream;
  HS_CHECK((hipError_t)launch_spans(p, rstart, rlen, rbucket, roff, R, tile_prefix, max_tiles,
                                    spans, s));
  hipLaunchKernelGGL(hs_join_pairs_kernel<false>, dim3(grid), dim3(JN_BLOCK), 0, s, *p,
                     tile_prefix, R, (const int64_t*)spans, tile_counts, (const int64_t*)nullptr,
                     (int64_t*)nullptr, (int64_t*)nullptr);
  return (int)hipGetLastError();
}

// Reuses the spans computed by hs_join_count.
int hs_join_emit(const JoinParams* p, int R, const int64_t* tile_prefix, const int64_t* spans,
                 int grid, const int64_t* tile_offsets, int64_t* out_l, int64_t* out_r,
                 void* stream) {
  hipLaunchKernelGGL(hs_join_pairs_kernel<true>, dim3(grid), dim3(JN_BLOCK), 0,
                     (hipStream_t)stream, *p, tile_prefix, R, spans, (int64_t*)nullptr,
                     tile_offsets, out_l, out_r);
  return (int)hipGetLastError();
}

}  // extern "C"
