// Predicate / aggregate templates shared by the scan and join kernels.
//
// Predicates are a CNF: preds with equal `group` are OR-ed, groups are AND-ed (the host pushes
// NOT into the leaves).  Unknown (null) is false, which is exact for a final WHERE truth value.
// Aggregate values are products of affine terms  prod_i (alpha_i + beta_i * col_i), which covers
// x, x*y, x*(1-y), x*(1-y)*(1+z) (TPC-H Q1/Q3/Q6 shapes) with no interpreter in the inner loop.
#pragma once
#include "hs_common.h"

enum PredKind : int32_t {
  PK_INT_LIT = 0, PK_FLT_LIT = 1, PK_INT_COL = 2, PK_FLT_COL = 3, PK_IS_NULL = 4,
  PK_NOT_NULL = 5, PK_IN_SET = 6, PK_BITMAP = 7, PK_TRUE = 8
};
enum CmpOp : int32_t { OP_EQ = 0, OP_NE = 1, OP_LT = 2, OP_LE = 3, OP_GT = 4, OP_GE = 5 };
enum AggKind : int32_t { AK_SUM = 0, AK_COUNT = 1, AK_MIN = 2, AK_MAX = 3, AK_COUNT_STAR = 4 };

struct Pred {
  int32_t kind;
  int32_t op;
  int32_t col;
  int32_t col2;
  int32_t group;
  int32_t set_len;
  int64_t ilit;
  double flit;
  const int64_t* set;  // sorted int64 values (IN_SET) or 64-bit words (BITMAP)
};

struct AggSpec {
  int32_t kind;
  int32_t nterms;
  int32_t col[HS_MAX_TERMS];
  int32_t pad;
  double alpha[HS_MAX_TERMS];
  double beta[HS_MAX_TERMS];
};

template <typename T>
__device__ __forceinline__ bool hs_cmp(T a, T b, int op) {
  switch (op) {
    case OP_EQ: return a == b;
    case OP_NE: return a != b;
    case OP_LT: return a < b;
    case OP_LE: return a <= b;
    case OP_GT: return a > b;
    default: return a >= b;
  }
}

// Resolve a column slot to (desc,row): slots >= side_split refer to the second (right) row.
struct RowRef {
  int64_t r0;
  int64_t r1;
};

__device__ __forceinline__ bool hs_eval_pred(const Pred& p, const ColDesc* cols, int side_split,
                                             RowRef rr) {
  const int64_t row = p.col >= side_split ? rr.r1 : rr.r0;
  const ColDesc& c = cols[p.col];
  switch (p.kind) {
    case PK_TRUE: return true;
    case PK_IS_NULL: return !col_valid(c, row);
    case PK_NOT_NULL: return col_valid(c, row);
    default: break;
  }
  if (!col_valid(c, row)) return false;
  switch (p.kind) {
    case PK_INT_LIT: return hs_cmp<int64_t>(load_i64(c, row), p.ilit, p.op);
    case PK_FLT_LIT: return hs_cmp<double>(load_f64(c, row), p.flit, p.op);
    case PK_INT_COL:
    case PK_FLT_COL: {
      const int64_t row2 = p.col2 >= side_split ? rr.r1 : rr.r0;
      const ColDesc& c2 = cols[p.col2];
      if (!col_valid(c2, row2)) return false;
      if (p.kind == PK_INT_COL) return hs_cmp<int64_t>(load_i64(c, row), load_i64(c2, row2), p.op);
      return hs_cmp<double>(load_f64(c, row), load_f64(c2, row2), p.op);
    }
    case PK_IN_SET: {
      const int64_t v = load_i64(c, row);
      int lo = 0, hi = p.set_len;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (p.set[mid] < v) lo = mid + 1; else hi = mid;
      }
      const bool found = lo < p.set_len && p.set[lo] == v;
      return p.op == OP_EQ ? found : !found;
    }
    case PK_BITMAP: {
      const int64_t v = load_i64(c, row) - p.ilit;   // bit (value - base)
      bool found = false;
      if (v >= 0 && v < (int64_t)p.set_len * 64)
        found = (((const uint64_t*)p.set)[v >> 6] >> (v & 63)) & 1ull;
      return p.op == OP_EQ ? found : !found;
    }
    default: return false;
  }
}

// CNF evaluation over preds [begin, end) (sorted by group).
__device__ __forceinline__ bool hs_eval_cnf(const Pred* preds, int begin, int end,
                                            const ColDesc* cols, int side_split, RowRef rr) {
  if (begin >= end) return true;
  bool result = true;
  int cur = preds[begin].group;
  bool gval = false;
  for (int i = begin; i < end; ++i) {
    const Pred& p = preds[i];
    if (p.group != cur) {
      result = result && gval;
      cur = p.group;
      gval = false;
    }
    if (!gval) gval = hs_eval_pred(p, cols, side_split, rr);
  }
  return result && gval;
}

// Value of an aggregate input for one row; returns false when an input is null.
__device__ __forceinline__ bool hs_agg_value(const AggSpec& a, const ColDesc* cols,
                                             int side_split, RowRef rr, double& v) {
  v = 1.0;
  for (int t = 0; t < a.nterms; ++t) {
    const int slot = a.col[t];
    const int64_t row = slot >= side_split ? rr.r1 : rr.r0;
    if (!col_valid(cols[slot], row)) return false;
    v *= a.alpha[t] + a.beta[t] * load_f64(cols[slot], row);
  }
  return true;
}

__device__ __forceinline__ void hs_lds_atomic_min(double* addr, double v) {
  unsigned long long* a = (unsigned long long*)addr;
  unsigned long long old = *a, assumed;
  do {
    assumed = old;
    if (__longlong_as_double((long long)assumed) <= v) break;
    old = atomicCAS(a, assumed, (unsigned long long)__double_as_longlong(v));
  } while (assumed != old);
}

__device__ __forceinline__ void hs_lds_atomic_max(double* addr, double v) {
  unsigned long long* a = (unsigned long long*)addr;
  unsigned long long old = *a, assumed;
  do {
    assumed = old;
    if (__longlong_as_double((long long)assumed) >= v) break;
    old = atomicCAS(a, assumed, (unsigned long long)__double_as_longlong(v));
  } while (assumed != old);
}

// ------------------------------------------------------------------------------------------------
// Block accumulator shared by the scan and join aggregate kernels.
//
// Global aggregates accumulate in registers (no atomics), one value per aggregate whose meaning
// follows its kind (sum / min / max) plus a 32-bit valid-row count: 3 VGPRs per aggregate instead
// of a full (sum, min, max, count) quad, which is what keeps the fused kernels at >= 4 waves/SIMD.
// Grouped aggregates are first reduced across the wave per distinct group (ballot / readfirstlane
// peeling, so a wave with k distinct groups issues k LDS atomics instead of 64) — low-cardinality
// GROUP BYs no longer serialize on one LDS address.
// ------------------------------------------------------------------------------------------------
struct AggAcc {
  double v[HS_MAX_AGGS];
  uint32_t c[HS_MAX_AGGS];
};

__device__ __forceinline__ double agg_identity(int kind) {
  return kind == AK_MIN ? __builtin_inf() : (kind == AK_MAX ? -__builtin_inf() : 0.0);
}

__device__ __forceinline__ void acc_init(AggAcc& acc, const AggSpec* aggs, int A) {
#pragma unroll
  for (int a = 0; a < HS_MAX_AGGS; ++a) {
    acc.v[a] = a < A ? agg_identity(aggs[a].kind) : 0.0;
    acc.c[a] = 0u;
  }
}

__device__ __forceinline__ void acc_add(AggAcc& acc, int a, int kind, double x) {
  if (kind == AK_MIN) acc.v[a] = fmin(acc.v[a], x);
  else if (kind == AK_MAX) acc.v[a] = fmax(acc.v[a], x);
  else acc.v[a] += x;
  acc.c[a] += 1u;
}

struct GroupLds {
  double* sum;
  double* mn;
  double* mx;
  unsigned long long* cnt;
};

__device__ __forceinline__ GroupLds group_lds(double* base, int GA) {
  return GroupLds{base, base + GA, base + 2 * GA, (unsigned long long*)(base + 3 * GA)};
}

__device__ __forceinline__ void group_lds_init(GroupLds g, int GA, int nthreads) {
  for (int i = threadIdx.x; i < GA; i += nthreads) {
    g.sum[i] = 0.0;
    g.mn[i] = __builtin_inf();
    g.mx[i] = -__builtin_inf();
    g.cnt[i] = 0ull;
  }
}

// Write this block's partials: global -> [blockIdx][A]; grouped -> [blockIdx][G*A].
template <bool GROUPED, int NT>
__device__ __forceinline__ void acc_flush(const AggAcc& acc, const AggSpec* aggs, int A, int GA,
                                          GroupLds gl, double* psum, int64_t* pcnt, double* pmin,
                                          double* pmax) {
  if (GROUPED) {
    __syncthreads();
    for (int i = threadIdx.x; i < GA; i += NT) {
      const int64_t o = (int64_t)blockIdx.x * GA + i;
      psum[o] = gl.sum[i];
      pcnt[o] = (int64_t)gl.cnt[i];
      pmin[o] = gl.mn[i];
      pmax[o] = gl.mx[i];
    }
    return;
  }
  __shared__ double r_v[NT / 64][HS_MAX_AGGS];
  __shared__ int64_t r_c[NT / 64][HS_MAX_AGGS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < HS_MAX_AGGS; ++a) {
    if (a >= A) break;
    const int kind = aggs[a].kind;
    double wv;
    if (kind == AK_MIN) wv = hs_wave_min(acc.v[a]);
    else if (kind == AK_MAX) wv = hs_wave_max(acc.v[a]);
    else wv = hs_wave_sum(acc.v[a]);
    const int64_t wc = hs_wave_sum((int64_t)acc.c[a]);
    if (lane == 0) {
      r_v[w][a] = wv;
      r_c[w][a] = wc;
    }
  }
  __syncthreads();
  if (threadIdx.x < A) {
    const int a = threadIdx.x;
    const int kind = aggs[a].kind;
    double tv = agg_identity(kind);
    int64_t tc = 0;
    for (int ww = 0; ww < NT / 64; ++ww) {
      const double x = r_v[ww][a];
      tv = kind == AK_MIN ? fmin(tv, x) : (kind == AK_MAX ? fmax(tv, x) : tv + x);
      tc += r_c[ww][a];
    }
    const int64_t o = (int64_t)blockIdx.x * A + a;
    psum[o] = (kind == AK_MIN || kind == AK_MAX) ? 0.0 : tv;
    pcnt[o] = tc;
    pmin[o] = kind == AK_MIN ? tv : __builtin_inf();
    pmax[o] = kind == AK_MAX ? tv : -__builtin_inf();
  }
}
