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
      const int64_t v = load_i64(c, row);
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
// Global aggregates accumulate in registers (no atomics).  Grouped aggregates are first reduced
// across the wave per distinct group (ballot / readfirstlane peeling, so a wave with k distinct
// groups issues k LDS atomics instead of 64) — low-cardinality GROUP BYs no longer serialize on
// one LDS address.  Callers must invoke acc_row with the whole wave converged.
// ------------------------------------------------------------------------------------------------
struct AggAcc {
  double s[HS_MAX_AGGS], mn[HS_MAX_AGGS], mx[HS_MAX_AGGS];
  int64_t c[HS_MAX_AGGS];
};

__device__ __forceinline__ void acc_init(AggAcc& acc) {
#pragma unroll
  for (int a = 0; a < HS_MAX_AGGS; ++a) {
    acc.s[a] = 0.0;
    acc.c[a] = 0;
    acc.mn[a] = __builtin_inf();
    acc.mx[a] = -__builtin_inf();
  }
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

template <bool GROUPED>
__device__ __forceinline__ void acc_row(AggAcc& acc, const AggSpec* aggs, int A, bool pass, int g,
                                        const ColDesc* cols, int split, RowRef rr, GroupLds gl) {
  double v[HS_MAX_AGGS];
  bool ok[HS_MAX_AGGS];
#pragma unroll
  for (int a = 0; a < HS_MAX_AGGS; ++a) {
    v[a] = 0.0;
    ok[a] = false;
    if (a < A && pass) {
      const AggSpec& ag = aggs[a];
      ok[a] = ag.kind == AK_COUNT_STAR ? true : hs_agg_value(ag, cols, split, rr, v[a]);
    }
  }
  if (!GROUPED) {
#pragma unroll
    for (int a = 0; a < HS_MAX_AGGS; ++a) {
      if (a < A && ok[a]) {
        acc.s[a] += v[a];
        acc.c[a] += 1;
        acc.mn[a] = fmin(acc.mn[a], v[a]);
        acc.mx[a] = fmax(acc.mx[a], v[a]);
      }
    }
    return;
  }
  const int lane = threadIdx.x & 63;
  bool todo = pass;
  while (true) {
    const uint64_t act = __ballot(todo);
    if (act == 0ull) break;
    const int leader = __ffsll((unsigned long long)act) - 1;
    const int g0 = __shfl(g, leader, 64);
    const bool mine = todo && g == g0;
#pragma unroll
    for (int a = 0; a < HS_MAX_AGGS; ++a) {
      if (a >= A) break;
      const bool m = mine && ok[a];
      const uint64_t cm = __ballot(m);
      if (cm == 0ull) continue;
      const double sv = hs_wave_sum(m ? v[a] : 0.0);
      const double mnv = hs_wave_min(m ? v[a] : __builtin_inf());
      const double mxv = hs_wave_max(m ? v[a] : -__builtin_inf());
      if (lane == leader) {
        const int slot = g0 * A + a;
        const int kind = aggs[a].kind;
        if (kind == AK_SUM) atomicAdd(&gl.sum[slot], sv);
        else if (kind == AK_MIN) hs_lds_atomic_min(&gl.mn[slot], mnv);
        else if (kind == AK_MAX) hs_lds_atomic_max(&gl.mx[slot], mxv);
        atomicAdd(&gl.cnt[slot], (unsigned long long)__popcll(cm));
      }
    }
    todo = todo && !mine;
  }
}

// Write this block's partials: global -> [blockIdx][A]; grouped -> [blockIdx][G*A].
template <bool GROUPED, int NT>
__device__ __forceinline__ void acc_flush(const AggAcc& acc, int A, int GA, GroupLds gl,
                                          double* psum, int64_t* pcnt, double* pmin,
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
  __shared__ double r_s[NT / 64][HS_MAX_AGGS], r_mn[NT / 64][HS_MAX_AGGS], r_mx[NT / 64][HS_MAX_AGGS];
  __shared__ int64_t r_c[NT / 64][HS_MAX_AGGS];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int a = 0; a < HS_MAX_AGGS; ++a) {
    if (a >= A) break;
    const double ws = hs_wave_sum(acc.s[a]);
    const int64_t wc = hs_wave_sum(acc.c[a]);
    const double wmn = hs_wave_min(acc.mn[a]);
    const double wmx = hs_wave_max(acc.mx[a]);
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
    for (int ww = 0; ww < NT / 64; ++ww) {
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
