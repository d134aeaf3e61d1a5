// Vectorised (row-batch) evaluation of the predicate / aggregate templates.
//
// A lane owns NI rows of a tile at once and walks the CNF *predicate-major*: for each predicate
// the column is loaded for all NI rows before any compare, so every lane keeps NI independent
// HBM loads in flight instead of one dependent chain per row (the interpreter's per-row
// short-circuit made each row a serial load->compare->load chain).  Column types, predicate kinds
// and ops are wave-uniform, so every switch below is a scalar branch taken once per batch.
// Rows already known false are masked off, so their loads are never issued.
#pragma once
#include "hs_scan.h"

template <int NI>
__device__ __forceinline__ void vvalid(const ColDesc& c, const int64_t (&row)[NI],
                                       const bool (&m)[NI], bool (&out)[NI]) {
  if (c.valid == nullptr) {
#pragma unroll
    for (int i = 0; i < NI; ++i) out[i] = m[i];
    return;
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) out[i] = m[i] && c.valid[row[i]] != 0;
}

template <int NI, typename T, typename U>
__device__ __forceinline__ void vload_as(const void* data, const int64_t (&row)[NI],
                                         const bool (&m)[NI], U (&v)[NI]) {
  const T* d = (const T*)data;
#pragma unroll
  for (int i = 0; i < NI; ++i) v[i] = m[i] ? (U)d[row[i]] : (U)0;
}

template <int NI>
__device__ __forceinline__ void vload_i64(const ColDesc& c, const int64_t (&row)[NI],
                                          const bool (&m)[NI], int64_t (&v)[NI]) {
  switch (c.type) {
    case HS_I32: vload_as<NI, int32_t>(c.data, row, m, v); break;
    case HS_I64: vload_as<NI, int64_t>(c.data, row, m, v); break;
    case HS_I16: vload_as<NI, int16_t>(c.data, row, m, v); break;
    case HS_I8: vload_as<NI, int8_t>(c.data, row, m, v); break;
    case HS_BOOL: vload_as<NI, uint8_t>(c.data, row, m, v); break;
    case HS_U32: vload_as<NI, uint32_t>(c.data, row, m, v); break;
    case HS_F64: vload_as<NI, double>(c.data, row, m, v); break;
    case HS_F32: vload_as<NI, float>(c.data, row, m, v); break;
    default: vload_as<NI, uint64_t>(c.data, row, m, v); break;
  }
}

template <int NI>
__device__ __forceinline__ void vload_f64(const ColDesc& c, const int64_t (&row)[NI],
                                          const bool (&m)[NI], double (&v)[NI]) {
  switch (c.type) {
    case HS_F64: vload_as<NI, double>(c.data, row, m, v); break;
    case HS_F32: vload_as<NI, float>(c.data, row, m, v); break;
    case HS_I32: vload_as<NI, int32_t>(c.data, row, m, v); break;
    case HS_I64: vload_as<NI, int64_t>(c.data, row, m, v); break;
    case HS_I16: vload_as<NI, int16_t>(c.data, row, m, v); break;
    case HS_I8: vload_as<NI, int8_t>(c.data, row, m, v); break;
    case HS_BOOL: vload_as<NI, uint8_t>(c.data, row, m, v); break;
    case HS_U32: vload_as<NI, uint32_t>(c.data, row, m, v); break;
    default: vload_as<NI, uint64_t>(c.data, row, m, v); break;
  }
}

template <int NI, typename T>
__device__ __forceinline__ void vcmp(const T (&a)[NI], const T (&b)[NI], int op, const bool (&m)[NI],
                                     bool (&out)[NI]) {
  switch (op) {
    case OP_EQ:
#pragma unroll
      for (int i = 0; i < NI; ++i) out[i] = m[i] && a[i] == b[i];
      break;
    case OP_NE:
#pragma unroll
      for (int i = 0; i < NI; ++i) out[i] = m[i] && a[i] != b[i];
      break;
    case OP_LT:
#pragma unroll
      for (int i = 0; i < NI; ++i) out[i] = m[i] && a[i] < b[i];
      break;
    case OP_LE:
#pragma unroll
      for (int i = 0; i < NI; ++i) out[i] = m[i] && a[i] <= b[i];
      break;
    case OP_GT:
#pragma unroll
      for (int i = 0; i < NI; ++i) out[i] = m[i] && a[i] > b[i];
      break;
    default:
#pragma unroll
      for (int i = 0; i < NI; ++i) out[i] = m[i] && a[i] >= b[i];
      break;
  }
}

template <int NI>
__device__ __forceinline__ void vsel_rows(bool second, const int64_t (&r0)[NI],
                                          const int64_t (&r1)[NI], int64_t (&row)[NI]) {
#pragma unroll
  for (int i = 0; i < NI; ++i) row[i] = second ? r1[i] : r0[i];
}

// One predicate over the batch; rows with m[i] == false yield false and issue no loads.
template <int NI>
__device__ __forceinline__ void veval_pred(const Pred& p, const ColDesc* cols, int split,
                                           const int64_t (&r0)[NI], const int64_t (&r1)[NI],
                                           const bool (&m)[NI], bool (&out)[NI]) {
  if (p.kind == PK_TRUE) {
#pragma unroll
    for (int i = 0; i < NI; ++i) out[i] = m[i];
    return;
  }
  int64_t row[NI];
  vsel_rows(p.col >= split, r0, r1, row);
  const ColDesc& c = cols[p.col];
  bool mv[NI];
  vvalid(c, row, m, mv);
  if (p.kind == PK_IS_NULL || p.kind == PK_NOT_NULL) {
    const bool want = p.kind == PK_NOT_NULL;
#pragma unroll
    for (int i = 0; i < NI; ++i) out[i] = m[i] && (mv[i] == want);
    return;
  }
  switch (p.kind) {
    case PK_INT_LIT: {
      int64_t x[NI], l[NI];
      vload_i64(c, row, mv, x);
#pragma unroll
      for (int i = 0; i < NI; ++i) l[i] = p.ilit;
      vcmp(x, l, p.op, mv, out);
      return;
    }
    case PK_FLT_LIT: {
      double x[NI], l[NI];
      vload_f64(c, row, mv, x);
#pragma unroll
      for (int i = 0; i < NI; ++i) l[i] = p.flit;
      vcmp(x, l, p.op, mv, out);
      return;
    }
    case PK_INT_COL:
    case PK_FLT_COL: {
      int64_t row2[NI];
      vsel_rows(p.col2 >= split, r0, r1, row2);
      const ColDesc& c2 = cols[p.col2];
      bool mv2[NI];
      vvalid(c2, row2, mv, mv2);
      if (p.kind == PK_INT_COL) {
        int64_t x[NI], y[NI];
        vload_i64(c, row, mv2, x);
        vload_i64(c2, row2, mv2, y);
        vcmp(x, y, p.op, mv2, out);
      } else {
        double x[NI], y[NI];
        vload_f64(c, row, mv2, x);
        vload_f64(c2, row2, mv2, y);
        vcmp(x, y, p.op, mv2, out);
      }
      return;
    }
    case PK_IN_SET: {
      int64_t x[NI];
      vload_i64(c, row, mv, x);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        int lo = 0, hi = p.set_len;
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (p.set[mid] < x[i]) lo = mid + 1; else hi = mid;
        }
        const bool found = lo < p.set_len && p.set[lo] == x[i];
        out[i] = mv[i] && (p.op == OP_EQ ? found : !found);
      }
      return;
    }
    case PK_BITMAP: {
      int64_t x[NI];
      vload_i64(c, row, mv, x);
      const uint64_t* words = (const uint64_t*)p.set;
      const int64_t nbits = (int64_t)p.set_len * 64;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const int64_t v = x[i] - p.ilit;     // bit (value - base), as hs_scan.h
        bool found = false;
        if (mv[i] && v >= 0 && v < nbits) found = (words[v >> 6] >> (v & 63)) & 1ull;
        out[i] = mv[i] && (p.op == OP_EQ ? found : !found);
      }
      return;
    }
    default:
#pragma unroll
      for (int i = 0; i < NI; ++i) out[i] = false;
      return;
  }
}

// CNF over preds [begin, end) (sorted by group): OR within a group, AND across groups.
template <int NI>
__device__ __forceinline__ void veval_cnf(const Pred* preds, int begin, int end,
                                          const ColDesc* cols, int split, const int64_t (&r0)[NI],
                                          const int64_t (&r1)[NI], const bool (&act)[NI],
                                          bool (&res)[NI]) {
#pragma unroll
  for (int i = 0; i < NI; ++i) res[i] = act[i];
  if (begin >= end) return;
  bool g[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) g[i] = false;
  int cur = preds[begin].group;
  for (int k = begin; k < end; ++k) {
    const Pred& p = preds[k];
    if (p.group != cur) {
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        res[i] = res[i] && g[i];
        g[i] = false;
      }
      cur = p.group;
    }
    bool need[NI], o[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) need[i] = res[i] && !g[i];
    veval_pred(p, cols, split, r0, r1, need, o);
#pragma unroll
    for (int i = 0; i < NI; ++i) g[i] = g[i] || o[i];
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) res[i] = res[i] && g[i];
}

// Aggregate input over the batch: v = prod_t (alpha_t + beta_t * col_t); ok = all inputs valid.
template <int NI>
__device__ __forceinline__ void vagg_value(const AggSpec& a, const ColDesc* cols, int split,
                                           const int64_t (&r0)[NI], const int64_t (&r1)[NI],
                                           const bool (&m)[NI], double (&v)[NI], bool (&ok)[NI]) {
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    v[i] = 1.0;
    ok[i] = m[i];
  }
  if (a.kind == AK_COUNT_STAR) return;
  for (int t = 0; t < a.nterms; ++t) {
    const int slot = a.col[t];
    int64_t row[NI];
    vsel_rows(slot >= split, r0, r1, row);
    bool mv[NI];
    vvalid(cols[slot], row, ok, mv);
    double x[NI];
    vload_f64(cols[slot], row, mv, x);
    const double al = a.alpha[t], be = a.beta[t];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      v[i] *= al + be * x[i];
      ok[i] = mv[i];
    }
  }
}

// Group index of each row (group column may sit on either side); clears pass when the key is
// null or outside the dense domain.
template <int NI>
__device__ __forceinline__ void vgroup(const ColDesc* cols, int gcol, int split, int64_t base,
                                       int G, const int64_t (&r0)[NI], const int64_t (&r1)[NI],
                                       bool (&pass)[NI], int (&g)[NI]) {
  int64_t row[NI];
  vsel_rows(gcol >= split, r0, r1, row);
  bool mv[NI];
  vvalid(cols[gcol], row, pass, mv);
  int64_t x[NI];
  vload_i64(cols[gcol], row, mv, x);
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int64_t gi = x[i] - base;
    pass[i] = mv[i] && gi >= 0 && gi < G;
    g[i] = pass[i] ? (int)gi : 0;
  }
}

// Accumulate the whole batch: aggregate-major so only NI values are live at a time.  The grouped
// path reuses the wave-peeled LDS atomics per (row slot, aggregate); the wave stays converged
// because every loop bound here is wave-uniform.
template <bool GROUPED, int NI>
__device__ __forceinline__ void vaccumulate(AggAcc& acc, const AggSpec* aggs, int A,
                                            const ColDesc* cols, int split, const int64_t (&r0)[NI],
                                            const int64_t (&r1)[NI], const bool (&pass)[NI],
                                            const int (&g)[NI], GroupLds gl) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int a = 0; a < HS_MAX_AGGS; ++a) {
    if (a >= A) break;
    double v[NI];
    bool ok[NI];
    vagg_value(aggs[a], cols, split, r0, r1, pass, v, ok);
    const int kind = aggs[a].kind;
    if (!GROUPED) {
#pragma unroll
      for (int i = 0; i < NI; ++i)
        if (ok[i]) acc_add(acc, a, kind, v[i]);
      continue;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      bool todo = ok[i];
      while (true) {
        const uint64_t act = __ballot(todo);
        if (act == 0ull) break;
        const int leader = __ffsll((unsigned long long)act) - 1;
        const int g0 = __shfl(g[i], leader, 64);
        const bool mine = todo && g[i] == g0;
        const double sv = hs_wave_sum(mine ? v[i] : 0.0);
        double mnv = 0.0, mxv = 0.0;
        if (kind == AK_MIN) mnv = hs_wave_min(mine ? v[i] : __builtin_inf());
        if (kind == AK_MAX) mxv = hs_wave_max(mine ? v[i] : -__builtin_inf());
        const uint64_t cm = __ballot(mine);
        if (lane == leader) {
          const int slot = g0 * A + a;
          if (kind == AK_SUM) atomicAdd(&gl.sum[slot], sv);
          else if (kind == AK_MIN) hs_lds_atomic_min(&gl.mn[slot], mnv);
          else if (kind == AK_MAX) hs_lds_atomic_max(&gl.mx[slot], mxv);
          atomicAdd(&gl.cnt[slot], (unsigned long long)__popcll(cm));
        }
        todo = todo && !mine;
      }
    }
  }
}

// Contiguous tile chunk of this block: [t0, t1).  Contiguous chunks stream each block through
// consecutive rows and need one range lookup per block instead of one per tile.
__device__ __forceinline__ void block_tile_chunk(int64_t ntiles, int64_t& t0, int64_t& t1) {
  const int64_t per = (ntiles + gridDim.x - 1) / gridDim.x;
  t0 = (int64_t)blockIdx.x * per;
  t1 = min(ntiles, t0 + per);
}

// Largest r with tile_prefix[r] <= t.
__device__ __forceinline__ int tile_range_of(const int64_t* tile_prefix, int R, int64_t t) {
  int lo = 0, hi = R;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (tile_prefix[mid] <= t) lo = mid; else hi = mid;
  }
  return lo;
}
