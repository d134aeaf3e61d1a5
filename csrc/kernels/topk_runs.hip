// Run top-K threshold (exec/hash_agg.py TopKPlan, generated walk exec/jit_runs.py): every
// wavefront of the key-run walk leaves its best K entries in K fixed slots (keys, unsigned
// smallest-first order images, per-aggregate sums / counts), its K-th best value (WTH) and the
// largest value it dropped (DMX), both as order-preserving signed 64-bit images.  One small
// kernel reduces those over wavefronts, with no atomics in the walk itself:
//
//   hs_topk_runs_threshold: ctl[0] = max WTH, ctl[2] = max DMX - every value the slots do not
//                           hold is at most max(ctl[0], ctl[2]).
//
//   hs_topk_runs_images:    smallest-first images of the slots and the table's split keys, one
//                           array, so hash_agg.hip's radix select (hs_topk_select) picks the
//                           top k of both at once;
//   hs_topk_runs_gather:    the selected candidates and the bounds packed into one block (one
//                           copy to the host); the host checks the bound against the k-th
//                           best value and finishes the exact sort;
//   hs_topk_runs_fd:        the right columns of the candidates' keys (functional-dependency
//                           grouping), into the same block.
//
// C ABI, launched by the Python executor on the query stream.
#include <hip/hip_runtime.h>

#include <climits>

#include "hs_common.h"
#include <cstdint>

namespace {

constexpr int kBlock = 256;

__device__ __forceinline__ long long wave_max(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const long long u = __shfl_xor(v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}

__global__ __launch_bounds__(kBlock) void topk_runs_threshold_kernel(
    const long long* __restrict__ wth, const long long* __restrict__ dmx, long long n,
    long long* __restrict__ ctl) {
  long long a = LLONG_MIN, b = LLONG_MIN;
  const long long stride = (long long)gridDim.x * kBlock;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    a = wth[i] > a ? wth[i] : a;
    b = dmx[i] > b ? dmx[i] : b;
  }
  a = wave_max(a);
  b = wave_max(b);
  if ((threadIdx.x & 63) == 0) {
    atomicMax(&ctl[0], a);
    atomicMax(&ctl[2], b);
  }
}

// Order-preserving image of a double (NaN last), as hash_agg.hip's top-k images.
__device__ __forceinline__ unsigned long long uimg(double d) {
  if (d != d) return ~0ull - 1ull;
  d = d == 0.0 ? 0.0 : d;
  const unsigned long long b = (unsigned long long)__double_as_longlong(d);
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

// Smallest-first images of every candidate: the n_slots slots (empty ones, image pattern
// `empty`, last), then the table's dense groups (count gtotal[0]; rows past it last).  The order
// value is aggregate `agg`'s sum or (src_count) count; table groups read their count at
// cnt_slot (< 0: none, every group non-empty) and a zero count makes a sum NULL (first when
// ascending, last when descending, as Spark orders).
__global__ __launch_bounds__(kBlock) void topk_runs_images_kernel(
    const long long* __restrict__ vimg, const double* __restrict__ ssum,
    const long long* __restrict__ scnt, long long scap, unsigned long long empty,
    const double* __restrict__ gsum, const long long* __restrict__ gcnt,
    const long long* __restrict__ gtotal, long long gcap, int agg, int cnt_slot, int src_count,
    int desc, unsigned long long* __restrict__ img) {
  const long long n = scap + gcap;
  const long long G = gtotal[0];
  const long long stride = (long long)gridDim.x * kBlock;
  for (long long i = (long long)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    unsigned long long o = ~0ull;
    if (i < scap) {
      if ((unsigned long long)vimg[i] != empty) {
        const long long ai = (long long)agg * scap + i;
        const double x = src_count ? (double)scnt[ai] : ssum[ai];
        o = desc ? ~uimg(x) : uimg(x);
      }
    } else if (i - scap < G) {
      const long long j = i - scap;
      const long long c = cnt_slot >= 0 ? gcnt[(long long)cnt_slot * gcap + j] : 1;
      if (!src_count && c == 0) {
        o = desc ? ~0ull : 0ull;
      } else {
        const double x = src_count ? (double)c : gsum[(long long)agg * gcap + j];
        o = desc ? ~uimg(x) : uimg(x);
      }
    }
    img[i] = o;
  }
}

// The selected candidates (sel[0 .. *count), slot index or scap + table row) packed into one
// int64 block for a single copy to the host:
//   [0] candidate count, [1] ctl[0], [2] ctl[2], [3] table groups, [4] table overflow flag,
//   [8 + j] key, [8 + OUT + j] flag (bit 0: NULL key, bit 1: empty slot, bit 2: table),
//   [8 + (2 + a) OUT + j] sum bits of aggregate a, [8 + (2 + NA + a) OUT + j] its count.
__global__ __launch_bounds__(kBlock) void topk_runs_gather_kernel(
    const unsigned* __restrict__ sel, const unsigned long long* __restrict__ count, int OUT,
    const unsigned long long* __restrict__ skeys, const long long* __restrict__ vimg,
    const double* __restrict__ ssum, const long long* __restrict__ scnt, long long scap,
    unsigned long long empty, const unsigned long long* __restrict__ gkeys,
    const unsigned char* __restrict__ gnull, const double* __restrict__ gsum,
    const long long* __restrict__ gcnt, long long gcap, const long long* __restrict__ gtotal,
    const long long* __restrict__ ctl, int NA, long long* __restrict__ out) {
  const long long nsel = (long long)*count;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = nsel;
    out[1] = ctl[0];
    out[2] = ctl[2];
    out[3] = gtotal[0];
    out[4] = gtotal[1];
  }
  const long long m = nsel < OUT ? nsel : OUT;
  for (long long j = (long long)blockIdx.x * kBlock + threadIdx.x; j < m;
       j += (long long)gridDim.x * kBlock) {
    const long long s = sel[j];
    long long key, flag;
    if (s < scap) {
      key = (long long)skeys[s];
      flag = (unsigned long long)vimg[s] == empty ? 2 : 0;
      for (int a = 0; a < NA; ++a) {
        out[8 + (long long)(2 + a) * OUT + j] = __double_as_longlong(ssum[(long long)a * scap + s]);
        out[8 + (long long)(2 + NA + a) * OUT + j] = scnt[(long long)a * scap + s];
      }
    } else {
      const long long t = s - scap;
      key = (long long)gkeys[t];
      flag = 4 | (gnull[t] ? 1 : 0);
      for (int a = 0; a < NA; ++a) {
        out[8 + (long long)(2 + a) * OUT + j] = __double_as_longlong(gsum[(long long)a * gcap + t]);
        out[8 + (long long)(2 + NA + a) * OUT + j] = gcnt[(long long)a * gcap + t];
      }
    }
    out[8 + j] = key;
    out[8 + OUT + j] = flag;
  }
}

// Functional-dependency lookup of the selected candidates (GROUP BY key, right columns over a
// unique right key, exec/gpu.py _fd_grouping): candidate j's group key (out[8 + j]; packed:
// ((k >> shift) & mask) + lo, raw: k) is the right key value v; its bucket is Spark's
// pmod(murmur3(v, 42), nb) and a binary search of the bucket's sorted key rows finds its row.
// fdo: [j] row (-1: none), [(1 + a) OUT + j] column a's value (64-bit: integer or double bits),
// [(1 + NF + a) OUT + j] its validity.
struct FdCols {
  ColDesc c[4];
  int n;
  int pad;
};

__global__ __launch_bounds__(kBlock) void topk_runs_fd_kernel(
    const long long* __restrict__ out, int OUT, int raw, long long lo, int shift,
    unsigned long long mask, ColDesc key, const long long* __restrict__ off, int nb, FdCols cols,
    long long* __restrict__ fdo) {
  const long long nsel = out[0];
  const long long m = nsel < OUT ? nsel : OUT;
  const int NF = cols.n;
  for (long long j = (long long)blockIdx.x * kBlock + threadIdx.x; j < m;
       j += (long long)gridDim.x * kBlock) {
    const unsigned long long k = (unsigned long long)out[8 + j];
    const long long v = raw ? (long long)k : (long long)((k >> shift) & mask) + lo;
    const uint32_t h = (key.type == HS_I64 || key.type == HS_U64)
                           ? hs_hash_long((uint64_t)v, 42u)
                           : hs_hash_int((uint32_t)(int32_t)v, 42u);
    int b = (int)((int32_t)h % nb);
    if (b < 0) b += nb;
    long long a0 = off[b], a1 = off[b + 1];
    while (a0 < a1) {
      const long long mid = (a0 + a1) >> 1;
      if (load_i64(key, mid) < v) a0 = mid + 1; else a1 = mid;
    }
    const long long row = (a0 < off[b + 1] && load_i64(key, a0) == v) ? a0 : -1;
    fdo[j] = row;
    for (int a = 0; a < NF; ++a) {
      const ColDesc& c = cols.c[a];
      long long x = 0, ok = 0;
      if (row >= 0) {
        x = (c.type == HS_F32 || c.type == HS_F64) ? __double_as_longlong(load_f64(c, row))
                                                    : load_i64(c, row);
        ok = col_valid(c, row) ? 1 : 0;
      }
      fdo[(long long)(1 + a) * OUT + j] = x;
      fdo[(long long)(1 + NF + a) * OUT + j] = ok;
    }
  }
}

int grid_for(long long n) {
  long long g = (n + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return (int)g;
}

}  // namespace

extern "C" {

int hs_topk_runs_threshold(const long long* wth, const long long* dmx, long long n, long long* ctl,
                           void* stream) {
  if (n <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(topk_runs_threshold_kernel, dim3(grid_for(n)), dim3(kBlock), 0,
                     (hipStream_t)stream, wth, dmx, n, ctl);
  return (int)hipGetLastError();
}

int hs_topk_runs_images(const long long* vimg, const double* ssum, const long long* scnt,
                        long long scap, unsigned long long empty, const double* gsum,
                        const long long* gcnt, const long long* gtotal, long long gcap, int agg,
                        int cnt_slot, int src_count, int desc, unsigned long long* img,
                        void* stream) {
  if (scap + gcap <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(topk_runs_images_kernel, dim3(grid_for(scap + gcap)), dim3(kBlock), 0,
                     (hipStream_t)stream, vimg, ssum, scnt, scap, empty, gsum, gcnt, gtotal, gcap,
                     agg, cnt_slot, src_count, desc, img);
  return (int)hipGetLastError();
}

int hs_topk_runs_gather(const unsigned* sel, const unsigned long long* count, int OUT,
                        const unsigned long long* skeys, const long long* vimg, const double* ssum,
                        const long long* scnt, long long scap, unsigned long long empty,
                        const unsigned long long* gkeys, const unsigned char* gnull,
                        const double* gsum, const long long* gcnt, long long gcap,
                        const long long* gtotal, const long long* ctl, int NA, long long* out,
                        void* stream) {
  if (OUT <= 0) return -1;
  (void)hipGetLastError();
  hipLaunchKernelGGL(topk_runs_gather_kernel, dim3(grid_for(OUT)), dim3(kBlock), 0,
                     (hipStream_t)stream, sel, count, OUT, skeys, vimg, ssum, scnt, scap, empty,
                     gkeys, gnull, gsum, gcnt, gcap, gtotal, ctl, NA, out);
  return (int)hipGetLastError();
}

int hs_topk_runs_fd(const long long* out, int OUT, int raw, long long lo, int shift,
                    unsigned long long mask, const ColDesc* key, const long long* off, int nb,
                    const ColDesc* cols, int ncols, long long* fdo, void* stream) {
  if (OUT <= 0 || ncols < 0 || ncols > 4 || nb <= 0) return -1;
  FdCols fc{};
  for (int a = 0; a < ncols; ++a) fc.c[a] = cols[a];
  fc.n = ncols;
  (void)hipGetLastError();
  hipLaunchKernelGGL(topk_runs_fd_kernel, dim3(grid_for(OUT)), dim3(kBlock), 0,
                     (hipStream_t)stream, out, OUT, raw, lo, shift, mask, *key, off, nb, fc, fdo);
  return (int)hipGetLastError();
}

}  // extern "C"
