// Run-length form of a bucket-sorted 32-bit key column (exec/encoding.py RunCompact) and the
// per-tile run windows the run-keyed merge join reads (exec/jit.py gen_merge_join_agg, MJ_RUNS).
//
// A covering index is sorted by its indexed columns inside every bucket, so its
// leading key column is a sequence of runs of equal values: TPC-H l_orderkey has 1-7 rows per
// key.  The merge join only needs, per left row, *which run* it belongs to and, per run, its
// key.  Stored as
//   gmask[g]   64-bit mask of the rows of 64-row group g that start a run (row 0 always does),
//   gruns[g]   index of the run holding row 64 * g,
//   runkeys[r] key code of run r,
// that is 12 bytes per 64 rows plus 4 bytes per run instead of 4 bytes per row: for l_orderkey
// (4 rows per run) the key stream drops from 4 to ~1.2 bytes per row.  run_of(row) =
// gruns[row >> 6] + popcount(gmask[row >> 6] & bits 1 .. row & 63).
//
// Build: two passes of one wavefront per 64-row group (ballot of "differs from the previous
// row"), with the exclusive scan of the per-group run counts between them (torch.cumsum).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__device__ __forceinline__ int64_t run_of(const uint64_t* __restrict__ gmask,
                                          const int32_t* __restrict__ gruns, int64_t row) {
  const int64_t g = row >> 6;
  // bits 1 .. (row & 63) of the group mask: (2 << i) - 2 (i = 63 wraps to all bits but bit 0)
  const uint64_t below = (2ull << (unsigned)(row & 63)) - 2ull;
  return (int64_t)gruns[g] + __popcll(gmask[g] & below);
}

__global__ __launch_bounds__(256) void hs_runs_mask_kernel(const int32_t* __restrict__ x,
                                                           int64_t n, uint64_t* __restrict__ gmask,
                                                           int64_t* __restrict__ gcnt) {
  const int lane = threadIdx.x & 63;
  const int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (g >= ((n + 63) >> 6)) return;   // wavefront-uniform
  const int64_t i = (g << 6) + lane;
  const bool s = i < n && (i == 0 || x[i] != x[i - 1]);
  const uint64_t m = __ballot(s);
  if (lane == 0) {
    gmask[g] = m;
    gcnt[g] = __popcll(m);
  }
}

__global__ __launch_bounds__(256) void hs_runs_fill_kernel(const int32_t* __restrict__ x,
                                                           int64_t n,
                                                           const uint64_t* __restrict__ gmask,
                                                           const int64_t* __restrict__ gexcl,
                                                           int32_t* __restrict__ gruns,
                                                           int32_t* __restrict__ runkeys) {
  const int lane = threadIdx.x & 63;
  const int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (g >= ((n + 63) >> 6)) return;
  const uint64_t m = gmask[g];
  const int64_t e = gexcl[g];
  if (lane == 0) gruns[g] = (int32_t)(e + (int64_t)(m & 1ull) - 1);
  const int64_t i = (g << 6) + lane;
  if (i < n && ((m >> lane) & 1ull))
    runkeys[e + __popcll(m & ((1ull << lane) - 1ull))] = x[i];
}

// Per tile of a merge join (spans from hs_join_spans_sampled: row0, rows, rs, re): the first
// run of its rows and the number of runs they touch.
__global__ __launch_bounds__(256) void hs_tile_runs_kernel(const int64_t* __restrict__ tile_prefix,
                                                           int R, const int64_t* __restrict__ spans,
                                                           const uint64_t* __restrict__ gmask,
                                                           const int32_t* __restrict__ gruns,
                                                           int32_t* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= tile_prefix[R]) return;
  const int64_t row0 = spans[4 * t], rows = spans[4 * t + 1];
  int32_t a = 0, nl = 0;
  if (rows > 0) {
    a = (int32_t)run_of(gmask, gruns, row0);
    nl = (int32_t)(run_of(gmask, gruns, row0 + rows - 1) + 1 - a);
  }
  out[2 * t] = a;
  out[2 * t + 1] = nl;
}

// Run tags (1 bit per run, exec/jit_runs.py phase 1) -> row mask (1 bit per row) over 64-row
// groups [g0, g1): bit i of out[g] = tag of the run holding row 64 g + i.  One thread per group:
// T = the tag bits of the group's runs (<= 64 runs from gruns[g]: a 3-word funnel), the change
// points c_k = T_k ^ T_{k-1} are deposited at the runs' start rows (a software bit deposit over
// the set bits of the start mask, ~rows/4 iterations) and a prefix XOR spreads each run's tag
// over its rows.  The streaming scan (phase 2) then reads 8 bytes per 64 rows, prefetched one
// tile ahead, and skips the predicate loads of rows no tagged run holds.
__global__ __launch_bounds__(256) void hs_run_rowmask_kernel(const uint64_t* __restrict__ gmask,
                                                             const int32_t* __restrict__ gruns,
                                                             const uint32_t* __restrict__ tags,
                                                             int64_t g0, int64_t g1,
                                                             uint64_t* __restrict__ out) {
  const int64_t g = g0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= g1) return;
  const uint64_t m = gmask[g] | 1ull;   // row 0 starts (or continues) the group's first run
  const int64_t r0 = gruns[g];
  const int64_t w = r0 >> 5;
  const unsigned sh = (unsigned)(r0 & 31);
  const uint64_t lo = (uint64_t)tags[w] | ((uint64_t)tags[w + 1] << 32);
  const uint64_t hi = (uint64_t)tags[w + 2];
  const uint64_t T = sh ? ((lo >> sh) | (hi << (64 - sh))) : lo;
  const uint64_t c = T ^ (T << 1);      // c_k = T_k ^ T_{k-1}, T_{-1} = 0
  uint64_t d = 0, mm = m, cc = c;
  while (mm) {                          // deposit c's low bits at m's set bits, in order
    const uint64_t low = mm & (0ull - mm);
    if (cc & 1ull) d |= low;
    cc >>= 1;
    mm ^= low;
  }
  d ^= d << 1; d ^= d << 2; d ^= d << 4; d ^= d << 8; d ^= d << 16; d ^= d << 32;  // prefix XOR
  out[g] = d;
}

// Semi-join probe over the run form: tag of run r = the build-key bitmap's bit for run r's key
// (one bitmap test per run instead of per row), 1 bit per run, stored as whole words by the
// wavefront that owns 64 consecutive runs (ballot), as exec/jit_runs.py phase 1 writes them.
// key value = code + code_off - lo is the bitmap position; codes out of [0, nbits) miss.
__global__ __launch_bounds__(256) void hs_run_bitmap_tags_kernel(const int32_t* __restrict__ runkeys,
                                                                 int64_t nruns, int64_t code_off,
                                                                 const uint64_t* __restrict__ words,
                                                                 int64_t nbits,
                                                                 uint32_t* __restrict__ tags) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  bool t = false;
  if (r < nruns) {
    const int64_t v = (int64_t)runkeys[r] + code_off;
    t = v >= 0 && v < nbits && ((words[v >> 6] >> (v & 63)) & 1ull);
  }
  const uint64_t b = __ballot(t);
  const int64_t g = r >> 6;                 // wavefront-uniform: 64 runs per wavefront
  if (lane < 2 && (g << 6) < nruns) tags[2 * g + lane] = (uint32_t)(b >> (32 * lane));
}

}  // namespace

extern "C" {

// tags: at least 2 * ceil(nruns / 64) words
int hs_run_bitmap_tags(const int32_t* runkeys, int64_t nruns, int64_t code_off,
                       const uint64_t* words, int64_t nbits, uint32_t* tags, void* stream) {
  if (nruns > 0)
    hipLaunchKernelGGL(hs_run_bitmap_tags_kernel, dim3((unsigned)((nruns + 255) / 256)),
                       dim3(256), 0, (hipStream_t)stream, runkeys, nruns, code_off, words, nbits,
                       tags);
  return (int)hipGetLastError();
}

// tags must hold 2 readable words past the last run's word (phase 1 allocates that slack)
int hs_run_rowmask(const uint64_t* gmask, const int32_t* gruns, const uint32_t* tags, int64_t g0,
                   int64_t g1, uint64_t* out, void* stream) {
  if (g1 > g0)
    hipLaunchKernelGGL(hs_run_rowmask_kernel, dim3((unsigned)((g1 - g0 + 255) / 256)), dim3(256),
                       0, (hipStream_t)stream, gmask, gruns, tags, g0, g1, out);
  return (int)hipGetLastError();
}

// Pass 1: gmask / per-group run counts of the int32 column x[0, n).
int hs_key_runs_mask(const int32_t* x, int64_t n, uint64_t* gmask, int64_t* gcnt, void* stream) {
  const int64_t ng = (n + 63) >> 6;
  if (ng > 0)
    hipLaunchKernelGGL(hs_runs_mask_kernel, dim3((unsigned)((ng + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, x, n, gmask, gcnt);
  return (int)hipGetLastError();
}

// Pass 2: gruns and runkeys from gmask and the exclusive prefix gexcl of the run counts.
int hs_key_runs_fill(const int32_t* x, int64_t n, const uint64_t* gmask, const int64_t* gexcl,
                     int32_t* gruns, int32_t* runkeys, void* stream) {
  const int64_t ng = (n + 63) >> 6;
  if (ng > 0)
    hipLaunchKernelGGL(hs_runs_fill_kernel, dim3((unsigned)((ng + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, x, n, gmask, gexcl, gruns, runkeys);
  return (int)hipGetLastError();
}

// out: 2 int32 per tile (first run, run count); max_tiles >= tile_prefix[R] sizes the grid.
int hs_tile_runs(const int64_t* tile_prefix, int R, const int64_t* spans, const uint64_t* gmask,
                 const int32_t* gruns, int64_t max_tiles, int32_t* out, void* stream) {
  if (max_tiles > 0)
    hipLaunchKernelGGL(hs_tile_runs_kernel, dim3((unsigned)((max_tiles + 255) / 256)), dim3(256),
                       0, (hipStream_t)stream, tile_prefix, R, spans, gmask, gruns, out);
  return (int)hipGetLastError();
}

}  // extern "C"
