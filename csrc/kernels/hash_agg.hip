// Grouped aggregation over a global open-addressing hash table, and device top-k.
//
// The generated scan / join kernels (hyperspace_amd/exec/jit.py, hash mode) insert one record per
// run of equal group keys: a wavefront first reduces adjacent equal keys with a segmented
// shuffle scan, then only the run's last lane probes the table (linear probing, 64-bit packed
// keys, atomicCAS on the key word) and adds its partial sums / counts with memory-side atomics.
// This file holds the table's fixed-shape kernels:
//
//   hs_hagg_init     fill a fresh table (keys = EMPTY, sums = 0, counts = 0, min = +inf, max = -inf)
//   hs_hagg_extract  occupied slots -> dense (key, null, aggregates) arrays in slot order
//                    (deterministic: per-block counts, one scan, then the writes), resetting the
//                    slots it read, so the next query reuses the table without a full memset
//   hs_hagg_merge    insert dense partial groups into a table (multi-rank combine)
//   hs_topk_*        ORDER BY <one expression> LIMIT k over the dense groups: an order-preserving
//                    u64 image per group, a 3-level radix select (12 bits per level, LDS
//                    histograms, the running prefix kept on the device), then every group whose
//                    image's top 36 bits are <= the selected prefix; the host sorts those few
//                    candidates by the full ORDER BY
//
// Layout (structure of arrays, so every pass over the table is coalesced):
//   keys[M + 2]           slot M holds the key ~0 (the EMPTY pattern itself), slot M + 1 the NULL
//                         key of an unpacked single-column key; both are addressed directly
//   sums[NA][M + 2], cnts[NA][M + 2], mins / maxs [NA][M + 2] (null when no MIN / MAX)
// Occupancy: keys[s] != EMPTY for s < M; cnts[star][s] > 0 for the two direct slots.
// Dense outputs use the same SoA form with row stride `cap` (the output capacity).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr unsigned long long kEmpty = ~0ull;
constexpr int kBlock = 256;
constexpr int kTopkBits = 12;
constexpr int kTopkBins = 1 << kTopkBits;
constexpr int kTopkLevels = 3;

__device__ __forceinline__ unsigned long long mix64(unsigned long long h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

__device__ __forceinline__ bool occupied(const unsigned long long* keys, const long long* cnts,
                                         long long M, int star, long long s) {
  return s < M ? keys[s] != kEmpty : cnts[(long long)star * (M + 2) + s] > 0;
}

__global__ __launch_bounds__(kBlock) void hagg_init_kernel(unsigned long long* keys, double* sums,
                                                           long long* cnts, double* mins,
                                                           double* maxs, long long M, int NA) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long nslot = M + 2;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < nslot * NA;
       i += stride) {
    if (i < nslot) keys[i] = kEmpty;
    sums[i] = 0.0;
    cnts[i] = 0;
    if (mins) mins[i] = __builtin_inf();
    if (maxs) maxs[i] = -__builtin_inf();
  }
}

// Block-exclusive prefix of one flag per thread (thread order); returns this thread's position
// among the block's flagged threads, and the block total through `tot`.
__device__ __forceinline__ int block_prefix(bool f, int* tot) {
  __shared__ int wt[kBlock / 64];
  const unsigned long long bm = __ballot(f);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) wt[w] = __popcll(bm);
  __syncthreads();
  int base = 0, t = 0;
  for (int k = 0; k < kBlock / 64; ++k) {
    base += k < w ? wt[k] : 0;
    t += wt[k];
  }
  *tot = t;
  return base + __popcll(bm & ((1ull << lane) - 1ull));
}

constexpr int kSlotsPerThread = 4;
constexpr int kChunk = kBlock * kSlotsPerThread;   // slots per extract block

// Per block (kChunk slots, lane-consecutive slots per step): number of occupied slots.
__global__ __launch_bounds__(kBlock) void hagg_count_kernel(
    const unsigned long long* __restrict__ keys, const long long* __restrict__ cnts, long long M,
    int star, long long* __restrict__ block_counts) {
  int c = 0;
#pragma unroll
  for (int k = 0; k < kSlotsPerThread; ++k) {
    const long long s = (long long)blockIdx.x * kChunk + k * kBlock + threadIdx.x;
    c += (s < M + 2 && occupied(keys, cnts, M, star, s)) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  __shared__ int ws[kBlock / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += ws[w];
    block_counts[blockIdx.x] = t;
  }
}

// One block: exclusive scan of nb counts in place; total[0] = sum, total[1] = *flag (the
// insert kernels' overflow flag), which is then cleared.
__global__ __launch_bounds__(1024) void hagg_scan_kernel(long long* __restrict__ v, long long nb,
                                                         long long* __restrict__ total,
                                                         long long* __restrict__ flag) {
  __shared__ long long part[1024];
  const long long per = (nb + blockDim.x - 1) / blockDim.x;
  const long long b = (long long)threadIdx.x * per;
  const long long e = b + per < nb ? b + per : nb;
  long long s = 0;
  for (long long i = b; i < e; ++i) s += v[i];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long run = 0;
    for (int i = 0; i < (int)blockDim.x; ++i) {
      const long long x = part[i];
      part[i] = run;
      run += x;
    }
    total[0] = run;
    total[1] = flag ? flag[0] : 0;
    if (flag) flag[0] = 0;
  }
  __syncthreads();
  long long run = part[threadIdx.x];
  for (long long i = b; i < e; ++i) {
    const long long x = v[i];
    v[i] = run;
    run += x;
  }
}

__global__ __launch_bounds__(kBlock) void hagg_emit_kernel(
    unsigned long long* __restrict__ keys, double* __restrict__ sums, long long* __restrict__ cnts,
    double* __restrict__ mins, double* __restrict__ maxs, long long M, int NA, int star,
    const long long* __restrict__ block_off, int reset, long long cap,
    unsigned long long* __restrict__ out_keys, unsigned char* __restrict__ out_null,
    double* __restrict__ out_sums, long long* __restrict__ out_cnts, double* __restrict__ out_mins,
    double* __restrict__ out_maxs) {
  const long long st = M + 2;
  long long base = block_off[blockIdx.x];
  for (int k = 0; k < kSlotsPerThread; ++k) {
  const long long s = (long long)blockIdx.x * kChunk + k * kBlock + threadIdx.x;
  const bool f = s < st && occupied(keys, cnts, M, star, s);
  int tot;
  const int r = block_prefix(f, &tot);
  __syncthreads();   // block_prefix's LDS words are reused by the next step
  const long long pos = base + r;
  base += tot;
  if (!f) continue;
  out_keys[pos] = s == M ? kEmpty : keys[s];
  out_null[pos] = s == M + 1 ? 1 : 0;
  for (int i = 0; i < NA; ++i) {
    const long long si = (long long)i * st + s, oi = (long long)i * cap + pos;
    out_sums[oi] = sums[si];
    out_cnts[oi] = cnts[si];
    if (mins) out_mins[oi] = mins[si];
    if (maxs) out_maxs[oi] = maxs[si];
    if (reset) {
      sums[si] = 0.0;
      cnts[si] = 0;
      if (mins) mins[si] = __builtin_inf();
      if (maxs) maxs[si] = -__builtin_inf();
    }
  }
  if (reset && s < M) keys[s] = kEmpty;
  }
}

// Slot of `key` (null: the NULL slot), inserting it if absent; -1 when the probe sequence
// exceeds max_probe (the caller flags overflow and re-runs with a larger table).
__device__ __forceinline__ long long probe_insert(unsigned long long* keys, long long M,
                                                  unsigned long long key, bool is_null,
                                                  int max_probe) {
  if (is_null) return M + 1;
  if (key == kEmpty) return M;
  unsigned long long h = mix64(key) & (unsigned long long)(M - 1);
  for (int p = 0; p < max_probe; ++p) {
    const unsigned long long prev = atomicCAS(&keys[h], kEmpty, key);
    if (prev == kEmpty || prev == key) return (long long)h;
    h = (h + 1) & (unsigned long long)(M - 1);
  }
  return -1;
}

// Insert n dense groups (SoA, row stride in_cap) into a table.
__global__ __launch_bounds__(kBlock) void hagg_merge_kernel(
    const unsigned long long* __restrict__ in_keys, const unsigned char* __restrict__ in_null,
    const double* __restrict__ in_sums, const long long* __restrict__ in_cnts,
    const double* __restrict__ in_mins, const double* __restrict__ in_maxs, long long n,
    long long in_cap, unsigned long long* keys, double* sums, long long* cnts, double* mins,
    double* maxs, long long M, int NA, long long* flag) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long st = M + 2;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += stride) {
    const long long s = probe_insert(keys, M, in_keys[g], in_null[g] != 0, 1 << 20);
    if (s < 0) {
      flag[0] = 1;
      continue;
    }
    for (int i = 0; i < NA; ++i) {
      const long long si = (long long)i * st + s, gi = (long long)i * in_cap + g;
      unsafeAtomicAdd(&sums[si], in_sums[gi]);
      if (in_cnts[gi]) atomicAdd((unsigned long long*)&cnts[si], (unsigned long long)in_cnts[gi]);
      if (mins) atomicMin(&mins[si], in_mins[gi]);
      if (maxs) atomicMax(&maxs[si], in_maxs[gi]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Top-k
// ------------------------------------------------------------------------------------------------
// Order-preserving image of a double (ascending); NaN sorts last like Spark.
__device__ __forceinline__ unsigned long long dimg(double d) {
  if (d != d) return ~0ull - 1ull;
  d = d == 0.0 ? 0.0 : d;
  const unsigned long long b = (unsigned long long)__double_as_longlong(d);
  return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

// Image sources: 0 sum, 1 count, 2 min, 3 max, 4 avg (sum / count) of aggregate `agg`;
// 5 packed key field (code = (key >> shift) & mask, 0 = null when nullable); 6 raw signed key;
// 7 raw double key (bits).  cnt_slot < 0: groups carry no count (every group is non-empty).
// Ascending: nulls first (image 0); descending: image complemented, nulls last (Spark's default
// null ordering).
__global__ __launch_bounds__(kBlock) void topk_images_kernel(
    const unsigned long long* __restrict__ keys, const unsigned char* __restrict__ nulls,
    const double* __restrict__ sums, const long long* __restrict__ cnts,
    const double* __restrict__ mins, const double* __restrict__ maxs, long long G, long long cap,
    int src, int agg, int cnt_slot, int shift, unsigned long long mask, int nullable, int desc,
    unsigned long long* __restrict__ img) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += stride) {
    bool isnull = false;
    unsigned long long v = 0;
    const long long ai = (long long)agg * cap + g;
    const long long c = cnt_slot >= 0 ? cnts[(long long)cnt_slot * cap + g] : 1;
    switch (src) {
      case 0: isnull = c == 0; v = dimg(sums[ai]); break;
      case 1: v = (unsigned long long)c ^ 0x8000000000000000ull; break;
      case 2: isnull = c == 0; v = dimg(mins[ai]); break;
      case 3: isnull = c == 0; v = dimg(maxs[ai]); break;
      case 4: isnull = c == 0; v = dimg(c ? sums[ai] / (double)c : 0.0); break;
      case 5: {
        const unsigned long long code = (keys[g] >> shift) & mask;
        isnull = nullable && code == 0;
        v = code;  // codes order like their values
        break;
      }
      case 6:
        isnull = nulls[g] != 0;
        v = keys[g] ^ 0x8000000000000000ull;
        break;
      default:
        isnull = nulls[g] != 0;
        v = dimg(__longlong_as_double((long long)keys[g]));
        break;
    }
    unsigned long long o = desc ? ~v : v;
    if (isnull) o = desc ? ~0ull : 0ull;
    img[g] = o;
  }
}

__global__ void topk_init_kernel(unsigned long long* st, unsigned long long k,
                                 unsigned long long* count) {
  st[0] = 0ull;
  st[1] = k;
  *count = 0ull;
}

// Radix-select state (device): st[0] = prefix of the selected bin path, st[1] = rank still to
// take inside it (1-based), hist[kTopkBins].
// Level L histograms bits [64 - 12 (L + 1), 64 - 12 L) of the images whose higher bits equal
// the prefix.
__global__ __launch_bounds__(kBlock) void topk_hist_kernel(const unsigned long long* __restrict__ img,
                                                           long long G, int level,
                                                           const unsigned long long* __restrict__ st,
                                                           unsigned int* __restrict__ hist) {
  __shared__ unsigned int h[kTopkBins];
  for (int i = threadIdx.x; i < kTopkBins; i += kBlock) h[i] = 0u;
  __syncthreads();
  const int shift = 64 - kTopkBits * (level + 1);
  const unsigned long long prefix = level ? st[0] : 0ull;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += stride) {
    const unsigned long long x = img[g];
    const bool in = level == 0 || (x >> (shift + kTopkBits)) == prefix;
    if (in) atomicAdd(&h[(x >> shift) & (kTopkBins - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kTopkBins; i += kBlock)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// One block: pick the bin holding the st[1]-th smallest image of this level, extend the
// prefix, subtract the ranks below it, and clear the histogram for the next level.
__global__ __launch_bounds__(kBlock) void topk_pick_kernel(int level, unsigned long long* st,
                                                           unsigned int* hist) {
  __shared__ unsigned long long part[kBlock];
  constexpr int per = kTopkBins / kBlock;
  const int b0 = threadIdx.x * per;
  unsigned long long s = 0;
  for (int i = 0; i < per; ++i) s += hist[b0 + i];
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned long long want = st[1];
    unsigned long long run = 0;
    int t = 0;
    while (t < kBlock - 1 && run + part[t] < want) run += part[t++];
    int b = t * per;
    while (b < kTopkBins - 1 && run + hist[b] < want) run += hist[b++];
    st[0] = ((level ? st[0] : 0ull) << kTopkBits) | (unsigned long long)b;
    st[1] = want - run;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kTopkBins; i += kBlock) hist[i] = 0u;
}

// Groups whose image's top 36 bits are <= the selected prefix: the exact top-k plus the ties
// of the k-th image at 36-bit resolution.
__global__ __launch_bounds__(kBlock) void topk_select_kernel(const unsigned long long* __restrict__ img,
                                                             long long G,
                                                             const unsigned long long* __restrict__ st,
                                                             unsigned* __restrict__ out,
                                                             unsigned long long* __restrict__ count) {
  const int shift = 64 - kTopkBits * kTopkLevels;
  const unsigned long long t = st[0];
  const long long stride = (long long)gridDim.x * blockDim.x;
  const int lane = threadIdx.x & 63;
  for (long long g0 = (long long)blockIdx.x * blockDim.x; g0 < G; g0 += stride) {
    const long long g = g0 + threadIdx.x;
    const bool sel = g < G && (img[g] >> shift) <= t;
    const unsigned long long bm = __ballot(sel);
    if (bm == 0ull) continue;
    unsigned long long base = 0;
    const int leader = __ffsll((long long)bm) - 1;
    if (lane == leader) base = atomicAdd(count, (unsigned long long)__popcll(bm));
    base = __shfl(base, leader, 64);
    if (sel) {
      const unsigned below = (unsigned)__popcll(bm & ((1ull << lane) - 1ull));
      out[base + below] = (unsigned)g;
    }
  }
}

__global__ __launch_bounds__(kBlock) void hagg_take_kernel(
    const unsigned* __restrict__ rows, long long n, const unsigned long long* __restrict__ keys,
    const unsigned char* __restrict__ nulls, const double* __restrict__ sums,
    const long long* __restrict__ cnts, const double* __restrict__ mins,
    const double* __restrict__ maxs, int NA, long long cap, long long ocap,
    unsigned long long* __restrict__ o_keys, unsigned char* __restrict__ o_nulls,
    double* __restrict__ o_sums, long long* __restrict__ o_cnts, double* __restrict__ o_mins,
    double* __restrict__ o_maxs) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const long long g = rows[i];
    o_keys[i] = keys[g];
    o_nulls[i] = nulls[g];
    for (int a = 0; a < NA; ++a) {
      o_sums[(long long)a * ocap + i] = sums[(long long)a * cap + g];
      o_cnts[(long long)a * ocap + i] = cnts[(long long)a * cap + g];
      if (mins) o_mins[(long long)a * ocap + i] = mins[(long long)a * cap + g];
      if (maxs) o_maxs[(long long)a * ocap + i] = maxs[(long long)a * cap + g];
    }
  }
}

inline unsigned grid_for(long long n, long long cap = 8192) {
  const long long b = (n + kBlock - 1) / kBlock;
  return (unsigned)(b < 1 ? 1 : (b > cap ? cap : b));
}

}  // namespace

extern "C" {

int hs_topk_levels() { return kTopkLevels; }
int hs_topk_bins() { return kTopkBins; }

int hs_hagg_init(unsigned long long* keys, double* sums, long long* cnts, double* mins,
                 double* maxs, long long M, int NA, void* stream) {
  if (M <= 0 || (M & (M - 1)) != 0 || NA <= 0) return -1;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hagg_init_kernel, dim3(grid_for((M + 2) * NA)), dim3(kBlock), 0,
                     (hipStream_t)stream, keys, sums, cnts, mins, maxs, M, NA);
  return (int)hipGetLastError();
}

// Workspace int64s of hs_hagg_extract for a table of M slots.
long long hs_hagg_extract_blocks(long long M) { return (M + 2 + kChunk - 1) / kChunk; }

// total: two int64s (the group count G, and the table's overflow flag, which is cleared).
// out_*: SoA with row stride `cap` >= G (M + 2 always suffices).
int hs_hagg_extract(unsigned long long* keys, double* sums, long long* cnts, double* mins,
                    double* maxs, long long M, int NA, int star, int reset, long long* ws,
                    long long* total, long long* flag, long long cap, unsigned long long* out_keys,
                    unsigned char* out_null, double* out_sums, long long* out_cnts,
                    double* out_mins, double* out_maxs, void* stream) {
  if (M <= 0 || NA <= 0 || star < 0 || star >= NA) return -1;
  (void)hipGetLastError();
  hipStream_t s = (hipStream_t)stream;
  const long long nb = hs_hagg_extract_blocks(M);
  hipLaunchKernelGGL(hagg_count_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, keys, cnts, M,
                     star, ws);
  hipLaunchKernelGGL(hagg_scan_kernel, dim3(1), dim3(1024), 0, s, ws, nb, total, flag);
  hipLaunchKernelGGL(hagg_emit_kernel, dim3((unsigned)nb), dim3(kBlock), 0, s, keys, sums, cnts,
                     mins, maxs, M, NA, star, (const long long*)ws, reset, cap, out_keys,
                     out_null, out_sums, out_cnts, out_mins, out_maxs);
  return (int)hipGetLastError();
}

int hs_hagg_merge(const unsigned long long* in_keys, const unsigned char* in_null,
                  const double* in_sums, const long long* in_cnts, const double* in_mins,
                  const double* in_maxs, long long n, long long in_cap, unsigned long long* keys,
                  double* sums, long long* cnts, double* mins, double* maxs, long long M, int NA,
                  long long* flag, void* stream) {
  if (n <= 0) return 0;
  if (M <= 0 || (M & (M - 1)) != 0) return -1;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hagg_merge_kernel, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream,
                     in_keys, in_null, in_sums, in_cnts, in_mins, in_maxs, n, in_cap, keys, sums,
                     cnts, mins, maxs, M, NA, flag);
  return (int)hipGetLastError();
}

int hs_topk_images(const unsigned long long* keys, const unsigned char* nulls, const double* sums,
                   const long long* cnts, const double* mins, const double* maxs, long long G,
                   long long cap, int src, int agg, int cnt_slot, int shift,
                   unsigned long long mask, int nullable, int desc, unsigned long long* img,
                   void* stream) {
  if (G <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(topk_images_kernel, dim3(grid_for(G)), dim3(kBlock), 0, (hipStream_t)stream,
                     keys, nulls, sums, cnts, mins, maxs, G, cap, src, agg, cnt_slot, shift, mask,
                     nullable, desc, img);
  return (int)hipGetLastError();
}

// Candidates of the k smallest of G images.  st: 2 u64 (zeroed here); hist: kTopkBins u32
// (zero on entry, left zero); out: G u32 row ids; count: 1 u64 (zeroed here).
int hs_topk_select(const unsigned long long* img, long long G, long long k, unsigned long long* st,
                   unsigned int* hist, unsigned* out, unsigned long long* count, void* stream) {
  if (G <= 0 || k <= 0) return -1;
  (void)hipGetLastError();
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(topk_init_kernel, dim3(1), dim3(1), 0, s, st, (unsigned long long)k, count);
  for (int level = 0; level < kTopkLevels; ++level) {
    hipLaunchKernelGGL(topk_hist_kernel, dim3(grid_for(G, 2048)), dim3(kBlock), 0, s, img, G,
                       level, (const unsigned long long*)st, hist);
    hipLaunchKernelGGL(topk_pick_kernel, dim3(1), dim3(kBlock), 0, s, level, st, hist);
  }
  hipLaunchKernelGGL(topk_select_kernel, dim3(grid_for(G, 4096)), dim3(kBlock), 0, s, img, G,
                     (const unsigned long long*)st, out, count);
  return (int)hipGetLastError();
}

int hs_hagg_take(const unsigned* rows, long long n, const unsigned long long* keys,
                 const unsigned char* nulls, const double* sums, const long long* cnts,
                 const double* mins, const double* maxs, int NA, long long cap, long long ocap,
                 unsigned long long* o_keys, unsigned char* o_nulls, double* o_sums,
                 long long* o_cnts, double* o_mins, double* o_maxs, void* stream) {
  if (n <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hagg_take_kernel, dim3(grid_for(n)), dim3(kBlock), 0, (hipStream_t)stream,
                     rows, n, keys, nulls, sums, cnts, mins, maxs, NA, cap, ocap, o_keys, o_nulls,
                     o_sums, o_cnts, o_mins, o_maxs);
  return (int)hipGetLastError();
}

}  // extern "C"
