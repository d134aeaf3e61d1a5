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
//                    (deterministic), and reset the slots it read, so the next query reuses the
//                    table without a memset of the whole table
//   hs_hagg_merge    insert dense partial groups into a table (multi-rank combine)
//   hs_topk_*        ORDER BY <one expression> LIMIT k over the dense groups: order-preserving
//                    u64 images, LDS bitonic top-k per 2048-row chunk (repeated until one chunk
//                    is left), then every group whose image is <= the k-th image is selected;
//                    the host sorts those few candidates by the full ORDER BY
//
// Table layout (M = power-of-two probe slots, NA = aggregate slots per group):
//   keys[M + 2]   slot M holds the key ~0 (the EMPTY pattern itself), slot M + 1 the NULL key of
//                 an unpacked single-column key; both are addressed directly, never probed
//   sums, cnts, mins, maxs [(M + 2) * NA]   (mins / maxs may be null when no MIN / MAX)
// Occupancy: keys[s] != EMPTY for s < M; cnts[s * NA + star] > 0 for the two special slots.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr unsigned long long kEmpty = ~0ull;
constexpr int kExtractItems = 8;                 // slots per thread of hs_hagg_extract
constexpr int kExtractBlock = 256;
constexpr int kExtractChunk = kExtractItems * kExtractBlock;
constexpr int kTopkChunk = 2048;                 // rows sorted in LDS per top-k block
constexpr int kTopkBlock = 256;

__device__ __forceinline__ unsigned long long mix64(unsigned long long h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

__device__ __forceinline__ bool occupied(const unsigned long long* keys, const long long* cnts,
                                         long long M, int NA, int star, long long s) {
  return s < M ? keys[s] != kEmpty : cnts[s * NA + star] > 0;
}

__global__ __launch_bounds__(256) void hagg_init_kernel(unsigned long long* keys, double* sums,
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

// Per block: number of occupied slots of its kExtractChunk slots.
__global__ __launch_bounds__(kExtractBlock) void hagg_count_kernel(
    const unsigned long long* __restrict__ keys, const long long* __restrict__ cnts, long long M,
    int NA, int star, long long* __restrict__ block_counts) {
  const long long nslot = M + 2;
  const long long s0 = (long long)blockIdx.x * kExtractChunk + (long long)threadIdx.x * kExtractItems;
  int c = 0;
#pragma unroll
  for (int k = 0; k < kExtractItems; ++k) {
    const long long s = s0 + k;
    c += (s < nslot && occupied(keys, cnts, M, NA, star, s)) ? 1 : 0;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  __shared__ int wsum[kExtractBlock / 64];
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int w = 0; w < kExtractBlock / 64; ++w) t += wsum[w];
    block_counts[blockIdx.x] = t;
  }
}

// One block: exclusive scan of nb block counts in place; total -> *total.
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
    total[1] = flag ? flag[0] : 0;   // overflow flag of the insert kernels, then cleared
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

__global__ __launch_bounds__(kExtractBlock) void hagg_emit_kernel(
    unsigned long long* __restrict__ keys, double* __restrict__ sums, long long* __restrict__ cnts,
    double* __restrict__ mins, double* __restrict__ maxs, long long M, int NA, int star,
    const long long* __restrict__ block_off, int reset, unsigned long long* __restrict__ out_keys,
    unsigned char* __restrict__ out_null, double* __restrict__ out_sums,
    long long* __restrict__ out_cnts, double* __restrict__ out_mins, double* __restrict__ out_maxs) {
  const long long nslot = M + 2;
  const long long s0 = (long long)blockIdx.x * kExtractChunk + (long long)threadIdx.x * kExtractItems;
  unsigned occ = 0u;
#pragma unroll
  for (int k = 0; k < kExtractItems; ++k) {
    const long long s = s0 + k;
    occ |= (s < nslot && occupied(keys, cnts, M, NA, star, s)) ? (1u << k) : 0u;
  }
  // block-exclusive prefix of the per-thread counts (thread order = slot order)
  const int c = __popc(occ);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int inc = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int u = __shfl_up(inc, d, 64);
    if (lane >= d) inc += u;
  }
  __shared__ int wtot[kExtractBlock / 64];
  if (lane == 63) wtot[w] = inc;
  __syncthreads();
  int wbase = 0;
  for (int k = 0; k < w; ++k) wbase += wtot[k];
  long long pos = block_off[blockIdx.x] + wbase + inc - c;
  for (int k = 0; k < kExtractItems; ++k) {
    if (!((occ >> k) & 1u)) continue;
    const long long s = s0 + k;
    out_keys[pos] = s == M ? kEmpty : keys[s];
    out_null[pos] = s == M + 1 ? 1 : 0;
    for (int i = 0; i < NA; ++i) {
      const long long si = s * NA + i, oi = pos * NA + i;
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
    ++pos;
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
    const unsigned long long k = keys[h];
    if (k == key) return (long long)h;
    if (k == kEmpty) {
      const unsigned long long prev = atomicCAS(&keys[h], kEmpty, key);
      if (prev == kEmpty || prev == key) return (long long)h;
    }
    h = (h + 1) & (unsigned long long)(M - 1);
  }
  return -1;
}

__global__ __launch_bounds__(256) void hagg_merge_kernel(
    const unsigned long long* __restrict__ in_keys, const unsigned char* __restrict__ in_null,
    const double* __restrict__ in_sums, const long long* __restrict__ in_cnts,
    const double* __restrict__ in_mins, const double* __restrict__ in_maxs, long long n,
    unsigned long long* keys, double* sums, long long* cnts, double* mins, double* maxs,
    long long M, int NA, long long* flag) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += stride) {
    const long long s = probe_insert(keys, M, in_keys[g], in_null[g] != 0, 1 << 20);
    if (s < 0) {
      flag[0] = 1;
      continue;
    }
    for (int i = 0; i < NA; ++i) {
      const long long si = s * NA + i, gi = g * NA + i;
      if (in_cnts[gi] == 0) continue;
      unsafeAtomicAdd(&sums[si], in_sums[gi]);
      atomicAdd((unsigned long long*)&cnts[si], (unsigned long long)in_cnts[gi]);
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
// 5 packed key field (code = (key >> shift) & mask, 0 = null when nullable, value = lo + code - 1
// (nullable) or lo + code); 6 raw signed key; 7 raw double key (bits).  Ascending: nulls first
// (image 0); descending: image complemented, nulls last.  Spark's default null ordering.
__global__ __launch_bounds__(256) void topk_images_kernel(
    const unsigned long long* __restrict__ keys, const unsigned char* __restrict__ nulls,
    const double* __restrict__ sums, const long long* __restrict__ cnts,
    const double* __restrict__ mins, const double* __restrict__ maxs, long long G, int NA,
    int src, int agg, int cnt_slot, int shift, unsigned long long mask, int nullable, int desc,
    unsigned long long* __restrict__ img) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x; g < G; g += stride) {
    bool isnull = false;
    unsigned long long v = 0;
    const long long ai = g * NA + agg;
    const long long c = cnts[g * NA + cnt_slot];
    switch (src) {
      case 0: isnull = c == 0; v = dimg(sums[ai]); break;
      case 1: v = (unsigned long long)c ^ 0x8000000000000000ull; break;
      case 2: isnull = c == 0; v = dimg(mins[ai]); break;
      case 3: isnull = c == 0; v = dimg(maxs[ai]); break;
      case 4: isnull = c == 0; v = dimg(c ? sums[ai] / (double)c : 0.0); break;
      case 5: {
        const unsigned long long code = (keys[g] >> shift) & mask;
        isnull = nullable && code == 0;
        v = code;  // codes are ordered like the values (lo + code)
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
    // asc: null -> 0, values -> v (v >= 0); desc: values -> ~v, null -> ~0
    unsigned long long o = desc ? ~v : v;
    if (isnull) o = desc ? ~0ull : 0ull;
    img[g] = o;
  }
}

// One block per kTopkChunk rows: bitonic sort of (image, row) in LDS, the k smallest written
// to out[blockIdx.x * k ...] (missing rows padded with image ~0).
__global__ __launch_bounds__(kTopkBlock) void topk_pass_kernel(
    const unsigned long long* __restrict__ img, const unsigned* __restrict__ idx, long long n,
    int k, unsigned long long* __restrict__ out_img, unsigned* __restrict__ out_idx) {
  __shared__ unsigned long long si[kTopkChunk];
  __shared__ unsigned sx[kTopkChunk];
  const long long base = (long long)blockIdx.x * kTopkChunk;
  for (int i = threadIdx.x; i < kTopkChunk; i += kTopkBlock) {
    const long long g = base + i;
    const bool ok = g < n;
    si[i] = ok ? img[g] : ~0ull;
    sx[i] = ok ? (idx ? idx[g] : (unsigned)g) : 0xFFFFFFFFu;
  }
  __syncthreads();
  for (int size = 2; size <= kTopkChunk; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < kTopkChunk / 2; t += kTopkBlock) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const unsigned long long a = si[lo], b = si[hi];
        const unsigned xa = sx[lo], xb = sx[hi];
        const bool gt = a > b || (a == b && xa > xb);
        if (gt == up) {
          si[lo] = b; si[hi] = a;
          sx[lo] = xb; sx[hi] = xa;
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < k; i += kTopkBlock) {
    out_img[(long long)blockIdx.x * k + i] = si[i];
    out_idx[(long long)blockIdx.x * k + i] = sx[i];
  }
}

// Rows whose image is <= *thr (the k-th smallest image): the exact top-k plus its ties.
__global__ __launch_bounds__(256) void topk_select_kernel(const unsigned long long* __restrict__ img,
                                                          long long G,
                                                          const unsigned long long* __restrict__ thr,
                                                          unsigned* __restrict__ out,
                                                          unsigned long long* __restrict__ count) {
  const unsigned long long t = *thr;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const int lane = threadIdx.x & 63;
  for (long long g0 = (long long)blockIdx.x * blockDim.x; g0 < G; g0 += stride) {
    const long long g = g0 + threadIdx.x;
    const bool sel = g < G && img[g] <= t;
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

__global__ __launch_bounds__(256) void hagg_take_kernel(
    const unsigned* __restrict__ rows, long long n, const unsigned long long* __restrict__ keys,
    const unsigned char* __restrict__ nulls, const double* __restrict__ sums,
    const long long* __restrict__ cnts, const double* __restrict__ mins,
    const double* __restrict__ maxs, int NA, unsigned long long* __restrict__ o_keys,
    unsigned char* __restrict__ o_nulls, double* __restrict__ o_sums, long long* __restrict__ o_cnts,
    double* __restrict__ o_mins, double* __restrict__ o_maxs) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const long long g = rows[i];
    o_keys[i] = keys[g];
    o_nulls[i] = nulls[g];
    for (int a = 0; a < NA; ++a) {
      o_sums[i * NA + a] = sums[g * NA + a];
      o_cnts[i * NA + a] = cnts[g * NA + a];
      if (mins) o_mins[i * NA + a] = mins[g * NA + a];
      if (maxs) o_maxs[i * NA + a] = maxs[g * NA + a];
    }
  }
}

inline unsigned grid_for(long long n, long long cap = 8192) {
  const long long b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > cap ? cap : b));
}

}  // namespace

extern "C" {

int hs_hagg_extract_chunk() { return kExtractChunk; }
int hs_topk_chunk() { return kTopkChunk; }

int hs_hagg_init(unsigned long long* keys, double* sums, long long* cnts, double* mins,
                 double* maxs, long long M, int NA, void* stream) {
  if (M <= 0 || (M & (M - 1)) != 0 || NA <= 0) return -1;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hagg_init_kernel, dim3(grid_for((M + 2) * NA)), dim3(256), 0,
                     (hipStream_t)stream, keys, sums, cnts, mins, maxs, M, NA);
  return (int)hipGetLastError();
}

// ws: at least hs_hagg_extract_blocks(M) int64s; total: two int64s (the group count G, and the
// table's overflow flag, which is cleared).
// out_*: capacity >= G rows (M + 2 is always enough).
long long hs_hagg_extract_blocks(long long M) {
  return (M + 2 + kExtractChunk - 1) / kExtractChunk;
}

int hs_hagg_extract(unsigned long long* keys, double* sums, long long* cnts, double* mins,
                    double* maxs, long long M, int NA, int star, int reset, long long* ws,
                    long long* total, long long* flag, unsigned long long* out_keys, unsigned char* out_null,
                    double* out_sums, long long* out_cnts, double* out_mins, double* out_maxs,
                    void* stream) {
  if (M <= 0 || NA <= 0 || star < 0 || star >= NA) return -1;
  (void)hipGetLastError();
  hipStream_t s = (hipStream_t)stream;
  const long long nb = hs_hagg_extract_blocks(M);
  hipLaunchKernelGGL(hagg_count_kernel, dim3((unsigned)nb), dim3(kExtractBlock), 0, s, keys, cnts,
                     M, NA, star, ws);
  hipLaunchKernelGGL(hagg_scan_kernel, dim3(1), dim3(1024), 0, s, ws, nb, total, flag);
  hipLaunchKernelGGL(hagg_emit_kernel, dim3((unsigned)nb), dim3(kExtractBlock), 0, s, keys, sums,
                     cnts, mins, maxs, M, NA, star, (const long long*)ws, reset, out_keys,
                     out_null, out_sums, out_cnts, out_mins, out_maxs);
  return (int)hipGetLastError();
}

int hs_hagg_merge(const unsigned long long* in_keys, const unsigned char* in_null,
                  const double* in_sums, const long long* in_cnts, const double* in_mins,
                  const double* in_maxs, long long n, unsigned long long* keys, double* sums,
                  long long* cnts, double* mins, double* maxs, long long M, int NA,
                  long long* flag, void* stream) {
  if (n <= 0) return 0;
  if (M <= 0 || (M & (M - 1)) != 0) return -1;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hagg_merge_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream,
                     in_keys, in_null, in_sums, in_cnts, in_mins, in_maxs, n, keys, sums, cnts,
                     mins, maxs, M, NA, flag);
  return (int)hipGetLastError();
}

int hs_topk_images(const unsigned long long* keys, const unsigned char* nulls, const double* sums,
                   const long long* cnts, const double* mins, const double* maxs, long long G,
                   int NA, int src, int agg, int cnt_slot, int shift, unsigned long long mask,
                   int nullable, int desc, unsigned long long* img, void* stream) {
  if (G <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(topk_images_kernel, dim3(grid_for(G)), dim3(256), 0, (hipStream_t)stream,
                     keys, nulls, sums, cnts, mins, maxs, G, NA, src, agg, cnt_slot, shift, mask,
                     nullable, desc, img);
  return (int)hipGetLastError();
}

// One reduction pass: n rows -> ceil(n / chunk) * k rows (the k smallest of each chunk, sorted).
int hs_topk_pass(const unsigned long long* img, const unsigned* idx, long long n, int k,
                 unsigned long long* out_img, unsigned* out_idx, void* stream) {
  if (k <= 0 || k > kTopkChunk) return -1;
  if (n <= 0) return 0;
  (void)hipGetLastError();
  const long long nb = (n + kTopkChunk - 1) / kTopkChunk;
  hipLaunchKernelGGL(topk_pass_kernel, dim3((unsigned)nb), dim3(kTopkBlock), 0, (hipStream_t)stream,
                     img, idx, n, k, out_img, out_idx);
  return (int)hipGetLastError();
}

int hs_topk_select(const unsigned long long* img, long long G, const unsigned long long* thr,
                   unsigned* out, unsigned long long* count, void* stream) {
  if (G <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(topk_select_kernel, dim3(grid_for(G, 4096)), dim3(256), 0,
                     (hipStream_t)stream, img, G, thr, out, count);
  return (int)hipGetLastError();
}

int hs_hagg_take(const unsigned* rows, long long n, const unsigned long long* keys,
                 const unsigned char* nulls, const double* sums, const long long* cnts,
                 const double* mins, const double* maxs, int NA, unsigned long long* o_keys,
                 unsigned char* o_nulls, double* o_sums, long long* o_cnts, double* o_mins,
                 double* o_maxs, void* stream) {
  if (n <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hagg_take_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, rows,
                     n, keys, nulls, sums, cnts, mins, maxs, NA, o_keys, o_nulls, o_sums, o_cnts,
                     o_mins, o_maxs);
  return (int)hipGetLastError();
}

}  // extern "C"
