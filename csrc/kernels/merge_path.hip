// K6: merge of sorted runs (OptimizeAction.scala:85-99,115-133).
//
// An optimize / incremental rewrite reads the files of a bucket, each already sorted by the
// indexed columns.  Instead of re-sorting the bucket from scratch (a full LSD radix sort: one
// 8-bit pass per key byte), the runs are merged pairwise in ceil(log2(runs per bucket)) rounds:
//
// * mp_make_keys: one u64 composite key per row, (valid bit, sortable - kmin) of every indexed
//   column, most significant first - the exact order hs_sort_columns produces (NULLS FIRST);
// * mp_merge: merge path.  Every thread owns MP_ITEMS consecutive OUTPUT positions: it finds its
//   pair of runs (binary search over the round's pair table), the split of its first output
//   diagonal between the two runs (binary search, ties to the left run = stable), then merges
//   sequentially.  Keys and the row permutation are written to the other buffer; a pair with an
//   empty right run is a copy.
//
// The result is the permutation a stable sort by (bucket, indexed columns) would produce: runs
// are in file order and ties always take the left (earlier) run.
#include "hs_common.h"

#define MP_BLOCK 256
#define MP_ITEMS 8
#define MP_MAX_KEYS 8

struct MergeKeys {
  ColDesc col[MP_MAX_KEYS];
  uint64_t kmin[MP_MAX_KEYS];
  int32_t bits[MP_MAX_KEYS];
  int32_t nullable[MP_MAX_KEYS];
  int32_t nkeys;
  int32_t pad;
};

__global__ __launch_bounds__(MP_BLOCK) void mp_make_keys(MergeKeys mk, int64_t n,
                                                         uint64_t* __restrict__ keys) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t k = 0;
    for (int c = 0; c < mk.nkeys; ++c) {
      const bool v = col_valid(mk.col[c], i);
      if (mk.nullable[c]) k = (k << 1) | (v ? 1ull : 0ull);
      if (mk.bits[c] > 0) {
        const uint64_t x = v ? hs_sortable(mk.col[c], i) - mk.kmin[c] : 0ull;
        k = (mk.bits[c] >= 64 ? 0ull : (k << mk.bits[c])) | x;
      }
    }
    keys[i] = k;
  }
}

// pairs: 3 int64 per pair {start, mid, end}: left run [start, mid), right run [mid, end); the
// pairs tile [0, n) in order.
__global__ __launch_bounds__(MP_BLOCK) void mp_merge(const uint64_t* __restrict__ kin,
                                                     const uint32_t* __restrict__ pin,
                                                     uint64_t* __restrict__ kout,
                                                     uint32_t* __restrict__ pout,
                                                     const int64_t* __restrict__ pairs,
                                                     int npairs, int64_t n) {
  const int64_t pos0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * MP_ITEMS;
  if (pos0 >= n) return;
  const int64_t pos_end = pos0 + MP_ITEMS < n ? pos0 + MP_ITEMS : n;
  int lo = 0, hi = npairs - 1;
  while (lo < hi) {
    const int md = (lo + hi + 1) >> 1;
    if (pairs[3 * md] <= pos0) lo = md; else hi = md - 1;
  }
  int p = lo;
  int64_t pos = pos0;
  while (pos < pos_end) {
    const int64_t s = pairs[3 * p], m = pairs[3 * p + 1], e = pairs[3 * p + 2];
    const int64_t a = m - s, b = e - m;
    const int64_t d = pos - s;
    // merge path split: i elements of A among the first d outputs
    int64_t l = d - b > 0 ? d - b : 0, h = d < a ? d : a;
    while (l < h) {
      const int64_t md = (l + h) >> 1;
      if (kin[s + md] <= kin[m + d - md - 1]) l = md + 1; else h = md;
    }
    int64_t i = l, j = d - l;
    const int64_t stop = pos_end < e ? pos_end : e;
    uint64_t ka = i < a ? kin[s + i] : 0ull, kb = j < b ? kin[m + j] : 0ull;
    for (; pos < stop; ++pos) {
      const bool take_a = i < a && (j >= b || ka <= kb);
      const int64_t src = take_a ? s + i : m + j;
      kout[pos] = take_a ? ka : kb;
      pout[pos] = pin ? pin[src] : (uint32_t)src;
      if (take_a) { ++i; ka = i < a ? kin[s + i] : 0ull; }
      else { ++j; kb = j < b ? kin[m + j] : 0ull; }
    }
    ++p;
  }
}

extern "C" {

int hs_merge_keys_size() { return (int)sizeof(MergeKeys); }

// Composite keys of the `nkeys` columns described in *mk (bits / kmin / nullable per column,
// total <= 64 bits) into keys[n].
int hs_merge_make_keys(const MergeKeys* mk, int64_t n, uint64_t* keys, void* stream) {
  if (n <= 0) return 0;
  if (mk->nkeys < 1 || mk->nkeys > MP_MAX_KEYS) return -2;
  int total = 0;
  for (int c = 0; c < mk->nkeys; ++c) total += mk->bits[c] + (mk->nullable[c] ? 1 : 0);
  if (total > 64) return -3;
  int64_t g = (n + MP_BLOCK - 1) / MP_BLOCK;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(mp_make_keys, dim3((unsigned)g), dim3(MP_BLOCK), 0, (hipStream_t)stream,
                     *mk, n, keys);
  return (int)hipGetLastError();
}

// One merge round over the device pair table `pairs` (npairs x {start, mid, end}).  `pin`
// null: the input permutation is the identity.
int hs_merge_round(const uint64_t* kin, const uint32_t* pin, uint64_t* kout, uint32_t* pout,
                   const int64_t* pairs, int npairs, int64_t n, void* stream) {
  if (n <= 0 || npairs <= 0) return 0;
  if (n > 0xFFFFFFFFll) return -2;
  const int64_t threads = (n + MP_ITEMS - 1) / MP_ITEMS;
  const int64_t g = (threads + MP_BLOCK - 1) / MP_BLOCK;
  hipLaunchKernelGGL(mp_merge, dim3((unsigned)g), dim3(MP_BLOCK), 0, (hipStream_t)stream, kin,
                     pin, kout, pout, pairs, npairs, n);
  return (int)hipGetLastError();
}

}  // extern "C"
