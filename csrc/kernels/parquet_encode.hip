// K4: Parquet page encoding on the MI355X (SURVEY.md §2.3 K4 "Parquet encode kernels").
//
// Dictionary-encoded index columns leave the GPU as bit-packed codes: one bit-packed run per
// data page (hybrid RLE/bit-packing, LSB-first, groups of 8 values).  One thread packs one group
// of 8 codes (<= 16 bits each -> <= 16 bytes) into its byte slot of the page, so packing is a
// single coalesced pass; pages are addressed through a small page table (row start, values,
// output byte offset, group prefix) searched per thread.  The host writer
// (csrc/runtime/hs_parquet_write.cpp) only frames the pages.
//
// Codes for fixed-width columns come from a dictionary lookup (hs_pq_dict_codes): binary search
// of each value's bit pattern in the sorted dictionary of bit patterns (so -0.0 / NaN payloads
// survive bit-exactly); a miss flags the column as not dictionary-encodable.
#include <hip/hip_runtime.h>

#include <cstdint>

struct HsPqPage {
  int64_t row0;       // first row of the page in the (bucket-major) column
  int64_t n;          // values in the page
  int64_t out_off;    // byte offset of the page's packed data in the output buffer
  int64_t gpre;       // exclusive prefix of groups (ceil(n/8)) over pages
};

__global__ __launch_bounds__(256) void hs_pq_pack_kernel(const int32_t* __restrict__ codes,
                                                         const HsPqPage* __restrict__ pages,
                                                         int npages, int64_t ngroups, int bw_all,
                                                         const int32_t* __restrict__ page_bw,
                                                         uint8_t* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  int lo = 0, hi = npages;  // page with gpre <= g < next gpre
  while (hi - lo > 1) {
    const int md = (lo + hi) >> 1;
    if (pages[md].gpre <= g) lo = md; else hi = md;
  }
  const HsPqPage pg = pages[lo];
  const int bw = page_bw ? page_bw[lo] : bw_all;  // per-page width: per-file dictionaries
  const int64_t j = g - pg.gpre;           // group within the page
  const int64_t r0 = pg.row0 + j * 8;
  const int64_t left = pg.n - j * 8;
  uint64_t w0 = 0, w1 = 0;                 // 128-bit accumulator (8 x <=16 bits)
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t c = k < left ? (uint64_t)(uint32_t)codes[r0 + k] : 0ull;
    const int bit = k * bw;
    if (bit < 64) {
      w0 |= c << bit;
      if (bit + bw > 64) w1 |= c >> (64 - bit);
    } else {
      w1 |= c << (bit - 64);
    }
  }
  uint8_t* o = out + pg.out_off + j * bw;  // 8 values x bw bits = bw bytes
  for (int k = 0; k < bw; ++k) o[k] = (uint8_t)(k < 8 ? (w0 >> (8 * k)) : (w1 >> (8 * (k - 8))));
}

// Per-file dictionaries.  Codes into a column's job-wide sorted dictionary (D entries) become
// codes into the sorted subset that one bucket file uses, so a file's bytes depend only on its
// own rows (not on which other buckets shared the encode call: one-pass, bucket-range-streamed
// and any-world-size builds write identical files).  Files are contiguous row ranges
// [fo[f], fo[f+1]) of the bucket-major column.
//
// Mark: one workgroup per CH-row chunk; the chunk's rows of each file it touches set bits of a
// D-bit LDS bitmap (low-cardinality columns hit a handful of words: LDS atomics, not HBM ones),
// whose non-zero words are OR-ed into present[f * DW + w].
constexpr int kDictChunk = 4096;
constexpr int kDictMaxWords = 2048;  // D <= 65536

__device__ __forceinline__ int file_of(const int64_t* fo, int nf, int64_t r) {
  int lo = 0, hi = nf;  // fo[lo] <= r < fo[lo + 1]
  while (hi - lo > 1) {
    const int md = (lo + hi) >> 1;
    if (fo[md] <= r) lo = md; else hi = md;
  }
  return lo;
}

__global__ __launch_bounds__(256) void hs_pq_dict_mark_kernel(const int32_t* __restrict__ codes,
                                                              const int64_t* __restrict__ fo,
                                                              int nf, int dw,
                                                              uint32_t* __restrict__ present) {
  __shared__ uint32_t bm[kDictMaxWords];
  const int64_t n = fo[nf];
  const int64_t r0 = (int64_t)blockIdx.x * kDictChunk;
  if (r0 >= n) return;
  const int64_t r1 = r0 + kDictChunk < n ? r0 + kDictChunk : n;
  int f = file_of(fo, nf, r0);
  for (int64_t s = r0; s < r1; ++f) {
    const int64_t e = fo[f + 1] < r1 ? fo[f + 1] : r1;
    for (int w = threadIdx.x; w < dw; w += blockDim.x) bm[w] = 0u;
    __syncthreads();
    for (int64_t r = s + threadIdx.x; r < e; r += blockDim.x) {
      const uint32_t c = (uint32_t)codes[r];
      atomicOr(&bm[c >> 5], 1u << (c & 31));
    }
    __syncthreads();
    for (int w = threadIdx.x; w < dw; w += blockDim.x)
      if (bm[w]) atomicOr(&present[(int64_t)f * dw + w], bm[w]);
    __syncthreads();
    s = e;
  }
}

// Remap: code -> its rank among the file's present codes (wpre = exclusive prefix of the
// present words' popcounts within each file).
// One workgroup per CH-row chunk, file segment by file segment (the file search runs once per
// chunk and segment, not per row); the file's present words and prefixes are read through L1.
__global__ __launch_bounds__(256) void hs_pq_dict_remap_kernel(int32_t* __restrict__ codes,
                                                               const int64_t* __restrict__ fo,
                                                               int nf, int dw,
                                                               const uint32_t* __restrict__ present,
                                                               const int32_t* __restrict__ wpre) {
  const int64_t n = fo[nf];
  const int64_t r0 = (int64_t)blockIdx.x * kDictChunk;
  if (r0 >= n) return;
  const int64_t r1 = r0 + kDictChunk < n ? r0 + kDictChunk : n;
  int f = file_of(fo, nf, r0);
  for (int64_t s = r0; s < r1; ++f) {
    const int64_t e = fo[f + 1] < r1 ? fo[f + 1] : r1;
    const uint32_t* pw = present + (int64_t)f * dw;
    const int32_t* pp = wpre + (int64_t)f * dw;
    for (int64_t r = s + threadIdx.x; r < e; r += blockDim.x) {
      const uint32_t c = (uint32_t)codes[r];
      codes[r] = pp[c >> 5] + __popc(pw[c >> 5] & ((1u << (c & 31)) - 1u));
    }
    s = e;
  }
}

// codes[i] = index of bits[i] in the sorted dictionary `dict` (n_dict entries); a value that is
// not in the dictionary sets *miss.
template <typename T>
__global__ __launch_bounds__(256) void hs_pq_dict_codes_kernel(const T* __restrict__ bits, int64_t n,
                                                               const T* __restrict__ dict,
                                                               int n_dict, int32_t* __restrict__ codes,
                                                               int32_t* __restrict__ miss) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const T v = bits[i];
  int lo = 0, hi = n_dict;
  while (lo < hi) {
    const int md = (lo + hi) >> 1;
    if (dict[md] < v) lo = md + 1; else hi = md;
  }
  if (lo >= n_dict || dict[lo] != v) {
    *miss = 1;
    lo = 0;
  }
  codes[i] = lo;
}

extern "C" {

// page_bw: per-page bit widths (each in 1..16, checked by the caller) or null for ``bw``
int hs_pq_pack(const int32_t* codes, const HsPqPage* pages, int npages, int64_t ngroups, int bw,
               const int32_t* page_bw, uint8_t* out, void* stream) {
  if (ngroups <= 0) return 0;
  if (!page_bw && (bw < 1 || bw > 16)) return -1;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hs_pq_pack_kernel, dim3((unsigned)((ngroups + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, codes, pages, npages, ngroups, bw, page_bw, out);
  return (int)hipGetLastError();
}

// present: zeroed uint32 [nf * dw]; fo: device int64 [nf + 1] file row offsets
int hs_pq_dict_mark(const int32_t* codes, const int64_t* fo, int nf, int64_t n, int dw,
                    uint32_t* present, void* stream) {
  if (n <= 0 || nf <= 0) return 0;
  if (dw < 1 || dw > kDictMaxWords) return -1;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hs_pq_dict_mark_kernel, dim3((unsigned)((n + kDictChunk - 1) / kDictChunk)),
                     dim3(256), 0, (hipStream_t)stream, codes, fo, nf, dw, present);
  return (int)hipGetLastError();
}

int hs_pq_dict_remap(int32_t* codes, const int64_t* fo, int nf, int64_t n, int dw,
                     const uint32_t* present, const int32_t* wpre, void* stream) {
  if (n <= 0 || nf <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hs_pq_dict_remap_kernel, dim3((unsigned)((n + kDictChunk - 1) / kDictChunk)),
                     dim3(256), 0,
                     (hipStream_t)stream, codes, fo, nf, dw, present, wpre);
  return (int)hipGetLastError();
}

// elem_bytes 4 or 8: values compared as signed bit patterns (the dictionary is sorted that way
// on the device with torch.sort of the int32/int64 view)
int hs_pq_dict_codes(const void* bits, int64_t n, int elem_bytes, const void* dict, int n_dict,
                     int32_t* codes, int32_t* miss, void* stream) {
  if (n <= 0) return 0;
  (void)hipGetLastError();
  const dim3 grid((unsigned)((n + 255) / 256));
  if (elem_bytes == 4)
    hipLaunchKernelGGL(hs_pq_dict_codes_kernel<int32_t>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const int32_t*)bits, n, (const int32_t*)dict, n_dict, codes, miss);
  else if (elem_bytes == 8)
    hipLaunchKernelGGL(hs_pq_dict_codes_kernel<int64_t>, grid, dim3(256), 0, (hipStream_t)stream,
                       (const int64_t*)bits, n, (const int64_t*)dict, n_dict, codes, miss);
  else
    return -1;
  return (int)hipGetLastError();
}

}  // extern "C"
