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
                                                         int npages, int64_t ngroups, int bw,
                                                         uint8_t* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  int lo = 0, hi = npages;  // page with gpre <= g < next gpre
  while (hi - lo > 1) {
    const int md = (lo + hi) >> 1;
    if (pages[md].gpre <= g) lo = md; else hi = md;
  }
  const HsPqPage pg = pages[lo];
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

int hs_pq_pack(const int32_t* codes, const HsPqPage* pages, int npages, int64_t ngroups, int bw,
               uint8_t* out, void* stream) {
  if (ngroups <= 0) return 0;
  if (bw < 1 || bw > 16) return -1;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hs_pq_pack_kernel, dim3((unsigned)((ngroups + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, codes, pages, npages, ngroups, bw, out);
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
