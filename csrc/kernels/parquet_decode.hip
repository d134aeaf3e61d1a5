// K1: Parquet page decode on the MI355X.
//
// The host page layer (csrc/runtime/hs_parquet.cpp) decompresses pages and cuts every
// RLE/bit-packed hybrid stream into a run table; the page bytes still hold dictionary indices
// at their encoded bit width.  Here one wave expands one run:
//   kind 0  RLE run         -> value (or dict[value]) repeated `count` times
//   kind 1  bit-packed run  -> unpack `bit_width`-bit fields (LSB first), optional dict gather
//   kind 2  PLAIN run       -> element copy
// Value runs write the dense (non-null) value index space; level runs write one validity byte
// per row.  Page data inside the staging buffer is only 16-byte aligned per page and PLAIN
// values can start at any byte (v1 pages put the definition levels first), so every read goes
// through aligned 32-bit loads and funnel shifts — consecutive lanes read consecutive bytes, so
// the dword loads of a wave coalesce.  The buffer carries >= 16 bytes of tail slack.
#include <hip/hip_runtime.h>

#include <cstdint>

struct HsPqRun {
  int64_t dst, count, src;
  int32_t kind, bit_width;
};

// 8 little-endian bytes starting at byte offset `off` of a 4-byte aligned buffer
__device__ __forceinline__ uint64_t load_u64_at(const uint8_t* buf, int64_t off) {
  const uint32_t* w = (const uint32_t*)(buf + (off & ~(int64_t)3));
  const int sh = (int)(off & 3) * 8;
  const uint64_t lo = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  if (sh == 0) return lo;
  const uint64_t hi = w[2];
  return (lo >> sh) | (hi << (64 - sh));
}

__device__ __forceinline__ uint32_t load_u32_at(const uint8_t* buf, int64_t off) {
  const uint32_t* w = (const uint32_t*)(buf + (off & ~(int64_t)3));
  const int sh = (int)(off & 3) * 8;
  if (sh == 0) return w[0];
  return (uint32_t)((((uint64_t)w[1] << 32) | w[0]) >> sh);
}

// i-th `bw`-bit field of a bit-packed run starting at byte `src` (bw <= 32)
__device__ __forceinline__ uint32_t unpack(const uint8_t* buf, int64_t src, int64_t i, int bw) {
  const int64_t bit = i * bw;
  const uint64_t win = load_u64_at(buf, src + (bit >> 3));
  const uint64_t mask = bw == 32 ? 0xffffffffull : ((1ull << bw) - 1);
  return (uint32_t)((win >> (bit & 7)) & mask);
}

template <typename T>
__device__ __forceinline__ T load_elem(const uint8_t* buf, int64_t off);
template <>
__device__ __forceinline__ uint32_t load_elem<uint32_t>(const uint8_t* buf, int64_t off) {
  return load_u32_at(buf, off);
}
template <>
__device__ __forceinline__ uint64_t load_elem<uint64_t>(const uint8_t* buf, int64_t off) {
  return load_u64_at(buf, off);
}

// T: uint32_t (INT32/FLOAT) or uint64_t (INT64/DOUBLE) — values are moved as raw bits
template <typename T>
__global__ __launch_bounds__(256) void hs_pq_values_kernel(
    const uint8_t* __restrict__ buf, const HsPqRun* __restrict__ runs, int64_t nruns,
    int64_t dict_off, int64_t dict_count, T* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nruns) return;
  const int lane = threadIdx.x & 63;
  const HsPqRun run = runs[r];
  T* o = out + run.dst;
  if (run.kind == 2) {
    for (int64_t i = lane; i < run.count; i += 64)
      o[i] = load_elem<T>(buf, run.src + i * (int64_t)sizeof(T));
    return;
  }
  // dictionary pages are 16-byte aligned; indices from a corrupt file must not read past the
  // dictionary, so out-of-range indices decode as 0 instead of faulting
  const T* dict = (const T*)(buf + dict_off);
  if (run.kind == 0) {
    const T v = (uint64_t)run.src < (uint64_t)dict_count ? dict[run.src] : (T)0;
    for (int64_t i = lane; i < run.count; i += 64) o[i] = v;
    return;
  }
  for (int64_t i = lane; i < run.count; i += 64) {
    const uint32_t k = unpack(buf, run.src, i, run.bit_width);
    o[i] = (int64_t)k < dict_count ? dict[k] : (T)0;
  }
}

__global__ __launch_bounds__(256) void hs_pq_levels_kernel(
    const uint8_t* __restrict__ buf, const HsPqRun* __restrict__ runs, int64_t nruns,
    uint8_t* __restrict__ valid) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nruns) return;
  const int lane = threadIdx.x & 63;
  const HsPqRun run = runs[r];
  uint8_t* o = valid + run.dst;
  if (run.kind == 0) {
    const uint8_t v = run.src != 0;
    for (int64_t i = lane; i < run.count; i += 64) o[i] = v;
    return;
  }
  for (int64_t i = lane; i < run.count; i += 64)
    o[i] = (uint8_t)(unpack(buf, run.src, i, run.bit_width) != 0);
}

extern "C" {

// Expand value runs into `out` (elem_bytes 4 or 8).  dict_off < 0: the chunk has no dictionary
// (then every run must be PLAIN).  Returns a HIP error code.
int hs_pq_decode_values(const uint8_t* buf, const HsPqRun* runs, int64_t nruns, int64_t dict_off,
                        int64_t dict_count, int elem_bytes, void* out, void* stream) {
  if (nruns <= 0) return 0;
  // staging worker threads share the thread-local HIP error slot with torch; clear anything
  // stale so the check below reports this launch only
  (void)hipGetLastError();
  const dim3 grid((unsigned)((nruns + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  if (elem_bytes == 4)
    hipLaunchKernelGGL(hs_pq_values_kernel<uint32_t>, grid, dim3(256), 0, s, buf, runs, nruns,
                       dict_off, dict_count, (uint32_t*)out);
  else if (elem_bytes == 8)
    hipLaunchKernelGGL(hs_pq_values_kernel<uint64_t>, grid, dim3(256), 0, s, buf, runs, nruns,
                       dict_off, dict_count, (uint64_t*)out);
  else
    return -1;
  return (int)hipGetLastError();
}

// Load the decode kernels' code objects from the calling thread (empty launches).  HIP loads a
// library's kernels lazily on first launch; doing that once from the main thread keeps the
// first launches of the staging worker threads from racing the load.
int hs_pq_warmup(void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(hs_pq_values_kernel<uint32_t>, dim3(1), dim3(256), 0, s, nullptr, nullptr,
                     (int64_t)0, (int64_t)0, (int64_t)0, (uint32_t*)nullptr);
  hipLaunchKernelGGL(hs_pq_values_kernel<uint64_t>, dim3(1), dim3(256), 0, s, nullptr, nullptr,
                     (int64_t)0, (int64_t)0, (int64_t)0, (uint64_t*)nullptr);
  hipLaunchKernelGGL(hs_pq_levels_kernel, dim3(1), dim3(256), 0, s, nullptr, nullptr, (int64_t)0,
                     (uint8_t*)nullptr);
  return (int)hipStreamSynchronize(s);
}

// Expand definition-level runs (max level 1) into one validity byte per row.
int hs_pq_decode_levels(const uint8_t* buf, const HsPqRun* runs, int64_t nruns, uint8_t* valid,
                        void* stream) {
  if (nruns <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hs_pq_levels_kernel, dim3((unsigned)((nruns + 3) / 4)), dim3(256), 0,
                     (hipStream_t)stream, buf, runs, nruns, valid);
  return (int)hipGetLastError();
}

}  // extern "C"
