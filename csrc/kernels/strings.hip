// String values addressed by (device address, length) pairs - the output of the PLAIN
// BYTE_ARRAY page expansion (parquet_decode.hip, eb-16 pages) - turned into dictionary codes
// without a host decode (io/native_parquet.StringCodes.finish_plain):
//
//   hs_str_hash64   one 64-bit hash per value (8-byte words, then a 64-bit finalizer);
//   hs_str_gather   the bytes of selected values packed back to back (the distinct values'
//                   representatives, copied to the host as the dictionary);
//   hs_str_differ   per value, whether its bytes differ from another value's (each value vs
//                   the representative of its hash: catches hash collisions exactly).
//
// One lane per value: the values of an index column are short (TPC-H / TPC-DS dimension
// strings: 1-30 bytes), so a lane's byte loop is short and the wavefront's loads of neighbouring
// values touch neighbouring bytes of the page.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

__device__ __forceinline__ uint64_t mix64(uint64_t h) {
  h ^= h >> 33;
  h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  return h ^ (h >> 33);
}

// little-endian word of up to 8 bytes at an unaligned address
__device__ __forceinline__ uint64_t load_bytes(const uint8_t* p, int n) {
  uint64_t w = 0;
  for (int i = 0; i < n; ++i) w |= (uint64_t)p[i] << (8 * i);
  return w;
}

__global__ __launch_bounds__(256) void hs_str_hash64_kernel(const uint64_t* __restrict__ ptr,
                                                            const int32_t* __restrict__ len,
                                                            int64_t n, uint64_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t* p = (const uint8_t*)(uintptr_t)ptr[i];
    const int l = len[i] > 0 ? len[i] : 0;
    uint64_t h = 0x9e3779b97f4a7c15ull ^ ((uint64_t)l * 0x2545f4914f6cdd1dull);
    int k = 0;
    for (; k + 8 <= l; k += 8) h = mix64(h ^ load_bytes(p + k, 8)) + 0x632be59bd9b4e019ull;
    if (k < l) h = mix64(h ^ load_bytes(p + k, l - k) ^ 0x8cb92ba72f3d8dd7ull);
    out[i] = mix64(h);
  }
}

__global__ __launch_bounds__(256) void hs_str_gather_kernel(const uint64_t* __restrict__ ptr,
                                                            const int32_t* __restrict__ len,
                                                            const int64_t* __restrict__ off,
                                                            int64_t n, uint8_t* __restrict__ out) {
  // one wavefront per value: its bytes are copied by the 64 lanes
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t i = wid; i < n; i += nw) {
    const uint8_t* p = (const uint8_t*)(uintptr_t)ptr[i];
    const int l = len[i] > 0 ? len[i] : 0;
    uint8_t* o = out + off[i];
    for (int k = lane; k < l; k += 64) o[k] = p[k];
  }
}

__global__ __launch_bounds__(256) void hs_str_differ_kernel(
    const uint64_t* __restrict__ a, const int32_t* __restrict__ alen,
    const uint64_t* __restrict__ b, const int32_t* __restrict__ blen, int64_t n,
    uint8_t* __restrict__ diff) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int l = alen[i];
    uint8_t d = l != blen[i];
    if (!d && l > 0) {
      const uint8_t* p = (const uint8_t*)(uintptr_t)a[i];
      const uint8_t* q = (const uint8_t*)(uintptr_t)b[i];
      if (p != q)
        for (int k = 0; k < l; ++k)
          if (p[k] != q[k]) { d = 1; break; }
    }
    diff[i] = d;
  }
}

unsigned grid_for(int64_t n, int per_block) {
  const int64_t g = (n + per_block - 1) / per_block;
  return (unsigned)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

}  // namespace

extern "C" {

int hs_str_hash64(const uint64_t* ptr, const int32_t* len, int64_t n, uint64_t* out,
                  void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(hs_str_hash64_kernel, dim3(grid_for(n, 256)), dim3(256), 0,
                     (hipStream_t)stream, ptr, len, n, out);
  return (int)hipGetLastError();
}

int hs_str_gather(const uint64_t* ptr, const int32_t* len, const int64_t* off, int64_t n,
                  uint8_t* out, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(hs_str_gather_kernel, dim3(grid_for(n, 4)), dim3(256), 0,
                     (hipStream_t)stream, ptr, len, off, n, out);
  return (int)hipGetLastError();
}

int hs_str_differ(const uint64_t* a, const int32_t* alen, const uint64_t* b,
                  const int32_t* blen, int64_t n, uint8_t* diff, void* stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(hs_str_differ_kernel, dim3(grid_for(n, 256)), dim3(256), 0,
                     (hipStream_t)stream, a, alen, b, blen, n, diff);
  return (int)hipGetLastError();
}

}  // extern "C"
