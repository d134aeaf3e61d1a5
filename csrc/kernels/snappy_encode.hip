// K4: Snappy compression of index Parquet pages on the MI355X (SURVEY.md §2.3 K4 "Parquet
// encode (+ Snappy)"; the reference writes Spark's default Snappy Parquet,
// DataFrameWriterExtensions.scala:57-66).
//
// The encoded pages (bit-packed dictionary codes or PLAIN values) are still in HBM after
// hs_pq_pack, so they are compressed there and only the compressed bytes cross PCIe.
//
// Work split: every page is cut into chunks of <= 64 KiB; one lane compresses one chunk with the
// greedy Snappy match finder (4-byte hash probe, skip acceleration over incompressible runs,
// copy extension).  A chunk's elements only reference bytes of the same chunk, so the element
// streams of consecutive chunks concatenate into one valid Snappy stream per page (the host
// writer prepends the varint length and the definition-level literal).  Each lane's hash table
// (512 x u16 positions) lives in LDS, interleaved by lane (entry h of lane l at h*64 + l), 64 KiB
// per 64-lane workgroup: two workgroups per CU.  Chunks are written to fixed-size slots
// (hs_snappy_max_compressed), then hs_snappy_pack concatenates the used bytes of every slot at
// host-computed offsets (a workgroup per chunk, dword copies when aligned).
//
// The same match finder is compiled for the host (hs_snappy_compress_host) so CPU tests check
// the element stream against an independent decoder.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kHashBits = 9;
constexpr int kHashSize = 1 << kHashBits;
constexpr int kLanes = 64;
constexpr int kChunk = 1 << 16;
constexpr int kInputMargin = 15;

__host__ __device__ inline uint32_t load32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__host__ __device__ inline uint32_t hash32(uint32_t v) {
  return (v * 0x1e35a7bdu) >> (32 - kHashBits);
}

__host__ __device__ inline uint8_t* emit_literal(uint8_t* op, const uint8_t* src, int n) {
  const uint32_t m = (uint32_t)n - 1;
  if (m < 60) {
    *op++ = (uint8_t)(m << 2);
  } else if (m < (1u << 8)) {
    *op++ = (uint8_t)(60 << 2);
    *op++ = (uint8_t)m;
  } else if (m < (1u << 16)) {
    *op++ = (uint8_t)(61 << 2);
    *op++ = (uint8_t)m;
    *op++ = (uint8_t)(m >> 8);
  } else {
    *op++ = (uint8_t)(62 << 2);
    *op++ = (uint8_t)m;
    *op++ = (uint8_t)(m >> 8);
    *op++ = (uint8_t)(m >> 16);
  }
  for (int i = 0; i < n; ++i) op[i] = src[i];
  return op + n;
}

__host__ __device__ inline uint8_t* emit_copy_le64(uint8_t* op, int offset, int len) {
  if (len < 12 && offset < 2048) {          // 1-byte offset form: len 4..11, offset < 2048
    *op++ = (uint8_t)(1 | ((len - 4) << 2) | ((offset >> 8) << 5));
    *op++ = (uint8_t)offset;
  } else {                                  // 2-byte offset form: len 1..64
    *op++ = (uint8_t)(2 | ((len - 1) << 2));
    *op++ = (uint8_t)offset;
    *op++ = (uint8_t)(offset >> 8);
  }
  return op;
}

__host__ __device__ inline uint8_t* emit_copy(uint8_t* op, int offset, int len) {
  while (len >= 68) {
    op = emit_copy_le64(op, offset, 64);
    len -= 64;
  }
  if (len > 64) {
    op = emit_copy_le64(op, offset, 60);
    len -= 60;
  }
  return emit_copy_le64(op, offset, len);
}

// Snappy elements (no length preamble) of in[0, n), n <= 64 KiB; `tab(h)` is this chunk's hash
// table slot h (positions within the chunk).  Returns the end of the output.
template <typename Tab>
__host__ __device__ uint8_t* compress_chunk(const uint8_t* in, int n, uint8_t* op, Tab tab) {
  for (int h = 0; h < kHashSize; ++h) tab(h) = 0;
  int next_emit = 0;
  if (n >= kInputMargin + 1) {
    const int ip_limit = n - kInputMargin;
    int ip = 1;
    for (;;) {
      int cand;
      uint32_t skip = 32;
      for (;;) {                              // find a 4-byte match
        if (ip > ip_limit) goto done;
        const uint32_t v = load32(in + ip);
        const uint32_t h = hash32(v);
        cand = tab(h);
        tab(h) = (uint16_t)ip;
        if (load32(in + cand) == v) break;
        ip += (int)(skip >> 5);
        ++skip;
      }
      op = emit_literal(op, in + next_emit, ip - next_emit);
      for (;;) {                              // emit copies while matches chain
        int m = 4;
        while (ip + m < n && in[cand + m] == in[ip + m]) ++m;
        op = emit_copy(op, ip - cand, m);
        ip += m;
        next_emit = ip;
        if (ip > ip_limit) goto done;
        tab(hash32(load32(in + ip - 1))) = (uint16_t)(ip - 1);
        const uint32_t v = load32(in + ip);
        const uint32_t h = hash32(v);
        cand = tab(h);
        tab(h) = (uint16_t)ip;
        if (load32(in + cand) != v) break;
      }
      ++ip;
    }
  }
done:
  if (next_emit < n) op = emit_literal(op, in + next_emit, n - next_emit);
  return op;
}

}  // namespace

struct HsSnappyChunk {
  const uint8_t* src;   // device pointer of the chunk's first input byte
  int64_t len;          // 1 .. 65536
};

__global__ __launch_bounds__(kLanes) void hs_snappy_compress_kernel(
    const HsSnappyChunk* __restrict__ chunks, int nchunks, uint8_t* __restrict__ slots,
    int64_t slot_bytes, int32_t* __restrict__ sizes) {
  __shared__ uint16_t tab[kHashSize * kLanes];
  const int lane = threadIdx.x;
  const int c = blockIdx.x * kLanes + lane;
  if (c >= nchunks) return;
  const HsSnappyChunk ch = chunks[c];
  uint8_t* out = slots + (int64_t)c * slot_bytes;
  uint16_t* t = tab + lane;
  uint8_t* end = compress_chunk(ch.src, (int)ch.len, out,
                                [t](int h) -> uint16_t& { return t[h * kLanes]; });
  sizes[c] = (int32_t)(end - out);
}

__global__ __launch_bounds__(256) void hs_snappy_pack_kernel(const uint8_t* __restrict__ slots,
                                                             int64_t slot_bytes,
                                                             const int32_t* __restrict__ sizes,
                                                             const int64_t* __restrict__ dst_off,
                                                             uint8_t* __restrict__ out) {
  const int c = blockIdx.x;
  const int n = sizes[c];
  const uint8_t* s = slots + (int64_t)c * slot_bytes;
  uint8_t* d = out + dst_off[c];
  if ((((uintptr_t)d) & 3) == 0) {            // slots are 16-byte aligned: dword copies
    const int nw = n >> 2;
    const uint32_t* s4 = (const uint32_t*)s;
    uint32_t* d4 = (uint32_t*)d;
    for (int i = threadIdx.x; i < nw; i += blockDim.x) d4[i] = s4[i];
    for (int i = (nw << 2) + threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
  } else {
    for (int i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
  }
}

extern "C" {

// worst-case element bytes of one chunk of `n` input bytes (Snappy's 32 + n + n/6 bound),
// rounded to 16 bytes so every slot stays aligned
int64_t hs_snappy_max_compressed(int64_t n) { return ((32 + n + n / 6) + 15) & ~(int64_t)15; }

int hs_snappy_chunk_bytes() { return kChunk; }

int hs_snappy_compress(const HsSnappyChunk* chunks, int nchunks, uint8_t* slots,
                       int64_t slot_bytes, int32_t* sizes, void* stream) {
  if (nchunks <= 0) return 0;
  if (slot_bytes < hs_snappy_max_compressed(kChunk)) return -1;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hs_snappy_compress_kernel, dim3((unsigned)((nchunks + kLanes - 1) / kLanes)),
                     dim3(kLanes), 0, (hipStream_t)stream, chunks, nchunks, slots, slot_bytes,
                     sizes);
  return (int)hipGetLastError();
}

int hs_snappy_pack(const uint8_t* slots, int64_t slot_bytes, const int32_t* sizes,
                   const int64_t* dst_off, int nchunks, uint8_t* out, void* stream) {
  if (nchunks <= 0) return 0;
  (void)hipGetLastError();
  hipLaunchKernelGGL(hs_snappy_pack_kernel, dim3((unsigned)nchunks), dim3(256), 0,
                     (hipStream_t)stream, slots, slot_bytes, sizes, dst_off, out);
  return (int)hipGetLastError();
}

// host build of the same match finder: elements of in[0, n) (n <= 64 KiB) into out (at least
// hs_snappy_max_compressed(n) bytes); returns the element byte count, or -1
int64_t hs_snappy_compress_host(const uint8_t* in, int64_t n, uint8_t* out) {
  if (n < 0 || n > kChunk) return -1;
  static thread_local uint16_t tab[kHashSize];
  uint8_t* end = compress_chunk(in, (int)n, out, [](int h) -> uint16_t& { return tab[h]; });
  return (int64_t)(end - out);
}

}  // extern "C"
