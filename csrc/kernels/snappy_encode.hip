// K4: Snappy compression of index Parquet pages on the MI355X (SURVEY.md §2.3 K4 "Parquet
// encode (+ Snappy)"; the reference writes Spark's default Snappy Parquet,
// DataFrameWriterExtensions.scala:57-66).
//
// The encoded pages (bit-packed dictionary codes or PLAIN values) are still in HBM after
// hs_pq_pack, so they are compressed there and only the compressed bytes cross PCIe.
//
// Work split: every page is cut into chunks of <= 64 KiB and one wavefront compresses one chunk
// (hs_snappy_compress_kernel below: 64 positions hashed and probed per step, ballots pick the
// greedy match, matches extend 64 bytes per step); its 4096-entry u16 hash table lives in LDS
// (8 KiB per wave, 4 waves per workgroup).  A chunk's elements only reference bytes of the same
// chunk, so the element streams of consecutive chunks concatenate into one valid Snappy stream
// per page (the host writer prepends the varint length and the definition-level literal).
// Chunks are written to fixed-size slots (hs_snappy_max_compressed), then hs_snappy_pack
// concatenates the used bytes of every slot at host-computed offsets (a workgroup per chunk,
// dword copies when aligned).
//
// A first version gave each lane its own chunk (serial greedy finder, 512-entry table per lane):
// 64 KiB of LDS per 64 lanes left ~24 waves on the chip per 96 MB batch and ran at ~1.2 GB/s
// (profiles/kernel_stats_sf100_r2_snappy_lane.csv).  That serial finder remains as the host
// compressor (hs_snappy_compress_host: dictionary pages, CPU tests).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kHashBits = 12;
constexpr int kHashSize = 1 << kHashBits;
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
  int64_t len;          // 0 .. 65536
};

namespace {

constexpr int kWaveHashBits = 12;
constexpr int kWaveHashSize = 1 << kWaveHashBits;
constexpr int kWavesPerBlock = 4;
constexpr uint16_t kNone = 0xFFFF;

__device__ inline uint32_t hash_wave(uint32_t v) { return (v * 0x1e35a7bdu) >> (32 - kWaveHashBits); }

__device__ inline uint8_t* wave_literal(uint8_t* op, const uint8_t* src, int n, int lane) {
  const uint32_t m = (uint32_t)n - 1;
  const int h = m < 60 ? 1 : (m < (1u << 8) ? 2 : (m < (1u << 16) ? 3 : 4));
  if (lane < h)   // tag (length in the tag, or 60..62 + 1..3 little-endian length bytes)
    op[lane] = lane == 0 ? (uint8_t)((h == 1 ? m : (uint32_t)(58 + h)) << 2)
                         : (uint8_t)(m >> (8 * (lane - 1)));
  for (int i = lane; i < n; i += 64) op[h + i] = src[i];
  return op + h + n;
}

__device__ inline uint8_t* wave_copy(uint8_t* op, int offset, int len, int lane) {
  // uniform element sequence; lane 0 stores the tags
  while (len > 0) {
    const int piece = len >= 68 ? 64 : (len > 64 ? 60 : len);
    if (lane == 0) emit_copy_le64(op, offset, piece);
    op += (piece < 12 && offset < 2048) ? 2 : 3;
    len -= piece;
  }
  return op;
}

}  // namespace

// One wavefront per chunk.  Every step takes the 64 positions [ip, ip + 64): each lane hashes
// its position's 4 bytes and probes the wave's LDS hash table (positions from earlier steps
// only, so every candidate precedes it), a ballot picks the first lane with a verified 4-byte
// match, the wave emits the pending literal and extends the match 64 bytes per step (ballot on
// the first mismatching byte), and all probed positions up to the match enter the table.
// Decisions are wave-uniform; lanes only parallelise hashing, probing, copying and comparing.
__global__ __launch_bounds__(64 * kWavesPerBlock) void hs_snappy_compress_kernel(
    const HsSnappyChunk* __restrict__ chunks, int nchunks, uint8_t* __restrict__ slots,
    int64_t slot_bytes, int32_t* __restrict__ sizes) {
  __shared__ uint16_t tabs[kWavesPerBlock][kWaveHashSize];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int c = blockIdx.x * kWavesPerBlock + w;
  if (c >= nchunks) return;
  uint16_t* tab = tabs[w];
  for (int i = lane; i < kWaveHashSize; i += 64) tab[i] = kNone;
  __builtin_amdgcn_wave_barrier();
  const HsSnappyChunk ch = chunks[c];
  const uint8_t* in = ch.src;
  const int n = (int)ch.len;
  uint8_t* const out0 = slots + (int64_t)c * slot_bytes;
  uint8_t* op = out0;
  int next_emit = 0;
  const int ip_limit = n - 4;       // last position with 4 readable bytes
  int ip = 0;
  while (ip <= ip_limit) {
    const int pos = ip + lane;
    const bool ok = pos <= ip_limit;
    uint32_t v = 0, h = 0;
    int cand = kNone;
    if (ok) {
      v = load32(in + pos);
      h = hash_wave(v);
      cand = tab[h];
    }
    const bool hit = ok && cand != kNone && load32(in + cand) == v;
    const uint64_t mask = __ballot(hit);
    __builtin_amdgcn_wave_barrier();
    if (mask == 0) {
      if (ok) tab[h] = (uint16_t)pos;
      __builtin_amdgcn_wave_barrier();
      ip += 64;
      continue;
    }
    const int m = __ffsll((unsigned long long)mask) - 1;
    if (ok && lane <= m) tab[h] = (uint16_t)pos;
    __builtin_amdgcn_wave_barrier();
    const int mpos = ip + m;
    const int mcand = __shfl(cand, m);
    if (mpos > next_emit) op = wave_literal(op, in + next_emit, mpos - next_emit, lane);
    int len = 4;
    for (;;) {                                // extend 64 bytes per step
      const int a = mpos + len + lane;
      const bool eq = a < n && in[mcand + len + lane] == in[a];
      const uint64_t miss = __ballot(!eq);
      if (miss) {
        len += __ffsll((unsigned long long)miss) - 1;
        break;
      }
      len += 64;
    }
    op = wave_copy(op, mpos - mcand, len, lane);
    ip = mpos + len;
    next_emit = ip;
  }
  if (next_emit < n) op = wave_literal(op, in + next_emit, n - next_emit, lane);
  if (lane == 0) sizes[c] = (int32_t)(op - out0);
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
  hipLaunchKernelGGL(hs_snappy_compress_kernel,
                     dim3((unsigned)((nchunks + kWavesPerBlock - 1) / kWavesPerBlock)),
                     dim3(64 * kWavesPerBlock), 0, (hipStream_t)stream, chunks, nchunks, slots,
                     slot_bytes, sizes);
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
