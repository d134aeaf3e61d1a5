// K4: Snappy compression of index Parquet pages on the MI355X (SURVEY.md §2.3 K4 "Parquet
// encode (+ Snappy)"; the reference writes Spark's default Snappy Parquet,
// DataFrameWriterExtensions.scala:57-66).
//
// The encoded pages (bit-packed dictionary codes or PLAIN values) are still in HBM after
// hs_pq_pack, so they are compressed there and only the compressed bytes cross PCIe.
//
// Work split: every page is cut into chunks of <= 64 KiB and one wavefront compresses one chunk
// (hs_snappy_compress_kernel below: 64 positions hashed and probed per step, ballots pick the
// greedy match, matches extend 64 bytes per step); its 2048-entry u16 hash table lives in LDS
// (4 KiB per wave, 4 waves per workgroup).  A chunk's elements only reference bytes of the same
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

constexpr int kWaveHashBits = 11;   // 4 KiB per wave: 10 waves per SIMD
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

// 4 bytes at p from aligned dword loads (a funnel shift joins the two words); p's aligned
// word is inside the buffer, and the second word is only read when p is unaligned, i.e. when
// it holds bytes p..p+3 needs
__device__ inline uint32_t load4(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t s = (uint32_t)(a & 3);
  const uint32_t lo = w[0];
  if (s == 0) return lo;
  return (uint32_t)((((uint64_t)w[1] << 32) | lo) >> (8u * s));   // v_alignbit_b32
}

// bytes p .. p+19 as five little-endian words from six aligned dword loads (p + 24 must be
// inside the buffer)
__device__ inline void load20(const uint8_t* p, uint32_t r[5]) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* w = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t s = 8u * (uint32_t)(a & 3);
  uint32_t x[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) x[k] = w[k];
#pragma unroll
  for (int k = 0; k < 5; ++k) r[k] = (uint32_t)((((uint64_t)x[k + 1] << 32) | x[k]) >> s);
}

// literal of the window bytes [a, b) held one per lane (b - a <= 64)
__device__ inline uint8_t* wave_literal_regs(uint8_t* op, uint32_t byte, int a, int b, int lane) {
  const int m = b - a - 1;
  const int h = m < 60 ? 1 : 2;
  if (lane == 0) {
    op[0] = (uint8_t)((m < 60 ? m : 60) << 2);
    if (h == 2) op[1] = (uint8_t)m;
  }
  if (lane >= a && lane < b) op[h + lane - a] = (uint8_t)byte;
  return op + h + (b - a);
}

// One wavefront per chunk, one window of 64 positions [ip, ip + 64) per step:
//   1. every lane loads its position's 4 bytes (aligned dword loads), hashes them and probes the
//      wave's LDS table (positions of earlier windows only, so candidates always precede);
//   2. lanes with a candidate verify it and measure their own match length (dword compares,
//      capped at 64 bytes) -- all in parallel, no serial dependence between positions;
//   3. the greedy parse of the window runs on wave-uniform values only: first matching lane at or
//      after the cursor -> literal of the bytes before it (straight from the lanes' registers) +
//      copy, cursor jumps past the match, repeat; a match may run past the window;
//   4. probed positions before the cursor enter the table and the next window starts there.
// Literals are emitted per window (<= 64 bytes, 1-2 byte tag), so no byte is ever re-read for
// output and each window costs two dependent memory round trips whatever its match count.
// (The first wave design emitted one greedy match per step, with a literal copy and a serial
// extension in between: 22 GB/s on sorted int64 keys, profiles/kernel_stats_build_r2_snappy_v2.csv.)
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
  int ip = 0;
  while (ip < n) {
    const int pos = ip + lane;
    const bool probe = pos <= n - 4;
    const bool fast = pos + 28 <= n;       // 20 bytes at pos and at any candidate < pos
    uint32_t pv[5];
    uint32_t v = 0, h = 0;
    int cand = kNone, len = 0;
    if (fast) {
      load20(in + pos, pv);
      v = pv[0];
    } else if (probe) {
      v = load4(in + pos);
    } else if (pos < n) {
      v = in[pos];
    }
    if (probe) {
      h = hash_wave(v);
      cand = tab[h];
    }
    if (cand != kNone) {
      if (fast) {                          // verify + first 20 bytes in one round trip
        uint32_t cv[5];
        load20(in + cand, cv);
        if (cv[0] == v) {
          len = 20;
#pragma unroll
          for (int k = 4; k >= 1; --k) {
            const uint32_t x = cv[k] ^ pv[k];
            if (x) len = 4 * k + (__builtin_ctz(x) >> 3);
          }
        }
      } else if (load4(in + cand) == v) {
        len = 4;
      }
      if (len == 20 || (len == 4 && !fast)) {   // longer matches: 4 bytes per step
        while (len < 64 && pos + len + 4 <= n) {
          const uint32_t x = load4(in + pos + len) ^ load4(in + cand + len);
          if (x) {
            len += __builtin_ctz(x) >> 3;
            break;
          }
          len += 4;
        }
        if (len > 64) len = 64;
        while (len < 64 && pos + len < n && in[cand + len] == in[pos + len]) ++len;
      }
    }
    const uint64_t hit = __ballot(len >= 4);
    const int wv = n - ip < 64 ? n - ip : 64;
    int cur = 0;
    while (cur < wv) {
      const uint64_t avail = hit & (~0ull << cur);
      if (avail == 0) {
        op = wave_literal_regs(op, v, cur, wv, lane);
        cur = wv;
        break;
      }
      const int m = __ffsll((unsigned long long)avail) - 1;
      if (m > cur) op = wave_literal_regs(op, v, cur, m, lane);
      const int ml = __shfl(len, m);
      const int mc = __shfl(cand, m);
      op = wave_copy(op, ip + m - mc, ml, lane);
      cur = m + ml;
    }
    __builtin_amdgcn_wave_barrier();
    if (probe && lane < cur) tab[h] = (uint16_t)pos;
    __builtin_amdgcn_wave_barrier();
    ip += cur;
  }
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
