// K1: Parquet page decode on the MI355X.  Two paths:
//   * device pages (hs_pq_decode_pages, below): raw compressed pages in, values out — Snappy,
//     RLE/bit-packed parsing and dictionary expansion all on the GPU;
//   * host run tables (hs_pq_decode_values / _levels): for chunks with nulls.
//
// Host run tables: the host page layer (csrc/runtime/hs_parquet.cpp) decompresses pages and cuts every
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

// ------------------------------------------------------------------------------------------------
// Device-resident page decode (no host decompression or run tables): the host preads the raw
// column chunks and lists their pages (csrc/runtime/hs_parquet.cpp hs_pq_plan_chunk); here
//   hs_pq_inflate_kernel  one wavefront per page: Snappy (or a copy) into the scratch buffer;
//   hs_pq_expand_kernel   one workgroup per data page: RLE / bit-packed dictionary indices or
//                         PLAIN values straight into the destination column.
// Two launches per source file instead of one per run batch of every chunk.
// dst: device address of the decompressed page (the caller turns the planner's scratch offsets
// into addresses; host-inflated pages, codec 2, point at their own device copy)
struct HsPqPage {
  int64_t src, dst, out, dict, row;
  int32_t csize, usize, nvals, codec, kind, enc, levels, eb, dict_page, nulls;
  int64_t valid;   // nulls != 0: device address of the page's first validity byte
};

enum : int { kErrCorrupt = 1, kErrDictRange = 2 };

// input bytes one wavefront parses per Snappy batch (up to 64 tags); LDS per workgroup scales
// with it (profiles/build_sweep_inflate_r3.jsonl)
#ifndef HS_SNAPPY_WIN
#define HS_SNAPPY_WIN 128
#endif

// Snappy raw-block decompression by one wavefront (input at byte offset `ib` of the 4-byte
// aligned buffer `base`, `n` bytes; output `out`, `cap` bytes).
//
// Tag parsing is data-parallel.  Each batch looks at a 512-byte window of the input: every
// lane speculatively decodes a tag at each of its 8 window offsets (length, source and the
// offset of the following tag), then pointer-jumping tables over "next tag" (6 rounds) give
// every lane j the position of the j-th tag after the window start, so up to 64 real tags
// are found in O(log) LDS steps instead of one dependent step per tag.  Then
//   1. literal bytes are copied byte-parallel over the batch (a batch that is one long literal,
//      as on incompressible pages, with aligned dword stores: two aligned loads and a funnel
//      shift per lane, four dwords in flight per lane);
//   2. copy bytes are resolved byte-parallel from output that is already final: a byte whose
//      source lies in an earlier batch or in a literal of this batch is read directly; a source
//      inside another copy of this batch follows that copy back (a run of copies with one
//      offset — RLE-like data — is one overlapping copy, left by a modulo), so every step moves
//      to an earlier tag.
// A fence between the passes and between batches makes the wavefront's stores visible to its
// later loads.
__device__ void snappy_wave(const uint8_t* __restrict__ base, int64_t ib, int n,
                            uint8_t* __restrict__ out, int cap, int w, int lane,
                            int* __restrict__ status) {
  constexpr int WIN = HS_SNAPPY_WIN, PER = WIN / 64, LOGT = 6;
  // pointer-jumping tables (2^k-th following tag; window offsets fit 16 bits): 6 KB per
  // wavefront instead of 12, so three workgroups fit a CU instead of two
  __shared__ short s_next[4][LOGT][WIN];
  __shared__ int s_skip[4][WIN];         // exact successor offset (a literal may jump far)
  __shared__ int s_len[4][WIN];          // speculative tag at each window offset: output bytes
  __shared__ int s_srcw[4][WIN];         //   and source (literal: input offset, copy: -offset)
  __shared__ uint8_t s_win[4][WIN + 8];
  __shared__ int s_start[4][65];
  __shared__ int s_src[4][64];
  __shared__ int s_root[4][64];          // output start of the tag's same-offset copy run
  const uint8_t* in = base + ib;
  int ip = 0;
  uint32_t len = 0;
  for (int shift = 0; ip < n && shift <= 28; shift += 7) {
    const uint8_t b = in[ip++];
    len |= (uint32_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) break;
  }
  if ((int)len != cap) { if (lane == 0) atomicOr(status, kErrCorrupt); return; }
  auto wsync = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  int op = 0;
  while (ip < n) {
#pragma unroll
    for (int k = 0; k < PER + 1; ++k) {
      const int x = lane * PER + k;
      if (x < WIN + 8) s_win[w][x] = ip + x < n ? in[ip + x] : 0;
    }
    wsync();
    // speculative decode at every window offset
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = lane * PER + k;
      const uint8_t* h = s_win[w] + i;
      const int tag = h[0], kind = tag & 3;
      int hl, l, src, ok = 1;
      if (kind == 0) {
        l = tag >> 2;
        hl = 1;
        if (l >= 60) {
          const int nb = l - 59;
          l = 0;
          for (int b = 0; b < nb; ++b) l |= (int)h[1 + b] << (8 * b);
          hl += nb;
        }
        l += 1;
        src = ip + i + hl;
        if (l <= 0) ok = 0;
      } else if (kind == 1) {
        l = 4 + ((tag >> 2) & 7); src = -(((tag >> 5) << 8) | h[1]); hl = 2;
      } else if (kind == 2) {
        l = 1 + (tag >> 2); src = -(h[1] | (h[2] << 8)); hl = 3;
      } else {
        l = 1 + (tag >> 2);
        src = -(h[1] | (h[2] << 8) | (h[3] << 16) | ((int)h[4] << 24));
        hl = 5;
      }
      // a header must lie inside the window (and the input): otherwise the offset absorbs
      ok = ok && i + hl <= WIN && ip + i + hl <= n;
      s_len[w][i] = l;
      s_srcw[w][i] = src;
      // a target beyond the window saturates at WIN (16 bits): only "< WIN" is ever tested,
      // except the last real tag's successor, kept exactly in s_skip
      const int nx = ok ? i + hl + (kind == 0 ? l : 0) : i;
      s_next[w][0][i] = (short)(nx < WIN ? nx : WIN);
      s_skip[w][i] = nx;
    }
    wsync();
    for (int t = 1; t < LOGT; ++t) {
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = lane * PER + k;
        const int a = s_next[w][t - 1][i];
        s_next[w][t][i] = (short)(a < WIN ? s_next[w][t - 1][a] : a);
      }
      wsync();
    }
    // lane j: position of the j-th tag of the batch
    int pos = 0;
#pragma unroll
    for (int t = 0; t < LOGT; ++t)
      if ((lane >> t) & 1) pos = pos < WIN ? s_next[w][t][pos] : pos;
    const bool real = pos < WIN && s_next[w][0][pos] != pos && ip + pos < n;
    const uint64_t rm = __ballot(real);
    const int cnt = rm == ~0ull ? 64 : __ffsll((long long)~rm) - 1;   // leading decodable tags
    if (cnt == 0) { if (lane == 0) atomicOr(status, kErrCorrupt); return; }
    const bool mine = lane < cnt;
    int l = mine ? s_len[w][pos] : 0;
    const int src = mine ? s_srcw[w][pos] : 0;
    // exclusive scan of the tag lengths -> output starts
    int incl = l;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    const int st = incl - l;
    const int total = __shfl(incl, cnt - 1, 64);
    const int nextpos = __shfl(mine ? s_skip[w][pos] : 0, cnt - 1, 64);
    // a copy may not reach before the output start; literals must end inside the input
    const bool bad = mine && (src < 0 ? (-src > op + st) : (src + l > n));
    if (__ballot(bad) != 0ull || op + total > cap) {
      if (lane == 0) atomicOr(status, kErrCorrupt);
      return;
    }
    const int prev = __shfl_up(src, 1, 64);
    const bool head = !(src < 0 && lane > 0 && prev == src);
    const uint64_t heads = __ballot(mine && head);
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int hl = 63 - __clzll((long long)(heads & upto));
    const int root = __shfl(st, hl < 0 ? 0 : hl, 64);
    if (mine) {
      s_start[w][lane] = st;
      s_src[w][lane] = src;
      s_root[w][lane] = root;
    }
    if (lane == 0) s_start[w][cnt] = total;
    wsync();
    ip += nextpos;
    // 1. literal bytes
    if (cnt == 1 && s_src[w][0] >= 0) {
      const int d0 = op, ll = total;
      const int64_t sabs = ib + s_src[w][0];
      const int mis = (int)((uintptr_t)out & 3);     // aligned in absolute address
      const int wa = ((d0 + mis) & ~3) - mis;
      const int nw = (d0 + ll - wa + 3) >> 2;
#pragma unroll 4
      for (int j = lane; j < nw; j += 64) {
        const int x = wa + 4 * j;
        if (x >= d0 && x + 4 <= d0 + ll) {
          *(uint32_t*)(out + x) = load_u32_at(base, sabs + (x - d0));
        } else {
          for (int y = x; y < x + 4; ++y)
            if (y >= d0 && y < d0 + ll) out[y] = base[sabs + (y - d0)];
        }
      }
    } else {
#pragma unroll 2
      for (int b = lane; b < total; b += 64) {
        int lo = 0, hi = cnt - 1;
        while (lo < hi) {
          const int m = (lo + hi + 1) >> 1;
          if (s_start[w][m] <= b) lo = m; else hi = m - 1;
        }
        const int sr = s_src[w][lo];
        if (sr >= 0) out[op + b] = base[ib + sr + (b - s_start[w][lo])];
      }
    }
    // the wavefront's own global stores must be visible to its own later loads: a
    // workgroup-scope fence (same CU) instead of a device-wide one
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    // 2. copy bytes
#pragma unroll 2
    for (int b = lane; b < total; b += 64) {
      int cur = 0, hi = cnt - 1;
      while (cur < hi) {
        const int m = (cur + hi + 1) >> 1;
        if (s_start[w][m] <= b) cur = m; else hi = m - 1;
      }
      if (s_src[w][cur] >= 0) continue;
      int p2 = b, q;
      for (;;) {
        const int off = -s_src[w][cur];
        const int cst = s_root[w][cur];
        q = p2 - off;
        if (q >= cst) q = cst - off + (p2 - cst) % off;
        if (q < 0) break;
        int lo = 0, h2 = cur - 1;
        while (lo < h2) {
          const int m = (lo + h2 + 1) >> 1;
          if (s_start[w][m] <= q) lo = m; else h2 = m - 1;
        }
        if (s_src[w][lo] >= 0) break;
        p2 = q;
        cur = lo;
      }
      out[op + b] = out[op + q];
    }
    // the wavefront's own global stores must be visible to its own later loads: a
    // workgroup-scope fence (same CU) instead of a device-wide one
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    op += total;
  }
  if (op != cap && lane == 0) atomicOr(status, kErrCorrupt);
}

__global__ __launch_bounds__(256) void hs_pq_inflate_kernel(
    const uint8_t* __restrict__ raw, uint8_t* __restrict__ scratch,
    const HsPqPage* __restrict__ pages, int npages, int* __restrict__ status) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pi = blockIdx.x * 4 + w;
  if (pi >= npages) return;               // wavefront-local from here on: no block barriers
  const HsPqPage p = pages[pi];
  if (p.codec == 2) return;               // inflated on the host (dst = its device copy)
  // raw == nullptr: the page table of a batched launch carries absolute source addresses
  const uint8_t* in = (const uint8_t*)((uintptr_t)raw + (uintptr_t)p.src);
  uint8_t* out = (uint8_t*)p.dst;
  const int lv = p.kind == 1 ? p.levels : 0;   // v2: level streams stored uncompressed first
  if (lv > p.csize || lv > p.usize) { if (lane == 0) atomicOr(status, kErrCorrupt); return; }
  for (int i = lane; i < lv; i += 64) out[i] = in[i];
  if (p.codec == 0) {
    for (int i = lv + lane; i < p.csize; i += 64) out[i] = in[i];
    return;
  }
  snappy_wave(in, lv, p.csize - lv, out + lv, p.usize - lv, w, lane, status);
}

template <typename T>
__device__ void expand_page(const HsPqPage& p, const uint8_t* __restrict__ pg,
                            const HsPqPage* __restrict__ pages, int nv, int* __restrict__ status) {
  __shared__ int r_start[129];
  __shared__ int64_t r_src[128];
  __shared__ int r_kind[128];
  __shared__ int r_meta[3];           // runs, next stream position, error
  T* out = (T*)p.out;
  const int n = p.usize;
  int voff = 0;
  if (p.kind == 0 && p.levels) voff = 4 + (int)load_u32_at(pg, 0);
  else if (p.kind == 1) voff = p.levels;
  if (voff < 0 || voff > n) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
  if (p.enc == 0) {                   // PLAIN
    if ((int64_t)nv * (int64_t)sizeof(T) > n - voff) {
      if (threadIdx.x == 0) atomicOr(status, kErrCorrupt);
      return;
    }
    for (int i = threadIdx.x; i < nv; i += blockDim.x)
      out[i] = load_elem<T>(pg, voff + (int64_t)i * (int64_t)sizeof(T));
    return;
  }
  // dictionary indices: bit width byte, then the RLE / bit-packed hybrid stream
  if (n - voff < 1 || p.dict_page < 0) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
  const int bw = pg[voff];
  if (bw > 32) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
  const int64_t s0 = voff + 1, send = n;
  const T* dict = (const T*)p.dict;
  const int64_t dcount = pages[p.dict_page].nvals;
  const int vbytes = (bw + 7) / 8;
  int64_t pos = s0;
  int done = 0;
  while (done < nv) {
    if (threadIdx.x == 0) {
      int k = 0, acc = 0, err = 0;
      int64_t q = pos;
      while (k < 128 && done + acc < nv) {
        uint64_t h = 0;
        int shift = 0;
        for (;;) {
          if (q >= send || shift > 35) { err = 1; break; }
          const uint8_t b = pg[q++];
          h |= (uint64_t)(b & 0x7f) << shift;
          if (!(b & 0x80)) break;
          shift += 7;
        }
        if (err) break;
        const int left = nv - done - acc;
        if (h & 1) {
          const int64_t groups = (int64_t)(h >> 1);
          const int64_t nbytes = groups * bw;
          if (q + nbytes > send) { err = 1; break; }
          const int64_t take = groups * 8 < left ? groups * 8 : left;
          r_kind[k] = 1;
          r_src[k] = q;
          r_start[k] = acc;
          acc += (int)take;
          q += nbytes;
        } else {
          const int64_t cnt = (int64_t)(h >> 1);
          if (q + vbytes > send) { err = 1; break; }
          uint64_t v = 0;
          for (int i = 0; i < vbytes; ++i) v |= (uint64_t)pg[q + i] << (8 * i);
          q += vbytes;
          if (cnt == 0) continue;
          r_kind[k] = 0;
          r_src[k] = (int64_t)v;
          r_start[k] = acc;
          acc += (int)(cnt < left ? cnt : left);
        }
        ++k;
      }
      r_start[k] = acc;
      r_meta[0] = k;
      r_meta[2] = err || (k == 0 && done < nv);
      pos = q;
    }
    __syncthreads();
    const int k = r_meta[0];
    const int err = r_meta[2];
    const int total = r_start[k];
    if (err) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
      int lo = 0, hi = k - 1;
      while (lo < hi) {
        const int m = (lo + hi + 1) >> 1;
        if (r_start[m] <= i) lo = m; else hi = m - 1;
      }
      uint32_t idx;
      if (r_kind[lo] == 0) {
        idx = (uint32_t)r_src[lo];
      } else {
        const int64_t bit = (int64_t)(i - r_start[lo]) * bw;
        const uint64_t win = load_u64_at(pg, r_src[lo] + (bit >> 3));
        const uint64_t mask = bw == 32 ? 0xffffffffull : ((1ull << bw) - 1);
        idx = (uint32_t)((win >> (bit & 7)) & mask);
      }
      T v = (T)0;
      if ((int64_t)idx < dcount) v = dict[idx];
      else atomicOr(status, kErrDictRange);
      out[done + i] = v;
    }
    __syncthreads();
    done += total;
  }
}

// BOOLEAN data page -> one byte (0 / 1) per value.  PLAIN: bit-packed LSB first; RLE (enc 3):
// a 4-byte length, then the RLE / bit-packed hybrid stream at bit width 1.  Runs are resolved
// per 64-value slice by one lane each (a run header is at most a few bytes), so the whole
// workgroup writes values.
__device__ void expand_bool(const HsPqPage& p, const uint8_t* __restrict__ pg, int nv,
                            int* __restrict__ status) {
  uint8_t* out = (uint8_t*)p.out;
  const int n = p.usize;
  int voff = 0;
  if (p.kind == 0 && p.levels) voff = 4 + (int)load_u32_at(pg, 0);
  else if (p.kind == 1) voff = p.levels;
  if (voff < 0 || voff > n) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
  if (p.enc == 0) {
    if ((nv + 7) / 8 > n - voff) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
    for (int i = threadIdx.x; i < nv; i += blockDim.x)
      out[i] = (uint8_t)((pg[voff + (i >> 3)] >> (i & 7)) & 1);
    return;
  }
  if (n - voff < 4) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
  const int64_t len = (int64_t)load_u32_at(pg, voff);
  const int64_t s0 = voff + 4, send = s0 + len;
  if (send > n) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
  __shared__ int r_start[129];
  __shared__ int64_t r_src[128];
  __shared__ int r_kind[128];
  __shared__ int r_meta[2];
  int64_t pos = s0;
  int done = 0;
  while (done < nv) {
    if (threadIdx.x == 0) {
      int k = 0, acc = 0, err = 0;
      int64_t q = pos;
      while (k < 128 && done + acc < nv) {
        uint64_t h = 0;
        int shift = 0;
        for (;;) {
          if (q >= send || shift > 35) { err = 1; break; }
          const uint8_t b = pg[q++];
          h |= (uint64_t)(b & 0x7f) << shift;
          if (!(b & 0x80)) break;
          shift += 7;
        }
        if (err) break;
        const int left = nv - done - acc;
        if (h & 1) {                       // bit-packed: groups of 8 values, 1 byte each
          const int64_t groups = (int64_t)(h >> 1);
          if (q + groups > send) { err = 1; break; }
          r_kind[k] = 1;
          r_src[k] = q;
          r_start[k] = acc;
          acc += (int)(groups * 8 < left ? groups * 8 : left);
          q += groups;
        } else {                           // RLE: count, then one value byte
          const int64_t cnt = (int64_t)(h >> 1);
          if (q + 1 > send) { err = 1; break; }
          const int v = pg[q++] & 1;
          if (cnt == 0) continue;
          r_kind[k] = 0;
          r_src[k] = v;
          r_start[k] = acc;
          acc += (int)(cnt < left ? cnt : left);
        }
        ++k;
      }
      r_start[k] = acc;
      r_meta[0] = k;
      r_meta[1] = err || (k == 0 && done < nv);
      pos = q;
    }
    __syncthreads();
    const int k = r_meta[0];
    if (r_meta[1]) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
    const int total = r_start[k];
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
      int lo = 0, hi = k - 1;
      while (lo < hi) {
        const int m = (lo + hi + 1) >> 1;
        if (r_start[m] <= i) lo = m; else hi = m - 1;
      }
      const int j = i - r_start[lo];
      out[done + i] = r_kind[lo] == 0 ? (uint8_t)r_src[lo]
                                      : (uint8_t)((pg[r_src[lo] + (j >> 3)] >> (j & 7)) & 1);
    }
    __syncthreads();
    done += total;
  }
}

// PLAIN BYTE_ARRAY data page (eb 16): `nv` length-prefixed values (4-byte little-endian length,
// then the bytes) -> per value the device address of its first byte (uint64 at p.out) and its
// length (int32 at p.dict).  The offsets are one dependent chain, so one lane walks it, 1024
// values per round into LDS, and the workgroup writes them out coalesced; the page's bytes stay
// where the inflate left them (the caller keeps the scratch alive until the strings are
// hashed: io/native_parquet.StringCodes.finish_plain).
__device__ void expand_plain_strings(const HsPqPage& p, const uint8_t* __restrict__ pg, int nv,
                                     int* __restrict__ status) {
  __shared__ int s_off[1024];
  __shared__ int s_len[1024];
  __shared__ int s_meta[2];
  uint64_t* optr = (uint64_t*)p.out;
  int32_t* olen = (int32_t*)p.dict;
  const int n = p.usize;
  int voff = 0;
  if (p.kind == 0 && p.levels) voff = 4 + (int)load_u32_at(pg, 0);
  else if (p.kind == 1) voff = p.levels;
  if (voff < 0 || voff > n) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
  int64_t q = voff;                       // lane 0's walk position
  int done = 0;
  while (done < nv) {
    if (threadIdx.x == 0) {
      int k = 0, err = 0;
      while (k < 1024 && done + k < nv) {
        if (q + 4 > n) { err = 1; break; }
        const int64_t l = (int64_t)load_u32_at(pg, q);
        q += 4;
        if (l > n - q) { err = 1; break; }
        s_off[k] = (int)q;
        s_len[k] = (int)l;
        q += l;
        ++k;
      }
      s_meta[0] = k;
      s_meta[1] = err;
    }
    __syncthreads();
    const int k = s_meta[0];
    if (s_meta[1]) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
    for (int i = threadIdx.x; i < k; i += blockDim.x) {
      optr[done + i] = (uint64_t)(uintptr_t)(pg + s_off[i]);
      olen[done + i] = s_len[i];
    }
    __syncthreads();
    done += k;
  }
}

// Block-wide sum of one int per thread (256 threads: 4 wavefronts).
__device__ __forceinline__ int block_sum(int v, int* __restrict__ s_part) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) s_part[threadIdx.x >> 6] = v;
  __syncthreads();
  return s_part[0] + s_part[1] + s_part[2] + s_part[3];
}

// Definition levels (max level 1) of a page with nulls -> one validity byte per row at
// `valid`; returns the page's non-null value count (every thread), or -1 on corruption.  v1
// pages carry a 4-byte length then the RLE / bit-packed hybrid stream; v2 pages the bare stream
// of `levels` bytes.  Runs are cut by one lane (headers are a few bytes), rows written by all.
__device__ int expand_levels(const HsPqPage& p, const uint8_t* __restrict__ pg,
                             uint8_t* __restrict__ valid) {
  __shared__ int r_start[129];
  __shared__ int64_t r_src[128];
  __shared__ int r_kind[128];
  __shared__ int r_meta[2];
  __shared__ int s_part[4];
  const int n = p.usize, nv = p.nvals;
  int64_t s0, send;
  if (p.kind == 0) {
    if (!p.levels || n < 4) return -1;
    s0 = 4;
    send = 4 + (int64_t)load_u32_at(pg, 0);
  } else {
    s0 = 0;
    send = p.levels;
  }
  if (send > n) return -1;
  int64_t pos = s0;
  int done = 0, ones = 0;
  while (done < nv) {
    if (threadIdx.x == 0) {
      int k = 0, acc = 0, err = 0;
      int64_t q = pos;
      while (k < 128 && done + acc < nv) {
        uint64_t h = 0;
        int shift = 0;
        for (;;) {
          if (q >= send || shift > 35) { err = 1; break; }
          const uint8_t b = pg[q++];
          h |= (uint64_t)(b & 0x7f) << shift;
          if (!(b & 0x80)) break;
          shift += 7;
        }
        if (err) break;
        const int left = nv - done - acc;
        if (h & 1) {
          const int64_t groups = (int64_t)(h >> 1);
          if (q + groups > send) { err = 1; break; }
          r_kind[k] = 1;
          r_src[k] = q;
          r_start[k] = acc;
          acc += (int)(groups * 8 < left ? groups * 8 : left);
          q += groups;
        } else {
          const int64_t cnt = (int64_t)(h >> 1);
          if (q + 1 > send) { err = 1; break; }
          const int v = pg[q++] & 1;
          if (cnt == 0) continue;
          r_kind[k] = 0;
          r_src[k] = v;
          r_start[k] = acc;
          acc += (int)(cnt < left ? cnt : left);
        }
        ++k;
      }
      r_start[k] = acc;
      r_meta[0] = k;
      r_meta[1] = err || (k == 0 && done < nv);
      pos = q;
    }
    __syncthreads();
    const int k = r_meta[0];
    if (r_meta[1]) return -1;
    const int total = r_start[k];
    for (int i = threadIdx.x; i < total; i += blockDim.x) {
      int lo = 0, hi = k - 1;
      while (lo < hi) {
        const int m = (lo + hi + 1) >> 1;
        if (r_start[m] <= i) lo = m; else hi = m - 1;
      }
      const int j = i - r_start[lo];
      const uint8_t v = r_kind[lo] == 0 ? (uint8_t)r_src[lo]
                                        : (uint8_t)((pg[r_src[lo] + (j >> 3)] >> (j & 7)) & 1);
      valid[done + i] = v;
      ones += v;
    }
    __syncthreads();
    done += total;
  }
  return block_sum(ones, s_part);
}

// In-place spread of a page's `nonnull` dense values (out[0, nonnull)) to their rows
// (out[row] for valid rows, 0 for nulls).  Rank(row) <= row, so 256-row chunks are processed
// from the last: a chunk only overwrites dense slots at or after its first row, which no
// earlier chunk reads, and within a chunk every source is loaded before any store.
template <typename T>
__device__ void spread_nulls(T* __restrict__ out, const uint8_t* __restrict__ valid, int nv,
                             int nonnull) {
  __shared__ int s_wave[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int base_end = nonnull;
  for (int c = ((nv + 255) >> 8) - 1; c >= 0; --c) {
    const int r = (c << 8) + (int)threadIdx.x;
    const bool v = r < nv && valid[r] != 0;
    const uint64_t bal = __ballot(v);
    const int rank_in_wave = __popcll(bal & ((1ull << lane) - 1ull));
    if (lane == 0) s_wave[w] = __popcll(bal);
    __syncthreads();
    int before = 0;
    for (int x = 0; x < w; ++x) before += s_wave[x];
    const int chunk = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    const int base = base_end - chunk;
    const T x = v ? out[base + before + rank_in_wave] : (T)0;
    __syncthreads();
    if (r < nv) out[r] = x;
    base_end = base;
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void hs_pq_expand_kernel(
    const uint8_t* __restrict__ scratch, const HsPqPage* __restrict__ pages, int npages,
    int* __restrict__ status) {
  const int pi = blockIdx.x;
  if (pi >= npages) return;
  const HsPqPage p = pages[pi];
  if (p.kind == 2 || p.nvals == 0) return;     // dictionary pages are read by the data pages
  const uint8_t* pg = (const uint8_t*)p.dst;
  int nv = p.nvals;
  uint8_t* valid = (uint8_t*)p.valid;
  if (p.nulls) {                               // levels first, then the non-null values dense
    if (!valid) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
    nv = expand_levels(p, pg, valid);
    if (nv < 0 || nv > p.nvals) { if (threadIdx.x == 0) atomicOr(status, kErrCorrupt); return; }
  }
  if (nv > 0) {
    if (p.eb == 16) expand_plain_strings(p, pg, nv, status);
    else if (p.eb == 4) expand_page<uint32_t>(p, pg, pages, nv, status);
    else if (p.eb == 8) expand_page<uint64_t>(p, pg, pages, nv, status);
    else if (p.eb == 1) expand_bool(p, pg, nv, status);
    else if (threadIdx.x == 0) atomicOr(status, kErrCorrupt);
  }
  if (!p.nulls) return;
  __syncthreads();
  if (p.eb == 16) {                        // (address, length) pairs; nulls get (0, 0)
    spread_nulls<uint64_t>((uint64_t*)p.out, valid, p.nvals, nv);
    spread_nulls<uint32_t>((uint32_t*)p.dict, valid, p.nvals, nv);
  } else if (p.eb == 4) spread_nulls<uint32_t>((uint32_t*)p.out, valid, p.nvals, nv);
  else if (p.eb == 8) spread_nulls<uint64_t>((uint64_t*)p.out, valid, p.nvals, nv);
  else if (p.eb == 1) spread_nulls<uint8_t>((uint8_t*)p.out, valid, p.nvals, nv);
}

extern "C" {

// Decode the pages planned by hs_pq_plan_chunk: inflate (one wavefront per page) then expand
// (one workgroup per page) on `stream`.  `raw`, `scratch`, `pages` and `status` are device
// pointers; errors accumulate as bits in *status.  With `raw` null the pages' `src` fields are
// absolute device addresses: one launch then decodes the pages of many files.
int hs_pq_decode_pages(const uint8_t* raw, uint8_t* scratch, const HsPqPage* pages, int npages,
                       int* status, void* stream) {
  if (npages <= 0) return 0;
  (void)hipGetLastError();
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(hs_pq_inflate_kernel, dim3((unsigned)((npages + 3) / 4)), dim3(256), 0, s,
                     raw, scratch, pages, npages, status);
  hipLaunchKernelGGL(hs_pq_expand_kernel, dim3((unsigned)npages), dim3(256), 0, s, scratch,
                     pages, npages, status);
  return (int)hipGetLastError();
}

int hs_pq_page_struct_size() { return (int)sizeof(HsPqPage); }

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
  hipLaunchKernelGGL(hs_pq_inflate_kernel, dim3(1), dim3(256), 0, s, nullptr, nullptr, nullptr, 0,
                     nullptr);
  hipLaunchKernelGGL(hs_pq_expand_kernel, dim3(1), dim3(256), 0, s, nullptr, nullptr, 0, nullptr);
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
