// K3: Spark-compatible Murmur3 bucketing + bucket histogram (SURVEY §2.3 K3, §7.4 hard part 1).
//
// bucket = pmod(murmur3(cols..., seed=42), numBuckets) with per-column seed chaining; nulls leave
// the running hash unchanged; strings use hashUnsafeBytes (Spark's per-byte tail).  One pass over
// the key columns also produces the per-bucket row counts (LDS-privatised histogram, one global
// atomic per non-empty bin per block) that the partitioner and the bucket offset table need.
#include "hs_common.h"

#define HS_HASH_MAX_COLS 8
#define HS_STR 100
#define HS_STRDICT 101   // int32 codes into a dictionary held as (offsets, chars) on the device

// Value transform applied before hashing, so a device column hashes like Spark's logical value:
//   HS_XF_DECIMAL | s : float64 storage of decimal(p<=15, s) -> unscaled long llrint(d * 10^s)
//   HS_XF_MUL | k     : int64 * 10^k   (timestamp[s]/[ms] -> microseconds)
//   HS_XF_FDIV | k    : floor(int64 / 10^k)  (timestamp[ns] -> microseconds)
#define HS_XF_NONE 0
#define HS_XF_DECIMAL 0x100
#define HS_XF_MUL 0x200
#define HS_XF_FDIV 0x300

struct HashCol {
  const void* data;        // values, chars for HS_STR, int32 codes for HS_STRDICT
  const uint8_t* valid;    // nullable
  const int64_t* offsets;  // HS_STR: n+1 row offsets; HS_STRDICT: dictionary offsets
  const void* aux;         // HS_STRDICT: dictionary chars
  int32_t type;            // HsType, HS_STR or HS_STRDICT
  int32_t xform;           // HS_XF_* | argument
};

__device__ __forceinline__ int64_t hs_pow10(int k) {
  int64_t p = 1;
  for (int i = 0; i < k; ++i) p *= 10;
  return p;
}

struct HashParams {
  HashCol cols[HS_HASH_MAX_COLS];
  int32_t ncols;
  int32_t num_buckets;
  uint32_t seed;
  int32_t pad;
};

__device__ __forceinline__ uint32_t hash_string(const uint8_t* chars, int64_t lo, int64_t hi,
                                                uint32_t h1) {
  const int64_t len = hi - lo;
  const int64_t aligned = len - (len & 3);
  int64_t i = 0;
  for (; i < aligned; i += 4) {
    const uint8_t* p = chars + lo + i;
    uint32_t w = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                 ((uint32_t)p[3] << 24);
    h1 = hs_mix_h1(h1, hs_mix_k1(w));
  }
  for (; i < len; ++i) {
    int32_t b = (int8_t)chars[lo + i];  // sign-extended, as Platform.getByte
    h1 = hs_mix_h1(h1, hs_mix_k1((uint32_t)b));
  }
  return hs_fmix(h1, (uint32_t)len);
}

__device__ __forceinline__ uint32_t hash_value(const HashCol& c, int64_t row, uint32_t h) {
  if (c.valid != nullptr && c.valid[row] == 0) return h;
  switch (c.type) {
    case HS_I8: return hs_hash_int((uint32_t)(int32_t)((const int8_t*)c.data)[row], h);
    case HS_I16: return hs_hash_int((uint32_t)(int32_t)((const int16_t*)c.data)[row], h);
    case HS_I32: return hs_hash_int((uint32_t)((const int32_t*)c.data)[row], h);
    case HS_BOOL: return hs_hash_int((uint32_t)(((const uint8_t*)c.data)[row] != 0), h);
    case HS_I64: {
      int64_t v = ((const int64_t*)c.data)[row];
      const int xk = c.xform & 0xff;
      if ((c.xform & 0xf00) == HS_XF_MUL) {
        v *= hs_pow10(xk);
      } else if ((c.xform & 0xf00) == HS_XF_FDIV) {
        const int64_t d = hs_pow10(xk);
        int64_t q = v / d;
        if ((v % d) != 0 && v < 0) --q;  // floor, like Math.floorDiv
        v = q;
      }
      return hs_hash_long((uint64_t)v, h);
    }
    // Spark 2.4.2 (the reference's pin, build.sbt:19) hashes floatToIntBits / doubleToLongBits:
    // NaN is canonicalised, -0.0 keeps its sign bit (the -0.0 -> 0.0 rewrite is Spark 3.x).
    case HS_F32: {
      float f = ((const float*)c.data)[row];
      const uint32_t bits = (f != f) ? 0x7fc00000u : __float_as_uint(f);
      return hs_hash_int(bits, h);
    }
    case HS_F64: {
      double d = ((const double*)c.data)[row];
      if ((c.xform & 0xf00) == HS_XF_DECIMAL) {  // decimal: Spark hashes the unscaled long
        return hs_hash_long((uint64_t)__double2ll_rn(d * (double)hs_pow10(c.xform & 0xff)), h);
      }
      const uint64_t bits = (d != d) ? 0x7ff8000000000000ull : (uint64_t)__double_as_longlong(d);
      return hs_hash_long(bits, h);
    }
    case HS_STR:
      return hash_string((const uint8_t*)c.data, c.offsets[row], c.offsets[row + 1], h);
    case HS_STRDICT: {   // the dictionary entry's bytes: same hash as the raw string
      const int32_t code = ((const int32_t*)c.data)[row];
      return hash_string((const uint8_t*)c.aux, c.offsets[code], c.offsets[code + 1], h);
    }
    default:
      return hs_hash_long(((const uint64_t*)c.data)[row], h);
  }
}

template <bool HIST_IN_LDS>
__global__ __launch_bounds__(256) void hs_murmur3_bucket_kernel(HashParams p, int64_t n,
                                                                int32_t* __restrict__ out_bucket,
                                                                int64_t* __restrict__ bucket_counts) {
  extern __shared__ __attribute__((aligned(16))) int32_t lds_hist[];
  if (HIST_IN_LDS && bucket_counts != nullptr) {
    for (int i = threadIdx.x; i < p.num_buckets; i += blockDim.x) lds_hist[i] = 0;
    __syncthreads();
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < n; row += stride) {
    uint32_t h = p.seed;
    for (int c = 0; c < p.ncols; ++c) h = hash_value(p.cols[c], row, h);
    int32_t b = (int32_t)((int64_t)(int32_t)h % p.num_buckets);
    if (b < 0) b += p.num_buckets;
    out_bucket[row] = b;
    if (bucket_counts != nullptr) {
      if (HIST_IN_LDS) atomicAdd(&lds_hist[b], 1);
      else atomicAdd((unsigned long long*)&bucket_counts[b], 1ull);
    }
  }
  if (HIST_IN_LDS && bucket_counts != nullptr) {
    __syncthreads();
    for (int i = threadIdx.x; i < p.num_buckets; i += blockDim.x)
      if (lds_hist[i]) atomicAdd((unsigned long long*)&bucket_counts[i], (unsigned long long)lds_hist[i]);
  }
}

// Raw 32-bit hash output (for tests / hash joins).
__global__ __launch_bounds__(256) void hs_murmur3_hash_kernel(HashParams p, int64_t n,
                                                              int32_t* __restrict__ out_hash) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < n; row += stride) {
    uint32_t h = p.seed;
    for (int c = 0; c < p.ncols; ++c) h = hash_value(p.cols[c], row, h);
    out_hash[row] = (int32_t)h;
  }
}

static int grid_for(int64_t n, int block) {
  int64_t g = (n + block - 1) / block;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" {

// bucket_counts may be null; must be zero-initialised by the caller otherwise.
int hs_murmur3_bucket(const HashParams* p, int64_t n, int32_t* out_bucket, int64_t* bucket_counts,
                      void* stream) {
  if (n == 0) return 0;
  const int block = 256;
  const int grid = grid_for(n, block);
  hipStream_t s = (hipStream_t)stream;
  if (p->num_buckets <= 16384) {
    size_t lds = bucket_counts ? (size_t)p->num_buckets * sizeof(int32_t) : 0;
    hipLaunchKernelGGL(hs_murmur3_bucket_kernel<true>, dim3(grid), dim3(block), lds, s, *p, n,
                       out_bucket, bucket_counts);
  } else {
    hipLaunchKernelGGL(hs_murmur3_bucket_kernel<false>, dim3(grid), dim3(block), 0, s, *p, n,
                       out_bucket, bucket_counts);
  }
  return (int)hipGetLastError();
}

int hs_murmur3_hash(const HashParams* p, int64_t n, int32_t* out_hash, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(hs_murmur3_hash_kernel, dim3(grid_for(n, 256)), dim3(256), 0,
                     (hipStream_t)stream, *p, n, out_hash);
  return (int)hipGetLastError();
}

int hs_hash_params_size() { return (int)sizeof(HashParams); }

}  // extern "C"
