// Avro object-container block decoder (host, columnar).
//
// The reference reads Avro sources through Spark's DataSource (DefaultFileBasedSource.scala:
// 43-48 lists avro among the default formats).  This is a native decoder for the flat record
// schemas a covering index can be built on: every top-level field is a primitive (boolean, int,
// long, float, double, bytes, string) or a two-branch union of "null" and a primitive.  The
// Python side (hyperspace_amd/io/avro.py) parses the container header (magic, metadata map,
// sync marker) and the schema JSON into a field program; this decoder walks the data blocks
// (count, size, payload, sync), inflates deflate / snappy blocks and decodes the records straight
// into columnar buffers (fixed-width values + validity bytes, or offsets + chars) that Python
// wraps as Arrow arrays without a per-value Python step.
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <exception>
#include <string>
#include <vector>

extern "C" int64_t hs_pq_snappy_decompress(const uint8_t* in, int64_t n, uint8_t* out,
                                           int64_t cap);   // hs_parquet.cpp

namespace {

enum AType : int32_t { A_NULL = 0, A_BOOL = 1, A_INT = 2, A_LONG = 3, A_FLOAT = 4, A_DOUBLE = 5,
                       A_BYTES = 6, A_STRING = 7 };
enum Codec : int32_t { C_NULL = 0, C_DEFLATE = 1, C_SNAPPY = 2 };

struct Col {
  int32_t type = 0;
  int32_t null_branch = -1;      // union branch index of "null"; -1 = not a union
  std::vector<uint8_t> data;     // fixed-width values, or chars
  std::vector<uint8_t> valid;    // one byte per row
  std::vector<int64_t> offs;     // string / bytes offsets (rows + 1)
};

struct Result {
  std::vector<Col> cols;
  int64_t rows = 0;
  std::string err;
};

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok = true;

  int64_t zz_long() {
    uint64_t v = 0;
    int shift = 0;
    while (true) {
      if (p >= end || shift > 63) { ok = false; return 0; }
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) break;
      shift += 7;
    }
    return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
  }
  bool take(void* dst, size_t n) {
    if ((size_t)(end - p) < n) { ok = false; return false; }
    std::memcpy(dst, p, n);
    p += n;
    return true;
  }
};

int width_of(int32_t t) {
  switch (t) {
    case A_BOOL: return 1;
    case A_INT: case A_FLOAT: return 4;
    case A_LONG: case A_DOUBLE: return 8;
    default: return 0;
  }
}

bool decode_value(Reader& r, Col& c) {
  switch (c.type) {
    case A_NULL: return true;
    case A_BOOL: { uint8_t b; if (!r.take(&b, 1)) return false; c.data.push_back(b ? 1 : 0); return true; }
    case A_INT: {
      const int32_t v = (int32_t)r.zz_long();
      const uint8_t* q = reinterpret_cast<const uint8_t*>(&v);
      c.data.insert(c.data.end(), q, q + 4);
      return r.ok;
    }
    case A_LONG: {
      const int64_t v = r.zz_long();
      const uint8_t* q = reinterpret_cast<const uint8_t*>(&v);
      c.data.insert(c.data.end(), q, q + 8);
      return r.ok;
    }
    case A_FLOAT: { uint8_t b[4]; if (!r.take(b, 4)) return false; c.data.insert(c.data.end(), b, b + 4); return true; }
    case A_DOUBLE: { uint8_t b[8]; if (!r.take(b, 8)) return false; c.data.insert(c.data.end(), b, b + 8); return true; }
    case A_BYTES: case A_STRING: {
      const int64_t n = r.zz_long();
      if (!r.ok || n < 0 || n > r.end - r.p) { r.ok = false; return false; }
      c.data.insert(c.data.end(), r.p, r.p + n);
      r.p += n;
      c.offs.push_back((int64_t)c.data.size());
      return true;
    }
    default: r.ok = false; return false;
  }
}

// placeholder for a null row: keeps fixed-width columns dense and offsets monotone
void decode_null(Col& c) {
  const int w = width_of(c.type);
  if (w) c.data.insert(c.data.end(), (size_t)w, 0);
  else if (c.type == A_BYTES || c.type == A_STRING) c.offs.push_back((int64_t)c.data.size());
}

bool decode_records(Reader& r, int64_t count, Result& res) {
  for (int64_t i = 0; i < count; ++i) {
    for (Col& c : res.cols) {
      bool present = true;
      if (c.null_branch >= 0) {
        const int64_t br = r.zz_long();
        if (!r.ok || br < 0 || br > 1) { res.err = "bad union branch"; return false; }
        present = br != c.null_branch;
      }
      if (present) {
        if (!decode_value(r, c)) { res.err = "truncated record"; return false; }
      } else {
        decode_null(c);
      }
      c.valid.push_back(present ? 1 : 0);
    }
  }
  res.rows += count;
  return true;
}

bool inflate_raw(const uint8_t* in, size_t n, std::vector<uint8_t>& out) {
  z_stream zs;
  std::memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, -15) != Z_OK) return false;   // raw deflate (RFC 1951), as Avro writes
  // DEFLATE expands at most ~1032:1: a larger output is a corrupt or hostile block, not data
  const size_t cap = std::min<size_t>(n * 1032 + 4096, (size_t)1 << 32);
  out.resize(std::min<size_t>(std::max<size_t>(n * 4, 4096), cap));
  zs.next_in = const_cast<Bytef*>(in);
  zs.avail_in = (uInt)n;
  int rc;
  do {
    if (zs.total_out == out.size()) {
      if (out.size() >= cap) { rc = Z_DATA_ERROR; break; }
      out.resize(std::min(out.size() * 2, cap));
    }
    zs.next_out = out.data() + zs.total_out;
    zs.avail_out = (uInt)(out.size() - zs.total_out);
    rc = inflate(&zs, Z_NO_FLUSH);
  } while (rc == Z_OK);
  const bool good = rc == Z_STREAM_END;
  out.resize(zs.total_out);
  inflateEnd(&zs);
  return good;
}

// snappy varint preamble = uncompressed length
bool snappy_block(const uint8_t* in, size_t n, std::vector<uint8_t>& out) {
  if (n < 4) return false;
  n -= 4;   // trailing big-endian CRC32 of the uncompressed bytes
  uint64_t len = 0;
  int shift = 0;
  size_t i = 0;
  while (i < n && shift < 35) {
    const uint8_t b = in[i++];
    len |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) break;
    shift += 7;
  }
  // a Snappy tag of k bytes emits at most 64 bytes (copy-2: 3 bytes -> 64), so a preamble
  // claiming more than ~32x the block is corrupt: never allocate from an untrusted length
  if (len > (uint64_t)n * 32 + 64) return false;
  out.resize(len);
  if (hs_pq_snappy_decompress(in, (int64_t)n, out.data(), (int64_t)len) != (int64_t)len)
    return false;
  const uint32_t want = ((uint32_t)in[n] << 24) | ((uint32_t)in[n + 1] << 16) |
                        ((uint32_t)in[n + 2] << 8) | (uint32_t)in[n + 3];
  return (uint32_t)crc32(0L, out.data(), (uInt)out.size()) == want;
}

}  // namespace

extern "C" {

// Decode every data block of a container whose header ends at ``buf`` (``len`` bytes of blocks
// follow).  types / null_branch: one entry per top-level field.  Returns an opaque result.
void* hs_avro_decode(const uint8_t* buf, int64_t len, const uint8_t* sync, int32_t codec,
                     int32_t nfields, const int32_t* types, const int32_t* null_branch) {
  Result* res = new Result();
  // no C++ exception may cross the C ABI (ctypes): allocation failures become res->err
  try {
  res->cols.resize((size_t)nfields);
  for (int f = 0; f < nfields; ++f) {
    res->cols[f].type = types[f];
    res->cols[f].null_branch = null_branch[f];
    if (types[f] == A_BYTES || types[f] == A_STRING) res->cols[f].offs.push_back(0);
  }
  Reader top{buf, buf + len};
  std::vector<uint8_t> scratch;
  while (top.p < top.end && res->err.empty()) {
    const int64_t count = top.zz_long();
    const int64_t size = top.zz_long();
    if (!top.ok || count < 0 || size < 0 || size > top.end - top.p) {
      res->err = "corrupt block header";
      break;
    }
    const uint8_t* body = top.p;
    top.p += size;
    if (top.end - top.p < 16 || std::memcmp(top.p, sync, 16) != 0) {
      res->err = "sync marker mismatch";
      break;
    }
    top.p += 16;
    const uint8_t* data = body;
    size_t dlen = (size_t)size;
    if (codec == C_DEFLATE) {
      if (!inflate_raw(body, (size_t)size, scratch)) { res->err = "deflate block"; break; }
      data = scratch.data();
      dlen = scratch.size();
    } else if (codec == C_SNAPPY) {
      if (!snappy_block(body, (size_t)size, scratch)) { res->err = "snappy block (or CRC)"; break; }
      data = scratch.data();
      dlen = scratch.size();
    } else if (codec != C_NULL) {
      res->err = "unsupported codec";
      break;
    }
    Reader r{data, data + dlen};
    if (!decode_records(r, count, *res)) break;
  }
  } catch (const std::exception& e) {
    res->err = std::string("avro decode: ") + e.what();
  } catch (...) {
    res->err = "avro decode: unknown error";
  }
  return res;
}

const char* hs_avro_error(void* h) {
  Result* r = static_cast<Result*>(h);
  return r->err.empty() ? nullptr : r->err.c_str();
}

int64_t hs_avro_rows(void* h) { return static_cast<Result*>(h)->rows; }

// which: 0 = data, 1 = validity, 2 = offsets
const void* hs_avro_buffer(void* h, int32_t field, int32_t which, int64_t* nbytes) {
  Col& c = static_cast<Result*>(h)->cols[(size_t)field];
  if (which == 0) { *nbytes = (int64_t)c.data.size(); return c.data.data(); }
  if (which == 1) { *nbytes = (int64_t)c.valid.size(); return c.valid.data(); }
  *nbytes = (int64_t)(c.offs.size() * sizeof(int64_t));
  return c.offs.data();
}

void hs_avro_free(void* h) { delete static_cast<Result*>(h); }

}  // extern "C"
