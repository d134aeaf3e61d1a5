// Native Parquet page layer for the MI355X decode path (SURVEY.md §2.3 K1, §7.1 "Parquet
// reader/writer page layer, thrift metadata parsed on the host in C++").
//
// Host side only: footer + page headers (Thrift compact protocol), page decompression
// (UNCOMPRESSED / SNAPPY; other codecs are reported as unsupported so the caller falls back),
// and a pre-parse of every RLE/bit-packed hybrid stream (definition levels, dictionary indices)
// into a flat *run table*.  The decompressed page bytes and the run table are what travel to the
// GPU; expanding runs into values (dictionary gather, bit unpacking, PLAIN copies) happens in
// csrc/kernels/parquet_decode.hip.  Dictionary-encoded data therefore crosses PCIe at its
// encoded width (e.g. 6 bits per TPC-H l_quantity instead of 64).
//
// Scope: flat schemas (no repetition), optional or required columns (definition levels), data
// pages V1 and V2.  Physical types INT32 / INT64 / FLOAT / DOUBLE (PLAIN and dictionary
// encodings; the INT32 / INT64 logical types DATE, TIMESTAMP, DECIMAL and INT8/16 included),
// BOOLEAN (bit-packed PLAIN or RLE), BYTE_ARRAY (dictionary pages parse on the host,
// hs_pq_plain_strings, and the codes decode on the device; PLAIN data pages decode on the device
// to value addresses + lengths, hashed into codes afterwards).  Anything else (INT96,
// FIXED_LEN_BYTE_ARRAY, DELTA_* encodings, codecs other than SNAPPY / UNCOMPRESSED) returns
// HS_PQ_UNSUPPORTED and the Python side reads that column with pyarrow instead.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

enum : int {
  HS_PQ_OK = 0,
  HS_PQ_IO = -1,
  HS_PQ_CORRUPT = -2,
  HS_PQ_UNSUPPORTED = -3,
  HS_PQ_CAPACITY = -4,
  HS_PQ_NULLS = -5,        // the chunk may hold nulls: not decodable by the device-only path
};

// ------------------------------------------------------------------ Thrift compact protocol
struct TReader {
  const uint8_t* p;
  const uint8_t* end;
  bool bad = false;

  uint8_t byte() {
    if (p >= end) { bad = true; return 0; }
    return *p++;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int shift = 0; shift < 64; shift += 7) {
      const uint8_t b = byte();
      v |= (uint64_t)(b & 0x7f) << shift;
      if (!(b & 0x80)) return v;
    }
    bad = true;
    return 0;
  }
  int64_t zigzag() {
    const uint64_t v = varint();
    return (int64_t)(v >> 1) ^ -(int64_t)(v & 1);
  }
  std::string binary() {
    const uint64_t n = varint();
    if ((uint64_t)(end - p) < n) { bad = true; return {}; }
    std::string s((const char*)p, n);
    p += n;
    return s;
  }
  // field header: returns type (0 = stop); id updated from the delta or an explicit i16
  int field(int16_t& id) {
    const uint8_t b = byte();
    if (b == 0) return 0;
    const int type = b & 0x0f;
    const int delta = b >> 4;
    id = delta ? (int16_t)(id + delta) : (int16_t)zigzag();
    return type;
  }
  void list_header(int& elem_type, int64_t& size) {
    const uint8_t b = byte();
    elem_type = b & 0x0f;
    size = b >> 4;
    if (size == 15) size = (int64_t)varint();
    // every element takes at least one byte: a longer list is a damaged length
    if (size < 0 || size > end - p) {
      bad = true;
      size = 0;
    }
  }
  void skip(int type) {
    switch (type) {
      case 1: case 2: return;                       // bool (value in the type nibble)
      case 3: byte(); return;
      case 4: case 5: case 6: zigzag(); return;
      case 7: p += 8; if (p > end) bad = true; return;
      case 8: binary(); return;
      case 9: case 10: {
        int et; int64_t n; list_header(et, n);
        for (int64_t i = 0; i < n && !bad; ++i) skip_elem(et);
        return;
      }
      case 11: {
        const uint64_t n = varint();
        if (n == 0) return;
        const uint8_t kv = byte();
        for (uint64_t i = 0; i < n && !bad; ++i) { skip_elem(kv >> 4); skip_elem(kv & 0x0f); }
        return;
      }
      case 12: skip_struct(); return;
      default: bad = true;
    }
  }
  void skip_elem(int type) {
    if (type == 1 || type == 2) { byte(); return; }  // bools inside containers take a byte
    skip(type);
  }
  void skip_struct() {
    int16_t id = 0;
    for (int t; (t = field(id)) != 0 && !bad;) skip(t);
  }
};

struct SchemaEl {
  int type = -1, type_length = 0, repetition = 0, num_children = 0;
  std::string name;
};

struct ChunkMeta {
  int type = -1, codec = 0;
  int64_t num_values = 0, total_compressed = 0, total_uncompressed = 0;
  int64_t data_page_offset = 0, dict_page_offset = -1;
  int64_t null_count = -1;   // from the chunk statistics; -1: not recorded
  std::vector<std::string> path;
};

struct RowGroupMeta {
  int64_t num_rows = 0;
  std::vector<ChunkMeta> cols;
};

}  // namespace

// One entry per RLE run or (chunk of a) bit-packed run / PLAIN page — the GPU's work items
// (layout shared with csrc/kernels/parquet_decode.hip).  Values are written to
// out[dst .. dst+count): the dense non-null value index for value runs, rows for level runs.
struct HsPqRun {
  int64_t dst;        // first output index
  int64_t count;      // values in this run
  int64_t src;        // byte offset of the data in the chunk buffer; RLE runs: the value
  int32_t kind;       // 0 RLE, 1 bit-packed, 2 PLAIN
  int32_t bit_width;  // bits per value (RLE / bit-packed); PLAIN: element bytes
};

struct HsPqChunkInfo {
  int64_t num_values;     // rows in the chunk
  int64_t num_nonnull;    // non-null values
  int64_t dict_off;       // byte offset of the PLAIN dictionary in the buffer (-1: none)
  int64_t dict_count;
  int64_t bytes_used;     // bytes of the buffer written
  int64_t nvalue_runs, nlevel_runs;
  int32_t dict_encoded;   // 1 if any data page is dictionary-encoded
  int32_t plain_pages;    // pages stored PLAIN
};

namespace {

struct File {
  int fd = -1;
  std::vector<HsPqRun> vruns, lruns;  // run tables of the last hs_pq_read_chunk
  int64_t size = 0;
  int64_t num_rows = 0;
  std::vector<SchemaEl> schema;      // flattened, as stored
  std::vector<int> leaves;           // schema index of each leaf column
  std::vector<RowGroupMeta> rgs;
  std::string error;
};

void parse_schema_el(TReader& r, SchemaEl& s) {
  int16_t id = 0;
  for (int t; (t = r.field(id)) != 0 && !r.bad;) {
    switch (id) {
      case 1: s.type = (int)r.zigzag(); break;
      case 2: s.type_length = (int)r.zigzag(); break;
      case 3: s.repetition = (int)r.zigzag(); break;
      case 4: s.name = r.binary(); break;
      case 5: s.num_children = (int)r.zigzag(); break;
      default: r.skip(t);
    }
  }
}

void parse_col_meta(TReader& r, ChunkMeta& m) {
  int16_t id = 0;
  for (int t; (t = r.field(id)) != 0 && !r.bad;) {
    switch (id) {
      case 1: m.type = (int)r.zigzag(); break;
      case 3: {
        int et; int64_t n; r.list_header(et, n);
        for (int64_t i = 0; i < n && !r.bad; ++i) m.path.push_back(r.binary());
        break;
      }
      case 4: m.codec = (int)r.zigzag(); break;
      case 5: m.num_values = r.zigzag(); break;
      case 6: m.total_uncompressed = r.zigzag(); break;
      case 7: m.total_compressed = r.zigzag(); break;
      case 9: m.data_page_offset = r.zigzag(); break;
      case 11: m.dict_page_offset = r.zigzag(); break;
      case 12: {  // Statistics: null_count is field 3
        int16_t sid = 0;
        for (int st; (st = r.field(sid)) != 0 && !r.bad;) {
          if (sid == 3 && st == 6) m.null_count = r.zigzag();
          else r.skip(st);
        }
        break;
      }
      default: r.skip(t);
    }
  }
}

void parse_row_group(TReader& r, RowGroupMeta& g) {
  int16_t id = 0;
  for (int t; (t = r.field(id)) != 0 && !r.bad;) {
    if (id == 1) {
      int et; int64_t n; r.list_header(et, n);
      g.cols.resize((size_t)n);
      for (int64_t i = 0; i < n && !r.bad; ++i) {
        int16_t cid = 0;  // ColumnChunk
        for (int ct; (ct = r.field(cid)) != 0 && !r.bad;) {
          if (cid == 3) parse_col_meta(r, g.cols[(size_t)i]);
          else r.skip(ct);
        }
      }
    } else if (id == 3) {
      g.num_rows = r.zigzag();
    } else {
      r.skip(t);
    }
  }
}

bool pread_all(int fd, void* buf, size_t n, int64_t off) {
  uint8_t* d = (uint8_t*)buf;
  while (n) {
    const ssize_t k = pread(fd, d, n, off);
    if (k <= 0) return false;
    d += k; n -= (size_t)k; off += k;
  }
  return true;
}

int open_file(const char* path, File& f) {
  f.fd = open(path, O_RDONLY | O_CLOEXEC);
  if (f.fd < 0) { f.error = "open failed"; return HS_PQ_IO; }
  struct stat st;
  if (fstat(f.fd, &st) != 0 || st.st_size < 12) { f.error = "not a parquet file"; return HS_PQ_IO; }
  f.size = st.st_size;
  uint8_t tail[8];
  if (!pread_all(f.fd, tail, 8, f.size - 8) || memcmp(tail + 4, "PAR1", 4) != 0) {
    f.error = "missing PAR1 footer";
    return HS_PQ_CORRUPT;
  }
  uint32_t flen;
  memcpy(&flen, tail, 4);
  if ((int64_t)flen + 12 > f.size) { f.error = "bad footer length"; return HS_PQ_CORRUPT; }
  std::vector<uint8_t> meta(flen);
  if (!pread_all(f.fd, meta.data(), flen, f.size - 8 - flen)) { f.error = "read"; return HS_PQ_IO; }
  TReader r{meta.data(), meta.data() + meta.size()};
  int16_t id = 0;
  for (int t; (t = r.field(id)) != 0 && !r.bad;) {
    if (id == 2) {
      int et; int64_t n; r.list_header(et, n);
      f.schema.resize((size_t)n);
      for (int64_t i = 0; i < n && !r.bad; ++i) parse_schema_el(r, f.schema[(size_t)i]);
    } else if (id == 3) {
      f.num_rows = r.zigzag();
    } else if (id == 4) {
      int et; int64_t n; r.list_header(et, n);
      f.rgs.resize((size_t)n);
      for (int64_t i = 0; i < n && !r.bad; ++i) parse_row_group(r, f.rgs[(size_t)i]);
    } else {
      r.skip(t);
    }
  }
  if (r.bad) { f.error = "corrupt footer"; return HS_PQ_CORRUPT; }
  for (size_t i = 1; i < f.schema.size(); ++i)
    if (f.schema[i].num_children == 0) f.leaves.push_back((int)i);
  // every row group must describe every leaf column (callers index cols[] by leaf)
  for (const RowGroupMeta& g : f.rgs) {
    if (g.cols.size() != f.leaves.size() || g.num_rows < 0) {
      f.error = "row group / schema mismatch";
      return HS_PQ_CORRUPT;
    }
    // sizes the buffer bounds derive from (hs_pq_chunk_bound etc.) must be sane
    for (const ChunkMeta& m : g.cols)
      if (m.total_compressed < 0 || m.total_compressed > f.size || m.total_uncompressed < 0 ||
          m.total_uncompressed > ((int64_t)1 << 40) || m.num_values < 0 ||
          // Snappy expands at most ~22x (a 64-byte copy in 3 bytes); plain pages not at all
          ((m.codec == 0 || m.codec == 1) &&
           m.total_uncompressed > 24 * m.total_compressed + 4096) ||
          m.data_page_offset < 0 || m.data_page_offset > f.size) {
        f.error = "corrupt column chunk metadata";
        return HS_PQ_CORRUPT;
      }
  }
  return HS_PQ_OK;
}

// ------------------------------------------------------------------ Snappy (raw block format)
// Host Snappy decompression.  Most tags of Parquet pages are short (literals and copies of
// <= 16-64 bytes), so the hot loop avoids variable-length memcpy calls: while at least 64 bytes
// of input and output slack remain, short literals move as one unaligned 16-byte copy and copies
// with offset >= 8 as 8-byte steps that may overrun into the slack (later tags overwrite it);
// short-offset copies (runs) expand their pattern in place.  The tail runs the exact checked
// loop.  (~4-8x the byte-wise loop on TPC-H price / key pages.)
static inline void copy8(uint8_t* d, const uint8_t* s) { uint64_t v; memcpy(&v, s, 8); memcpy(d, &v, 8); }
static inline void copy16(uint8_t* d, const uint8_t* s) {
  uint64_t a, b; memcpy(&a, s, 8); memcpy(&b, s + 8, 8); memcpy(d, &a, 8); memcpy(d + 8, &b, 8);
}

bool snappy_decompress(const uint8_t* in, size_t n, uint8_t* out, size_t cap, size_t* out_len) {
  const uint8_t* ip = in;
  const uint8_t* iend = in + n;
  uint64_t len = 0;
  for (int shift = 0; ip < iend; shift += 7) {
    const uint8_t b = *ip++;
    len |= (uint64_t)(b & 0x7f) << shift;
    if (!(b & 0x80)) break;
    if (shift > 28) return false;
  }
  if (len > cap) return false;
  uint8_t* op = out;
  uint8_t* oend = out + len;
  // fast loop: every tag header fits (<= 5 bytes) and every short move may overrun by < 64
  while (iend - ip >= 64 && oend - op >= 64) {
    const uint8_t tag = *ip++;
    const int kind = tag & 3;
    if (kind == 0) {
      size_t l = (size_t)(tag >> 2) + 1;
      if (l <= 16) {
        copy16(op, ip);                         // input slack >= 63, output slack >= 64
        ip += l; op += l;
        continue;
      }
      if (l > 60) {
        const int nb = (int)l - 60;
        l = 0;
        for (int i = 0; i < nb; ++i) l |= (size_t)ip[i] << (8 * i);
        ip += nb;
        l += 1;
      }
      if ((size_t)(iend - ip) < l || (size_t)(oend - op) < l) return false;
      memcpy(op, ip, l);
      ip += l; op += l;
      continue;
    }
    size_t l, off;
    if (kind == 1) {
      l = 4 + ((tag >> 2) & 7);
      off = ((size_t)(tag >> 5) << 8) | *ip++;
    } else if (kind == 2) {
      l = 1 + (tag >> 2);
      off = (size_t)ip[0] | ((size_t)ip[1] << 8);
      ip += 2;
    } else {
      l = 1 + (tag >> 2);
      off = (size_t)ip[0] | ((size_t)ip[1] << 8) | ((size_t)ip[2] << 16) | ((size_t)ip[3] << 24);
      ip += 4;
    }
    if (off == 0 || off > (size_t)(op - out) || (size_t)(oend - op) < l) return false;
    const uint8_t* src = op - off;
    if (off >= 8 && l <= 16) {
      // two unconditional 8-byte steps (output slack >= 64); the second may read bytes the
      // first wrote (8 <= off < 16), which is the copy's meaning
      copy8(op, src);
      copy8(op + 8, src + 8);
    } else if (off >= 8 && (size_t)(oend - op) >= l + 8) {
      for (size_t i = 0; i < l; i += 8) copy8(op + i, src + i);   // chunks never overlap
    } else if (off >= l) {
      memcpy(op, src, l);
    } else {
      for (size_t i = 0; i < l; ++i) op[i] = src[i];             // run: pattern of period off
    }
    op += l;
  }
  while (ip < iend) {
    const uint8_t tag = *ip++;
    const int kind = tag & 3;
    if (kind == 0) {  // literal
      size_t l = tag >> 2;
      if (l >= 60) {
        const int nb = (int)l - 59;
        if (ip + nb > iend) return false;
        l = 0;
        for (int i = 0; i < nb; ++i) l |= (size_t)ip[i] << (8 * i);
        ip += nb;
      }
      l += 1;
      if (ip + l > iend || op + l > oend) return false;
      memcpy(op, ip, l);
      ip += l; op += l;
      continue;
    }
    size_t l, off;
    if (kind == 1) {
      if (ip >= iend) return false;
      l = 4 + ((tag >> 2) & 7);
      off = ((size_t)(tag >> 5) << 8) | *ip++;
    } else if (kind == 2) {
      if (ip + 2 > iend) return false;
      l = 1 + (tag >> 2);
      off = (size_t)ip[0] | ((size_t)ip[1] << 8);
      ip += 2;
    } else {
      if (ip + 4 > iend) return false;
      l = 1 + (tag >> 2);
      off = (size_t)ip[0] | ((size_t)ip[1] << 8) | ((size_t)ip[2] << 16) | ((size_t)ip[3] << 24);
      ip += 4;
    }
    if (off == 0 || off > (size_t)(op - out) || op + l > oend) return false;
    const uint8_t* src = op - off;
    if (off >= l) {
      memcpy(op, src, l);
      op += l;
    } else {
      for (size_t i = 0; i < l; ++i) *op++ = src[i];  // overlapping copy (run extension)
    }
  }
  if (op != oend) return false;
  *out_len = len;
  return true;
}

}  // namespace

namespace {

constexpr int64_t kChunk = 4096;  // split long runs so each GPU work item stays short
// device plans inflate Snappy dictionary pages larger than this on the host (plan_chunk)
constexpr int kHostDictMin = 64 << 10;
constexpr int64_t kDeviceInflateMax = 2 << 20;   // largest page a wavefront inflates
std::atomic<int> g_host_inflate{2};   // hs_pq_set_host_inflate
std::atomic<int> g_device_nulls{1};   // hs_pq_set_device_nulls
std::atomic<int> g_plain_strings{1};  // hs_pq_set_plain_strings

// Parse an RLE/bit-packed hybrid stream of `count` values into runs (dst starts at `dst0`).
// `base` is the stream's byte offset in the chunk buffer.  Returns the number of non-zero
// values when `count_ones` (definition levels, bit width 1), 0 otherwise; -1 on corruption.
int64_t parse_hybrid(const uint8_t* s, int64_t len, int64_t base, int bw, int64_t count,
                     int64_t dst0, std::vector<HsPqRun>& runs, bool count_ones) {
  TReader r{s, s + len};
  int64_t done = 0, ones = 0;
  const int vbytes = (bw + 7) / 8;
  while (done < count) {
    if (r.p >= r.end) return -1;
    const uint64_t h = r.varint();
    if (r.bad) return -1;
    if (h & 1) {  // bit-packed: (h>>1) groups of 8 values, bw bytes per group
      const uint64_t g64 = h >> 1;
      // a damaged header can claim ~2^63 groups: bound it by the bytes left before multiplying
      if (bw > 0 && g64 > (uint64_t)(r.end - r.p) / (uint64_t)bw) return -1;
      const int64_t left = count - done;
      const int64_t groups = g64 > (uint64_t)((left + 7) / 8) && bw == 0 ? (left + 7) / 8
                                                                           : (int64_t)g64;
      const int64_t nbytes = groups * bw;
      const int64_t take = groups < (left + 7) / 8 ? groups * 8 : left;
      const int64_t off = base + (r.p - s);
      for (int64_t c = 0; c < take; c += kChunk)   // kChunk % 8 == 0: chunks stay byte aligned
        runs.push_back({dst0 + done + c, take - c < kChunk ? take - c : kChunk,
                        off + c * bw / 8, 1, bw});
      if (count_ones)
        for (int64_t i = 0; i < take; ++i) ones += (r.p[i >> 3] >> (i & 7)) & 1;
      r.p += nbytes;
      done += take;
    } else {  // RLE: (h>>1) repeats of one value stored in ceil(bw/8) bytes
      const int64_t nvals = (int64_t)(h >> 1);
      if (r.end - r.p < vbytes) return -1;
      uint64_t v = 0;
      for (int i = 0; i < vbytes; ++i) v |= (uint64_t)r.p[i] << (8 * i);
      r.p += vbytes;
      if (nvals == 0) continue;
      const int64_t take = nvals < count - done ? nvals : count - done;
      for (int64_t c = 0; c < take; c += kChunk)
        runs.push_back({dst0 + done + c, take - c < kChunk ? take - c : kChunk, (int64_t)v, 0,
                        bw});
      if (count_ones && v) ones += take;
      done += take;
    }
  }
  return count_ones ? ones : 0;
}

struct PageHdr {
  int type = -1, usize = 0, csize = 0;
  int nvals = 0, enc = 0, def_enc = 3, v2_def_len = 0, v2_rep_len = 0;
  bool v2 = false, v2_compressed = true;
  int dict_nvals = 0;
};

bool parse_page_header(TReader& r, PageHdr& h) {
  int16_t id = 0;
  for (int t; (t = r.field(id)) != 0 && !r.bad;) {
    switch (id) {
      case 1: h.type = (int)r.zigzag(); break;
      case 2: h.usize = (int)r.zigzag(); break;
      case 3: h.csize = (int)r.zigzag(); break;
      case 5: {  // DataPageHeader
        int16_t d = 0;
        for (int dt; (dt = r.field(d)) != 0 && !r.bad;) {
          if (d == 1) h.nvals = (int)r.zigzag();
          else if (d == 2) h.enc = (int)r.zigzag();
          else if (d == 3) h.def_enc = (int)r.zigzag();
          else r.skip(dt);
        }
        break;
      }
      case 7: {  // DictionaryPageHeader
        int16_t d = 0;
        for (int dt; (dt = r.field(d)) != 0 && !r.bad;) {
          if (d == 1) h.dict_nvals = (int)r.zigzag();
          else if (d == 2) h.enc = (int)r.zigzag();
          else r.skip(dt);
        }
        break;
      }
      case 8: {  // DataPageHeaderV2
        h.v2 = true;
        int16_t d = 0;
        for (int dt; (dt = r.field(d)) != 0 && !r.bad;) {
          if (d == 1) h.nvals = (int)r.zigzag();
          else if (d == 4) h.enc = (int)r.zigzag();
          else if (d == 5) h.v2_def_len = (int)r.zigzag();
          else if (d == 6) h.v2_rep_len = (int)r.zigzag();
          else if (d == 7) h.v2_compressed = (dt == 1);
          else r.skip(dt);
        }
        break;
      }
      default: r.skip(t);
    }
  }
  // counts and lengths of a damaged header can decode negative (found by the ASan corpus run,
  // scripts/sanitize_hostio.py): reject them here so no caller sizes a copy from them
  if (h.usize < 0 || h.csize < 0 || h.nvals < 0 || h.dict_nvals < 0 || h.v2_def_len < 0 ||
      h.v2_rep_len < 0 || h.v2_def_len > h.csize || h.v2_def_len > h.usize)
    return false;
  return !r.bad;
}

int elem_bytes(int type) {
  switch (type) {
    case 1: case 4: return 4;   // INT32, FLOAT
    case 2: case 5: return 8;   // INT64, DOUBLE
    default: return 0;
  }
}

// decompress `csize` bytes into dst (capacity cap): bytes written, -1 corrupt, -2 unsupported
int64_t inflate(int codec, const uint8_t* src, int64_t csize, uint8_t* dst, int64_t cap) {
  if (codec == 0) {
    if (csize > cap) return -1;
    memcpy(dst, src, (size_t)csize);
    return csize;
  }
  if (codec == 1) {
    size_t n = 0;
    if (!snappy_decompress(src, (size_t)csize, dst, (size_t)cap, &n)) return -1;
    return (int64_t)n;
  }
  return -2;
}

int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

int read_chunk(File* f, int rg, int col, uint8_t* buf, int64_t cap, HsPqChunkInfo* info) {
  memset(info, 0, sizeof(*info));
  info->dict_off = -1;
  f->vruns.clear();
  f->lruns.clear();
  const ChunkMeta& m = f->rgs[(size_t)rg].cols[(size_t)col];
  const SchemaEl& s = f->schema[(size_t)f->leaves[(size_t)col]];
  if (s.repetition == 2) return HS_PQ_UNSUPPORTED;
  const int eb = elem_bytes(m.type);
  if (!eb) return HS_PQ_UNSUPPORTED;
  if (m.codec != 0 && m.codec != 1) return HS_PQ_UNSUPPORTED;
  const bool optional = s.repetition == 1;
  const int64_t start = m.dict_page_offset > 0 && m.dict_page_offset < m.data_page_offset
                            ? m.dict_page_offset : m.data_page_offset;
  const int64_t len = m.total_compressed;
  if (start < 4 || len < 0 || start + len > f->size) return HS_PQ_CORRUPT;
  std::vector<uint8_t> raw((size_t)len);
  if (!pread_all(f->fd, raw.data(), (size_t)len, start)) return HS_PQ_IO;
  int64_t used = 0, rows = 0, dense = 0;
  TReader r{raw.data(), raw.data() + raw.size()};
  while (rows < m.num_values) {
    PageHdr ph;
    if (!parse_page_header(r, ph)) return HS_PQ_CORRUPT;
    if (ph.csize < 0 || ph.usize < 0 || r.end - r.p < ph.csize) return HS_PQ_CORRUPT;
    const uint8_t* payload = r.p;
    r.p += ph.csize;
    const int64_t at = align16(used);
    if (ph.type == 2) {  // dictionary page: PLAIN values
      if (ph.enc != 0 && ph.enc != 2) return HS_PQ_UNSUPPORTED;
      if (at + ph.usize > cap) return HS_PQ_CAPACITY;
      const int64_t got = inflate(m.codec, payload, ph.csize, buf + at, cap - at);
      if (got < 0) return got == -2 ? HS_PQ_UNSUPPORTED : HS_PQ_CORRUPT;
      if (got < (int64_t)ph.dict_nvals * eb) return HS_PQ_CORRUPT;
      info->dict_off = at;
      info->dict_count = ph.dict_nvals;
      used = at + got;
      continue;
    }
    if (ph.type != 0 && ph.type != 3) continue;  // index pages and the like carry no rows
    const bool dict = ph.enc == 2 || ph.enc == 8;
    if (!dict && ph.enc != 0) return HS_PQ_UNSUPPORTED;
    if (at + ph.usize + 8 > cap) return HS_PQ_CAPACITY;
    uint8_t* page = buf + at;
    int64_t plen, vbase = 0, levels_len = 0;
    const uint8_t* levels = nullptr;
    if (ph.v2) {  // levels stay uncompressed ahead of the (optionally compressed) values
      if (ph.v2_rep_len) return HS_PQ_UNSUPPORTED;
      const int64_t lv = ph.v2_def_len;
      if (lv > ph.csize) return HS_PQ_CORRUPT;
      memcpy(page, payload, (size_t)lv);
      const int64_t got = inflate(ph.v2_compressed ? m.codec : 0, payload + lv, ph.csize - lv,
                                  page + lv, cap - at - lv);
      if (got < 0) return got == -2 ? HS_PQ_UNSUPPORTED : HS_PQ_CORRUPT;
      plen = lv + got;
      levels = page;
      levels_len = lv;
      vbase = lv;
    } else {
      plen = inflate(m.codec, payload, ph.csize, page, cap - at);
      if (plen < 0) return plen == -2 ? HS_PQ_UNSUPPORTED : HS_PQ_CORRUPT;
      if (optional) {
        if (ph.def_enc != 3) return HS_PQ_UNSUPPORTED;  // deprecated BIT_PACKED levels
        if (plen < 4) return HS_PQ_CORRUPT;
        uint32_t l32;
        memcpy(&l32, page, 4);
        levels = page + 4;
        levels_len = l32;
        vbase = 4 + (int64_t)l32;
        if (vbase > plen) return HS_PQ_CORRUPT;
      }
    }
    int64_t nonnull = ph.nvals;
    if (optional) {
      const int64_t ones = parse_hybrid(levels, levels_len, at + (levels - page), 1, ph.nvals,
                                        rows, f->lruns, true);
      if (ones < 0) return HS_PQ_CORRUPT;
      nonnull = ones;
    }
    const uint8_t* vals = page + vbase;
    const int64_t vlen = plen - vbase;
    if (dict) {
      if (info->dict_off < 0) return HS_PQ_CORRUPT;
      if (nonnull > 0) {
        if (vlen < 1) return HS_PQ_CORRUPT;
        const int bw = vals[0];
        if (bw > 32) return HS_PQ_CORRUPT;
        if (parse_hybrid(vals + 1, vlen - 1, at + vbase + 1, bw, nonnull, dense, f->vruns,
                         false) < 0)
          return HS_PQ_CORRUPT;
      }
      info->dict_encoded = 1;
    } else {
      if (vlen < nonnull * eb) return HS_PQ_CORRUPT;
      for (int64_t c = 0; c < nonnull; c += kChunk)
        f->vruns.push_back({dense + c, nonnull - c < kChunk ? nonnull - c : kChunk,
                            at + vbase + c * eb, 2, eb});
      info->plain_pages += 1;
    }
    rows += ph.nvals;
    dense += nonnull;
    used = at + plen;
  }
  info->num_values = rows;
  info->num_nonnull = dense;
  info->bytes_used = used;
  info->nvalue_runs = (int64_t)f->vruns.size();
  info->nlevel_runs = (int64_t)f->lruns.size();
  return HS_PQ_OK;
}

}  // namespace

// ------------------------------------------------------------------ device-decode page plan
// One entry per page of a column chunk whose decompression, RLE/bit-packed parsing and value
// expansion all run on the GPU (csrc/kernels/parquet_decode.hip: hs_pq_inflate /
// hs_pq_expand).  The host only preads the raw (compressed) chunk and walks the page headers.
// Layout shared with the kernels; `out` and `dict` are absolute device addresses the caller
// fills in once the device buffers exist.
struct HsPqPage {
  int64_t src;      // payload offset in the raw (compressed) buffer
  int64_t dst;      // offset of the decompressed page in the scratch buffer (16-byte aligned)
  int64_t out;      // device address of the page's first output value (data pages)
  int64_t dict;     // device address of the chunk's decompressed dictionary (0: none)
  int64_t row;      // first row of the page within its chunk
  int32_t csize;    // payload bytes as stored
  int32_t usize;    // bytes after decompression (levels included)
  int32_t nvals;    // rows of the page (data pages) / dictionary entries (dictionary page)
  int32_t codec;    // 0 uncompressed, 1 snappy
  int32_t kind;     // 0 data v1, 1 data v2, 2 dictionary
  int32_t enc;      // 0 PLAIN, 2 / 8 dictionary indices, 3 RLE (booleans)
  int32_t levels;   // v1: 1 if a length-prefixed definition-level stream precedes the values;
                    // v2: byte length of the (never compressed) level streams
  int32_t eb;       // element bytes (4 / 8; 1: BOOLEAN, one byte per value)
  int32_t dict_page;  // index (within the plan) of the chunk's dictionary page, -1: none
  int32_t nulls;    // 1: the page may hold nulls - its definition levels decode to validity
                    // bytes at `valid` and the dense values spread to their rows
  int64_t valid;    // device address of the page's first validity byte (caller fills it in)
};

namespace {

// Plan one chunk: pread its raw bytes to `raw + at` and describe every page.  `dst_at` is the
// scratch offset where this chunk's first decompressed page goes; returns the scratch bytes
// used via *dst_used.  Chunks with repetition, unsupported codecs or encodings are reported as
// HS_PQ_UNSUPPORTED (the caller decodes them another way).
int plan_chunk(File* f, int rg, int col, uint8_t* raw, int64_t raw_cap, int64_t raw_at,
               int64_t dst_at, HsPqPage* pages, int max_pages, int* npages, int64_t* raw_used,
               int64_t* dst_used, uint8_t* hbuf, int64_t hcap, int64_t h_at, int64_t* h_used) {
  *npages = 0;
  const ChunkMeta& m = f->rgs[(size_t)rg].cols[(size_t)col];
  const SchemaEl& s = f->schema[(size_t)f->leaves[(size_t)col]];
  if (s.repetition == 2) return HS_PQ_UNSUPPORTED;
  // BYTE_ARRAY: only dictionary-encoded chunks.  The dictionary page is inflated here (the
  // caller parses its strings, hs_pq_plain_strings) and the data pages decode on the device to
  // 4-byte dictionary codes through a code table the caller supplies in `dict`.
  const bool strings = m.type == 6;
  // BOOLEAN: bit-packed PLAIN or length-prefixed RLE (bit width 1) values, one byte per row out
  const bool boolean = m.type == 0;
  const int eb = strings ? 4 : (boolean ? 1 : elem_bytes(m.type));
  if (!eb) return HS_PQ_UNSUPPORTED;
  if (strings && !hbuf) return HS_PQ_UNSUPPORTED;
  if (m.codec != 0 && m.codec != 1) return HS_PQ_UNSUPPORTED;
  const bool optional = s.repetition == 1;
  // chunks with nulls (or without a null count): the kernels decode the definition levels too,
  // unless disabled (hs_pq_set_device_nulls), in which case another path decodes the chunk
  const bool nullable = optional && m.null_count != 0;
  if (nullable && !g_device_nulls.load(std::memory_order_relaxed)) return HS_PQ_NULLS;
  const int64_t start = m.dict_page_offset > 0 && m.dict_page_offset < m.data_page_offset
                            ? m.dict_page_offset : m.data_page_offset;
  const int64_t len = m.total_compressed;
  if (start < 4 || len < 0 || start + len > f->size) return HS_PQ_CORRUPT;
  if (raw_at + len > raw_cap) return HS_PQ_CAPACITY;
  uint8_t* base = raw + raw_at;
  if (!pread_all(f->fd, base, (size_t)len, start)) return HS_PQ_IO;
  TReader r{base, base + len};
  int64_t rows = 0, dst = dst_at, hat = h_at;
  int dict_idx = -1;
  while (rows < m.num_values) {
    PageHdr ph;
    if (!parse_page_header(r, ph)) return HS_PQ_CORRUPT;
    if (ph.csize < 0 || ph.usize < 0 || r.end - r.p < ph.csize) return HS_PQ_CORRUPT;
    const int64_t payload = raw_at + (r.p - base);
    r.p += ph.csize;
    if (ph.type != 0 && ph.type != 2 && ph.type != 3) continue;   // index pages etc.
    if (*npages >= max_pages) return HS_PQ_CAPACITY;
    HsPqPage& p = pages[*npages];
    memset(&p, 0, sizeof(p));
    p.src = payload;
    p.dst = (dst + 15) & ~(int64_t)15;
    p.csize = ph.csize;
    p.codec = m.codec;
    p.eb = eb;
    p.dict_page = -1;
    if (ph.type == 2) {
      if (boolean || (ph.enc != 0 && ph.enc != 2)) return HS_PQ_UNSUPPORTED;
      p.kind = 2;
      p.usize = ph.usize;
      p.nvals = ph.dict_nvals;
      if ((int64_t)ph.dict_nvals * (strings ? 4 : eb) > ph.usize || ph.dict_nvals < 0)
        return HS_PQ_CORRUPT;
      dict_idx = *npages;
    } else {
      const bool dict = !boolean && (ph.enc == 2 || ph.enc == 8);
      if (!dict && ph.enc != 0 && !(boolean && ph.enc == 3)) return HS_PQ_UNSUPPORTED;
      // PLAIN strings (eb 16): each value's address and length; the caller hashes them into
      // codes (io/native_parquet.StringCodes.finish_plain)
      if (strings && !dict) {
        if (ph.enc != 0 || !g_plain_strings.load(std::memory_order_relaxed))
          return HS_PQ_UNSUPPORTED;
        p.eb = 16;
      }
      if (dict && dict_idx < 0) return HS_PQ_CORRUPT;
      p.enc = ph.enc;
      p.nvals = ph.nvals;
      p.row = rows;
      p.nulls = nullable ? 1 : 0;
      p.dict_page = dict ? dict_idx : -1;
      if (ph.v2) {
        if (ph.v2_rep_len) return HS_PQ_UNSUPPORTED;
        if (ph.v2_def_len > ph.csize) return HS_PQ_CORRUPT;
        p.kind = 1;
        p.levels = ph.v2_def_len;
        if (!ph.v2_compressed) p.codec = 0;
        p.usize = ph.usize;
      } else {
        if (optional && ph.def_enc != 3) return HS_PQ_UNSUPPORTED;
        p.kind = 0;
        p.levels = optional ? 1 : 0;
        p.usize = ph.usize;
      }
      rows += ph.nvals;
    }
    if (p.codec == 0 && p.csize != p.usize) return HS_PQ_CORRUPT;
    // Snappy pages that actually compressed are chains of short tags (a tag every few bytes),
    // which a wavefront resolves at ~14 us per 64 tags; literal-dominated pages (bit-packed
    // dictionary indices, random values) inflate on the device at copy speed.  Inflate the
    // former here, like large dictionary pages (a dense chain of short copies): codec 2 =
    // host-inflated, `src` = offset in the handle's host_pages buffer (levels included).
    const int mode = g_host_inflate.load(std::memory_order_relaxed);
    const bool big_dict = p.kind == 2 && p.usize > kHostDictMin;
    const bool str_dict = strings && p.kind == 2;
    bool dense = str_dict || (p.codec == 1 && mode > 0 &&
        (big_dict || (mode > 1 && (int64_t)p.usize * 10 >= (int64_t)p.csize * 11)));
    // mode 3: every third tag-dense data page stays on the device, so host and device inflate
    // concurrently (a batched device decode keeps up with about half the host's share)
    if (mode == 3 && dense && !str_dict && !big_dict && p.kind != 2 &&
        p.usize <= kDeviceInflateMax && (*npages % 3) == 2)
      dense = false;
    // one wavefront inflates one page on the device: a multi-MB Snappy page left to it runs for
    // seconds (profiles/cold_load_r2.jsonl: 58 s for an index of 1M-row pages), so such a
    // column goes to the host page layer instead
    if (p.codec == 1 && !(dense && hbuf) && p.usize > kDeviceInflateMax) return HS_PQ_UNSUPPORTED;
    if (dense && hbuf) {
      const int lv = p.kind == 1 ? p.levels : 0;
      const uint8_t* src = base + (payload - raw_at);
      const int64_t at = (hat + 15) & ~(int64_t)15;
      if (at + p.usize + 16 > hcap) return HS_PQ_CAPACITY;
      memcpy(hbuf + at, src, (size_t)lv);
      if (p.codec == 0) {
        memcpy(hbuf + at, src, (size_t)p.usize);
      } else {
        size_t got = 0;
        if (!snappy_decompress(src + lv, (size_t)(p.csize - lv), hbuf + at + lv,
                               (size_t)(p.usize - lv), &got) ||
            got != (size_t)(p.usize - lv))
          return HS_PQ_CORRUPT;
      }
      p.codec = 2;
      p.src = at;
      hat = at + p.usize + 16;
      ++*npages;
      continue;                      // occupies no device scratch
    }
    dst = p.dst + p.usize + 16;   // + slack: the kernels read 8-byte windows
    ++*npages;
  }
  if (rows != m.num_values) return HS_PQ_CORRUPT;
  *raw_used = len;
  *dst_used = dst - dst_at;
  *h_used = hat - h_at;
  return HS_PQ_OK;
}

}  // namespace

extern "C" {

const char* hs_pq_error(void* h) { return h ? ((File*)h)->error.c_str() : "null handle"; }

// Raw (compressed) bytes of a chunk as stored: the pread size of hs_pq_plan_chunk.
int64_t hs_pq_chunk_raw_bytes(void* h, int rg, int col) {
  return ((File*)h)->rgs[(size_t)rg].cols[(size_t)col].total_compressed;
}

// Upper bound of the pages of a chunk (uncompressed bytes / 1 KiB + 64): sizes the page table.
int64_t hs_pq_chunk_max_pages(void* h, int rg, int col) {
  const ChunkMeta& m = ((File*)h)->rgs[(size_t)rg].cols[(size_t)col];
  return m.total_uncompressed / 1024 + m.num_values / 1024 + 64;
}

// `hbuf` (capacity `hcap`, next free offset `h_at`): where pages the host inflates go (codec 2,
// `src` = offset in hbuf); null keeps every page for the device.  Sized by the caller from
// hs_pq_chunk_host_bound.
int hs_pq_plan_chunk(void* h, int rg, int col, uint8_t* raw, int64_t raw_cap, int64_t raw_at,
                     int64_t dst_at, HsPqPage* pages, int max_pages, int* npages,
                     int64_t* raw_used, int64_t* dst_used, uint8_t* hbuf, int64_t hcap,
                     int64_t h_at, int64_t* h_used) {
  return plan_chunk((File*)h, rg, col, raw, raw_cap, raw_at, dst_at, pages, max_pages, npages,
                    raw_used, dst_used, hbuf, hcap, h_at, h_used);
}

// Bytes that bound what hs_pq_plan_chunk may inflate into the host buffer for this chunk.
// Which Snappy pages the planner inflates on the host (codec 2): 0 none (every page inflates
// on the device), 1 large dictionary pages only, 2 those and tag-dense data pages (default),
// 3 as 2 but every third tag-dense data page is left to the device.
void hs_pq_set_host_inflate(int mode) { g_host_inflate.store(mode, std::memory_order_relaxed); }

// 1 (default): device page plans accept chunks with nulls (levels decoded on the device);
// 0: such chunks report HS_PQ_NULLS and go through the host page layer.
void hs_pq_set_device_nulls(int on) { g_device_nulls.store(on, std::memory_order_relaxed); }

// 1 (default): PLAIN BYTE_ARRAY data pages plan as eb-16 pages (value addresses + lengths on
// the device); 0: such chunks report HS_PQ_UNSUPPORTED and are read another way.
void hs_pq_set_plain_strings(int on) { g_plain_strings.store(on, std::memory_order_relaxed); }

int64_t hs_pq_chunk_host_bound(void* h, int rg, int col) {
  const ChunkMeta& m = ((File*)h)->rgs[(size_t)rg].cols[(size_t)col];
  return m.total_uncompressed + 32 * hs_pq_chunk_max_pages(h, rg, col) + 64;
}

int hs_pq_page_size() { return (int)sizeof(HsPqPage); }

// A PLAIN BYTE_ARRAY stream (`n` values of 4-byte little-endian length + bytes, as in a
// dictionary page) to Arrow string layout: offsets[n + 1] (int32) and the concatenated bytes in
// `chars` (capacity `cap`, at most `len`).  Returns the byte count, or -1 when the stream is
// shorter than its lengths say.
int64_t hs_pq_plain_strings(const uint8_t* src, int64_t len, int64_t n, int32_t* offsets,
                            uint8_t* chars, int64_t cap) {
  int64_t at = 0, out = 0;
  offsets[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (at + 4 > len) return -1;
    uint32_t l;
    memcpy(&l, src + at, 4);
    at += 4;
    if ((int64_t)l > len - at || out + (int64_t)l > cap || out + (int64_t)l > INT32_MAX)
      return -1;
    memcpy(chars + out, src + at, l);
    at += l;
    out += l;
    offsets[i + 1] = (int32_t)out;
  }
  return out;
}


// Opens a file and parses its footer.  Always returns a handle (check hs_pq_ok / hs_pq_error;
// release with hs_pq_close).
void* hs_pq_open(const char* path) {
  File* f = new File();
  open_file(path, *f);
  return f;
}

int hs_pq_ok(void* h) { return ((File*)h)->fd >= 0 && ((File*)h)->error.empty() ? 1 : 0; }

void hs_pq_close(void* h) {
  File* f = (File*)h;
  if (!f) return;
  if (f->fd >= 0) close(f->fd);
  delete f;
}

int64_t hs_pq_num_rows(void* h) { return ((File*)h)->num_rows; }
int hs_pq_num_row_groups(void* h) { return (int)((File*)h)->rgs.size(); }
int64_t hs_pq_row_group_rows(void* h, int rg) { return ((File*)h)->rgs[(size_t)rg].num_rows; }
int hs_pq_num_columns(void* h) { return (int)((File*)h)->leaves.size(); }

// Leaf column by top-level name in a flat schema; -1 if absent (or the schema is nested).
int hs_pq_find_column(void* h, const char* name) {
  File* f = (File*)h;
  if (f->schema.size() != f->leaves.size() + 1) return -1;
  for (size_t i = 0; i < f->leaves.size(); ++i)
    if (f->schema[(size_t)f->leaves[i]].name == name) return (int)i;
  return -1;
}

// physical type, max definition level (0 required / 1 optional), element bytes (0: the native
// path does not decode this column)
int hs_pq_column_info(void* h, int col, int* type, int* max_def, int* ebytes) {
  File* f = (File*)h;
  const SchemaEl& s = f->schema[(size_t)f->leaves[(size_t)col]];
  *type = s.type;
  *max_def = s.repetition == 1 ? 1 : 0;
  *ebytes = s.repetition == 2 ? 0 : elem_bytes(s.type);
  return HS_PQ_OK;
}

// Buffer bytes that suffice for hs_pq_read_chunk of this column chunk.
int64_t hs_pq_chunk_bound(void* h, int rg, int col) {
  const ChunkMeta& m = ((File*)h)->rgs[(size_t)rg].cols[(size_t)col];
  return m.total_uncompressed + 16 * 64 + 64;  // + per-page alignment / slack
}

// Read, decompress and pre-parse one column chunk into `buf` (dictionary page first, then the
// data pages back to back, each 16-byte aligned).  The run tables stay in the handle until the
// next call; fetch them with hs_pq_copy_runs.
int hs_pq_read_chunk(void* h, int rg, int col, uint8_t* buf, int64_t cap, HsPqChunkInfo* info) {
  return read_chunk((File*)h, rg, col, buf, cap, info);
}

// Copy the last chunk's run tables out, adding `src_base` to every buffer offset (so several
// chunks can share one device buffer) and `dst_base` to every output index.
int hs_pq_copy_runs(void* h, HsPqRun* vdst, HsPqRun* ldst, int64_t src_base, int64_t dst_base) {
  File* f = (File*)h;
  for (size_t i = 0; i < f->vruns.size(); ++i) {
    HsPqRun r = f->vruns[i];
    if (r.kind != 0) r.src += src_base;
    r.dst += dst_base;
    vdst[i] = r;
  }
  for (size_t i = 0; i < f->lruns.size(); ++i) {
    HsPqRun r = f->lruns[i];
    if (r.kind != 0) r.src += src_base;
    r.dst += dst_base;
    ldst[i] = r;
  }
  return HS_PQ_OK;
}

int hs_pq_run_size() { return (int)sizeof(HsPqRun); }
int hs_pq_info_size() { return (int)sizeof(HsPqChunkInfo); }

// Snappy decompression hook for tests.
int64_t hs_pq_snappy_decompress(const uint8_t* in, int64_t n, uint8_t* out, int64_t cap) {
  size_t got = 0;
  return snappy_decompress(in, (size_t)n, out, (size_t)cap, &got) ? (int64_t)got : -1;
}

}  // extern "C"
