// Native Parquet writer for index bucket files (SURVEY.md §2.3 K4 "Parquet encode").
//
// The MI355X does the encoding work — dictionary build, code assignment and bit-packing run in
// HIP kernels (exec/pq_encode.py + csrc/kernels/parquet_encode.hip) — so a column chunk arrives
// here as ready page payload in pinned host memory: PLAIN values, or bit-packed dictionary codes.
// This file only frames it: Thrift-compact page headers, definition levels (all valid: one RLE
// run), the dictionary page, and the footer; payload bytes go to the file with pwritev straight
// from the pinned buffers (no host-side copy or re-encode).
//
// Output: Parquet format 1 files with data page V1, codec UNCOMPRESSED, optional flat columns,
// readable by Spark, pyarrow and the native reader in hs_parquet.cpp.
#include <fcntl.h>
#include <sys/uio.h>
#include <unistd.h>

#include <cerrno>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace {

// ------------------------------------------------------------------ Thrift compact writer
struct TWriter {
  std::vector<uint8_t> b;
  std::vector<int16_t> last{0};

  void byte(uint8_t v) { b.push_back(v); }
  void varint(uint64_t v) {
    while (v >= 0x80) { b.push_back((uint8_t)(v | 0x80)); v >>= 7; }
    b.push_back((uint8_t)v);
  }
  void zz(int64_t v) { varint(((uint64_t)v << 1) ^ (uint64_t)(v >> 63)); }
  void field(int16_t id, int type) {
    const int16_t d = (int16_t)(id - last.back());
    if (d > 0 && d <= 15) byte((uint8_t)((d << 4) | type));
    else { byte((uint8_t)type); zz(id); }
    last.back() = id;
  }
  void i32(int16_t id, int64_t v) { field(id, 5); zz(v); }
  void i64(int16_t id, int64_t v) { field(id, 6); zz(v); }
  void str(int16_t id, const std::string& s) { field(id, 8); varint(s.size()); bin(s); }
  void bin(const std::string& s) { b.insert(b.end(), s.begin(), s.end()); }
  void begin_struct(int16_t id) { field(id, 12); last.push_back(0); }
  void begin_anon_struct() { last.push_back(0); }  // list element
  void end_struct() { byte(0); last.pop_back(); }
  void list(int16_t id, int elem_type, int64_t n) {
    field(id, 9);
    if (n < 15) byte((uint8_t)((n << 4) | elem_type));
    else { byte((uint8_t)(0xf0 | elem_type)); varint((uint64_t)n); }
  }
};

}  // namespace

// Per column chunk (one row group) handed over by Python.
struct HsPqWCol {
  const char* name;
  int32_t ptype;          // 1 INT32, 2 INT64, 4 FLOAT, 5 DOUBLE, 6 BYTE_ARRAY
  int32_t logical;        // 0 none, 1 DATE, 2 STRING
  int32_t dict;           // 1: payload is bit-packed dictionary codes
  int32_t bit_width;      // dict code width
  const uint8_t* dict_page;  // PLAIN dictionary values (fixed width, or BYTE_ARRAY len+bytes)
  int64_t dict_bytes;
  int64_t dict_count;
  const uint8_t* payload;    // PLAIN values or packed codes (ceil(n/8)*bit_width bytes)
  int64_t payload_bytes;
  // codec 1 (SNAPPY): dict_page is a whole Snappy stream of dict_raw_bytes; payload holds the
  // Snappy elements (no length preamble) of payload_raw_bytes encoded bytes, compressed on the
  // device (csrc/kernels/snappy_encode.hip)
  int64_t dict_raw_bytes;
  int64_t payload_raw_bytes;
  int32_t codec;             // 0 UNCOMPRESSED, 1 SNAPPY
  int32_t pad;
};

namespace {

struct ColPos {
  int64_t dict_off = -1, data_off = 0, total = 0, raw_total = 0;
};

void put_varint(std::vector<uint8_t>& v, uint64_t x) {
  while (x >= 0x80) { v.push_back((uint8_t)(x | 0x80)); x >>= 7; }
  v.push_back((uint8_t)x);
}

void def_levels_all_valid(std::vector<uint8_t>& v, int64_t n) {
  // 4-byte length prefix + one RLE run (header (n << 1), value 1 in one byte)
  std::vector<uint8_t> run;
  uint64_t h = (uint64_t)n << 1;
  while (h >= 0x80) { run.push_back((uint8_t)(h | 0x80)); h >>= 7; }
  run.push_back((uint8_t)h);
  run.push_back(1);
  const uint32_t len = (uint32_t)run.size();
  v.insert(v.end(), (const uint8_t*)&len, (const uint8_t*)&len + 4);
  v.insert(v.end(), run.begin(), run.end());
}

std::vector<uint8_t> page_header(int type, int64_t size, int64_t nvals, int enc,
                                 int64_t raw_size = -1) {
  TWriter w;
  w.i32(1, type);
  w.i32(2, raw_size < 0 ? size : raw_size);   // uncompressed_page_size
  w.i32(3, size);                             // compressed_page_size
  if (type == 2) {
    w.begin_struct(7);
    w.i32(1, nvals);
    w.i32(2, enc);
    w.end_struct();
  } else {
    w.begin_struct(5);
    w.i32(1, nvals);
    w.i32(2, enc);
    w.i32(3, 3);  // definition levels: RLE
    w.i32(4, 3);  // repetition levels: RLE
    w.end_struct();
  }
  w.byte(0);
  return w.b;
}

bool write_all(int fd, std::vector<iovec>& iov, int64_t& pos) {
  size_t i = 0;
  while (i < iov.size()) {
    const int cnt = (int)std::min<size_t>(iov.size() - i, 512);
    ssize_t k = pwritev(fd, iov.data() + i, cnt, pos);
    if (k < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    pos += k;
    while (k > 0 && i < iov.size()) {   // advance past fully written vectors
      if ((size_t)k >= iov[i].iov_len) { k -= (ssize_t)iov[i].iov_len; ++i; }
      else {
        iov[i].iov_base = (uint8_t*)iov[i].iov_base + k;
        iov[i].iov_len -= (size_t)k;
        k = 0;
      }
    }
  }
  return true;
}

}  // namespace

extern "C" {

// Write one Parquet file: `ncols` columns x `nrg` row groups (cols[rg * ncols + c]),
// rg_rows[rg] rows each, no nulls.  Returns 0 or -errno.
int hs_pq_write_file(const char* path, int ncols, int nrg, const int64_t* rg_rows,
                     const HsPqWCol* cols, const char* created_by) {
  const std::string tmp = std::string(path);
  const int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) return -errno;
  int64_t pos = 0;
  std::vector<std::vector<uint8_t>> keep;   // header bytes referenced by iovecs
  keep.reserve((size_t)ncols * nrg * 4 + 4);
  std::vector<iovec> iov;
  static const char magic[4] = {'P', 'A', 'R', '1'};
  iov.push_back({(void*)magic, 4});
  int64_t off = 4;
  std::vector<ColPos> posv((size_t)ncols * nrg);
  for (int g = 0; g < nrg; ++g) {
    const int64_t n = rg_rows[g];
    for (int c = 0; c < ncols; ++c) {
      const HsPqWCol& col = cols[(size_t)g * ncols + c];
      ColPos& p = posv[(size_t)g * ncols + c];
      const int64_t start = off;
      const bool snappy = col.codec == 1;
      if (col.dict) {
        const int64_t raw = snappy ? col.dict_raw_bytes : col.dict_bytes;
        keep.push_back(page_header(2, col.dict_bytes, col.dict_count, 0, raw));
        p.dict_off = off;
        iov.push_back({keep.back().data(), keep.back().size()});
        iov.push_back({(void*)col.dict_page, (size_t)col.dict_bytes});
        off += (int64_t)keep.back().size() + col.dict_bytes;
        p.raw_total += (int64_t)keep.back().size() + raw;
      }
      std::vector<uint8_t> pre;
      def_levels_all_valid(pre, n);
      if (col.dict) {
        pre.push_back((uint8_t)col.bit_width);
        uint64_t h = ((uint64_t)((n + 7) / 8) << 1) | 1;  // one bit-packed run
        while (h >= 0x80) { pre.push_back((uint8_t)(h | 0x80)); h >>= 7; }
        pre.push_back((uint8_t)h);
      }
      int64_t raw_psize = (int64_t)pre.size() + col.payload_bytes;
      if (snappy) {
        // Snappy stream: varint(uncompressed size), the levels/width prefix as one literal
        // element, then the device-compressed elements of the payload
        raw_psize = (int64_t)pre.size() + col.payload_raw_bytes;
        std::vector<uint8_t> z;
        put_varint(z, (uint64_t)raw_psize);
        z.push_back((uint8_t)((pre.size() - 1) << 2));   // prefix < 60 bytes
        z.insert(z.end(), pre.begin(), pre.end());
        pre.swap(z);
      }
      const int64_t psize = (int64_t)pre.size() + col.payload_bytes;
      keep.push_back(page_header(0, psize, n, col.dict ? 8 : 0, raw_psize));
      p.data_off = off;
      iov.push_back({keep.back().data(), keep.back().size()});
      off += (int64_t)keep.back().size();
      p.raw_total += (int64_t)keep.back().size() + raw_psize;
      keep.push_back(std::move(pre));
      iov.push_back({keep.back().data(), keep.back().size()});
      if (col.payload_bytes) iov.push_back({(void*)col.payload, (size_t)col.payload_bytes});
      off += psize;
      p.total = off - start;
    }
  }
  // footer
  TWriter w;
  w.i32(1, 1);
  w.list(2, 12, ncols + 1);
  w.begin_anon_struct();
  w.str(4, "schema");
  w.i32(5, ncols);
  w.end_struct();
  for (int c = 0; c < ncols; ++c) {
    const HsPqWCol& col = cols[c];
    w.begin_anon_struct();
    w.i32(1, col.ptype);
    w.i32(3, 1);  // OPTIONAL
    w.str(4, col.name);
    if (col.logical == 1) w.i32(6, 6);        // converted type DATE
    else if (col.logical == 2) w.i32(6, 0);   // UTF8
    if (col.logical) {
      w.begin_struct(10);                       // LogicalType union
      w.begin_struct(col.logical == 1 ? 6 : 1);  // DateType / StringType
      w.end_struct();
      w.end_struct();
    }
    w.end_struct();
  }
  int64_t total_rows = 0;
  for (int g = 0; g < nrg; ++g) total_rows += rg_rows[g];
  w.i64(3, total_rows);
  w.list(4, 12, nrg);
  for (int g = 0; g < nrg; ++g) {
    w.begin_anon_struct();
    w.list(1, 12, ncols);
    int64_t rg_bytes = 0;
    for (int c = 0; c < ncols; ++c) {
      const HsPqWCol& col = cols[(size_t)g * ncols + c];
      const ColPos& p = posv[(size_t)g * ncols + c];
      rg_bytes += p.raw_total;
      w.begin_anon_struct();                   // ColumnChunk
      w.i64(2, p.dict_off >= 0 ? p.dict_off : p.data_off);
      w.begin_struct(3);                       // ColumnMetaData
      w.i32(1, col.ptype);
      if (col.dict) {
        w.list(2, 5, 3);
        w.zz(0); w.zz(3); w.zz(8);              // PLAIN, RLE, RLE_DICTIONARY
      } else {
        w.list(2, 5, 2);
        w.zz(0); w.zz(3);                       // PLAIN, RLE
      }
      w.list(3, 8, 1);
      w.varint(strlen(col.name));
      w.bin(col.name);
      w.i32(4, col.codec == 1 ? 1 : 0);         // SNAPPY / UNCOMPRESSED
      w.i64(5, rg_rows[g]);
      w.i64(6, p.raw_total);                    // total_uncompressed_size
      w.i64(7, p.total);                        // total_compressed_size
      w.i64(9, p.data_off);
      if (p.dict_off >= 0) w.i64(11, p.dict_off);
      // Statistics { 3: null_count = 0 }: every index column the device encoder writes is
      // null-free, and readers (our device page planner, hs_parquet.cpp) take the null-free
      // decode path only when the footer says so
      w.begin_struct(12);
      w.i64(3, 0);
      w.end_struct();
      w.end_struct();
      w.end_struct();
    }
    w.i64(2, rg_bytes);
    w.i64(3, rg_rows[g]);
    w.end_struct();
  }
  w.str(6, created_by ? created_by : "hyperspace_amd");
  w.byte(0);
  keep.push_back(std::move(w.b));
  const uint32_t flen = (uint32_t)keep.back().size();
  iov.push_back({keep.back().data(), keep.back().size()});
  std::vector<uint8_t> tail(8);
  memcpy(tail.data(), &flen, 4);
  memcpy(tail.data() + 4, magic, 4);
  keep.push_back(std::move(tail));
  iov.push_back({keep.back().data(), 8});
  const bool ok = write_all(fd, iov, pos);
  const int err = ok ? 0 : -errno;
  if (close(fd) != 0 && ok) return -errno;
  return err;
}

// ------------------------------------------------------------------ general writer (v2)
// One data page of a column chunk.  Definition levels (nullable columns) and values arrive as
// separate device-encoded segments: the level bits of one bit-packed run (1 bit per row, LSB
// first) and the value payload (PLAIN values of the non-null rows, bit-packed dictionary codes,
// or bit-packed BOOLEANs).  With codec 1 each segment holds the Snappy elements of its raw bytes
// (no preamble); the small host parts of the page (level length + run header, dictionary bit
// width + run header) go in as literal elements.
struct HsPqWPage {
  const uint8_t* levels;
  int64_t levels_bytes;
  int64_t levels_raw;     // ceil(nvals / 8)
  const uint8_t* payload;
  int64_t payload_bytes;
  int64_t payload_raw;
  int64_t nvals;          // rows of the page (nulls included)
  int64_t nonnull;        // non-null rows (= values encoded)
};

struct HsPqWCol2 {
  const char* name;
  int32_t ptype;          // 0 BOOLEAN, 1 INT32, 2 INT64, 4 FLOAT, 5 DOUBLE, 6 BYTE_ARRAY
  int32_t logical;        // 0 none, 1 DATE, 2 STRING, 3 INT, 4 TIMESTAMP, 5 DECIMAL
  int32_t lp0;            // INT: bit width | TIMESTAMP: unit 0 ms, 1 us, 2 ns | DECIMAL: precision
  int32_t lp1;            // INT: signed | TIMESTAMP: adjusted to UTC | DECIMAL: scale
  int32_t dict;
  int32_t bit_width;
  int32_t codec;
  int32_t nullable;
  const uint8_t* dict_page;
  int64_t dict_bytes;
  int64_t dict_count;
  int64_t dict_raw_bytes;
  int64_t null_count;
  const HsPqWPage* pages;
  int32_t npages;
  int32_t pad;
};

namespace {

void literal(std::vector<uint8_t>& z, const std::vector<uint8_t>& raw) {
  // Snappy literal element(s) of a small host byte string
  size_t i = 0;
  while (i < raw.size()) {
    const size_t n = std::min<size_t>(raw.size() - i, 60);
    z.push_back((uint8_t)((n - 1) << 2));
    z.insert(z.end(), raw.begin() + (long)i, raw.begin() + (long)(i + n));
    i += n;
  }
}

void schema_element(TWriter& w, const HsPqWCol2& col) {
  w.begin_anon_struct();
  w.i32(1, col.ptype);
  w.i32(3, 1);   // OPTIONAL (as Spark writes every column of a DataFrame)
  w.str(4, col.name);
  // converted_type (6) for older readers, scale (7) / precision (8) for DECIMAL
  switch (col.logical) {
    case 1: w.i32(6, 6); break;                                   // DATE
    case 2: w.i32(6, 0); break;                                   // UTF8
    case 3: w.i32(6, (col.lp1 ? 15 : 11) + (col.lp0 == 8 ? 0 : col.lp0 == 16 ? 1 :
                                             col.lp0 == 32 ? 2 : 3)); break;   // INT_x / UINT_x
    case 4: if (col.lp0 <= 1) w.i32(6, col.lp0 == 0 ? 9 : 10); break;          // TIMESTAMP_*
    case 5: w.i32(6, 5); w.i32(7, col.lp1); w.i32(8, col.lp0); break;         // DECIMAL
    default: break;
  }
  if (col.logical) {
    w.begin_struct(10);               // LogicalType union
    switch (col.logical) {
      case 1: w.begin_struct(6); w.end_struct(); break;          // DATE
      case 2: w.begin_struct(1); w.end_struct(); break;          // STRING
      case 3:                                                    // INTEGER
        w.begin_struct(10);
        w.field(1, 3); w.byte((uint8_t)col.lp0);                 // i8 bitWidth
        w.field(2, col.lp1 ? 1 : 2);                             // bool isSigned
        w.end_struct();
        break;
      case 4:                                                    // TIMESTAMP
        w.begin_struct(8);
        w.field(1, col.lp1 ? 1 : 2);                             // isAdjustedToUTC
        w.begin_struct(2);                                       // TimeUnit union
        w.begin_struct(col.lp0 == 0 ? 1 : col.lp0 == 1 ? 2 : 3); w.end_struct();
        w.end_struct();
        w.end_struct();
        break;
      case 5:                                                    // DECIMAL
        w.begin_struct(5);
        w.i32(1, col.lp1);                                       // scale
        w.i32(2, col.lp0);                                       // precision
        w.end_struct();
        break;
      default: break;
    }
    w.end_struct();
  }
  w.end_struct();
}

}  // namespace

// Write one Parquet file: `ncols` columns x `nrg` row groups (cols[rg * ncols + c]), each
// column chunk one optional dictionary page plus `npages` data pages.  Returns 0 or -errno.
int hs_pq_write_file2(const char* path, int ncols, int nrg, const int64_t* rg_rows,
                      const HsPqWCol2* cols, const char* created_by) {
  const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) return -errno;
  int64_t pos = 0;
  std::vector<std::vector<uint8_t>> keep;
  std::vector<iovec> iov;
  static const char magic[4] = {'P', 'A', 'R', '1'};
  iov.push_back({(void*)magic, 4});
  int64_t off = 4;
  std::vector<ColPos> posv((size_t)ncols * nrg);
  size_t reserve = 4;
  for (int i = 0; i < ncols * nrg; ++i) reserve += 8 + 6 * (size_t)cols[i].npages;
  keep.reserve(reserve);   // iovecs point into keep's elements: never reallocate
  for (int g = 0; g < nrg; ++g) {
    for (int c = 0; c < ncols; ++c) {
      const HsPqWCol2& col = cols[(size_t)g * ncols + c];
      ColPos& p = posv[(size_t)g * ncols + c];
      const int64_t start = off;
      const bool snappy = col.codec == 1;
      if (col.dict) {
        const int64_t raw = snappy ? col.dict_raw_bytes : col.dict_bytes;
        keep.push_back(page_header(2, col.dict_bytes, col.dict_count, 0, raw));
        p.dict_off = off;
        iov.push_back({keep.back().data(), keep.back().size()});
        iov.push_back({(void*)col.dict_page, (size_t)col.dict_bytes});
        off += (int64_t)keep.back().size() + col.dict_bytes;
        p.raw_total += (int64_t)keep.back().size() + raw;
      }
      p.data_off = off;
      for (int q = 0; q < col.npages; ++q) {
        const HsPqWPage& pg = col.pages[q];
        // host parts: level length + run header, value run header
        std::vector<uint8_t> lpre, vpre;
        if (col.nullable) {
          std::vector<uint8_t> run;
          put_varint(run, ((uint64_t)((pg.nvals + 7) / 8) << 1) | 1);
          const uint32_t len = (uint32_t)(run.size() + pg.levels_raw);
          lpre.insert(lpre.end(), (const uint8_t*)&len, (const uint8_t*)&len + 4);
          lpre.insert(lpre.end(), run.begin(), run.end());
        } else {
          def_levels_all_valid(lpre, pg.nvals);   // one RLE run of 1s, no device bytes
        }
        if (col.dict) {
          vpre.push_back((uint8_t)col.bit_width);
          if (pg.nonnull > 0) put_varint(vpre, ((uint64_t)((pg.nonnull + 7) / 8) << 1) | 1);
        }
        const int64_t lraw = col.nullable ? pg.levels_raw : 0;
        const int64_t raw_size = (int64_t)lpre.size() + lraw + (int64_t)vpre.size() +
                                 pg.payload_raw;
        std::vector<uint8_t> head, mid;   // bytes before the level bits / before the payload
        if (snappy) {
          put_varint(head, (uint64_t)raw_size);
          if (!lpre.empty()) literal(head, lpre);
          if (!vpre.empty()) literal(mid, vpre);
        } else {
          head = lpre;
          mid = vpre;
        }
        const int64_t lbytes = col.nullable ? pg.levels_bytes : 0;
        const int64_t psize = (int64_t)head.size() + lbytes + (int64_t)mid.size() +
                              pg.payload_bytes;
        keep.push_back(page_header(0, psize, pg.nvals, col.dict ? 8 : 0, raw_size));
        iov.push_back({keep.back().data(), keep.back().size()});
        off += (int64_t)keep.back().size();
        p.raw_total += (int64_t)keep.back().size() + raw_size;
        if (!head.empty()) {
          keep.push_back(std::move(head));
          iov.push_back({keep.back().data(), keep.back().size()});
        }
        if (lbytes) iov.push_back({(void*)pg.levels, (size_t)lbytes});
        if (!mid.empty()) {
          keep.push_back(std::move(mid));
          iov.push_back({keep.back().data(), keep.back().size()});
        }
        if (pg.payload_bytes) iov.push_back({(void*)pg.payload, (size_t)pg.payload_bytes});
        off += psize;
      }
      p.total = off - start;
    }
  }
  TWriter w;
  w.i32(1, 1);
  w.list(2, 12, ncols + 1);
  w.begin_anon_struct();
  w.str(4, "schema");
  w.i32(5, ncols);
  w.end_struct();
  for (int c = 0; c < ncols; ++c) schema_element(w, cols[c]);
  int64_t total_rows = 0;
  for (int g = 0; g < nrg; ++g) total_rows += rg_rows[g];
  w.i64(3, total_rows);
  w.list(4, 12, nrg);
  for (int g = 0; g < nrg; ++g) {
    w.begin_anon_struct();
    w.list(1, 12, ncols);
    int64_t rg_bytes = 0;
    for (int c = 0; c < ncols; ++c) {
      const HsPqWCol2& col = cols[(size_t)g * ncols + c];
      const ColPos& p = posv[(size_t)g * ncols + c];
      rg_bytes += p.raw_total;
      w.begin_anon_struct();
      w.i64(2, p.dict_off >= 0 ? p.dict_off : p.data_off);
      w.begin_struct(3);
      w.i32(1, col.ptype);
      if (col.dict) {
        w.list(2, 5, 3);
        w.zz(0); w.zz(3); w.zz(8);
      } else {
        w.list(2, 5, 2);
        w.zz(0); w.zz(3);
      }
      w.list(3, 8, 1);
      w.varint(strlen(col.name));
      w.bin(col.name);
      w.i32(4, col.codec == 1 ? 1 : 0);
      w.i64(5, rg_rows[g]);
      w.i64(6, p.raw_total);
      w.i64(7, p.total);
      w.i64(9, p.data_off);
      if (p.dict_off >= 0) w.i64(11, p.dict_off);
      w.begin_struct(12);               // Statistics { 3: null_count }
      w.i64(3, col.null_count);
      w.end_struct();
      w.end_struct();
      w.end_struct();
    }
    w.i64(2, rg_bytes);
    w.i64(3, rg_rows[g]);
    w.end_struct();
  }
  w.str(6, created_by ? created_by : "hyperspace_amd");
  w.byte(0);
  keep.push_back(std::move(w.b));
  const uint32_t flen = (uint32_t)keep.back().size();
  iov.push_back({keep.back().data(), keep.back().size()});
  std::vector<uint8_t> tail(8);
  memcpy(tail.data(), &flen, 4);
  memcpy(tail.data() + 4, magic, 4);
  keep.push_back(std::move(tail));
  iov.push_back({keep.back().data(), 8});
  const bool ok = write_all(fd, iov, pos);
  const int err = ok ? 0 : -errno;
  if (close(fd) != 0 && ok) return -errno;
  return err;
}

}  // extern "C"
