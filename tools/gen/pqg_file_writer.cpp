// pqg_file_writer.cpp — test/bench tooling: alltypes row groups (pqg_gen_alltypes) written as a
// parquet file, so the file-to-device path (pqg_file_* + pqg_rgr_*) can be run end to end on the
// BASELINE config-5 workload. Layout as SerializedFileWriter / SerializedRowGroupWriter /
// SerializedPageWriter produce it (file/writer.rs): "PAR1", per row group and column the pages
// (thrift-compact PageHeader + payload), then the thrift-compact FileMetaData, its length and
// "PAR1". Codecs: 0 none, 1 SNAPPY (raw format, greedy 4-byte-hash matcher), 2 GZIP (zlib).
// Not part of the decode library.
#include <stdio.h>
#include <string.h>
#include <zlib.h>

#include <algorithm>
#include <string>
#include <vector>

#include "pqg_gen.h"

namespace {

// Thrift compact protocol writer (field deltas, zigzag varints, list headers).
struct Tw {
  std::vector<uint8_t>& b;
  int16_t last = 0;
  std::vector<int16_t> stack;
  explicit Tw(std::vector<uint8_t>& out) : b(out) {}
  void varint(uint64_t v) {
    while (v >= 0x80) {
      b.push_back((uint8_t)(v | 0x80));
      v >>= 7;
    }
    b.push_back((uint8_t)v);
  }
  void zz(int64_t v) { varint(((uint64_t)v << 1) ^ (uint64_t)(v >> 63)); }
  void field(int16_t id, int type) {
    const int d = id - last;
    if (d > 0 && d <= 15) {
      b.push_back((uint8_t)(d << 4 | type));
    } else {
      b.push_back((uint8_t)type);
      zz(id);
    }
    last = id;
  }
  void i32(int16_t id, int32_t v) {
    field(id, 5);
    zz(v);
  }
  void i64(int16_t id, int64_t v) {
    field(id, 6);
    zz(v);
  }
  void str(int16_t id, const std::string& s) {
    field(id, 8);
    varint(s.size());
    b.insert(b.end(), s.begin(), s.end());
  }
  void list(int16_t id, int elem, uint32_t n) {
    field(id, 9);
    if (n < 15) {
      b.push_back((uint8_t)(n << 4 | elem));
    } else {
      b.push_back((uint8_t)(0xF0 | elem));
      varint(n);
    }
  }
  void begin() {  // a struct value (field header already written, or a list element)
    stack.push_back(last);
    last = 0;
  }
  void end() {
    b.push_back(0);
    last = stack.back();
    stack.pop_back();
  }
  void struct_field(int16_t id) {
    field(id, 12);
    begin();
  }
};

void snappy_compress(const uint8_t* in, size_t n, std::vector<uint8_t>& out) {
  out.clear();
  {
    uint64_t v = n;
    while (v >= 0x80) {
      out.push_back((uint8_t)(v | 0x80));
      v >>= 7;
    }
    out.push_back((uint8_t)v);
  }
  auto literal = [&](size_t from, size_t to) {
    while (from < to) {
      const size_t len = std::min<size_t>(to - from, 65536);
      if (len <= 60) {
        out.push_back((uint8_t)((len - 1) << 2));
      } else if (len <= 256) {
        out.push_back(60 << 2);
        out.push_back((uint8_t)(len - 1));
      } else {
        out.push_back(61 << 2);
        out.push_back((uint8_t)((len - 1) & 255));
        out.push_back((uint8_t)((len - 1) >> 8));
      }
      out.insert(out.end(), in + from, in + from + len);
      from += len;
    }
  };
  std::vector<int64_t> table(1 << 14, -1);
  size_t i = 0, lit = 0;
  while (i + 4 <= n) {
    uint32_t v;
    memcpy(&v, in + i, 4);
    const uint32_t h = (v * 0x1E35A7BDu) >> 18;
    const int64_t c = table[h];
    table[h] = (int64_t)i;
    if (c >= 0 && i - (size_t)c <= 65535 && memcmp(in + c, in + i, 4) == 0) {
      literal(lit, i);
      size_t m = 4;
      while (i + m < n && in[c + m] == in[i + m]) ++m;
      const size_t off = i - (size_t)c;
      for (size_t rem = m; rem;) {  // copies with a 2-byte offset, 1..64 bytes each
        const size_t len = std::min<size_t>(rem, 64);
        out.push_back((uint8_t)(((len - 1) << 2) | 2));
        out.push_back((uint8_t)(off & 255));
        out.push_back((uint8_t)(off >> 8));
        rem -= len;
      }
      i += m;
      lit = i;
    } else {
      ++i;
    }
  }
  literal(lit, n);
}

int gzip_compress(const uint8_t* in, size_t n, std::vector<uint8_t>& out) {
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (deflateInit2(&zs, 1, Z_DEFLATED, 16 + MAX_WBITS, 8, Z_DEFAULT_STRATEGY) != Z_OK) return -1;
  out.resize(deflateBound(&zs, n) + 64);
  zs.next_in = const_cast<uint8_t*>(in);
  zs.avail_in = (uInt)n;
  zs.next_out = out.data();
  zs.avail_out = (uInt)out.size();
  const int rc = deflate(&zs, Z_FINISH);
  out.resize(zs.total_out);
  deflateEnd(&zs);
  return rc == Z_STREAM_END ? 0 : -1;
}

const char* at_name[11] = {"id",        "bool_col",   "tinyint_col",     "smallint_col", "int_col",      "bigint_col",
                           "float_col", "double_col", "date_string_col", "string_col",   "timestamp_col"};
const int at_type[11] = {PQG_INT32, PQG_BOOLEAN, PQG_INT32, PQG_INT32, PQG_INT32, PQG_INT64,
                         PQG_FLOAT, PQG_DOUBLE, PQG_BYTE_ARRAY, PQG_BYTE_ARRAY, PQG_INT96};

struct ChunkMeta {
  int64_t num_values = 0, uncompressed = 0, compressed = 0, data_off = -1, dict_off = -1, start = 0;
  std::vector<int> encodings;
};

}  // namespace

extern "C" {

int pqg_write_alltypes_file(const char* path, uint64_t rows_per_group, uint32_t row_groups, uint64_t row0,
                            double p_null, uint64_t seed, int codec, int threads) {
  if (!path || codec < 0 || codec > 2) return PQG_ERR_INVALID;
  FILE* f = fopen(path, "wb");
  if (!f) return PQG_ERR_GENERAL;
  int64_t pos = 0;
  auto put = [&](const void* p, size_t n) {
    fwrite(p, 1, n, f);
    pos += (int64_t)n;
  };
  put("PAR1", 4);
  std::vector<std::vector<ChunkMeta>> meta(row_groups, std::vector<ChunkMeta>(11));
  std::vector<int64_t> rg_bytes(row_groups, 0);
  std::vector<uint8_t> blob, comp, hdr;
  for (uint32_t g = 0; g < row_groups; ++g) {
    pqg_alltypes_info info;
    void* h = pqg_gen_alltypes(rows_per_group, row0 + (uint64_t)g * rows_per_group, p_null, seed, threads, &info);
    if (!h) {
      fclose(f);
      return PQG_ERR_GENERAL;
    }
    blob.assign(info.blob_len + 64, 0);
    std::vector<pqg_page> pages(info.npages);
    pqg_alltypes_copy(h, blob.data(), blob.size(), pages.data(), info.npages);
    pqg_alltypes_free(h);
    for (int c = 0; c < 11; ++c) {
      ChunkMeta& m = meta[g][c];
      m.start = pos;
      m.num_values = (int64_t)rows_per_group;
      for (uint32_t k = info.chunk_first[c]; k < info.chunk_first[c + 1]; ++k) {
        const pqg_page& pg = pages[k];
        const uint8_t* payload = blob.data() + pg.offset;
        const uint8_t* body = payload;
        size_t blen = pg.nbytes;
        if (codec == 1) {
          snappy_compress(payload, pg.nbytes, comp);
          body = comp.data();
          blen = comp.size();
        } else if (codec == 2) {
          if (gzip_compress(payload, pg.nbytes, comp)) {
            fclose(f);
            return PQG_ERR_GENERAL;
          }
          body = comp.data();
          blen = comp.size();
        }
        hdr.clear();
        Tw w(hdr);  // PageHeader
        w.i32(1, pg.page_type);
        w.i32(2, (int32_t)pg.nbytes);
        w.i32(3, (int32_t)blen);
        if (pg.page_type == PQG_PAGE_DICTIONARY) {
          w.struct_field(7);  // DictionaryPageHeader
          w.i32(1, (int32_t)pg.num_values);
          w.i32(2, pg.encoding);
          w.end();
          m.dict_off = pos;
        } else {
          w.struct_field(5);  // DataPageHeader
          w.i32(1, (int32_t)pg.num_values);
          w.i32(2, pg.encoding);
          w.i32(3, pg.def_encoding);
          w.i32(4, pg.rep_encoding);
          w.end();
          if (m.data_off < 0) m.data_off = pos;
        }
        hdr.push_back(0);
        bool seen = false;
        for (int e : m.encodings) seen |= e == pg.encoding;
        if (!seen) m.encodings.push_back(pg.encoding);
        put(hdr.data(), hdr.size());
        put(body, blen);
        m.uncompressed += (int64_t)(hdr.size() + pg.nbytes);
        m.compressed += (int64_t)(hdr.size() + blen);
      }
      bool rle = false;
      for (int e : m.encodings) rle |= e == PQG_RLE;
      if (!rle) m.encodings.push_back(PQG_RLE);  // the def levels
      rg_bytes[g] += m.uncompressed;
    }
  }
  std::vector<uint8_t> fm;
  Tw w(fm);  // FileMetaData
  w.i32(1, 1);
  w.list(2, 12, 12);
  w.begin();  // root
  w.str(4, "schema");
  w.i32(5, 11);
  w.end();
  for (int c = 0; c < 11; ++c) {
    w.begin();
    w.i32(1, at_type[c]);
    w.i32(3, 1);  // OPTIONAL
    w.str(4, at_name[c]);
    w.end();
  }
  w.i64(3, (int64_t)rows_per_group * row_groups);
  w.list(4, 12, row_groups);
  for (uint32_t g = 0; g < row_groups; ++g) {
    w.begin();  // RowGroup
    w.list(1, 12, 11);
    for (int c = 0; c < 11; ++c) {
      const ChunkMeta& m = meta[g][c];
      w.begin();  // ColumnChunk
      w.i64(2, m.start);
      w.struct_field(3);  // ColumnMetaData
      w.i32(1, at_type[c]);
      w.list(2, 5, (uint32_t)m.encodings.size());
      for (int e : m.encodings) w.zz(e);
      w.list(3, 8, 1);
      w.varint(strlen(at_name[c]));
      w.b.insert(w.b.end(), at_name[c], at_name[c] + strlen(at_name[c]));
      w.i32(4, codec);
      w.i64(5, m.num_values);
      w.i64(6, m.uncompressed);
      w.i64(7, m.compressed);
      w.i64(9, m.data_off);
      if (m.dict_off >= 0) w.i64(11, m.dict_off);
      w.end();
      w.end();
    }
    w.i64(2, rg_bytes[g]);
    w.i64(3, (int64_t)rows_per_group);
    w.end();
  }
  w.str(6, "pqgtools alltypes writer");
  fm.push_back(0);
  put(fm.data(), fm.size());
  const uint32_t flen = (uint32_t)fm.size();
  put(&flen, 4);
  put("PAR1", 4);
  const bool ok = ferror(f) == 0;
  return fclose(f) == 0 && ok ? PQG_OK : PQG_ERR_GENERAL;
}

}  // extern "C"
