// file_reader.cpp — footer, thrift compact protocol, page reader, decompression.
//
// The thrift structures come from parquet-format 2.5.0 (parquet.thrift); the reference reads
// them through the `parquet-format`/`thrift` crates (file/reader.rs:38-43,186-189,412-416).
// Only the fields the reader uses are decoded; everything else is skipped by type.
#include "file_reader.hpp"

#include <string.h>
#include <zlib.h>

namespace pqg {

namespace {

// ------------------------------------------------------------------ compact protocol
enum CType { CT_STOP = 0, CT_TRUE = 1, CT_FALSE = 2, CT_BYTE = 3, CT_I16 = 4, CT_I32 = 5, CT_I64 = 6,
             CT_DOUBLE = 7, CT_BINARY = 8, CT_LIST = 9, CT_SET = 10, CT_MAP = 11, CT_STRUCT = 12 };

struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool bad = false;
  std::string why;

  uint8_t byte() {
    if (p >= end) {
      fail("unexpected end of thrift data");
      return 0;
    }
    return *p++;
  }
  void fail(const char* m) {
    if (!bad) why = m;
    bad = true;
    p = end;
  }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 70; s += 7) {
      uint8_t b = byte();
      if (bad) return 0;
      v |= (uint64_t)(b & 0x7F) << s;
      if (!(b & 0x80)) return v;
    }
    fail("varint too long");
    return 0;
  }
  int64_t zz() {
    uint64_t u = varint();
    return (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
  }
  int32_t i32() { return (int32_t)zz(); }
  int64_t i64() { return zz(); }
  std::string binary() {
    uint64_t n = varint();
    if (bad || n > (uint64_t)(end - p)) {
      fail("binary length out of range");
      return {};
    }
    std::string s((const char*)p, (size_t)n);
    p += n;
    return s;
  }
  // field header: returns type; id updated (short delta or explicit i16)
  int field(int16_t& id) {
    uint8_t b = byte();
    if (bad) return CT_STOP;
    int t = b & 0x0F;
    if (t == CT_STOP) return CT_STOP;
    int delta = b >> 4;
    if (delta) id = (int16_t)(id + delta);
    else id = (int16_t)i32();
    return t;
  }
  void list_header(int& etype, uint64_t& n) {
    uint8_t b = byte();
    etype = b & 0x0F;
    n = b >> 4;
    if (n == 15) n = varint();
  }
  void skip(int t, int depth = 0) {
    if (depth > 64) {
      fail("thrift nesting too deep");
      return;
    }
    switch (t) {
      case CT_TRUE: case CT_FALSE: return;
      case CT_BYTE: byte(); return;
      case CT_I16: case CT_I32: case CT_I64: varint(); return;
      case CT_DOUBLE:
        if (end - p < 8) fail("short double");
        else p += 8;
        return;
      case CT_BINARY: binary(); return;
      case CT_LIST: case CT_SET: {
        int et;
        uint64_t n;
        list_header(et, n);
        for (uint64_t i = 0; i < n && !bad; ++i) skip(et == CT_TRUE ? CT_BYTE : et, depth + 1);
        return;
      }
      case CT_MAP: {
        uint64_t n = varint();
        if (n == 0) return;
        uint8_t kv = byte();
        for (uint64_t i = 0; i < n && !bad; ++i) {
          skip(kv >> 4, depth + 1);
          skip(kv & 0x0F, depth + 1);
        }
        return;
      }
      case CT_STRUCT: {
        int16_t id = 0;
        for (;;) {
          int ft = field(id);
          if (bad || ft == CT_STOP) return;
          skip(ft, depth + 1);
        }
      }
      default: fail("unknown thrift type");
    }
  }
  bool boolean(int t) { return t == CT_TRUE; }
};

// ------------------------------------------------------------------ structures
void read_schema_element(Reader& r, SchemaNode& s) {
  int16_t id = 0;
  for (;;) {
    int t = r.field(id);
    if (r.bad || t == CT_STOP) return;
    switch (id) {
      case 1: s.type = r.i32(); break;
      case 2: s.type_length = r.i32(); break;
      case 3: s.repetition = r.i32(); break;
      case 4: s.name = r.binary(); break;
      case 5: s.num_children = r.i32(); break;
      case 6: s.converted_type = r.i32(); break;
      case 7: s.scale = r.i32(); break;
      case 8: s.precision = r.i32(); break;
      default: r.skip(t);
    }
  }
}

void read_column_metadata(Reader& r, ColumnChunkMeta& c) {
  int16_t id = 0;
  for (;;) {
    int t = r.field(id);
    if (r.bad || t == CT_STOP) return;
    switch (id) {
      case 1: c.type = r.i32(); break;
      case 2: {
        int et;
        uint64_t n;
        r.list_header(et, n);
        for (uint64_t i = 0; i < n && !r.bad; ++i) c.encodings.push_back(r.i32());
        break;
      }
      case 3: {
        int et;
        uint64_t n;
        r.list_header(et, n);
        for (uint64_t i = 0; i < n && !r.bad; ++i) c.path.push_back(r.binary());
        break;
      }
      case 4: c.codec = r.i32(); break;
      case 5: c.num_values = r.i64(); break;
      case 6: c.total_uncompressed_size = r.i64(); break;
      case 7: c.total_compressed_size = r.i64(); break;
      case 9: c.data_page_offset = r.i64(); break;
      case 11:
        c.dictionary_page_offset = r.i64();
        c.has_dict_offset = true;
        break;
      default: r.skip(t);
    }
  }
}

bool read_column_chunk(Reader& r, ColumnChunkMeta& c) {
  int16_t id = 0;
  bool has_meta = false;
  for (;;) {
    int t = r.field(id);
    if (r.bad || t == CT_STOP) return has_meta;
    if (id == 3 && t == CT_STRUCT) {
      read_column_metadata(r, c);
      has_meta = true;
    } else {
      r.skip(t);
    }
  }
}

bool read_row_group(Reader& r, RowGroupMeta& g) {
  int16_t id = 0;
  bool ok = true;
  for (;;) {
    int t = r.field(id);
    if (r.bad || t == CT_STOP) return ok;
    switch (id) {
      case 1: {
        int et;
        uint64_t n;
        r.list_header(et, n);
        for (uint64_t i = 0; i < n && !r.bad; ++i) {
          ColumnChunkMeta c;
          ok &= read_column_chunk(r, c);
          g.columns.push_back(std::move(c));
        }
        break;
      }
      case 2: g.total_byte_size = r.i64(); break;
      case 3: g.num_rows = r.i64(); break;
      default: r.skip(t);
    }
  }
}

// schema/types.rs:737-793: OPTIONAL -> def+1, REPEATED -> def+1 & rep+1; leaves in order.
void build_leaves(const std::vector<SchemaNode>& s, size_t& idx, int16_t def, int16_t rep,
                  const std::string& prefix, std::vector<LeafColumn>& out, bool& ok) {
  if (idx >= s.size()) {
    ok = false;
    return;
  }
  const SchemaNode& n = s[idx++];
  if (n.repetition == 1) def++;
  else if (n.repetition == 2) {
    def++;
    rep++;
  }
  std::string path = prefix.empty() ? n.name : prefix + "." + n.name;
  if (n.num_children <= 0 && n.type >= 0) {
    out.push_back(LeafColumn{path, n.type, n.type_length, def, rep});
    return;
  }
  for (int c = 0; c < n.num_children && ok; ++c) build_leaves(s, idx, def, rep, path, out, ok);
}

}  // namespace

int parse_file_metadata(const uint8_t* data, uint64_t len, FileMeta& meta, std::string& err) {
  // file/reader.rs:155-211
  if (len < 8) {
    err = "Invalid Parquet file. Size is smaller than footer";
    return PQG_ERR_GENERAL;
  }
  if (memcmp(data + len - 4, "PAR1", 4) != 0) {
    err = "Invalid Parquet file. Corrupt footer";
    return PQG_ERR_GENERAL;
  }
  int32_t mlen;
  memcpy(&mlen, data + len - 8, 4);
  if (mlen < 0) {
    err = "Invalid Parquet file. Metadata length is less than zero";
    return PQG_ERR_GENERAL;
  }
  int64_t start = (int64_t)len - 8 - mlen;
  if (start < 0) {
    err = "Invalid Parquet file. Metadata start is less than zero";
    return PQG_ERR_GENERAL;
  }
  Reader r{data + start, data + start + mlen};
  int16_t id = 0;
  for (;;) {
    int t = r.field(id);
    if (r.bad || t == CT_STOP) break;
    switch (id) {
      case 1: meta.version = r.i32(); break;
      case 2: {
        int et;
        uint64_t n;
        r.list_header(et, n);
        for (uint64_t i = 0; i < n && !r.bad; ++i) {
          SchemaNode s;
          read_schema_element(r, s);
          meta.schema.push_back(std::move(s));
        }
        break;
      }
      case 3: meta.num_rows = r.i64(); break;
      case 4: {
        int et;
        uint64_t n;
        r.list_header(et, n);
        for (uint64_t i = 0; i < n && !r.bad; ++i) {
          RowGroupMeta g;
          if (!read_row_group(r, g) && !r.bad) {
            err = "Expected to have column metadata";
            return PQG_ERR_GENERAL;
          }
          meta.row_groups.push_back(std::move(g));
        }
        break;
      }
      case 6: meta.created_by = r.binary(); break;
      default: r.skip(t);
    }
  }
  if (r.bad) {
    err = "Could not parse metadata: " + r.why;
    return PQG_ERR_GENERAL;
  }
  if (meta.schema.empty()) {
    err = "Could not parse metadata: empty schema";
    return PQG_ERR_GENERAL;
  }
  // root's children only (the root itself carries no repetition level)
  bool ok = true;
  size_t idx = 1;
  for (int c = 0; c < meta.schema[0].num_children && ok; ++c)
    build_leaves(meta.schema, idx, 0, 0, "", meta.leaves, ok);
  if (!ok) {
    err = "Could not parse metadata: malformed schema tree";
    return PQG_ERR_GENERAL;
  }
  return PQG_OK;
}

int parse_page_header(const uint8_t* p, uint64_t avail, PageHeaderInfo& h, uint64_t& used,
                      std::string& err) {
  Reader r{p, p + avail};
  int16_t id = 0;
  for (;;) {
    int t = r.field(id);
    if (r.bad || t == CT_STOP) break;
    switch (id) {
      case 1: h.type = r.i32(); break;
      case 2: h.uncompressed_size = r.i32(); break;
      case 3: h.compressed_size = r.i32(); break;
      case 5: {  // DataPageHeader
        h.has_v1 = true;
        int16_t fid = 0;
        for (;;) {
          int ft = r.field(fid);
          if (r.bad || ft == CT_STOP) break;
          switch (fid) {
            case 1: h.num_values = r.i32(); break;
            case 2: h.encoding = r.i32(); break;
            case 3: h.def_encoding = r.i32(); break;
            case 4: h.rep_encoding = r.i32(); break;
            default: r.skip(ft);
          }
        }
        break;
      }
      case 7: {  // DictionaryPageHeader
        h.has_dict = true;
        int16_t fid = 0;
        for (;;) {
          int ft = r.field(fid);
          if (r.bad || ft == CT_STOP) break;
          switch (fid) {
            case 1: h.num_values = r.i32(); break;
            case 2: h.encoding = r.i32(); break;
            case 3: h.is_sorted = r.boolean(ft); break;
            default: r.skip(ft);
          }
        }
        break;
      }
      case 8: {  // DataPageHeaderV2
        h.has_v2 = true;
        int16_t fid = 0;
        for (;;) {
          int ft = r.field(fid);
          if (r.bad || ft == CT_STOP) break;
          switch (fid) {
            case 1: h.num_values = r.i32(); break;
            case 2: h.num_nulls = r.i32(); break;
            case 3: h.num_rows = r.i32(); break;
            case 4: h.encoding = r.i32(); break;
            case 5: h.def_len = r.i32(); break;
            case 6: h.rep_len = r.i32(); break;
            case 7: h.is_compressed = r.boolean(ft); break;
            default: r.skip(ft);
          }
        }
        break;
      }
      default: r.skip(t);
    }
  }
  if (r.bad) {
    err = "underlying Thrift error: " + r.why;
    return PQG_ERR_GENERAL;
  }
  used = (uint64_t)(r.p - p);
  return PQG_OK;
}

// ------------------------------------------------------------------ snappy (raw format)
static int snappy_decompress(const uint8_t* in, uint64_t n, uint8_t* out, uint64_t out_len,
                             uint64_t& produced, std::string& err) {
  uint64_t ip = 0, ulen = 0;
  for (int s = 0; s < 35; s += 7) {  // preamble: uncompressed length (varint)
    if (ip >= n) {
      err = "snappy: truncated preamble";
      return PQG_ERR_GENERAL;
    }
    uint8_t b = in[ip++];
    ulen |= (uint64_t)(b & 0x7F) << s;
    if (!(b & 0x80)) break;
  }
  if (ulen > out_len) {
    err = "snappy: output larger than expected";
    return PQG_ERR_GENERAL;
  }
  uint64_t op = 0;
  while (ip < n) {
    uint8_t tag = in[ip++];
    uint32_t kind = tag & 3;
    if (kind == 0) {  // literal
      uint64_t len = (tag >> 2) + 1;
      if ((tag >> 2) >= 60) {
        uint32_t nb = (tag >> 2) - 59;
        if (ip + nb > n) break;
        len = 0;
        for (uint32_t k = 0; k < nb; ++k) len |= (uint64_t)in[ip + k] << (8 * k);
        len += 1;
        ip += nb;
      }
      if (ip + len > n || op + len > ulen) {
        err = "snappy: literal out of range";
        return PQG_ERR_GENERAL;
      }
      memcpy(out + op, in + ip, len);
      ip += len;
      op += len;
    } else {
      uint64_t len, off;
      if (kind == 1) {
        if (ip + 1 > n) break;
        len = ((tag >> 2) & 7) + 4;
        off = ((uint64_t)(tag >> 5) << 8) | in[ip];
        ip += 1;
      } else if (kind == 2) {
        if (ip + 2 > n) break;
        len = (tag >> 2) + 1;
        off = in[ip] | ((uint64_t)in[ip + 1] << 8);
        ip += 2;
      } else {
        if (ip + 4 > n) break;
        len = (tag >> 2) + 1;
        off = in[ip] | ((uint64_t)in[ip + 1] << 8) | ((uint64_t)in[ip + 2] << 16) | ((uint64_t)in[ip + 3] << 24);
        ip += 4;
      }
      if (off == 0 || off > op || op + len > ulen) {
        err = "snappy: bad copy";
        return PQG_ERR_GENERAL;
      }
      if (off >= len) {
        memcpy(out + op, out + op - off, len);
      } else if (off >= 8) {  // overlapping: 8-byte steps never read bytes not yet written
        uint64_t k = 0;
        for (; k + 8 <= len; k += 8) memcpy(out + op + k, out + op - off + k, 8);
        for (; k < len; ++k) out[op + k] = out[op - off + k];
      } else {
        for (uint64_t k = 0; k < len; ++k) out[op + k] = out[op - off + k];  // a short repeat
      }
      op += len;
    }
  }
  if (op != ulen) {
    err = "snappy: truncated input";
    return PQG_ERR_GENERAL;
  }
  produced = op;
  return PQG_OK;
}

int decompress(int codec, const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_len,
               std::string& err) {
  uint64_t produced = 0;
  int st = PQG_OK;
  if (codec == 1) {
    st = snappy_decompress(in, in_len, out, out_len, produced, err);
  } else if (codec == 2) {  // GZIP (flate2 GzDecoder)
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) {
      err = "gzip: inflateInit2 failed";
      return PQG_ERR_GENERAL;
    }
    zs.next_in = const_cast<uint8_t*>(in);
    zs.avail_in = (uInt)in_len;
    zs.next_out = out;
    zs.avail_out = (uInt)out_len;
    int rc = inflate(&zs, Z_FINISH);
    produced = zs.total_out;
    inflateEnd(&zs);
    if (rc != Z_STREAM_END && rc != Z_OK && rc != Z_BUF_ERROR) {
      err = "gzip: inflate failed";
      return PQG_ERR_GENERAL;
    }
  } else {
    err = "compression codec is not supported (compression.rs is out of scope; SNAPPY and GZIP are)";
    return PQG_ERR_NYI;
  }
  if (st) return st;
  if (produced != out_len) {  // file/reader.rs:455-461
    err = "Actual decompressed size doesn't match the expected one";
    return PQG_ERR_GENERAL;
  }
  return PQG_OK;
}

int plan_chunk_pages(const uint8_t* file, uint64_t file_len, const ColumnChunkMeta& cc,
                     std::vector<PagePlan>& plan, uint64_t& blob_len, std::string& err) {
  blob_len = 64;
  // get_column_page_reader, file/reader.rs:314-330
  int64_t start = cc.has_dict_offset ? cc.dictionary_page_offset : cc.data_page_offset;
  int64_t len = cc.total_compressed_size;
  if (start < 0 || len < 0 || (uint64_t)(start + len) > file_len) {
    err = "column chunk out of file range";
    return PQG_ERR_EOF;
  }
  const uint8_t* p = file + start;
  uint64_t avail = (uint64_t)len, pos = 0, at = 0;
  int64_t seen = 0;
  // on a failure `plan` keeps the pages before it (their payloads can still be filled and decoded,
  // so that a failure on an earlier page is reported first, as the reference's page-by-page reads do)
  // SerializedPageReader::get_next_page, file/reader.rs:420-522
  while (seen < cc.num_values) {
    PageHeaderInfo h;
    uint64_t used = 0;
    int st = parse_page_header(p + pos, avail - pos, h, used, err);
    if (st) return st;
    pos += used;
    uint64_t offset = 0;
    bool can_decompress = true;
    if (h.has_v2) {
      offset = (uint64_t)(h.def_len + h.rep_len);
      can_decompress = h.is_compressed;
    }
    if (h.compressed_size < 0 || (uint64_t)h.compressed_size < offset ||
        (uint64_t)h.uncompressed_size < offset) {
      err = "bad page sizes";
      return PQG_ERR_GENERAL;
    }
    uint64_t clen = (uint64_t)h.compressed_size - offset;
    uint64_t ulen = (uint64_t)h.uncompressed_size - offset;
    if (pos + offset + clen > avail) {
      err = "failed to fill whole buffer";  // read_exact
      return PQG_ERR_EOF;
    }
    PagePlan pp;
    pp.src = p + pos;
    pp.prefix = offset;
    pp.clen = clen;
    pp.decompress = cc.codec != 0 && can_decompress;
    pos += offset + clen;
    const uint64_t out_len = pp.decompress ? offset + ulen : offset + clen;
    pqg_page& pg = pp.page;
    memset(&pg, 0, sizeof(pg));
    pg.offset = at;  // 64-byte aligned payload in the chunk's blob
    pg.nbytes = (uint32_t)out_len;
    if (h.type == PQG_PAGE_DICTIONARY && h.has_dict) {
      pg.page_type = PQG_PAGE_DICTIONARY;
      pg.num_values = (uint32_t)h.num_values;
      pg.encoding = h.encoding;
    } else if (h.type == PQG_PAGE_DATA && h.has_v1) {
      pg.page_type = PQG_PAGE_DATA;
      pg.num_values = (uint32_t)h.num_values;
      pg.encoding = h.encoding;
      pg.def_encoding = h.def_encoding;
      pg.rep_encoding = h.rep_encoding;
      seen += h.num_values;
    } else if (h.type == PQG_PAGE_DATA_V2 && h.has_v2) {
      pg.page_type = PQG_PAGE_DATA_V2;
      pg.num_values = (uint32_t)h.num_values;
      pg.encoding = h.encoding;
      pg.def_len = (uint32_t)h.def_len;
      pg.rep_len = (uint32_t)h.rep_len;
      seen += h.num_values;
    } else if (h.type == PQG_PAGE_DICTIONARY || h.type == PQG_PAGE_DATA || h.type == PQG_PAGE_DATA_V2) {
      err = "page header without its page-type header";  // assert! in the reference
      return PQG_ERR_PANIC;
    } else {
      continue;  // unknown page type (INDEX_PAGE): skipped (file/reader.rs:512-515)
    }
    plan.push_back(pp);
    at = (at + out_len + 63) & ~63ull;
    blob_len = at + 64;
  }
  blob_len = at + 64;  // tail slack
  return PQG_OK;
}

int fill_page(const PagePlan& pp, int codec, uint8_t* chunk_blob, std::string& err) {
  uint8_t* dst = chunk_blob + pp.page.offset;
  memcpy(dst, pp.src, pp.prefix);  // v2 levels are never compressed
  if (pp.decompress)
    return decompress(codec, pp.src + pp.prefix, pp.clen, dst + pp.prefix, pp.page.nbytes - pp.prefix, err);
  memcpy(dst + pp.prefix, pp.src + pp.prefix, pp.clen);
  return PQG_OK;
}

int read_chunk_pages(const uint8_t* file, uint64_t file_len, const ColumnChunkMeta& cc,
                     std::vector<uint8_t>& blob, std::vector<pqg_page>& pages, std::string& err) {
  std::vector<PagePlan> plan;
  uint64_t len = 0;
  std::string herr;
  const int hst = plan_chunk_pages(file, file_len, cc, plan, len, herr);
  // the pages before a header failure are read first: a decompression failure on one of them is
  // the reference's first error (get_next_page reads and decompresses page by page)
  blob.assign(len, 0);
  for (const PagePlan& pp : plan) {
    const int st = fill_page(pp, cc.codec, blob.data(), err);
    if (st) return st;
    pages.push_back(pp.page);
  }
  if (hst) err = herr;
  return hst;
}

}  // namespace pqg
