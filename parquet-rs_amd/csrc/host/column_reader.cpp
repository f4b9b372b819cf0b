// column_reader.cpp — pqg_file_* (SerializedFileReader, file/reader.rs:140-330) and
// pqg_column_reader_* (ColumnReaderImpl::read_batch over a GPU-decoded chunk,
// column/reader.rs:159-265).
//
// read_batch is the reference's loop (column/reader.rs:159-265) replayed page by page over the
// decoded chunk: the batch clamped to the slices, per iteration iter_batch_size clamped to the page
// and the slices, def levels counted for the values to read (or iter_batch_size values without def
// levels), num_decoded_values advanced by max(levels, values). The def / rep / value
// positions within a page move independently, as the reference's three decoders do.
// Chunk errors surface lazily, like the reference: batches that end before the first bad
// page succeed; the batch that reaches it returns the page's status.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>

#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "file_reader.hpp"
#include "staging.hpp"

using namespace pqg;

struct pqg_column_reader {
  pqg_column col{};
  bool is_ba = false;
  int es = 0;
  uint64_t total_levels = 0;   // sum of data-page num_values
  uint64_t total_values = 0;
  std::vector<int16_t> def, rep;
  std::vector<uint8_t> values;
  std::vector<int64_t> offsets;
  // data pages in file order: level count (num_values), first level, first dense value, dense
  // (non-null) value count, value encoding
  std::vector<uint64_t> pN, pL, pV, pK;
  std::vector<int32_t> pEnc;
  // ColumnReaderImpl's page state (column/reader.rs:106-137): the current data page, its
  // num_decoded_values, and the positions of its def / rep level decoders and of its value
  // decoder, which read_batch advances independently (:212-259)
  int64_t pg = -1;
  uint64_t buffered = 0, nd = 0, dpos = 0, rpos = 0, vpos = 0;
  uint64_t V = 0;              // absolute dense-value cursor (vstart of the page + vpos)
  int status = 0;              // chunk status
  int64_t bad_page = INT64_MAX;  // data-page index whose read_new_page fails (npages: after the last)
  std::string err;
};

struct ColumnStaging {
  int device = -1;
  hipStream_t s = nullptr;
  Buf h_blob, d_blob, d_def, d_rep, d_val, d_off, h_def, h_rep, h_val, h_off;
  ColumnStaging() { h_blob.host = h_def.host = h_rep.host = h_val.host = h_off.host = true; }
  ~ColumnStaging() {
    if (s) {
      hipStreamSynchronize(s);
      hipStreamDestroy(s);
    }
    for (Buf* b : {&h_blob, &d_blob, &d_def, &d_rep, &d_val, &d_off, &h_def, &h_rep, &h_val, &h_off}) b->release();
  }
};

pqg_file_reader::~pqg_file_reader() {
  delete staging;
  if (map) munmap(map, map_len);
}

static int value_size(int t, int tl) {
  switch (t) {
    case PQG_BOOLEAN: return 1;
    case PQG_INT32: case PQG_FLOAT: return 4;
    case PQG_INT64: case PQG_DOUBLE: return 8;
    case PQG_INT96: return 12;
    case PQG_FIXED_LEN_BYTE_ARRAY: return tl;
    default: return 0;
  }
}

static ChunkPages* get_chunk(pqg_file_reader* r, int rg, int col) {
  auto key = std::make_pair(rg, col);
  auto it = r->chunks.find(key);
  if (it != r->chunks.end()) return it->second.get();
  std::unique_ptr<ChunkPages> c(new ChunkPages());
  const ColumnChunkMeta& cc = r->meta.row_groups[rg].columns[col];
  c->status = read_chunk_pages(r->data, r->len, cc, c->blob, c->pages, c->err);
  ChunkPages* p = c.get();
  r->chunks[key] = std::move(c);
  return p;
}

static bool valid_chunk(pqg_file_reader* r, int rg, int col) {
  return r && rg >= 0 && rg < (int)r->meta.row_groups.size() && col >= 0 &&
         col < (int)r->meta.row_groups[rg].columns.size() && col < (int)r->meta.leaves.size();
}

extern "C" {

int pqg_file_open_memory(const uint8_t* data, uint64_t len, pqg_file_reader** out) {
  if (!out || (!data && len)) return PQG_ERR_INVALID;
  pqg_file_reader* r = new pqg_file_reader();
  r->owned.assign(data, data + len);
  r->data = r->owned.data();
  r->len = len;
  int st = parse_file_metadata(r->data, r->len, r->meta, r->err);
  *out = r;  // returned even on error so pqg_file_error can explain; caller closes
  return st;
}

int pqg_file_open(const char* path, pqg_file_reader** out) {
  if (!out || !path) return PQG_ERR_INVALID;
  *out = nullptr;
  FILE* f = fopen(path, "rb");
  if (!f) {
    pqg_file_reader* r = new pqg_file_reader();
    r->err = std::string("cannot open ") + path;
    *out = r;
    return PQG_ERR_GENERAL;
  }
  pqg_file_reader* r = new pqg_file_reader();
  // mapped, not read: a row group's pages are then read from the page cache by the threads that
  // fill the pinned staging (pqg_rgr_*), and a large file costs no copy at open
  fseek(f, 0, SEEK_END);
  const long sz = ftell(f);
  if (sz > 0) {
    void* m = mmap(nullptr, (size_t)sz, PROT_READ, MAP_PRIVATE, fileno(f), 0);
    if (m != MAP_FAILED) {
      r->map = m;
      r->map_len = (size_t)sz;
      r->data = (const uint8_t*)m;
      r->len = (uint64_t)sz;
    }
  }
  if (!r->map && sz > 0) {  // not mappable: read it
    fseek(f, 0, SEEK_SET);
    r->owned.resize((size_t)sz);
    r->owned.resize(fread(r->owned.data(), 1, (size_t)sz, f));
    r->data = r->owned.data();
    r->len = r->owned.size();
  }
  fclose(f);
  int st = parse_file_metadata(r->data, r->len, r->meta, r->err);
  *out = r;
  return st;
}

void pqg_file_close(pqg_file_reader* r) { delete r; }
const char* pqg_file_error(pqg_file_reader* r) { return r ? r->err.c_str() : "null reader"; }
int64_t pqg_file_num_rows(pqg_file_reader* r) { return r ? r->meta.num_rows : -1; }
int pqg_file_num_row_groups(pqg_file_reader* r) { return r ? (int)r->meta.row_groups.size() : -1; }
int pqg_file_num_columns(pqg_file_reader* r) { return r ? (int)r->meta.leaves.size() : -1; }

int pqg_file_column(pqg_file_reader* r, int col, pqg_column* out, char* path, size_t path_cap) {
  if (!r || !out || col < 0 || col >= (int)r->meta.leaves.size()) return PQG_ERR_INVALID;
  const LeafColumn& l = r->meta.leaves[col];
  out->physical_type = l.physical_type;
  out->type_length = l.type_length;
  out->max_def = l.max_def;
  out->max_rep = l.max_rep;
  if (path && path_cap) {
    snprintf(path, path_cap, "%s", l.path.c_str());
  }
  return PQG_OK;
}

int64_t pqg_row_group_num_rows(pqg_file_reader* r, int rg) {
  if (!r || rg < 0 || rg >= (int)r->meta.row_groups.size()) return -1;
  return r->meta.row_groups[rg].num_rows;
}

int pqg_chunk_pages(pqg_file_reader* r, int rg, int col, pqg_page* pages, uint32_t cap) {
  if (!valid_chunk(r, rg, col)) return -PQG_ERR_INVALID;
  ChunkPages* c = get_chunk(r, rg, col);
  if (c->status) {
    r->err = c->err;
    return -c->status;
  }
  uint32_t n = (uint32_t)c->pages.size();
  if (pages) memcpy(pages, c->pages.data(), (n < cap ? n : cap) * sizeof(pqg_page));
  return (int)n;
}

int pqg_chunk_blob(pqg_file_reader* r, int rg, int col, const uint8_t** blob, uint64_t* len) {
  if (!valid_chunk(r, rg, col) || !blob || !len) return PQG_ERR_INVALID;
  ChunkPages* c = get_chunk(r, rg, col);
  if (c->status) {
    r->err = c->err;
    return c->status;
  }
  *blob = c->blob.data();
  *len = c->blob.size();
  return PQG_OK;
}

// Decodes the whole chunk on the ctx's device, then keeps the decoded streams on the host. The
// page bytes go through the file's pinned staging (async H2D), the outputs come back into pinned
// buffers (async D2H) on the staging stream; device and pinned buffers are reused chunk after chunk.
int pqg_column_reader_open(pqg_file_reader* r, int rg, int col, pqg_ctx* ctx,
                           pqg_column_reader** out) {
  if (!valid_chunk(r, rg, col) || !ctx || !out) return PQG_ERR_INVALID;
  *out = nullptr;
  ChunkPages* c = get_chunk(r, rg, col);
  // a header / decompression failure on page k: the pages before it are decoded and served, the
  // batch that reaches page k returns its status (read_new_page -> get_next_page, column/reader.rs:269-275)
  const int host_st = c->status;
  std::unique_ptr<pqg_column_reader> cr(new pqg_column_reader());
  const LeafColumn& l = r->meta.leaves[col];
  cr->col.physical_type = l.physical_type;
  cr->col.type_length = l.type_length;
  cr->col.max_def = l.max_def;
  cr->col.max_rep = l.max_rep;
  cr->is_ba = l.physical_type == PQG_BYTE_ARRAY || l.physical_type == PQG_FIXED_LEN_BYTE_ARRAY;
  cr->es = value_size(l.physical_type, l.type_length);
  std::vector<int64_t> data_index;  // per page: index among the data pages read before it
  for (const pqg_page& p : c->pages) {
    data_index.push_back((int64_t)cr->pN.size());
    if (p.page_type == PQG_PAGE_DATA || p.page_type == PQG_PAGE_DATA_V2) {
      cr->pN.push_back(p.num_values);
      cr->pL.push_back(cr->total_levels);
      cr->pEnc.push_back(p.encoding);
      cr->total_levels += p.num_values;
    }
  }
  const uint64_t n = cr->total_levels;
  if (host_st && c->pages.empty()) {  // nothing before the failure: the first batch fails
    cr->status = host_st;
    cr->err = c->err;
    cr->bad_page = 0;
    *out = cr.release();
    return PQG_OK;
  }
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  if (!r->staging || r->staging->device != dev) {
    delete r->staging;
    r->staging = new ColumnStaging();
    r->staging->device = dev;
    if (hipStreamCreateWithFlags(&r->staging->s, hipStreamNonBlocking) != hipSuccess) {
      r->err = "hipStreamCreate failed";
      return PQG_ERR_HIP;
    }
  }
  ColumnStaging& S = *r->staging;
  // BYTE_ARRAY output bytes are bounded by the page bytes except for DELTA_BYTE_ARRAY prefix
  // sharing and dictionary repeats; the decode reports the exact size on CAPACITY, so retry once.
  uint64_t vcap = cr->is_ba && l.physical_type == PQG_BYTE_ARRAY ? c->blob.size() + 64
                                                                 : (uint64_t)cr->es * n + 64;
  const size_t blen = c->blob.size();
  bool ok = S.h_blob.need(blen + 64) == hipSuccess && S.d_blob.need(blen + 64) == hipSuccess &&
            S.d_def.need(n * 2 + 64) == hipSuccess && S.d_rep.need(n * 2 + 64) == hipSuccess &&
            S.h_def.need(n * 2 + 64) == hipSuccess && S.h_rep.need(n * 2 + 64) == hipSuccess &&
            (!cr->is_ba || (S.d_off.need((n + 1) * 8 + 64) == hipSuccess && S.h_off.need((n + 1) * 8 + 64) == hipSuccess));
  if (ok) {
    memcpy(S.h_blob.p, c->blob.data(), blen);
    ok = hipMemcpyAsync(S.d_blob.p, S.h_blob.p, blen, hipMemcpyHostToDevice, S.s) == hipSuccess;
  }
  if (!ok) {
    r->err = "HIP allocation/copy failed";
    return PQG_ERR_HIP;
  }
  int st = PQG_OK, bad = -1;
  std::string msg;
  pqg_output o{};
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (S.d_val.need(vcap) != hipSuccess) {
      r->err = "HIP allocation failed";
      return PQG_ERR_HIP;
    }
    o = pqg_output{};
    o.def_levels = l.max_def > 0 ? (int16_t*)S.d_def.p : nullptr;
    o.rep_levels = l.max_rep > 0 ? (int16_t*)S.d_rep.p : nullptr;
    o.values = S.d_val.p;
    o.values_capacity = vcap;
    o.offsets = cr->is_ba ? (int64_t*)S.d_off.p : nullptr;
    o.offsets_capacity = cr->is_ba ? n + 1 : 0;
    st = pqg_decode_chunk(ctx, &cr->col, (const uint8_t*)S.d_blob.p, blen, c->pages.data(),
                          (uint32_t)c->pages.size(), &o, S.s);
    if (st == PQG_OK) st = pqg_sync(ctx, &bad);
    msg = pqg_error_message(ctx);
    if (st == PQG_ERR_CAPACITY && attempt == 0 && o.num_bytes > vcap) {
      vcap = o.num_bytes + 64;
      continue;
    }
    break;
  }
  if (st == PQG_ERR_HIP || st == PQG_ERR_INVALID) {
    r->err = msg;
    return st;
  }
  cr->total_values = o.num_values;
  uint64_t vb = cr->is_ba ? o.num_bytes : o.num_values * (uint64_t)cr->es;
  if (vb > vcap) vb = vcap;
  const uint64_t noff = cr->is_ba ? o.num_values + 1 : 0;
  ok = S.h_val.need(vb + 64) == hipSuccess;
  if (ok && l.max_def > 0 && n) ok = hipMemcpyAsync(S.h_def.p, S.d_def.p, n * 2, hipMemcpyDeviceToHost, S.s) == hipSuccess;
  if (ok && l.max_rep > 0 && n) ok = hipMemcpyAsync(S.h_rep.p, S.d_rep.p, n * 2, hipMemcpyDeviceToHost, S.s) == hipSuccess;
  if (ok && vb) ok = hipMemcpyAsync(S.h_val.p, S.d_val.p, vb, hipMemcpyDeviceToHost, S.s) == hipSuccess;
  if (ok && noff) ok = hipMemcpyAsync(S.h_off.p, S.d_off.p, noff * 8, hipMemcpyDeviceToHost, S.s) == hipSuccess;
  if (ok) ok = hipStreamSynchronize(S.s) == hipSuccess;
  if (!ok) {
    r->err = "HIP copy failed";
    return PQG_ERR_HIP;
  }
  cr->def.resize(n);
  cr->rep.resize(n);
  if (l.max_def > 0 && n) memcpy(cr->def.data(), S.h_def.p, n * 2);
  if (l.max_rep > 0 && n) memcpy(cr->rep.data(), S.h_rep.p, n * 2);
  cr->values.resize(vb);
  if (vb) memcpy(cr->values.data(), S.h_val.p, vb);
  if (noff) {
    cr->offsets.resize(noff);
    memcpy(cr->offsets.data(), S.h_off.p, noff * 8);
  }
  cr->status = st;
  cr->err = msg;
  if (st != PQG_OK) {
    // the failing page's read_new_page (set_data) or first get fails the batch that reaches it; a
    // bad dictionary page (any failure before the first data page) fails the first batch
    cr->bad_page = (bad >= 0 && bad < (int)data_index.size()) ? data_index[bad] : 0;
  } else if (host_st) {  // every page before the host failure decoded: it fails the batch after them
    cr->status = host_st;
    cr->err = c->err;
    cr->bad_page = (int64_t)cr->pN.size();
  }
  // dense values per data page: the levels equal to max_def (the count read_batch makes,
  // column/reader.rs:216-220), or every level slot of a column without def levels; pages at or
  // after a failing page are never served
  const size_t np = cr->pN.size();
  cr->pV.assign(np, 0);
  cr->pK.assign(np, 0);
  uint64_t vs = 0;
  for (size_t i = 0; i < np && (int64_t)i < cr->bad_page; ++i) {
    uint64_t k = cr->pN[i];
    if (l.max_def > 0) {
      k = 0;
      const int16_t* d = cr->def.data() + cr->pL[i];
      for (uint64_t j = 0; j < cr->pN[i]; ++j) k += d[j] == l.max_def;
    }
    cr->pV[i] = vs;
    cr->pK[i] = k;
    vs += k;
  }
  if (cr->status == PQG_OK && vs != cr->total_values) {  // the decode's count disagrees with the levels
    cr->status = PQG_ERR_GENERAL;
    cr->err = "decoded value count does not match the def levels";
    cr->bad_page = 0;
  }
  *out = cr.release();
  return PQG_OK;
}

void pqg_column_reader_close(pqg_column_reader* cr) { delete cr; }

// has_next (column/reader.rs:416-430) with read_new_page (:269-380): the next data page is loaded
// when the current one is used up or empty; loading the failing page fails.
static int rb_has_next(pqg_column_reader* cr, bool* more) {
  *more = true;
  if (cr->pg >= 0 && cr->buffered != 0 && cr->nd != cr->buffered) return PQG_OK;
  const int64_t next = cr->pg + 1;
  if (cr->status != PQG_OK && next >= cr->bad_page) return cr->status;
  if (next >= (int64_t)cr->pN.size()) {  // no page left
    *more = false;
    return PQG_OK;
  }
  cr->pg = next;
  cr->buffered = cr->pN[next];
  cr->nd = cr->dpos = cr->rpos = cr->vpos = 0;
  *more = cr->buffered != 0;  // an empty page ends this call's loop
  return PQG_OK;
}

// Value decoder get (read_values, column/reader.rs:451-460) asking `want` values of the current
// page: how many the page's decoder returns, or its error. The page holds K dense values; asked past
// them (read_batch without def levels on a column with nulls) each decoder does what
// its get does once its stream is used up:
//  PLAIN fixed width / INT96 / FLBA: min(want, num_values left of the N set) values, EOF when the
//    value bytes run short ("Not enough bytes to decode", decoding.rs:138-156, 158-186, 228-247);
//  PLAIN BYTE_ARRAY: the length prefix read past the end panics (read_num_bytes!, bit_util.rs:30-43);
//  DELTA_BINARY_PACKED / DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY: min(want, values left of the
//    header's count) (decoding.rs:535-572, 697-711, 794-822);
//  dictionary indices and booleans (PLAIN, RLE): the reference goes on into the stream's padding
//    bits; not replayed here (NYI).
static int rb_values(pqg_column_reader* cr, uint64_t want, uint64_t* got) {
  const uint64_t N = cr->pN[cr->pg], K = cr->pK[cr->pg], v = cr->vpos;
  const int enc = cr->pEnc[cr->pg];
  *got = 0;
  switch (enc) {
    case PQG_DELTA_BINARY_PACKED:
    case PQG_DELTA_LENGTH_BYTE_ARRAY:
    case PQG_DELTA_BYTE_ARRAY:
      *got = want < K - v ? want : K - v;
      return PQG_OK;
    case PQG_PLAIN:
      if (cr->col.physical_type != PQG_BOOLEAN) {
        const uint64_t n = want < N - v ? want : N - v;
        if (v + n > K) {
          if (cr->col.physical_type == PQG_BYTE_ARRAY) {
            cr->err = "assertion failed: 4 <= src.len() (PLAIN BYTE_ARRAY length read past the page)";
            return PQG_ERR_PANIC;
          }
          cr->err = "Not enough bytes to decode";
          return PQG_ERR_EOF;
        }
        *got = n;
        return PQG_OK;
      }
      break;
    default:
      break;
  }
  if (v + want > K) {
    cr->err = "read_batch without def levels past a page's non-null values: the reference reads "
              "the stream's padding here (dictionary / boolean encodings), not replayed";
    return PQG_ERR_NYI;
  }
  *got = want;
  return PQG_OK;
}

// ColumnReaderImpl::read_batch (column/reader.rs:159-265) replayed over the decoded chunk, with the
// reference's slice lengths: values_cap values, def_cap / rep_cap levels (when given).
int pqg_column_reader_read_batch_caps(pqg_column_reader* cr, size_t batch_size, int16_t* def,
                                      size_t def_cap, int16_t* rep, size_t rep_cap, void* values,
                                      size_t values_cap, uint64_t values_bytes_cap, uint32_t* lengths,
                                      size_t* values_read, size_t* levels_read) {
  if (!cr || !values_read || !levels_read) return PQG_ERR_INVALID;
  *values_read = *levels_read = 0;
  // the smallest batch the slices allow (:170-177)
  uint64_t batch = batch_size < values_cap ? batch_size : values_cap;
  if (def && def_cap < batch) batch = def_cap;
  if (rep && rep_cap < batch) batch = rep_cap;
  const int16_t md = cr->col.max_def;
  const bool read_def = md > 0 && def, read_rep = cr->col.max_rep > 0 && rep;
  uint64_t vr = 0, lr = 0, bytes = 0;
  while ((vr > lr ? vr : lr) < batch) {
    bool more;
    int st = rb_has_next(cr, &more);
    if (st != PQG_OK) return st;
    if (!more) break;
    // iter_batch_size (:187-205)
    uint64_t iter = batch < cr->buffered - cr->nd ? batch : cr->buffered - cr->nd;
    if (values_cap - vr < iter) iter = values_cap - vr;
    if (def && def_cap - lr < iter) iter = def_cap - lr;
    if (rep && rep_cap - lr < iter) iter = rep_cap - lr;
    const uint64_t N = cr->buffered, lbase = cr->pL[cr->pg];
    uint64_t to_read = iter, ndef = 0, nrep = 0;
    if (read_def) {  // LevelDecoder::get clamps to the page's levels left (levels.rs:249-271)
      ndef = iter < N - cr->dpos ? iter : N - cr->dpos;
      const int16_t* src = cr->def.data() + lbase + cr->dpos;
      memcpy(def + lr, src, ndef * 2);
      to_read = 0;
      for (uint64_t i = 0; i < ndef; ++i) to_read += src[i] == md;
    }
    if (read_rep) {
      nrep = iter < N - cr->rpos ? iter : N - cr->rpos;
      memcpy(rep + lr, cr->rep.data() + lbase + cr->rpos, nrep * 2);
      if (def && ndef != nrep) {  // assert_eq! (:233-239)
        cr->err = "Number of decoded rep / def levels did not match";
        return PQG_ERR_PANIC;
      }
    }
    uint64_t nv = 0;
    st = rb_values(cr, to_read, &nv);
    if (st != PQG_OK) return st;
    const uint64_t v0 = cr->pV[cr->pg] + cr->vpos;
    if (cr->is_ba) {
      const uint64_t b0 = (uint64_t)cr->offsets[v0], b1 = (uint64_t)cr->offsets[v0 + nv];
      if (bytes + (b1 - b0) > values_bytes_cap) return PQG_ERR_CAPACITY;
      if (values && b1 > b0) memcpy((uint8_t*)values + bytes, cr->values.data() + b0, b1 - b0);
      if (lengths)
        for (uint64_t i = 0; i < nv; ++i)
          lengths[vr + i] = (uint32_t)(cr->offsets[v0 + i + 1] - cr->offsets[v0 + i]);
      bytes += b1 - b0;
    } else {
      const uint64_t nb = nv * (uint64_t)cr->es;
      if ((vr + nv) * (uint64_t)cr->es > values_bytes_cap) return PQG_ERR_CAPACITY;
      if (values && nb) memcpy((uint8_t*)values + vr * cr->es, cr->values.data() + v0 * cr->es, nb);
    }
    const uint64_t nlev = ndef > nrep ? ndef : nrep;
    const uint64_t adv = nlev > nv ? nlev : nv;
    if (adv == 0) {  // no progress: the reference's loop never ends
      cr->err = "read_batch makes no progress (the reference loops forever)";
      return PQG_ERR_HANG;
    }
    cr->dpos += ndef;
    cr->rpos += nrep;
    cr->vpos += nv;
    cr->nd += adv;  // num_decoded_values (:259)
    cr->V = cr->pV[cr->pg] + cr->vpos;
    lr += nlev;
    vr += nv;
  }
  *values_read = vr;
  *levels_read = lr;
  return PQG_OK;
}

// The original entry: every slice holds batch_size elements (values: batch_size values, their
// bytes bounded by values_bytes_cap).
int pqg_column_reader_read_batch(pqg_column_reader* cr, size_t batch_size, int16_t* def,
                                 int16_t* rep, void* values, uint64_t values_bytes_cap,
                                 uint32_t* lengths, size_t* values_read, size_t* levels_read) {
  return pqg_column_reader_read_batch_caps(cr, batch_size, def, batch_size, rep, batch_size, values,
                                           batch_size, values_bytes_cap, lengths, values_read,
                                           levels_read);
}

}  // extern "C"

// ---------------------------------------------------------------------------- triplets
// TypedTripletIter (record/triplet.rs:168-330) over a column reader: `batch_size` levels at a
// time through read_batch, values spaced onto the level slots whose def == max_def. The
// reference moves the dense values into place with swaps (triplet.rs:300-318); here slot i
// reads dense value k(i) = the count of max_def levels before it, the same triplets.
struct pqg_triplet_iter {
  pqg_column_reader* cr = nullptr;
  size_t batch = 0;
  std::vector<int16_t> def, rep;
  std::vector<uint8_t> vals;      // dense values of the batch (fixed width or BYTE_ARRAY bytes)
  std::vector<uint32_t> lens;     // BYTE_ARRAY lengths
  std::vector<uint64_t> slot;     // per triplet: dense value index, ~0 for a null slot
  std::vector<uint64_t> boff;     // BYTE_ARRAY: byte offset of each dense value
  size_t cur = 0, left = 0;
  bool has_next = false;
};

extern "C" {

int pqg_triplet_iter_open(pqg_column_reader* cr, size_t batch_size, pqg_triplet_iter** out) {
  if (!cr || !out || batch_size == 0) return PQG_ERR_INVALID;
  auto it = std::make_unique<pqg_triplet_iter>();
  it->cr = cr;
  it->batch = batch_size;
  if (cr->col.max_def > 0) it->def.resize(batch_size);
  if (cr->col.max_rep > 0) it->rep.resize(batch_size);
  it->slot.resize(batch_size);
  if (cr->is_ba) {
    it->lens.resize(batch_size);
    it->boff.resize(batch_size + 1);
  } else {
    it->vals.resize(batch_size * (size_t)cr->es + 16);
  }
  *out = it.release();
  return PQG_OK;
}

void pqg_triplet_iter_close(pqg_triplet_iter* it) { delete it; }

int pqg_triplet_iter_read_next(pqg_triplet_iter* it, int* has_next) {
  if (!it || !has_next) return PQG_ERR_INVALID;
  *has_next = 0;
  it->cur += 1;
  if (it->cur < it->left) {
    *has_next = it->has_next = true;
    return PQG_OK;
  }
  pqg_column_reader* cr = it->cr;
  size_t vr = 0, lr = 0;
  int st;
  if (cr->is_ba) {
    // the batch's bytes: at most the chunk's remaining bytes
    const uint64_t cap = (uint64_t)cr->offsets[cr->total_values] - (uint64_t)cr->offsets[cr->V] + 1;
    if (it->vals.size() < cap) it->vals.resize(cap);
    st = pqg_column_reader_read_batch(cr, it->batch, it->def.empty() ? nullptr : it->def.data(),
                                      it->rep.empty() ? nullptr : it->rep.data(), it->vals.data(),
                                      it->vals.size(), it->lens.data(), &vr, &lr);
  } else {
    st = pqg_column_reader_read_batch(cr, it->batch, it->def.empty() ? nullptr : it->def.data(),
                                      it->rep.empty() ? nullptr : it->rep.data(), it->vals.data(),
                                      it->vals.size(), nullptr, &vr, &lr);
  }
  if (st != PQG_OK) return st;
  if (vr == 0 && lr == 0) {  // no more values or levels
    it->has_next = false;
    return PQG_OK;
  }
  if (cr->is_ba) {
    it->boff[0] = 0;
    for (size_t k = 0; k < vr; ++k) it->boff[k + 1] = it->boff[k] + it->lens[k];
  }
  if (lr == 0 || vr == lr) {  // required column, or every level holds a value
    for (size_t i = 0; i < vr; ++i) it->slot[i] = i;
    it->left = vr;
  } else if (vr < lr) {       // spacing (triplet.rs:300-318)
    size_t k = 0;
    for (size_t i = 0; i < lr; ++i) it->slot[i] = it->def[i] == cr->col.max_def ? k++ : ~0ull;
    it->left = lr;
  } else {
    cr->err = "Spacing of values/levels is wrong, values_read: " + std::to_string(vr) +
              ", levels_read: " + std::to_string(lr);
    return PQG_ERR_GENERAL;
  }
  it->cur = 0;
  *has_next = it->has_next = true;
  return PQG_OK;
}

int pqg_triplet_iter_has_next(pqg_triplet_iter* it) { return it && it->has_next ? 1 : 0; }

int16_t pqg_triplet_iter_def_level(pqg_triplet_iter* it) {
  return it->def.empty() ? it->cr->col.max_def : it->def[it->cur];
}

int16_t pqg_triplet_iter_rep_level(pqg_triplet_iter* it) {
  return it->rep.empty() ? it->cr->col.max_rep : it->rep[it->cur];
}

int pqg_triplet_iter_is_null(pqg_triplet_iter* it) {
  return pqg_triplet_iter_def_level(it) < it->cr->col.max_def ? 1 : 0;
}

int pqg_triplet_iter_value(pqg_triplet_iter* it, void* out, size_t cap, size_t* len) {
  if (!it || !it->has_next || !len) return PQG_ERR_INVALID;
  // "Cannot extract value, max definition level: ..., current level: ..." (triplet.rs:236-243)
  if (pqg_triplet_iter_def_level(it) != it->cr->col.max_def) return PQG_ERR_PANIC;
  const uint64_t k = it->slot[it->cur];
  const uint8_t* src;
  size_t n;
  if (it->cr->is_ba) {
    src = it->vals.data() + it->boff[k];
    n = it->lens[k];
  } else {
    n = (size_t)it->cr->es;
    src = it->vals.data() + k * n;
  }
  *len = n;
  if (n > cap) return PQG_ERR_CAPACITY;
  if (out && n) memcpy(out, src, n);
  return PQG_OK;
}

}  // extern "C"
