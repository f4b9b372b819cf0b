// column_reader.cpp — pqg_file_* (SerializedFileReader, file/reader.rs:140-330) and
// pqg_column_reader_* (ColumnReaderImpl::read_batch over a GPU-decoded chunk,
// column/reader.rs:159-265).
//
// read_batch contract served here (derived from the loop at column/reader.rs:175-262):
//  * def levels requested and max_def > 0: every call returns exactly
//    min(batch_size, levels left in the chunk) levels and the values whose def == max_def;
//  * otherwise values = min(batch_size, levels left) (each level slot is one value), and
//    levels_read = values when rep levels are requested and max_rep > 0, else 0.
// Chunk errors surface lazily, like the reference: batches that end before the first bad
// page succeed; the batch that reaches it returns the page's status.
#include <hip/hip_runtime.h>
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
  uint64_t L = 0, V = 0;       // level / value cursors
  int status = 0;              // chunk status
  uint64_t bad_level = ~0ull;  // first level index of the failing page
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
  std::vector<uint64_t> page_start;  // level start of each page (data pages)
  for (const pqg_page& p : c->pages) {
    page_start.push_back(cr->total_levels);
    if (p.page_type == PQG_PAGE_DATA || p.page_type == PQG_PAGE_DATA_V2) cr->total_levels += p.num_values;
  }
  const uint64_t n = cr->total_levels;
  if (host_st && c->pages.empty()) {  // nothing before the failure: the first batch fails
    cr->status = host_st;
    cr->err = c->err;
    cr->bad_level = 0;
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
    cr->bad_level = (bad >= 0 && bad < (int)page_start.size()) ? page_start[bad] : 0;
    // a bad dictionary page (or any failure before the first data page) fails the first batch
  } else if (host_st) {  // every page before the host failure decoded: it fails the batch after them
    cr->status = host_st;
    cr->err = c->err;
    cr->bad_level = n;
  }
  *out = cr.release();
  return PQG_OK;
}

void pqg_column_reader_close(pqg_column_reader* cr) { delete cr; }

int pqg_column_reader_read_batch(pqg_column_reader* cr, size_t batch_size, int16_t* def,
                                 int16_t* rep, void* values, uint64_t values_bytes_cap,
                                 uint32_t* lengths, size_t* values_read, size_t* levels_read) {
  if (!cr || !values_read || !levels_read) return PQG_ERR_INVALID;
  *values_read = *levels_read = 0;
  const bool use_def = def && cr->col.max_def > 0;
  const bool use_rep = rep && cr->col.max_rep > 0;
  // The chunk was decoded with its def levels; reading an optional column without them would
  // make the reference decode one value per level slot, which this reader does not replay.
  if (cr->col.max_def > 0 && !def) return PQG_ERR_INVALID;
  uint64_t left = cr->total_levels - cr->L;
  uint64_t nlev = batch_size < left ? batch_size : left;
  // The reference's loop (column/reader.rs:181-262) keeps reading while fewer than batch_size
  // levels are in hand, so a call whose requested range reaches the failing page (or a failure
  // after the last decoded page: has_next -> read_new_page fails) returns its error, whatever was
  // read before it in that call; batch_size 0 never enters the loop (Ok((0, 0))).
  if (cr->status != PQG_OK && batch_size && cr->L + batch_size > cr->bad_level) return cr->status;
  if (nlev == 0) return PQG_OK;
  uint64_t nval = nlev;
  if (use_def) {
    nval = 0;
    const int16_t md = cr->col.max_def;
    for (uint64_t i = 0; i < nlev; ++i) nval += cr->def[cr->L + i] == md;
  }
  if (cr->V + nval > cr->total_values) return PQG_ERR_GENERAL;  // inconsistent chunk
  if (cr->is_ba) {
    uint64_t b0 = (uint64_t)cr->offsets[cr->V], b1 = (uint64_t)cr->offsets[cr->V + nval];
    if (b1 - b0 > values_bytes_cap) return PQG_ERR_CAPACITY;
    if (values && b1 > b0) memcpy(values, cr->values.data() + b0, b1 - b0);
    if (lengths)
      for (uint64_t i = 0; i < nval; ++i)
        lengths[i] = (uint32_t)(cr->offsets[cr->V + i + 1] - cr->offsets[cr->V + i]);
  } else {
    uint64_t nb = nval * (uint64_t)cr->es;
    if (nb > values_bytes_cap) return PQG_ERR_CAPACITY;
    if (values && nb) memcpy(values, cr->values.data() + cr->V * cr->es, nb);
  }
  if (use_def) memcpy(def, cr->def.data() + cr->L, nlev * 2);
  if (use_rep) memcpy(rep, cr->rep.data() + cr->L, nlev * 2);
  cr->L += nlev;
  cr->V += nval;
  *values_read = nval;
  *levels_read = (use_def || use_rep) ? nlev : 0;
  return PQG_OK;
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
