// chunk_decoder.cpp — pqg_ctx / pqg_decode_chunk / pqg_sync: the host half of the C ABI.
//
// Replaces ColumnReaderImpl's decode driving (column/reader.rs:159-488) for a whole chunk:
// validates the page sequence the way read_new_page / set_current_page_encoding /
// configure_dictionary would (column/reader.rs:269-488, decoding.rs:60-79), uploads the page
// table, and enqueues the kernels of device/*.hip on one HIP stream.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../../include/pqgpu.h"
#include "../pqg_internal.hpp"

using namespace pqg;

extern "C" {
hipError_t pqg_launch_prepare(const uint8_t*, uint64_t, PageWork*, int, ColumnParams, uint32_t*,
                              ChunkResult*, PrepInit, hipStream_t);
hipError_t pqg_launch_run_index(const uint8_t*, uint64_t, PageWork*, int, ColumnParams, int, int,
                                RunTables, ChunkResult*, hipStream_t);
hipError_t pqg_launch_levels(const uint8_t*, uint64_t, PageWork*, int, uint32_t, ColumnParams, int,
                             const uint32_t*, RunTables, LevelTables, int16_t*, ChunkResult*,
                             hipStream_t, hipEvent_t*, int, uint64_t);
hipError_t pqg_launch_scan(PageWork*, int, ChunkResult*, int es, uint64_t cap_bytes,
                           hipStream_t);
hipError_t pqg_launch_dict(const uint8_t*, uint64_t, PageWork*, int, uint32_t, ColumnParams, int,
                           int, const uint32_t*, RunTables, LevelTables, uint8_t*, ChunkResult*, hipStream_t,
                           hipEvent_t*, int);
hipError_t pqg_launch_plain_copy(const uint8_t*, uint64_t, PageWork*, int, int, int, uint64_t,
                                 uint8_t*, ChunkResult*, hipStream_t);
hipError_t pqg_launch_plain_bool(const uint8_t*, PageWork*, int, uint64_t, uint8_t*,
                                 ChunkResult*, hipStream_t);
hipError_t pqg_launch_rle_bool(const uint8_t*, uint64_t, PageWork*, int, uint32_t, ColumnParams,
                               const uint32_t*, RunTables, LevelTables, uint8_t*, ChunkResult*,
                               hipStream_t);
hipError_t pqg_launch_delta(const uint8_t*, uint64_t, PageWork*, int, int, uint8_t*,
                            ChunkResult*, hipStream_t);
hipError_t pqg_launch_space(const int16_t*, uint64_t, int16_t, const void*, int, uint64_t*, void*, hipStream_t);
uint64_t pqg_space_tiles(uint64_t n);
hipError_t pqg_launch_delta_tiled(const uint8_t*, uint64_t, PageWork*, int, uint32_t, const uint32_t*,
                                  DeltaTables, uint32_t, int, uint8_t*, ChunkResult*, hipStream_t,
                                  hipEvent_t*);
hipError_t pqg_launch_ba_dict_prep(const uint8_t*, uint64_t, PageWork*, int, int, uint64_t*,
                                   uint32_t*, ChunkResult*, hipStream_t);
hipError_t pqg_launch_bytes(const uint8_t*, uint64_t, PageWork*, int, int, bool, uint64_t*, uint32_t*,
                            uint32_t*, uint64_t, int64_t*, uint8_t*, uint64_t, uint64_t*, ChunkResult*,
                            hipStream_t);
hipError_t pqg_launch_badict_expand(const uint8_t*, uint64_t, PageWork*, uint32_t, RunTables, int,
                                    uint64_t*, uint32_t*, uint64_t*, uint32_t*, ChunkResult*, hipStream_t);
hipError_t pqg_launch_tile_desc(const uint8_t*, PageWork*, uint32_t, const uint32_t*, RunTables,
                                ColumnParams, int, int, hipStream_t);
hipError_t pqg_launch_page_counts(PageWork*, int, RunTables, int, hipStream_t);
hipError_t pqg_launch_lv_badict(const uint8_t*, uint64_t, PageWork*, int, ColumnParams, int, RunTables,
                                LevelTables, const uint64_t*, const uint32_t*, uint64_t*, uint32_t*,
                                ChunkResult*, hipStream_t);
}

// Two staging slots so consecutive async decodes never overwrite pinned memory that an
// in-flight H2D/D2H copy still reads (slot i is reused only after its last decode ended).
struct Slot {
  PageWork* d_pages = nullptr;
  size_t pages_cap = 0;
  PageWork* h_pages = nullptr;  // pinned staging
  ChunkResult* d_res = nullptr;
  ChunkResult* h_res = nullptr;  // pinned
  hipEvent_t ev[10] = {};  // 0-5 stage boundaries; 6-7 / 8-9 around the def-level path / values kernel
  bool kl = false, kv = false;  // events 6-7 / 8-9 recorded by the last decode
  bool used = false;     // a decode was enqueued and its timings not yet harvested
  bool pending = false;  // a decode was enqueued and its results not yet delivered
  uint64_t seq = 0;      // issue order of that decode
  // the decode's own result delivery (pqg_sync, or the slot's reuse): its output struct, the
  // level count read_batch reports, and what the host checks found before the launch
  pqg_output* out = nullptr;
  uint64_t total_levels = 0;
  int host_status = 0;
  int host_bad_page = -1;
  std::string host_msg;
  // BYTE_ARRAY / FLBA scratch: per value source address, length, DELTA_BYTE_ARRAY prefix;
  // per dictionary entry source address and length
  uint64_t* vsrc = nullptr;
  uint32_t* vlen = nullptr;
  uint32_t* vpre = nullptr;
  uint64_t* tsum = nullptr;  // BYTE_ARRAY copy: per page and tile of 4096 values, bytes then start
  size_t tsumcap = 0;
  size_t vcap = 0;
  uint64_t* dsrc = nullptr;
  uint32_t* dlen = nullptr;
  size_t dcap = 0;
  // hybrid-stream expand tiles: tile -> page map and one checkpoint array per stream kind
  uint32_t* tile_page = nullptr;
  RunTables rt[3] = {};  // def, rep, values (index-pass outputs)
  size_t tcap = 0;
  size_t pfcap = 0;      // pages the rt[].pflag arrays hold
  DeltaTables dt = {};   // DELTA_BINARY_PACKED tiled path
  size_t dt_tcap = 0, dt_pcap = 0;
  // level path (def, rep, RLE booleans): buffers of LevelTables (pqg_internal.hpp), grown on demand
  static constexpr int LV_BUFS = 13;  // wbase, wbase2, wfirst, rec, tab, win, sbase, bexit, seg, srec, spos, dense, ctr
  void* lvbuf[3][LV_BUFS] = {};
  size_t lvcap[3][LV_BUFS] = {};
  LevelTables lt(int k) const {
    LevelTables t{};
    t.wbase = (uint32_t*)lvbuf[k][0];
    t.wbase2 = (uint32_t*)lvbuf[k][1];
    t.wfirst = (uint32_t*)lvbuf[k][2];
    t.rec = (uint2*)lvbuf[k][3];
    t.tab = (uint2*)lvbuf[k][4];
    t.win = (uint2*)lvbuf[k][5];
    t.sbase = (uint32_t*)lvbuf[k][6];
    t.bexit = (uint32_t*)lvbuf[k][7];
    t.seg = (LvSeg*)lvbuf[k][8];
    t.srec = (uint2*)lvbuf[k][9];
    t.spos = (uint32_t*)lvbuf[k][10];
    t.dense = (uint32_t*)lvbuf[k][11];
    t.ctr = (uint32_t*)lvbuf[k][12];
    return t;
  }
};

struct pqg_ctx {
  int device = 0;
  Slot slot[2];
  int cur = 0;          // slot of the last decode
  PageWork* d_pages = nullptr;
  PageWork* h_pages = nullptr;
  ChunkResult* d_res = nullptr;
  ChunkResult* h_res = nullptr;
  hipEvent_t* ev = nullptr;
  hipStream_t stream = nullptr;
  bool timing = false;
  uint64_t seq = 0;     // decodes issued
  // first failure among decodes delivered at a slot's reuse, reported by the next pqg_sync
  int held_status = 0;
  int held_page = -1;
  uint64_t held_seq = 0;
  std::string held_msg;
  double acc_ms[7] = {};
  uint32_t epoch = 0;  // decode counter: look-back flags of older decodes never match
  uint64_t* dbgbuf = nullptr;  // diagnostics (PQG_DEBUG bit 4)
  size_t dbg_cap = 0;
  uint32_t dbg_n = 0;
  uint64_t acc_n = 0;
  uint32_t values_kernel = 0;
  uint64_t* sp_tiles = nullptr;  // pqg_space_values: per tile of levels, max_def count then base
  size_t sp_cap = 0;
  std::string msg;
};

// Adds the stage and kernel times of a finished decode to the accumulators.
static void harvest_times(double* acc, const hipEvent_t* ev, bool kl, bool kv) {
  float ms[7] = {};
  hipEventElapsedTime(&ms[0], ev[0], ev[1]);
  hipEventElapsedTime(&ms[1], ev[1], ev[2]);
  hipEventElapsedTime(&ms[2], ev[2], ev[3]);
  hipEventElapsedTime(&ms[3], ev[3], ev[4]);
  hipEventElapsedTime(&ms[4], ev[0], ev[5]);
  if (kl) hipEventElapsedTime(&ms[5], ev[6], ev[7]);
  if (kv) hipEventElapsedTime(&ms[6], ev[8], ev[9]);
  for (int k = 0; k < 7; ++k) acc[k] += ms[k];
}

static int set_err(pqg_ctx* c, int st, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  c->msg = buf;
  return st;
}

static int hip_fail(pqg_ctx* c, hipError_t e, const char* what) {
  return set_err(c, PQG_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

static const char* status_name(int st) {
  static const char* names[] = {"OK", "General", "NYI", "EOF", "panic", "hang", "capacity", "invalid", "hip"};
  return st >= 0 && st < 9 ? names[st] : "?";
}

// Delivers the results of slot sl's finished decode into its output struct; returns its status
// (the host checks' status when they rejected a page no later than the first failing one)
// and writes the failing page and a message.
static int finish_slot(Slot& sl, int* page_out, std::string& msg) {
  const ChunkResult& r = *sl.h_res;
  pqg_output* out = sl.out;
  out->num_levels = sl.total_levels;
  out->num_values = r.total_values;
  out->num_bytes = r.total_bytes;
  int st = 0, page = -1;
  if (r.bad != ~0ull) {
    page = (int)(r.bad >> 32);
    st = (int)(uint32_t)r.bad;
  }
  if (sl.host_status && (page < 0 || sl.host_bad_page <= page)) {
    page = sl.host_bad_page;
    st = sl.host_status;
    msg = sl.host_msg;
  } else if (st) {
    char buf[160];
    snprintf(buf, sizeof(buf), "page %d: %s (reference: %s)", page, status_name(st),
             st == PQG_ERR_PANIC ? "panics" : st == PQG_ERR_HANG ? "loops forever" : "returns Err");
    msg = buf;
  }
  sl.pending = false;
  *page_out = page;
  return st;
}

#define HIPCHK(expr, what)                      \
  do {                                          \
    hipError_t _e = (expr);                     \
    if (_e != hipSuccess) return hip_fail(ctx, _e, what); \
  } while (0)

static int log2_ceil(uint64_t x) {  // bit_util.rs:91-104
  if (x == 1) return 0;
  x -= 1;
  int r = 0;
  while (x) {
    x >>= 1;
    r++;
  }
  return r;
}

// Entries a level-path window table keeps per window (device/pqg_levels.hip lv_ent).
static uint32_t lv_ent(uint32_t w) {
  return w == 1 ? 64u : w == 2 ? 128u : w <= 4 ? 256u : w <= 8 ? 512u : 1024u;
}
static const uint64_t LV_WIN = 1024;

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

extern "C" {

int pqg_ctx_create(int device, pqg_ctx** out) {
  if (!out) return PQG_ERR_INVALID;
  *out = nullptr;
  pqg_ctx* ctx = new pqg_ctx();
  ctx->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete ctx;
    return PQG_ERR_HIP;
  }
  for (Slot& sl : ctx->slot) {
    if (hipMalloc(&sl.d_res, sizeof(ChunkResult)) != hipSuccess ||
        hipHostMalloc(&sl.h_res, sizeof(ChunkResult), hipHostMallocDefault) != hipSuccess) {
      delete ctx;
      return PQG_ERR_HIP;
    }
    for (auto& ev : sl.ev) hipEventCreate(&ev);
  }
  ctx->cur = 1;
  *out = ctx;
  return PQG_OK;
}

int pqg_ctx_destroy(pqg_ctx* ctx) {
  if (!ctx) return PQG_OK;
  hipSetDevice(ctx->device);
  for (Slot& sl : ctx->slot) {
    if (sl.used || sl.pending) hipEventSynchronize(sl.ev[5]);
    hipFree(sl.d_pages);
    hipHostFree(sl.h_pages);
    hipFree(sl.d_res);
    hipHostFree(sl.h_res);
    hipFree(sl.vsrc);
    hipFree(sl.vlen);
    hipFree(sl.vpre);
    hipFree(sl.tsum);
    hipFree(sl.dsrc);
    hipFree(sl.dlen);
    hipFree(sl.tile_page);
    for (RunTables& t : sl.rt) {
      hipFree(t.ck);
      hipFree(t.runs);
      hipFree(t.nruns);
      hipFree(t.desc);
      hipFree(t.qcount);
      hipFree(t.pflag);
      hipFree(t.nfall);
    }
    hipFree(sl.dt.page);
    hipFree(sl.dt.blocks);
    hipFree(sl.dt.agg);
    hipFree(sl.dt.inc);
    hipFree(sl.dt.flag);
    hipFree(sl.dt.nfall);
    for (int k = 0; k < 3; ++k) {
      for (void* b : sl.lvbuf[k]) hipFree(b);
    }
    for (auto& ev : sl.ev) hipEventDestroy(ev);
  }
  hipFree(ctx->sp_tiles);
  delete ctx;
  return PQG_OK;
}

int pqg_ctx_set_timing(pqg_ctx* ctx, int enabled) {
  if (!ctx) return PQG_ERR_INVALID;
  ctx->timing = enabled != 0;
  return PQG_OK;
}

const char* pqg_error_message(pqg_ctx* ctx) { return ctx ? ctx->msg.c_str() : "null ctx"; }

// Host-side checks that read_new_page / set_current_page_encoding / configure_dictionary /
// get_decoder would make before touching page bytes. Returns the status of the first page
// they reject (or 0) and writes that page's index.
static int validate_pages(const pqg_column* col, const pqg_page* pages, uint32_t n, int* bad,
                          int* dict_page, std::string& why) {
  *dict_page = -1;
  const int t = col->physical_type;
  for (uint32_t i = 0; i < n; ++i) {
    const pqg_page& p = pages[i];
    *bad = (int)i;
    if (p.page_type == PQG_PAGE_DICTIONARY) {
      if (*dict_page >= 0) {
        why = "Column cannot have more than one dictionary";
        return PQG_ERR_GENERAL;  // column/reader.rs:469-471
      }
      if (p.encoding != PQG_PLAIN && p.encoding != PQG_PLAIN_DICTIONARY) {
        why = "Invalid/Unsupported encoding type for dictionary";
        return PQG_ERR_NYI;  // column/reader.rs:483-486
      }
      *dict_page = (int)i;
      continue;
    }
    if (p.page_type != PQG_PAGE_DATA && p.page_type != PQG_PAGE_DATA_V2) continue;
    int enc = p.encoding;
    if (enc == PQG_PLAIN_DICTIONARY) enc = PQG_RLE_DICTIONARY;
    switch (enc) {
      case PQG_RLE_DICTIONARY:
        if (*dict_page < 0) {
          why = "Decoder for dict should have been set";
          return PQG_ERR_PANIC;  // column/reader.rs:396-399
        }
        break;
      case PQG_PLAIN:
        break;
      case PQG_RLE:
        if (t != PQG_BOOLEAN) {
          why = "RleValueDecoder only supports BoolType";
          return PQG_ERR_PANIC;  // decoding.rs:355-357
        }
        break;
      case PQG_DELTA_BINARY_PACKED:
        if (t != PQG_INT32 && t != PQG_INT64) {
          why = "DeltaBitPackDecoder only supports Int32Type and Int64Type";
          return PQG_ERR_PANIC;
        }
        break;
      case PQG_DELTA_LENGTH_BYTE_ARRAY:
        if (t != PQG_BYTE_ARRAY) {
          why = "DeltaLengthByteArrayDecoder only support ByteArrayType";
          return PQG_ERR_GENERAL;
        }
        break;
      case PQG_DELTA_BYTE_ARRAY:
        if (t != PQG_BYTE_ARRAY && t != PQG_FIXED_LEN_BYTE_ARRAY) {
          why = "DeltaByteArrayDecoder only supports ByteArrayType and FixedLenByteArrayType";
          return PQG_ERR_GENERAL;
        }
        break;
      default:
        why = "Encoding is not supported";
        return PQG_ERR_NYI;  // get_decoder, decoding.rs:76
    }
  }
  *bad = -1;
  return PQG_OK;
}

int pqg_decode_chunk(pqg_ctx* ctx, const pqg_column* col, const uint8_t* blob, uint64_t blob_len,
                     const pqg_page* pages, uint32_t npages, pqg_output* out, void* stream_v) {
  if (!ctx || !col || !out || (npages && !pages)) return PQG_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream_v;
  // ---- argument checks first: a rejected call leaves the context (and a decode still in
  // flight on it) untouched, so a later pqg_sync reports that decode's own status
  auto misaligned = [](const void* p) { return p && ((uintptr_t)p & 15u); };
  if (misaligned(out->def_levels) || misaligned(out->rep_levels) || misaligned(out->values))
    return set_err(ctx, PQG_ERR_INVALID, "output buffers must be 16-byte aligned");
  const int t = col->physical_type;
  if (t < 0 || t > 7) return set_err(ctx, PQG_ERR_INVALID, "bad physical type %d", t);
  if (t == PQG_FIXED_LEN_BYTE_ARRAY && col->type_length <= 0)
    return set_err(ctx, PQG_ERR_PANIC, "FLBA requires type_length > 0");
  if ((t == PQG_BYTE_ARRAY || t == PQG_FIXED_LEN_BYTE_ARRAY) && out->values) {
    uint64_t nlev = 0;
    for (uint32_t i = 0; i < npages; ++i)
      if (pages[i].page_type == PQG_PAGE_DATA || pages[i].page_type == PQG_PAGE_DATA_V2)
        nlev += pages[i].num_values;
    if (!out->offsets || out->offsets_capacity < nlev + 1)
      return set_err(ctx, PQG_ERR_INVALID, "BYTE_ARRAY/FLBA output needs offsets[num_levels + 1]");
  }
  HIPCHK(hipSetDevice(ctx->device), "hipSetDevice");
  ctx->stream = s;
  out->num_levels = out->num_values = out->num_bytes = 0;

  // ---- staging slot: wait until its previous decode has finished, harvest its timings and
  // deliver its results (a failure is held for the next pqg_sync)
  ctx->cur ^= 1;
  Slot& sl = ctx->slot[ctx->cur];
  if (sl.used || sl.pending) {
    HIPCHK(hipEventSynchronize(sl.ev[5]), "slot wait");
    if (sl.used && ctx->timing) {
      harvest_times(ctx->acc_ms, sl.ev, sl.kl, sl.kv);
      ctx->acc_n++;
    }
    sl.used = false;
    if (sl.pending) {
      int page;
      std::string m;
      const int st = finish_slot(sl, &page, m);
      if (st && !ctx->held_status) {
        ctx->held_status = st;
        ctx->held_page = page;
        ctx->held_seq = sl.seq;
        ctx->held_msg = m;
      }
    }
  }
  sl.out = out;
  sl.host_status = 0;
  sl.host_bad_page = -1;
  sl.host_msg.clear();
  // page table and the chunk result go up in one copy: the result sits after the pages
  const size_t res_off = ((size_t)npages * sizeof(PageWork) + 63) & ~(size_t)63;
  if (npages > sl.pages_cap) {
    size_t cap = npages < 1024 ? 1024 : npages;
    hipFree(sl.d_pages);
    hipHostFree(sl.h_pages);
    sl.d_pages = nullptr;
    sl.h_pages = nullptr;
    const size_t bytes = ((cap * sizeof(PageWork) + 63) & ~(size_t)63) + sizeof(ChunkResult);
    HIPCHK(hipMalloc(&sl.d_pages, bytes), "hipMalloc pages");
    HIPCHK(hipHostMalloc(&sl.h_pages, bytes, hipHostMallocDefault), "hipHostMalloc");
    sl.pages_cap = cap;
  }
  ctx->d_pages = sl.d_pages;
  ctx->h_pages = sl.h_pages;
  ctx->d_res = (ChunkResult*)((char*)sl.d_pages + res_off);
  ctx->h_res = sl.h_res;
  ctx->ev = sl.ev;
  sl.kl = sl.kv = false;
  int bad = -1, dict_page = -1;
  std::string why;
  int vst = validate_pages(col, pages, npages, &bad, &dict_page, why);
  uint64_t level_out = 0, max_page_bytes = 0, max_page_vals = 0;
  uint32_t total_tiles = 0;
  bool enc_present[16] = {};
  uint64_t nwin = 0;           // level-path windows, upper bound (a stream is part of its page)
  for (uint32_t i = 0; i < npages; ++i) {
    PageWork& w = ctx->h_pages[i];
    memset(&w, 0, sizeof(w));
    w.base = pages[i].offset;
    w.nbytes = pages[i].nbytes;
    w.num_values = pages[i].num_values;
    w.page_type = pages[i].page_type;
    w.encoding = pages[i].encoding;
    if (w.page_type != PQG_PAGE_DICTIONARY && w.encoding == PQG_PLAIN_DICTIONARY)
      w.encoding = PQG_RLE_DICTIONARY;  // column/reader.rs:391-393
    w.def_encoding = pages[i].def_encoding;
    w.rep_encoding = pages[i].rep_encoding;
    w.def_len = pages[i].def_len;
    w.rep_len = pages[i].rep_len;
    w.level_out = level_out;
    w.ltile0 = total_tiles;
    w.ntiles = 0;
    if (w.page_type == PQG_PAGE_DATA || w.page_type == PQG_PAGE_DATA_V2) {
      w.ntiles = (uint32_t)(((uint64_t)w.num_values + RUN_TILE - 1) / RUN_TILE);
      total_tiles += w.ntiles;
      level_out += w.num_values;
      if (w.encoding >= 0 && w.encoding < 16) enc_present[w.encoding] = true;
      if (w.nbytes > max_page_bytes) max_page_bytes = w.nbytes;
      if (w.num_values > max_page_vals) max_page_vals = w.num_values;
      nwin += (w.nbytes + LV_WIN - 1) / LV_WIN;
    }
    if (vst && (int)i == bad) w.status = vst;
    if (vst && (int)i > bad) w.status = -1;  // never reached by the reference
  }
  if (vst) {
    sl.host_status = vst;
    sl.host_bad_page = bad;
    sl.host_msg = why;
  }
  const bool want_def = col->max_def > 0 && out->def_levels;
  const bool want_rep = col->max_rep > 0 && out->rep_levels;
  const uint64_t lev_needed = level_out;
  // read_batch reports levels only for the streams it reads (column/reader.rs:259)
  sl.total_levels = (want_def || want_rep) ? lev_needed : 0;

  ColumnParams cp{};
  cp.physical_type = t;
  cp.type_length = col->type_length;
  cp.max_def = col->max_def;
  cp.max_rep = col->max_rep;
  cp.def_bit_width = log2_ceil((uint64_t)(int64_t)col->max_def + 1);
  cp.rep_bit_width = log2_ceil((uint64_t)(int64_t)col->max_rep + 1);
  cp.want_def = want_def;
  cp.want_rep = want_rep;
  // byte-array entries (address + length per value) take every index width; 4- / 8-byte values
  // up to 8 bits (wider: a large dictionary, gathered faster by the tiled expand)
  cp.dict_maxw = (t == PQG_BYTE_ARRAY || t == PQG_FIXED_LEN_BYTE_ARRAY) ? 16u : 8u;
  // Diagnostic kernel modes exist only in a PQG_DIAG build (make DIAG=1); the shipped library
  // never reads the environment and always runs the production path.
#ifdef PQG_DIAG
  static const int dbg_env = getenv("PQG_DEBUG") ? atoi(getenv("PQG_DEBUG")) : 0;
#else
  const int dbg_env = 0;
#endif
  cp.debug = dbg_env;
  cp.dbgbuf = nullptr;
  if (dbg_env & (16 | 32 | 64 | 128)) {
    size_t need = (size_t)(total_tiles * 4 > (uint64_t)npages * 2 ? total_tiles * 4 : (uint64_t)npages * 2) * 16;
    if (need < (size_t)npages * 64) need = (size_t)npages * 64;
    if (dbg_env & 128) need = (size_t)(nwin / LW_SEGW + npages + 1) * 32;  // per level-stream segment
    if (need > ctx->dbg_cap) {
      hipFree(ctx->dbgbuf);
      ctx->dbgbuf = nullptr;
      HIPCHK(hipMalloc(&ctx->dbgbuf, need), "hipMalloc dbg");
      ctx->dbg_cap = need;
    }
    ctx->dbg_n = (dbg_env & 32) ? (uint32_t)npages : total_tiles * 4;
    cp.dbgbuf = ctx->dbgbuf;
  }

  ChunkResult r0{};
  r0.total_levels = sl.total_levels;
  r0.bad = ~0ull;
  r0.dict_page = dict_page < 0 ? 0xFFFFFFFFu : (uint32_t)dict_page;
  *(ChunkResult*)((char*)ctx->h_pages + res_off) = r0;
  HIPCHK(hipMemcpyAsync(ctx->d_pages, ctx->h_pages, res_off + sizeof(ChunkResult), hipMemcpyHostToDevice, s),
         "H2D pages");

  const bool is_ba = t == PQG_BYTE_ARRAY || t == PQG_FIXED_LEN_BYTE_ARRAY;
  const int es = is_ba ? 0 : value_size(t, col->type_length);
  const int np = (int)npages;
  if (is_ba && out->values) {
    size_t need = lev_needed ? lev_needed : 1;
    if (need > sl.vcap) {
      hipFree(sl.vsrc);
      hipFree(sl.vlen);
      hipFree(sl.vpre);
      sl.vsrc = nullptr;
      sl.vlen = sl.vpre = nullptr;
      HIPCHK(hipMalloc(&sl.vsrc, need * 8), "hipMalloc vsrc");
      HIPCHK(hipMalloc(&sl.vlen, need * 4), "hipMalloc vlen");
      HIPCHK(hipMalloc(&sl.vpre, need * 4), "hipMalloc vpre");
      sl.vcap = need;
    }
    const size_t tneed = (size_t)np * ((max_page_vals + 4095) / 4096) + 1;
    if (tneed > sl.tsumcap) {
      hipFree(sl.tsum);
      sl.tsum = nullptr;
      sl.tsumcap = 0;
      HIPCHK(hipMalloc(&sl.tsum, tneed * 8), "hipMalloc byte-array tiles");
      sl.tsumcap = tneed;
    }
    size_t dn = dict_page >= 0 && pages[dict_page].num_values ? pages[dict_page].num_values : 1;
    if (dn > sl.dcap) {
      hipFree(sl.dsrc);
      hipFree(sl.dlen);
      sl.dsrc = nullptr;
      sl.dlen = nullptr;
      HIPCHK(hipMalloc(&sl.dsrc, dn * 8), "hipMalloc dsrc");
      HIPCHK(hipMalloc(&sl.dlen, dn * 4), "hipMalloc dlen");
      sl.dcap = dn;
    }
  }
  // expand-tile bookkeeping of the hybrid streams (tile -> page, checkpoints per stream kind)
  if (total_tiles + 1 > sl.tcap) {
    hipFree(sl.tile_page);
    sl.tile_page = nullptr;
    for (RunTables& r : sl.rt) {
      hipFree(r.ck);
      hipFree(r.runs);
      hipFree(r.nruns);
      hipFree(r.desc);
      hipFree(r.qcount);
      hipFree(r.pflag);
      hipFree(r.nfall);
      r = RunTables{};
    }
    sl.tcap = 0;
    sl.pfcap = 0;
    size_t cap = (size_t)total_tiles + 1024;
    HIPCHK(hipMalloc(&sl.tile_page, cap * sizeof(uint32_t)), "hipMalloc tile_page");
    sl.tcap = cap;
  }
  // run tables are allocated per stream kind on first use
  auto tables = [&](int k) -> hipError_t {
    RunTables& r = sl.rt[k];
    if (r.ck) return hipSuccess;
    hipError_t e = hipMalloc(&r.ck, (sl.tcap + 1) * sizeof(RunCkpt));
    if (e == hipSuccess) e = hipMalloc(&r.runs, sl.tcap * RUN_CAPT * sizeof(uint2));
    if (e == hipSuccess) e = hipMalloc(&r.nruns, sl.tcap * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&r.desc, sl.tcap * 4 * sizeof(QDesc));
    if (e == hipSuccess) e = hipMalloc(&r.qcount, sl.tcap * 4 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&r.nfall, sizeof(uint32_t));
    return e;
  };
  // page-pass flags, sized by pages (all stream kinds together)
  if ((size_t)np > sl.pfcap) {
    const size_t pc = (size_t)np < 4096 ? 4096 : (size_t)np * 2;
    for (RunTables& r : sl.rt) {
      hipFree(r.pflag);
      r.pflag = nullptr;
    }
    sl.pfcap = 0;
    for (RunTables& r : sl.rt) HIPCHK(hipMalloc(&r.pflag, pc * sizeof(uint32_t)), "hipMalloc page flags");
    sl.pfcap = pc;
  }
  const bool hybrid_values = enc_present[PQG_RLE_DICTIONARY] || (enc_present[PQG_RLE] && t == PQG_BOOLEAN);
  if (want_def) HIPCHK(tables(0), "hipMalloc run tables");
  if (want_rep) HIPCHK(tables(1), "hipMalloc run tables");
  if (hybrid_values && out->values) HIPCHK(tables(2), "hipMalloc run tables");
  const uint32_t nt = total_tiles;
  // Level path buffers (normalized streams) per stream kind, grown on demand.
  const bool rle_bool = enc_present[PQG_RLE] && t == PQG_BOOLEAN && out->values;
  // 4- / 8-byte dictionary values: their index streams take the same path (pqg_launch_dict)
  bool dict_lv = enc_present[PQG_RLE_DICTIONARY] && !is_ba && out->values && (es == 4 || es == 8);
  // byte-array dictionary indices: entry addresses and lengths from the same path
  bool badict_lv = enc_present[PQG_RLE_DICTIONARY] && is_ba && out->values;
#ifdef PQG_DIAG
  if (cp.debug & 256) dict_lv = badict_lv = false;  // diagnostics: dictionary indices through the general decoder
#endif
  dict_lv = dict_lv || badict_lv;
  const bool need_lv[3] = {want_def, want_rep, rle_bool || dict_lv};
  auto grow = [&](void** p, size_t* cap, size_t need, size_t elem, const char* what) -> int {
    if (need <= *cap) return PQG_OK;
    hipFree(*p);
    *p = nullptr;
    *cap = 0;
    const size_t c = need + need / 8 + 1024;
    HIPCHK(hipMalloc(p, c * elem), what);
    *cap = c;
    return PQG_OK;
  };
  for (int k = 0; k < 3; ++k) {
    if (!need_lv[k]) continue;
    int st;
    const size_t ent = lv_ent(k == 2 ? 1u : (uint32_t)(k == 0 ? cp.def_bit_width : cp.rep_bit_width));
    const size_t nseg = nwin / LW_SEGW + npages + 1;  // segments, upper bound
    const size_t need[Slot::LV_BUFS] = {(size_t)npages + 1, (size_t)npages + 1, nwin + npages + 1,
                                        64 * (nwin + 2 * (size_t)npages) + 1, (nwin + 1) * ent, nwin + 1,
                                        (size_t)npages + 1, nseg, nseg, nseg * LW_SCAP, nseg * LW_SCAP,
                                        (size_t)npages + 1, 16};
    const size_t elem[Slot::LV_BUFS] = {4, 4, 4, sizeof(uint2), sizeof(uint2), sizeof(uint2),
                                        4, 4, sizeof(LvSeg), sizeof(uint2), 4, 4, 4};
    const bool fresh_ctr = sl.lvbuf[k][12] == nullptr;
    for (int b = 0; b < Slot::LV_BUFS; ++b)
      if ((st = grow(&sl.lvbuf[k][b], &sl.lvcap[k][b], need[b], elem[b], "hipMalloc level tables"))) return st;
    // the tickets start at zero once; every launch using them leaves them at zero
    if (fresh_ctr) HIPCHK(hipMemsetAsync(sl.lvbuf[k][12], 0, sl.lvcap[k][12] * 4, s), "memset level tickets");
  }
  // Hybrid-stream flags: the level path (def, rep, RLE booleans) sets every page's flag and counts
  // the streams it hands back; dictionary indices always take the general decoder. k_prepare
  // sets them (no memset launches), and runs the fixed-width dictionary page's checks.
  PrepInit ini{};
  int nw_ = 0, nz = 0;
  for (int k = 0; k < 3; ++k) {
    if (!sl.rt[k].nfall) continue;
    const bool lvpath = k < 2 || rle_bool || dict_lv;
    ini.word[nw_] = sl.rt[k].nfall;
    ini.val[nw_++] = lvpath ? 0u : 0xFFFFFFFFu;
    if (!lvpath) ini.pzero[nz++] = sl.rt[k].pflag;
  }
  uint8_t* vo = (uint8_t*)out->values;
  const bool delta_vals = np && vo && !is_ba && enc_present[PQG_DELTA_BINARY_PACKED] && (t == PQG_INT32 || t == PQG_INT64);
  if (delta_vals) {  // DELTA_BINARY_PACKED tables (tiled fallback path), grown on demand
    if (nt > sl.dt_tcap || (size_t)np > sl.dt_pcap) {
      hipFree(sl.dt.page);
      hipFree(sl.dt.blocks);
      hipFree(sl.dt.agg);
      hipFree(sl.dt.inc);
      hipFree(sl.dt.flag);
      hipFree(sl.dt.nfall);
      sl.dt = DeltaTables{};
      sl.dt_tcap = sl.dt_pcap = 0;
      const size_t tc = sl.tcap, pc = (size_t)np < 1024 ? 1024 : np;
      HIPCHK(hipMalloc(&sl.dt.page, pc * sizeof(DeltaPage)), "hipMalloc delta pages");
      HIPCHK(hipMalloc(&sl.dt.blocks, tc * DELTA_BCAP * sizeof(DeltaBlock)), "hipMalloc delta blocks");
      HIPCHK(hipMalloc(&sl.dt.agg, tc * sizeof(uint64_t)), "hipMalloc delta agg");
      HIPCHK(hipMalloc(&sl.dt.inc, tc * sizeof(uint64_t)), "hipMalloc delta inc");
      HIPCHK(hipMalloc(&sl.dt.flag, tc * sizeof(uint32_t)), "hipMalloc delta flags");
      HIPCHK(hipMalloc(&sl.dt.nfall, sizeof(uint32_t)), "hipMalloc delta fallback count");
      HIPCHK(hipMemsetAsync(sl.dt.flag, 0, tc * sizeof(uint32_t), s), "memset delta flags");
      sl.dt_tcap = tc;
      sl.dt_pcap = pc;
    }
    ctx->epoch = (ctx->epoch + 1) & 0x3FFFFFFFu;
    if (ctx->epoch == 0) {  // wrapped: flags from 2^30 decodes ago could match
      HIPCHK(hipMemsetAsync(sl.dt.flag, 0, sl.dt_tcap * sizeof(uint32_t), s), "memset delta flags");
      ctx->epoch = 1;
    }
    ini.word[nw_] = sl.dt.nfall;
    ini.val[nw_++] = 0u;
  }
  ini.dict_page = dict_page;
  // configure_dictionary decodes the dictionary page whenever the reader reaches it, whatever the
  // data pages' encodings and whether values are read (column/reader.rs:463-481)
  ini.dict_es = (np && dict_page >= 0 && !is_ba) ? es : 0;
  ini.dense_def = need_lv[0] ? sl.lt(0).dense : nullptr;
  ini.dense_rep = need_lv[1] ? sl.lt(1).dense : nullptr;
  ini.dense_zero = (need_lv[2] && dict_lv) ? sl.lt(2).dense : nullptr;
  if (ctx->timing) hipEventRecord(ctx->ev[0], s);
  if (np) HIPCHK(pqg_launch_prepare(blob, blob_len, ctx->d_pages, np, cp, sl.tile_page, ctx->d_res, ini, s), "prepare");
  if (ctx->timing) hipEventRecord(ctx->ev[1], s);
  // the value-offset scan runs in the def stream's last kernel when no rep stream follows it
  // (timed runs take the same kernel sequence: the stage events bracket the fused kernel)
  const bool fused_scan = np && want_def && !want_rep;
  if (np && want_def) {
    HIPCHK(pqg_launch_levels(blob, blob_len, ctx->d_pages, np, nt, cp, 0, sl.tile_page, sl.rt[0],
                             sl.lt(0), out->def_levels, ctx->d_res, s,
                             ctx->timing ? &sl.ev[6] : nullptr, fused_scan ? es : -1, out->values_capacity),
           "def levels");
    sl.kl = ctx->timing;
  }
  if (np && want_rep)
    HIPCHK(pqg_launch_levels(blob, blob_len, ctx->d_pages, np, nt, cp, 1, sl.tile_page, sl.rt[1],
                             sl.lt(1), out->rep_levels, ctx->d_res, s, nullptr, -1, 0),
           "rep levels");
  if (ctx->timing) hipEventRecord(ctx->ev[2], s);
  if (!fused_scan) HIPCHK(pqg_launch_scan(ctx->d_pages, np, ctx->d_res, es, out->values_capacity, s), "scan");
  if (ctx->timing) hipEventRecord(ctx->ev[3], s);
  ctx->values_kernel = 0;
  if (np && vo && is_ba) {
    ctx->values_kernel = enc_present[PQG_RLE_DICTIONARY] ? PQG_RLE_DICTIONARY
                         : enc_present[PQG_DELTA_BYTE_ARRAY] ? PQG_DELTA_BYTE_ARRAY
                         : enc_present[PQG_DELTA_LENGTH_BYTE_ARRAY] ? PQG_DELTA_LENGTH_BYTE_ARRAY
                                                                     : PQG_PLAIN;
    const int tl = t == PQG_FIXED_LEN_BYTE_ARRAY ? col->type_length : 0;
    if (enc_present[PQG_RLE_DICTIONARY]) {
      HIPCHK(pqg_launch_ba_dict_prep(blob, blob_len, ctx->d_pages, dict_page, tl, sl.dsrc, sl.dlen,
                                     ctx->d_res, s), "byte-array dictionary");
      if (badict_lv)  // (nfall 0: the flags the plan sets decide which pages the index pass takes)
        HIPCHK(pqg_launch_lv_badict(blob, blob_len, ctx->d_pages, np, cp, dict_page, sl.rt[2], sl.lt(2), sl.dsrc,
                                    sl.dlen, sl.vsrc, sl.vlen, ctx->d_res, s), "dictionary indices");
      HIPCHK(pqg_launch_run_index(blob, blob_len, ctx->d_pages, np, cp, 2 /* SS_DICT */, dict_page,
                                  sl.rt[2], ctx->d_res, s), "dictionary index pass");
      HIPCHK(pqg_launch_tile_desc(blob, ctx->d_pages, nt, sl.tile_page, sl.rt[2], cp, 2, dict_page, s),
             "dictionary tiles");
      HIPCHK(pqg_launch_badict_expand(blob, blob_len, ctx->d_pages, nt, sl.rt[2], dict_page, sl.vsrc,
                                      sl.vlen, sl.dsrc, sl.dlen, ctx->d_res, s), "dictionary expand");
      HIPCHK(pqg_launch_page_counts(ctx->d_pages, np, sl.rt[2], 1, s), "dictionary byte counts");
    }
    HIPCHK(pqg_launch_bytes(blob, blob_len, ctx->d_pages, np, tl, enc_present[PQG_DELTA_BYTE_ARRAY],
                            sl.vsrc, sl.vlen, sl.vpre, out->values_capacity, out->offsets, vo, max_page_vals,
                            sl.tsum, ctx->d_res, s),
           "byte arrays");
  } else if (np && vo) {
    if (enc_present[PQG_PLAIN]) {
      ctx->values_kernel = PQG_PLAIN;
      if (t == PQG_BOOLEAN)
        HIPCHK(pqg_launch_plain_bool(blob, ctx->d_pages, np, max_page_vals, vo, ctx->d_res, s), "plain bool");
      else if (es > 0) {
        if (ctx->timing) hipEventRecord(sl.ev[8], s);
        HIPCHK(pqg_launch_plain_copy(blob, blob_len, ctx->d_pages, np, es, PQG_PLAIN, max_page_bytes, vo,
                                     ctx->d_res, s), "plain");
        if (ctx->timing) hipEventRecord(sl.ev[9], s);
        sl.kv = true;
      }
    }
    if (enc_present[PQG_RLE_DICTIONARY]) {
      ctx->values_kernel = PQG_RLE_DICTIONARY;
      // a dictionary of at most 2^dict_maxw entries: the writer's index width is within the level
      // path's limit, so the general decoder only sees the rare pages it hands back
      const int small_dict = dict_page >= 0 && pages[dict_page].num_values <= (1u << cp.dict_maxw);
      HIPCHK(pqg_launch_dict(blob, blob_len, ctx->d_pages, np, nt, cp, dict_page, es, sl.tile_page,
                             sl.rt[2], sl.lt(2), vo, ctx->d_res, s, ctx->timing ? &sl.ev[8] : nullptr, small_dict),
             "dict");
      sl.kv = ctx->timing;
    }
    if (delta_vals) {
      ctx->values_kernel = PQG_DELTA_BINARY_PACKED;
      sl.dt.dbg = (cp.debug & 32) ? cp.dbgbuf : nullptr;
      HIPCHK(pqg_launch_delta_tiled(blob, blob_len, ctx->d_pages, np, nt, sl.tile_page, sl.dt, ctx->epoch,
                                    es, vo, ctx->d_res, s, ctx->timing ? &sl.ev[8] : nullptr), "delta");
      sl.kv = true;
    }
    if (enc_present[PQG_RLE] && t == PQG_BOOLEAN) {
      ctx->values_kernel = PQG_RLE;
      HIPCHK(pqg_launch_rle_bool(blob, blob_len, ctx->d_pages, np, nt, cp, sl.tile_page, sl.rt[2],
                                 sl.lt(2), vo, ctx->d_res, s), "rle bool");
    }
  }
  if (ctx->timing) hipEventRecord(ctx->ev[4], s);
  HIPCHK(hipMemcpyAsync(ctx->h_res, ctx->d_res, sizeof(ChunkResult), hipMemcpyDeviceToHost, s), "D2H res");
  HIPCHK(hipEventRecord(ctx->ev[5], s), "event");
  sl.used = true;
  sl.pending = true;
  sl.seq = ++ctx->seq;
  return PQG_OK;
}

// Device-side record assembly of a decoded chunk (pqg_launch_space, device/pqg_kernels.hip).
int pqg_space_values(pqg_ctx* ctx, const int16_t* def_levels, uint64_t num_levels, int16_t max_def,
                     const void* values, int value_size, void* spaced, void* stream) {
  if (!ctx || (num_levels && (!def_levels || !spaced || !values)) ||
      (value_size != 1 && value_size != 4 && value_size != 8 && value_size != 12))
    return PQG_ERR_INVALID;
  if (num_levels == 0) return PQG_OK;
  const size_t nt = (size_t)pqg_space_tiles(num_levels);
  if (nt > ctx->sp_cap) {
    hipFree(ctx->sp_tiles);
    ctx->sp_tiles = nullptr;
    ctx->sp_cap = 0;
    if (hipMalloc(&ctx->sp_tiles, nt * 8) != hipSuccess) return set_err(ctx, PQG_ERR_HIP, "hipMalloc spacing tiles");
    ctx->sp_cap = nt;
  }
  const hipError_t e = pqg_launch_space(def_levels, num_levels, max_def, values, value_size, ctx->sp_tiles, spaced,
                                        stream ? (hipStream_t)stream : ctx->stream);
  return e == hipSuccess ? PQG_OK : set_err(ctx, PQG_ERR_HIP, "spacing launch: %s", hipGetErrorString(e));
}

// pqg_sync that also names the failing decode by its issue number (pqg_decode_seq); the
// row-group decoder maps it back to its own call (row_group.cpp).
int pqg_sync_seq(pqg_ctx* ctx, int* first_bad_page, uint64_t* bad_seq);

int pqg_sync(pqg_ctx* ctx, int* first_bad_page) { return pqg_sync_seq(ctx, first_bad_page, nullptr); }

// Issue number of the last decode enqueued on ctx (1, 2, ...; 0 before the first).
uint64_t pqg_decode_seq(pqg_ctx* ctx) { return ctx ? ctx->seq : 0; }

int pqg_sync_seq(pqg_ctx* ctx, int* first_bad_page, uint64_t* bad_seq) {
  if (!ctx) return PQG_ERR_INVALID;
  if (first_bad_page) *first_bad_page = -1;
  if (bad_seq) *bad_seq = 0;
  Slot* order[2] = {&ctx->slot[ctx->cur ^ 1], &ctx->slot[ctx->cur]};
  if (order[0]->pending && order[1]->pending && order[0]->seq > order[1]->seq) std::swap(order[0], order[1]);
  if (!order[0]->pending && !order[1]->pending && !ctx->held_status)
    return set_err(ctx, PQG_ERR_INVALID, "no decode pending");
  // every pending decode is delivered, in issue order; the first failure is reported
  int st = ctx->held_status, page = ctx->held_page;
  uint64_t seq = ctx->held_seq;
  std::string msg = ctx->held_msg;
  ctx->held_status = 0;
  ctx->held_page = -1;
  ctx->held_seq = 0;
  ctx->held_msg.clear();
  hipError_t herr = hipSuccess;
  for (Slot* sl : order) {
    if (!sl->pending) continue;
    const hipError_t e = hipEventSynchronize(sl->ev[5]);
    if (e != hipSuccess) {
      sl->pending = false;
      if (herr == hipSuccess) herr = e;
      continue;
    }
    if (sl->used && ctx->timing) {
      harvest_times(ctx->acc_ms, sl->ev, sl->kl, sl->kv);
      ctx->acc_n++;
    }
    sl->used = false;
    int pg;
    std::string m;
    const uint64_t sq = sl->seq;
    const int s2 = finish_slot(*sl, &pg, m);
    if (s2 && !st) {
      st = s2;
      page = pg;
      seq = sq;
      msg = m;
    }
  }
  if (herr != hipSuccess) return hip_fail(ctx, herr, "hipEventSynchronize");
  ctx->msg = msg;
  if (first_bad_page) *first_bad_page = page;
  if (bad_seq) *bad_seq = st ? seq : 0;
  return st;
}

// Average per-stage device time over every decode since the last reset (HIP events recorded
// on the decode stream between the stages).
int pqg_get_timings(pqg_ctx* ctx, pqg_timings* t) {
  if (!ctx || !t) return PQG_ERR_INVALID;
  memset(t, 0, sizeof(*t));
  if (!ctx->timing || ctx->acc_n == 0) return PQG_ERR_INVALID;
  double n = (double)ctx->acc_n;
  t->prepare_ms = (float)(ctx->acc_ms[0] / n);
  t->levels_ms = (float)(ctx->acc_ms[1] / n);
  t->scan_ms = (float)(ctx->acc_ms[2] / n);
  t->values_ms = (float)(ctx->acc_ms[3] / n);
  t->total_ms = (float)(ctx->acc_ms[4] / n);
  t->levels_kernel_ms = (float)(ctx->acc_ms[5] / n);
  t->values_kernel_ms = (float)(ctx->acc_ms[6] / n);
  t->values_kernel = ctx->values_kernel;
  return PQG_OK;
}

// Diagnostics: average per-wave phase cycles of the last decode's wave expand kernel
// (PQG_DEBUG bit 4). out[0..2] = desc, expand, tail cycles; out[3] = waves.
// Diagnostics: raw copy of the debug buffer (PQG_DIAG builds; u64 words).
int pqg_debug_read(pqg_ctx* ctx, uint64_t* out, size_t n) {
  if (!ctx || !ctx->dbgbuf || !out || n * 8 > ctx->dbg_cap) return PQG_ERR_INVALID;
  return hipMemcpy(out, ctx->dbgbuf, n * 8, hipMemcpyDeviceToHost) == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

int pqg_debug_stamps(pqg_ctx* ctx, double* out4) {
  if (!ctx || !ctx->dbgbuf || !out4) return PQG_ERR_INVALID;
  std::vector<uint32_t> h((size_t)ctx->dbg_n * 4);
  if (hipMemcpy(h.data(), ctx->dbgbuf, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return PQG_ERR_HIP;
  double a = 0, b = 0, c = 0;
  uint64_t n = 0;
  for (uint32_t i = 0; i < ctx->dbg_n; ++i) {
    a += h[4 * i];
    b += h[4 * i + 1];
    c += h[4 * i + 2];
    ++n;
  }
  out4[0] = a / (double)(n ? n : 1);
  out4[1] = b / (double)(n ? n : 1);
  out4[2] = c / (double)(n ? n : 1);
  out4[3] = (double)n;
  return PQG_OK;
}

int pqg_reset_timings(pqg_ctx* ctx) {
  if (!ctx) return PQG_ERR_INVALID;
  for (double& x : ctx->acc_ms) x = 0;
  ctx->acc_n = 0;
  return PQG_OK;
}

}  // extern "C"
