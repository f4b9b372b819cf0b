// chunk_decoder.cpp — pqg_ctx / pqg_decode_chunk(s) / pqg_sync: the host half of the C ABI.
//
// Replaces ColumnReaderImpl's decode driving (column/reader.rs:159-488) for whole column chunks:
// validates each chunk's page sequence the way read_new_page / set_current_page_encoding /
// configure_dictionary would (column/reader.rs:269-488, decoding.rs:60-79), uploads one page
// table for the decode, and enqueues the kernels of device/*.hip on one HIP stream.
//
// A decode is a batch of column chunks (pqg_decode_chunks; pqg_decode_chunk is a batch of one):
// the chunks share nothing in the reference (every column chunk has its own page reader and
// column reader, file/reader.rs:252-260, 306-330), so their pages go into one page table (each
// page naming its chunk, ChunkWork in pqg_internal.hpp) and every kernel runs once over all of
// them. A row group of 11 columns, or several row groups, then costs the ~30 launches one chunk
// costs instead of ~30 per chunk.
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
hipError_t pqg_launch_prepare(const uint8_t*, uint64_t, PageWork*, int, ChunkWork*, uint32_t*, PrepInit, hipStream_t);
hipError_t pqg_launch_run_index(const uint8_t*, uint64_t, PageWork*, int, ChunkWork*, int, RunTables, hipStream_t);
hipError_t pqg_launch_levels(const uint8_t*, uint64_t, PageWork*, int, ChunkWork*, int, uint32_t, const uint32_t*,
                             RunTables, LevelTables, hipStream_t, hipEvent_t*, int, hipEvent_t);
hipError_t pqg_launch_scan(PageWork*, int, ChunkWork*, hipStream_t);
hipError_t pqg_launch_lv(const uint8_t*, uint64_t, PageWork*, int, ChunkWork*, int, uint32_t, const uint64_t*,
                         const uint32_t*, uint64_t*, uint32_t*, RunTables, LevelTables, hipStream_t, hipEvent_t = nullptr);
hipError_t pqg_launch_dict(const uint8_t*, uint64_t, PageWork*, int, ChunkWork*, const uint32_t*, uint32_t,
                           const uint32_t* const*, const uint32_t*, const uint32_t*, uint32_t, const uint32_t* const*,
                           const uint32_t*, uint16_t*, RunTables, hipStream_t, hipEvent_t*);
hipError_t pqg_launch_plain(const uint8_t*, uint64_t, PageWork*, ChunkWork*, const uint32_t*, const uint32_t*, uint32_t,
                            uint64_t, const uint32_t*, uint32_t, hipStream_t);
hipError_t pqg_launch_plain_spec(const uint8_t*, uint64_t, PageWork*, int, ChunkWork*, const uint32_t*, uint32_t,
                                 uint32_t, hipStream_t);
hipError_t pqg_launch_plain_fix(const uint8_t*, uint64_t, PageWork*, ChunkWork*, const uint32_t*, uint32_t,
                                hipStream_t);
hipError_t pqg_launch_rle_bool(const uint8_t*, uint64_t, PageWork*, int, ChunkWork*, const uint32_t*, const uint32_t*,
                               uint32_t, RunTables, LevelTables, hipStream_t);
hipError_t pqg_launch_delta_tiled(const uint8_t*, uint64_t, PageWork*, int, ChunkWork*, uint32_t, const uint32_t*,
                                  DeltaTables, uint32_t, hipStream_t, hipEvent_t*);
hipError_t pqg_launch_space(const int16_t*, uint64_t, int16_t, const void*, int, uint64_t*, void*, hipStream_t);
uint64_t pqg_space_tiles(uint64_t n);
hipError_t pqg_launch_ba_dict_prep(const uint8_t*, uint64_t, PageWork*, ChunkWork*, int, uint64_t*, uint32_t*,
                                   hipStream_t);
hipError_t pqg_launch_badict_general(const uint8_t*, uint64_t, PageWork*, int, ChunkWork*, const uint32_t*,
                                     const uint32_t*, uint32_t, RunTables, uint64_t*, uint32_t*, uint64_t*, uint32_t*,
                                     int, hipStream_t);
hipError_t pqg_launch_bytes(const uint8_t*, uint64_t, PageWork*, int, ChunkWork*, const uint32_t*, const uint32_t*,
                            uint32_t, bool, bool, uint64_t*, uint32_t*, uint32_t*, const uint64_t*, const uint32_t*,
                            uint64_t*, uint32_t*, uint32_t*, const uint32_t*, uint32_t, uint32_t, uint8_t*, uint32_t,
                            hipStream_t);
}

// Stream kinds of the hybrid-stream tables: def, rep, dictionary indices, RLE booleans.
enum { K_DEF = 0, K_REP = 1, K_DICT = 2, K_BOOL = 3, K_N = 4 };
constexpr int SS_DICT = 2;  // device/pqg_runs.hpp StreamSel: dictionary indices

// Tile lists the kernels over one kind of page take (host-built, uploaded with the page table):
// general-path dictionary tiles by value size (1, 4, 8, 12) and all of them, byte-array
// dictionary tiles off the level path, byte-array copy tiles, RLE boolean tiles, PLAIN
// fixed-width pages (a page list) and PLAIN boolean tiles.
// TL_PSPEC: PLAIN pages of the chunks whose values are copied speculatively (ChunkWork::spec).
// TL_W4 / TL_W8: general-path dictionary tiles of 4- / 8-byte values whose dictionary has at most
// DW_MAXD entries (indices to a buffer, then the gather through LDS windows: k_dict_win).
// TL_BLEN: the large DELTA_LENGTH / DELTA_BYTE_ARRAY pages (a page list) whose length streams the
// multi-workgroup kernels decode (pqg_balen.hpp).
enum { TL_D1 = 0, TL_D4, TL_D8, TL_D12, TL_DALL, TL_BADICT, TL_BA, TL_BOOL, TL_PLAIN, TL_PBOOL, TL_PSPEC, TL_W4, TL_W8,
       TL_BLEN, TL_N };
constexpr uint32_t BL_MIN_VALUES = 65536;  // pqg_balen.hpp BL_MIN
#ifndef PQG_DWIN
#define PQG_DWIN 1  // (0: every general-path dictionary gather served from L2, for A/B runs)
#endif
constexpr uint32_t DW_MAXD = 65536;  // 16-bit indices

// What the host knows of one chunk of a decode until its results are delivered.
struct ChunkHost {
  pqg_output* out = nullptr;
  uint64_t total_levels = 0;  // the level count read_batch reports (column/reader.rs:259)
  int host_status = 0;        // what the host checks found before the launch
  int host_bad_page = -1;
  std::string host_msg;
};

// Two staging slots so consecutive async decodes never overwrite pinned memory that an
// in-flight H2D/D2H copy still reads (slot i is reused only after its last decode ended).
struct Slot {
  uint8_t* d_tab = nullptr;  // page table | chunk table | tile lists (one H2D copy)
  uint8_t* h_tab = nullptr;  // pinned staging
  size_t tab_cap = 0;
  ChunkWork* h_res = nullptr;  // pinned: the chunk table copied back after the decode
  size_t res_cap = 0;
  hipEvent_t ev[10] = {};  // 0-5 stage boundaries; 6-7 / 8-9 around the def-level path / values kernel
  hipEvent_t fork = nullptr, join = nullptr;  // the side stream's speculative PLAIN copy
  bool kl = false, kv = false;  // events 6-7 / 8-9 recorded by the last decode
  bool used = false;     // a decode was enqueued and its timings not yet harvested
  bool pending = false;  // a decode was enqueued and its results not yet delivered
  uint64_t seq = 0;      // issue order of that decode
  int call = 0;          // its index among the decodes since the last pqg_sync
  std::vector<ChunkHost> ch;  // per chunk of that decode
  // BYTE_ARRAY / FLBA scratch: per value source address, length, DELTA_BYTE_ARRAY prefix (slots
  // per chunk from ChunkWork::scr_base); per dictionary entry source and length (dscr_base)
  uint64_t* vsrc = nullptr;
  uint32_t* vlen = nullptr;
  uint32_t* vpre = nullptr;
  size_t vcap = 0;
  uint64_t* dsrc = nullptr;
  uint32_t* dlen = nullptr;
  size_t dcap = 0;
  uint64_t* tsum = nullptr;  // byte-array copy: per tile, bytes then start
  uint32_t* vaux = nullptr;  // DELTA_BYTE_ARRAY: per value, the previous smaller prefix length's value
  size_t vaux_cap = 0;
  uint32_t* dtile = nullptr;  // DELTA_BYTE_ARRAY: per tile, prefix-length minima and tile jumps
  size_t dtile_cap = 0;
  uint16_t* didx = nullptr;  // TL_W4 / TL_W8 tiles: RUN_TILE dictionary indices each
  size_t didx_cap = 0;
  uint8_t* blbuf = nullptr;  // TL_BLEN pages: per page, per tile and per block state (pqg_balen.hpp)
  size_t blcap = 0;
  // hybrid-stream expand tiles: tile -> page map and the index-pass tables per stream kind
  uint32_t* tile_page = nullptr;
  RunTables rt[K_N] = {};
  size_t tcap = 0;
  size_t pfcap = 0;      // pages the rt[].pflag arrays hold
  DeltaTables dt = {};   // DELTA_BINARY_PACKED tiled path
  size_t dt_tcap = 0, dt_pcap = 0;
  // level path (pqg_levels.hip): buffers of LevelTables per stream kind, grown on demand
  static constexpr int LV_BUFS = 14;  // wbase, wbase2, wfirst, rec, tab, win, sbase, bexit, seg, srec, spos, dense, ctr, bmp
  void* lvbuf[K_N][LV_BUFS] = {};
  size_t lvcap[K_N][LV_BUFS] = {};
  uint32_t* bail = nullptr;  // PQG_DIAG, PQG_DEBUG 512: LevelTables::bail of the def stream
  LevelTables lt(int k, uint32_t tstride) const {
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
    t.bmp = (uint16_t*)lvbuf[k][13];
    t.tstride = tstride;
    t.bail = k == K_DEF ? bail : nullptr;
    return t;
  }
};

struct pqg_ctx {
  int device = 0;
  Slot slot[2];
  int cur = 0;          // slot of the last decode
  hipStream_t stream = nullptr;
  bool timing = false;
  int overlap = 0;  // speculative PLAIN copy on the side stream (pqg_ctx_set_overlap): 0 off, 1 early, 2 late
  hipStream_t side = nullptr;  // lowest-priority stream of that copy
  uint64_t seq = 0;     // decodes issued
  int calls = 0;        // decodes issued since the last pqg_sync
  // first failure among decodes delivered at a slot's reuse, reported by the next pqg_sync
  int held_status = 0;
  int held_call = -1, held_chunk = -1, held_page = -1;
  std::string held_msg;
  double acc_ms[7] = {};
  uint64_t* dbgbuf = nullptr;  // diagnostics (PQG_DIAG builds)
  size_t dbg_cap = 0;
  uint32_t dbg_n = 0;
  uint64_t acc_n = 0;
  uint32_t values_kernel = 0;
  uint32_t paths = 0;  // PQG_PATH_* of the last decode
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

// Delivers the results of slot sl's finished decode into its chunks' output structs; returns the
// status of its first failing chunk (lowest index; per chunk the host checks' status when they
// rejected a page no later than the first failing one) and writes that chunk, its page and a
// message.
static int finish_slot(Slot& sl, int* chunk_out, int* page_out, std::string& msg) {
  int st0 = 0, chunk0 = -1, page0 = -1;
  for (size_t j = 0; j < sl.ch.size(); ++j) {
    const ChunkHost& h = sl.ch[j];
    const ChunkResult& r = sl.h_res[j].res;
    pqg_output* out = h.out;
    out->num_levels = h.total_levels;
    out->num_values = r.total_values;
    out->num_bytes = r.total_bytes;
    int st = 0, page = -1;
    if (r.bad != ~0ull) {
      page = (int)(r.bad >> 32);
      st = (int)(uint32_t)r.bad;
    }
    std::string m;
    if (h.host_status && (page < 0 || h.host_bad_page <= page)) {
      page = h.host_bad_page;
      st = h.host_status;
      m = h.host_msg;
    } else if (st) {
      char buf[160];
      snprintf(buf, sizeof(buf), "page %d: %s (reference: %s)", page, status_name(st),
               st == PQG_ERR_PANIC ? "panics" : st == PQG_ERR_HANG ? "loops forever" : "returns Err");
      m = buf;
    }
    if (st && !st0) {
      st0 = st;
      chunk0 = (int)j;
      page0 = page;
      msg = m;
    }
  }
  sl.pending = false;
  *chunk_out = chunk0;
  *page_out = page0;
  return st0;
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

static void free_run_tables(RunTables& r) {
  hipFree(r.ck);
  hipFree(r.runs);
  hipFree(r.nruns);
  hipFree(r.desc);
  hipFree(r.qcount);
  hipFree(r.pflag);
  hipFree(r.nfall);
  hipFree(r.hard);
  r = RunTables{};
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
    for (auto& ev : sl.ev) hipEventCreate(&ev);
    hipEventCreateWithFlags(&sl.fork, hipEventDisableTiming);
    hipEventCreateWithFlags(&sl.join, hipEventDisableTiming);
  }
  int least = 0, greatest = 0;
  hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (hipStreamCreateWithPriority(&ctx->side, hipStreamNonBlocking, least) != hipSuccess) {
    delete ctx;
    return PQG_ERR_HIP;
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
    hipFree(sl.d_tab);
    hipHostFree(sl.h_tab);
    hipHostFree(sl.h_res);
    hipFree(sl.vsrc);
    hipFree(sl.vlen);
    hipFree(sl.vpre);
    hipFree(sl.tsum);
    hipFree(sl.vaux);
    hipFree(sl.dtile);
    hipFree(sl.dsrc);
    hipFree(sl.dlen);
    hipFree(sl.didx);
    hipFree(sl.blbuf);
    hipFree(sl.tile_page);
    for (RunTables& t : sl.rt) free_run_tables(t);
    hipFree(sl.dt.page);
    hipFree(sl.dt.blocks);
    hipFree(sl.dt.agg);
    hipFree(sl.dt.inc);
    hipFree(sl.dt.flag);
    hipFree(sl.dt.nfall);
    for (int k = 0; k < K_N; ++k) {
      for (void* b : sl.lvbuf[k]) hipFree(b);
    }
    for (auto& ev : sl.ev) hipEventDestroy(ev);
    hipEventDestroy(sl.fork);
    hipEventDestroy(sl.join);
  }
  if (ctx->side) {
    hipStreamSynchronize(ctx->side);
    hipStreamDestroy(ctx->side);
  }
  hipFree(ctx->sp_tiles);
  hipFree(ctx->dbgbuf);
  delete ctx;
  return PQG_OK;
}

int pqg_ctx_set_timing(pqg_ctx* ctx, int enabled) {
  if (!ctx) return PQG_ERR_INVALID;
  ctx->timing = enabled != 0;
  return PQG_OK;
}

int pqg_ctx_set_overlap(pqg_ctx* ctx, int enabled) {
  if (!ctx) return PQG_ERR_INVALID;
  ctx->overlap = enabled < 0 ? 0 : enabled > 2 ? 2 : enabled;
  return PQG_OK;
}

const char* pqg_error_message(pqg_ctx* ctx) { return ctx ? ctx->msg.c_str() : "null ctx"; }

}  // extern "C"

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

// Argument checks of one chunk: a rejected call leaves the context (and decodes still in flight
// on it) untouched.
static int check_chunk(pqg_ctx* ctx, uint32_t j, const pqg_column* col, const pqg_page* pages, uint32_t npages,
                       const pqg_output* out) {
  if (!col || !out || (npages && !pages)) return set_err(ctx, PQG_ERR_INVALID, "chunk %u: null argument", j);
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
      if (pages[i].page_type == PQG_PAGE_DATA || pages[i].page_type == PQG_PAGE_DATA_V2) nlev += pages[i].num_values;
    if (!out->offsets || out->offsets_capacity < nlev + 1)
      return set_err(ctx, PQG_ERR_INVALID, "BYTE_ARRAY/FLBA output needs offsets[num_levels + 1]");
  }
  return PQG_OK;
}

// Grows a device buffer to at least `need` elements (+1/8 headroom).
static int grow(pqg_ctx* ctx, void** p, size_t* cap, size_t need, size_t elem, const char* what) {
  if (need <= *cap) return PQG_OK;
  hipFree(*p);
  *p = nullptr;
  *cap = 0;
  const size_t c = need + need / 8 + 1024;
  HIPCHK(hipMalloc(p, c * elem), what);
  *cap = c;
  return PQG_OK;
}

// The decode of a batch of column chunks (see the top of this file).
static int decode_batch(pqg_ctx* ctx, uint32_t nc, const pqg_column* cols, const uint8_t* blob, uint64_t blob_len,
                        const pqg_page* const* pages, const uint32_t* npages, pqg_output* outs, hipStream_t s) {
  if (!ctx || (nc && (!cols || !pages || !npages || !outs))) return PQG_ERR_INVALID;
  for (uint32_t j = 0; j < nc; ++j) {
    const int st = check_chunk(ctx, j, &cols[j], pages[j], npages[j], &outs[j]);
    if (st) return st;
  }
  HIPCHK(hipSetDevice(ctx->device), "hipSetDevice");
  ctx->stream = s;
  for (uint32_t j = 0; j < nc; ++j) outs[j].num_levels = outs[j].num_values = outs[j].num_bytes = 0;

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
      int chunk, page;
      std::string m;
      const int st = finish_slot(sl, &chunk, &page, m);
      if (st && !ctx->held_status) {
        ctx->held_status = st;
        ctx->held_call = sl.call;
        ctx->held_chunk = chunk;
        ctx->held_page = page;
        ctx->held_msg = m;
      }
    }
  }
  sl.kl = sl.kv = false;

  // ---- the batch's shape: pages, tiles, windows, per-chunk parameters and scratch slots
  uint32_t np = 0;
  for (uint32_t j = 0; j < nc; ++j) np += npages[j];
  sl.ch.assign(nc, ChunkHost{});
  std::vector<ChunkWork> cw(nc);
  std::vector<uint32_t> tl[TL_N];
  std::vector<PageWork> pw(np);
  uint32_t total_tiles = 0;
  uint32_t bl_maxtiles = 0;
  uint64_t nwin = 0, plain_max = 0, spec_max = 0, scr = 0, dscr = 0;
  uint32_t def_w = 0, rep_w = 0;  // bit masks of the level streams' widths
  bool any_def = false, any_rep = false, any_plain = false, any_pbool = false, any_ba = false, any_dba = false;
  bool any_badict = false, ba_lv = false, any_rbool = false, fixed_gen = false;
  uint32_t lv_es = 0, delta_es = 0;  // value sizes of the level-path dictionary chunks / DELTA chunks
  int nlvdict = 0;
#ifdef PQG_DIAG
  static const int dbg_env = getenv("PQG_DEBUG") ? atoi(getenv("PQG_DEBUG")) : 0;
#else
  const int dbg_env = 0;  // diagnostic kernel modes exist only in a PQG_DIAG build (make DIAG=1)
#endif
  uint32_t p0 = 0;
  for (uint32_t j = 0; j < nc; ++j) {
    const pqg_column* col = &cols[j];
    const pqg_page* pg = pages[j];
    const uint32_t n = npages[j];
    pqg_output* out = &outs[j];
    ChunkHost& h = sl.ch[j];
    ChunkWork& c = cw[j];
    memset(&c, 0, sizeof(c));
    h.out = out;
    const int t = col->physical_type;
    const bool is_ba = t == PQG_BYTE_ARRAY || t == PQG_FIXED_LEN_BYTE_ARRAY;
    const int es = is_ba ? 0 : value_size(t, col->type_length);
    int bad = -1, dict_page = -1;
    std::string why;
    const int vst = validate_pages(col, pg, n, &bad, &dict_page, why);
    if (vst) {
      h.host_status = vst;
      h.host_bad_page = bad;
      h.host_msg = why;
    }
    ColumnParams& cp = c.cp;
    cp.physical_type = t;
    cp.type_length = col->type_length;
    cp.max_def = col->max_def;
    cp.max_rep = col->max_rep;
    cp.def_bit_width = log2_ceil((uint64_t)(int64_t)col->max_def + 1);
    cp.rep_bit_width = log2_ceil((uint64_t)(int64_t)col->max_rep + 1);
    cp.want_def = col->max_def > 0 && out->def_levels;
    cp.want_rep = col->max_rep > 0 && out->rep_levels;
    // byte-array entries (address + length per value) take every index width; 4- / 8-byte values
    // up to 8 bits (wider: a large dictionary, gathered faster by the tiled expand)
#ifndef PQG_DICT_MAXW
#define PQG_DICT_MAXW 8u
#endif
    cp.dict_maxw = is_ba ? 16u : PQG_DICT_MAXW;
    cp.debug = dbg_env;
    c.def_out = out->def_levels;
    c.rep_out = out->rep_levels;
    c.val_out = (uint8_t*)out->values;
    c.off_out = out->offsets;
    c.val_cap = out->values_capacity;
    c.es = es;
    c.first_page = p0;
    c.npages = n;
    c.dict_page = dict_page < 0 ? -1 : (int32_t)(p0 + dict_page);
    c.res.bad = ~0ull;
    // configure_dictionary decodes the dictionary page whenever the reader reaches it, whatever
    // the data pages' encodings and whether values are read (column/reader.rs:463-481)
    c.dict_es = (dict_page >= 0 && !is_ba) ? es : 0;
    const bool vo = out->values != nullptr;
    bool enc[16] = {};
    uint64_t lev = 0;
    for (uint32_t i = 0; i < n; ++i) {
      PageWork& w = pw[p0 + i];
      memset(&w, 0, sizeof(w));
      w.base = pg[i].offset;
      w.nbytes = pg[i].nbytes;
      w.num_values = pg[i].num_values;
      w.page_type = pg[i].page_type;
      w.encoding = pg[i].encoding;
      if (w.page_type != PQG_PAGE_DICTIONARY && w.encoding == PQG_PLAIN_DICTIONARY)
        w.encoding = PQG_RLE_DICTIONARY;  // column/reader.rs:391-393
      w.def_encoding = pg[i].def_encoding;
      w.rep_encoding = pg[i].rep_encoding;
      w.def_len = pg[i].def_len;
      w.rep_len = pg[i].rep_len;
      w.level_out = lev;
      w.ltile0 = total_tiles;
      w.chunk = j;
      if (w.page_type == PQG_PAGE_DATA || w.page_type == PQG_PAGE_DATA_V2) {
        w.ntiles = (uint32_t)(((uint64_t)w.num_values + RUN_TILE - 1) / RUN_TILE);
        total_tiles += w.ntiles;
        lev += w.num_values;
        if (w.encoding >= 0 && w.encoding < 16) enc[w.encoding] = true;
        nwin += (w.nbytes + LV_WIN - 1) / LV_WIN;
      }
      if (vst && (int)i == bad) w.status = vst;
      if (vst && (int)i > bad) w.status = -1;  // never reached by the reference
    }
    // read_batch reports levels only for the streams it reads (column/reader.rs:259)
    h.total_levels = (cp.want_def || cp.want_rep) ? lev : 0;
    if (cp.want_def) {
      any_def = true;
      def_w |= 1u << cp.def_bit_width;
    }
    if (cp.want_rep) {
      any_rep = true;
      rep_w |= 1u << cp.rep_bit_width;
    }
    if (n && vo) {
      const uint32_t ndict = dict_page >= 0 ? pg[dict_page].num_values : 0u;
      auto list_tiles = [&](int which, int encoding) {  // tiles of this chunk's data pages (of an encoding)
        for (uint32_t i = 0; i < n; ++i) {
          const PageWork& w = pw[p0 + i];
          if (w.ntiles && (encoding < 0 || w.encoding == encoding))
            for (uint32_t k = 0; k < w.ntiles; ++k) tl[which].push_back(w.ltile0 + k);
        }
      };
      if (is_ba) {
        any_ba = true;
        c.scr_base = scr;
        scr += lev ? lev : 1;
        list_tiles(TL_BA, -1);
        if (enc[PQG_DELTA_BYTE_ARRAY]) any_dba = true;
        if (t == PQG_BYTE_ARRAY && (enc[PQG_DELTA_BYTE_ARRAY] || enc[PQG_DELTA_LENGTH_BYTE_ARRAY]))
          for (uint32_t i = 0; i < n; ++i) {
            const PageWork& w = pw[p0 + i];
            if ((w.encoding == PQG_DELTA_BYTE_ARRAY || w.encoding == PQG_DELTA_LENGTH_BYTE_ARRAY) &&
                w.num_values >= BL_MIN_VALUES && w.ntiles) {
              tl[TL_BLEN].push_back(p0 + i);
              if (w.ntiles > bl_maxtiles) bl_maxtiles = w.ntiles;
            }
          }
        if (enc[PQG_RLE_DICTIONARY]) {
          any_badict = true;
          c.dscr_base = dscr;
          dscr += ndict ? ndict : 1;
          if (dict_page >= 0 && ndict <= (1u << cp.dict_maxw)) {
            c.lvdict = 1;
            ba_lv = true;
          } else {  // (no dictionary page: the index pass reports the reference's panic)
            list_tiles(TL_BADICT, PQG_RLE_DICTIONARY);
          }
        }
      } else {
        if (enc[PQG_PLAIN]) {
          if (t == PQG_BOOLEAN) {
            any_pbool = true;
            list_tiles(TL_PBOOL, PQG_PLAIN);
          } else if (es > 0) {
            // values of a chunk whose data pages are all PLAIN, behind def levels: copied at the
            // offsets the value sections give, beside the level decode (checked by the scan)
            bool only_plain = true;
            for (int e = 0; e < 16; ++e) only_plain &= !enc[e] || e == PQG_PLAIN;
            c.spec = ctx->overlap && es >= 4 && cp.want_def && only_plain ? 1u : 0u;
            if (!c.spec) any_plain = true;
            for (uint32_t i = 0; i < n; ++i) {
              const PageWork& w = pw[p0 + i];
              if (w.ntiles && w.encoding == PQG_PLAIN) {
                tl[c.spec ? TL_PSPEC : TL_PLAIN].push_back(p0 + i);
                uint64_t& mx = c.spec ? spec_max : plain_max;
                if (w.nbytes > mx) mx = w.nbytes;
              }
            }
          }
        }
        if (enc[PQG_RLE_DICTIONARY]) {
          if ((es == 4 || es == 8) && dict_page >= 0 && ndict <= (1u << cp.dict_maxw)) {
            c.lvdict = 1;
            lv_es |= (uint32_t)es;
          } else {
            fixed_gen = true;
            const bool win = PQG_DWIN && (es == 4 || es == 8) && dict_page >= 0 && ndict <= DW_MAXD;
            list_tiles(win ? (es == 4 ? TL_W4 : TL_W8)
                           : es == 1 ? TL_D1 : es == 4 ? TL_D4 : es == 8 ? TL_D8 : TL_D12,
                       PQG_RLE_DICTIONARY);
            list_tiles(TL_DALL, PQG_RLE_DICTIONARY);
          }
        }
        if (enc[PQG_DELTA_BINARY_PACKED] && (t == PQG_INT32 || t == PQG_INT64)) delta_es |= (uint32_t)es;
        if (enc[PQG_RLE] && t == PQG_BOOLEAN) {
          any_rbool = true;
          list_tiles(TL_BOOL, PQG_RLE);
        }
      }
      if (c.lvdict) ++nlvdict;
    }
    p0 += n;
  }
#ifdef PQG_DIAG
  if (dbg_env & (16 | 32 | 64 | 128 | 256 | 512 | 1024 | 2048 | 4096 | 8192)) {
    size_t need = (size_t)(total_tiles * 4 > (uint64_t)np * 2 ? total_tiles * 4 : (uint64_t)np * 2) * 16;
    if (need < (size_t)np * 64) need = (size_t)np * 64;
    if (dbg_env & 128) need = (size_t)(nwin / LW_SEGW + np + 1) * 32;  // per level-stream segment
    if (dbg_env & 256) need = (size_t)2048 * 64 * 4 * 32;                 // per wave of k_lv_emit (grids <= 64 x)
    if (dbg_env & 1024) need = (size_t)2048 * 64 * 4 * 32;                // per wave of k_lv_emit_walk
    if (dbg_env & 2048) need = (size_t)2048 * 64 * 4 * 32;                // per wave of k_lv_win
    if (dbg_env & 4096) need = (size_t)(total_tiles / 8 + 64) * 64;       // per workgroup of k_dict_win
    if (dbg_env & 8192) need = (size_t)2 * 2048 * 64;                    // per workgroup of k_d1_tab / k_d1_emit
    if (dbg_env & 512) need = (size_t)np * 20 + 64;  // per page: its hand-back site, then the failing window
    if (need > ctx->dbg_cap) {
      hipFree(ctx->dbgbuf);
      ctx->dbgbuf = nullptr;
      HIPCHK(hipMalloc(&ctx->dbgbuf, need), "hipMalloc dbg");
      ctx->dbg_cap = need;
    }
    ctx->dbg_n = (dbg_env & 32) ? np : total_tiles * 4;
    sl.bail = nullptr;
    if (dbg_env & 512) {
      sl.bail = (uint32_t*)ctx->dbgbuf;
      HIPCHK(hipMemsetAsync(sl.bail, 0, (size_t)np * 20, s), "memset bail sites");
    }
    if (dbg_env & (1024 | 2048)) HIPCHK(hipMemsetAsync(ctx->dbgbuf, 0, (size_t)2048 * 64 * 64, s), "memset stamps");
    if (dbg_env & (4096 | 8192)) HIPCHK(hipMemsetAsync(ctx->dbgbuf, 0, need, s), "memset stamps");
    for (ChunkWork& c : cw) c.cp.dbgbuf = ctx->dbgbuf;
  }
#endif

  // ---- staging: page table | chunk table | tile lists, one H2D copy
  const size_t pw_bytes = ((size_t)np * sizeof(PageWork) + 63) & ~(size_t)63;
  const size_t cw_bytes = ((size_t)nc * sizeof(ChunkWork) + 63) & ~(size_t)63;
  size_t tl_off[TL_N], tl_total = 0;
  for (int k = 0; k < TL_N; ++k) {
    tl_off[k] = tl_total;
    tl_total += tl[k].size();
  }
  const size_t tab_bytes = pw_bytes + cw_bytes + tl_total * 4 + 64;
  if (tab_bytes > sl.tab_cap) {
    hipFree(sl.d_tab);
    hipHostFree(sl.h_tab);
    sl.d_tab = sl.h_tab = nullptr;
    sl.tab_cap = 0;
    const size_t cap = tab_bytes < (1u << 20) ? (1u << 20) : tab_bytes + tab_bytes / 4;
    HIPCHK(hipMalloc(&sl.d_tab, cap), "hipMalloc page table");
    HIPCHK(hipHostMalloc(&sl.h_tab, cap, hipHostMallocDefault), "hipHostMalloc page table");
    sl.tab_cap = cap;
  }
  if ((size_t)nc > sl.res_cap) {
    hipHostFree(sl.h_res);
    sl.h_res = nullptr;
    sl.res_cap = 0;
    const size_t cap = nc < 64 ? 64 : (size_t)nc * 2;
    HIPCHK(hipHostMalloc(&sl.h_res, cap * sizeof(ChunkWork), hipHostMallocDefault), "hipHostMalloc results");
    sl.res_cap = cap;
  }
  PageWork* d_pages = (PageWork*)sl.d_tab;
  ChunkWork* d_chunks = (ChunkWork*)(sl.d_tab + pw_bytes);
  const uint32_t* d_tl = (const uint32_t*)(sl.d_tab + pw_bytes + cw_bytes);
  const uint32_t* tlp[TL_N];
  uint32_t ntl[TL_N];
  for (int k = 0; k < TL_N; ++k) {
    tlp[k] = d_tl + tl_off[k];
    ntl[k] = (uint32_t)tl[k].size();
  }

  // ---- scratch, grown on demand
  const int ni = (int)np;
  if (any_ba) {
    int st;
    const size_t vcap0 = sl.vcap;
    if ((st = grow(ctx, (void**)&sl.vsrc, &sl.vcap, scr, 8, "hipMalloc vsrc"))) return st;
    if (sl.vcap != vcap0) {  // vlen / vpre share vsrc's capacity
      hipFree(sl.vlen);
      hipFree(sl.vpre);
      sl.vlen = sl.vpre = nullptr;
      HIPCHK(hipMalloc(&sl.vlen, sl.vcap * 4), "hipMalloc vlen");
      HIPCHK(hipMalloc(&sl.vpre, sl.vcap * 4), "hipMalloc vpre");
    }
    const size_t dcap0 = sl.dcap;
    if ((st = grow(ctx, (void**)&sl.dsrc, &sl.dcap, dscr ? dscr : 1, 8, "hipMalloc dsrc"))) return st;
    if (sl.dcap != dcap0) {
      hipFree(sl.dlen);
      sl.dlen = nullptr;
      HIPCHK(hipMalloc(&sl.dlen, sl.dcap * 4), "hipMalloc dlen");
    }
  }
  if (!tl[TL_BLEN].empty()) {  // BlPage per page, BlTile per tile, two streams' block offsets per tile
    int st;
    const size_t need = (size_t)np * 64 + ((size_t)total_tiles + 1) * (48 + 2 * 32 * 4);
    if ((st = grow(ctx, (void**)&sl.blbuf, &sl.blcap, need, 1, "hipMalloc byte-array length state"))) return st;
  }
  if (any_dba) {
    int st;
    if ((st = grow(ctx, (void**)&sl.vaux, &sl.vaux_cap, scr, 4, "hipMalloc vaux"))) return st;
    if ((st = grow(ctx, (void**)&sl.dtile, &sl.dtile_cap, ((size_t)total_tiles + 1) * 66, 4, "hipMalloc dtile")))
      return st;
  }
  if (ntl[TL_W4] + ntl[TL_W8]) {
    const int st = grow(ctx, (void**)&sl.didx, &sl.didx_cap, (size_t)(ntl[TL_W4] + ntl[TL_W8]) * RUN_TILE, 2,
                        "hipMalloc dictionary indices");
    if (st) return st;
  }
  // expand-tile bookkeeping (tile -> page, byte-array tile sums, index tables per stream kind)
  if ((size_t)total_tiles + 1 > sl.tcap) {
    hipFree(sl.tile_page);
    hipFree(sl.tsum);
    sl.tile_page = nullptr;
    sl.tsum = nullptr;
    for (RunTables& r : sl.rt) free_run_tables(r);
    sl.tcap = 0;
    sl.pfcap = 0;
    const size_t cap = (size_t)total_tiles + 1024;
    HIPCHK(hipMalloc(&sl.tile_page, cap * sizeof(uint32_t)), "hipMalloc tile_page");
    HIPCHK(hipMalloc(&sl.tsum, cap * sizeof(uint64_t)), "hipMalloc byte-array tiles");
    sl.tcap = cap;
  }
  auto tables = [&](int k) -> hipError_t {  // run tables per stream kind, on first use
    RunTables& r = sl.rt[k];
    if (r.ck) return hipSuccess;
    hipError_t e = hipMalloc(&r.ck, (sl.tcap + 1) * sizeof(RunCkpt));
    if (e == hipSuccess) e = hipMalloc(&r.runs, sl.tcap * RUN_CAPT * sizeof(uint2));
    if (e == hipSuccess) e = hipMalloc(&r.nruns, sl.tcap * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&r.desc, sl.tcap * 4 * sizeof(QDesc));
    if (e == hipSuccess) e = hipMalloc(&r.qcount, sl.tcap * 4 * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&r.nfall, sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&r.hard, (sl.tcap + 2) * sizeof(uint32_t));
    return e;
  };
  if ((size_t)np > sl.pfcap) {  // page-pass flags, sized by pages
    const size_t pc = (size_t)np < 4096 ? 4096 : (size_t)np * 2;
    for (RunTables& r : sl.rt) {
      hipFree(r.pflag);
      r.pflag = nullptr;
    }
    sl.pfcap = 0;
    for (RunTables& r : sl.rt) HIPCHK(hipMalloc(&r.pflag, pc * sizeof(uint32_t)), "hipMalloc page flags");
    sl.pfcap = pc;
  }
  const bool dict_any = nlvdict > 0 || fixed_gen || any_badict;
  const bool need_tables[K_N] = {any_def, any_rep, dict_any, any_rbool};
  for (int k = 0; k < K_N; ++k)
    if (need_tables[k]) HIPCHK(tables(k), "hipMalloc run tables");
  // level path buffers per stream kind, grown on demand; window tables of a uniform row stride
  uint32_t tstride[K_N] = {64, 64, 64, 64};
  for (int w = 1; w <= 31; ++w) {
    if ((def_w >> w) & 1u) tstride[K_DEF] = lv_ent((uint32_t)w) > tstride[K_DEF] ? lv_ent((uint32_t)w) : tstride[K_DEF];
    if ((rep_w >> w) & 1u) tstride[K_REP] = lv_ent((uint32_t)w) > tstride[K_REP] ? lv_ent((uint32_t)w) : tstride[K_REP];
  }
  const bool need_lv[K_N] = {any_def, any_rep, nlvdict > 0, any_rbool};
  for (int k = 0; k < K_N; ++k) {
    if (!need_lv[k]) continue;
    int st;
    const size_t ent = tstride[k];
    const size_t nseg = nwin / LW_SEGW + np + 1;  // segments, upper bound
    const size_t need[Slot::LV_BUFS] = {(size_t)np + 1, (size_t)np + 1, nwin + np + 1,
                                        64 * (nwin + 2 * (size_t)np) + 1, (nwin + 1) * ent, nwin + 1,
                                        (size_t)np + 1, nseg, nseg, nseg * LW_SCAP, nseg * LW_SCAP,
                                        (size_t)np + 1, 16, (nwin + 1) * 64};
    const size_t elem[Slot::LV_BUFS] = {4, 4, 4, sizeof(uint2), sizeof(uint2), sizeof(uint2),
                                        4, 4, sizeof(LvSeg), sizeof(uint2), 4, 4, 4, 2};
    const bool fresh_ctr = sl.lvbuf[k][12] == nullptr;
    for (int bb = 0; bb < Slot::LV_BUFS; ++bb)
      if ((st = grow(ctx, &sl.lvbuf[k][bb], &sl.lvcap[k][bb], need[bb], elem[bb], "hipMalloc level tables"))) return st;
    // the tickets start at zero once; every launch using them leaves them at zero
    if (fresh_ctr) HIPCHK(hipMemsetAsync(sl.lvbuf[k][12], 0, sl.lvcap[k][12] * 4, s), "memset level tickets");
  }
  // Hybrid-stream counters and flags, set by k_prepare (no memset launches): the level path (def,
  // rep, dictionary indices, RLE booleans) sets every page's flag and counts the streams it hands
  // back; the general dictionary path's kernels run when it has listed tiles.
  PrepInit ini{};
  int nw_ = 0, nz = 0;
  for (int k = 0; k < K_N; ++k) {
    if (!need_tables[k]) continue;
    ini.word[nw_] = sl.rt[k].nfall;
    ini.val[nw_++] = (k == K_DICT && (ntl[TL_DALL] || ntl[TL_BADICT])) ? 1u : 0u;
    if (!need_lv[k]) ini.pzero[nz++] = sl.rt[k].pflag;
  }
  if (delta_es) {  // DELTA_BINARY_PACKED tables (tiled fallback path), grown on demand
    if (total_tiles > sl.dt_tcap || (size_t)np > sl.dt_pcap) {
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
      sl.dt_tcap = tc;
      sl.dt_pcap = pc;
    }
    ini.word[nw_] = sl.dt.nfall;
    ini.val[nw_++] = 0u;
    sl.dt.dbg = (dbg_env & 32) ? ctx->dbgbuf : nullptr;

  }
  ini.dense_def = need_lv[K_DEF] ? sl.lt(K_DEF, 0).dense : nullptr;
  ini.dense_rep = need_lv[K_REP] ? sl.lt(K_REP, 0).dense : nullptr;
  ini.dense_zero = need_lv[K_DICT] ? sl.lt(K_DICT, 0).dense : nullptr;

  // ---- upload the tables
  memcpy(sl.h_tab, pw.data(), (size_t)np * sizeof(PageWork));
  memcpy(sl.h_tab + pw_bytes, cw.data(), (size_t)nc * sizeof(ChunkWork));
  for (int k = 0; k < TL_N; ++k)
    if (!tl[k].empty()) memcpy(sl.h_tab + pw_bytes + cw_bytes + tl_off[k] * 4, tl[k].data(), tl[k].size() * 4);
  HIPCHK(hipMemcpyAsync(sl.d_tab, sl.h_tab, pw_bytes + cw_bytes + tl_total * 4, hipMemcpyHostToDevice, s), "H2D pages");

  // ---- kernels
  const uint8_t* b = blob;
  hipEvent_t* ev = sl.ev;
  if (ctx->timing) hipEventRecord(ev[0], s);
  if (np) HIPCHK(pqg_launch_prepare(b, blob_len, d_pages, ni, d_chunks, sl.tile_page, ini, s), "prepare");
  const bool spec = np && ntl[TL_PSPEC];
  // fork: the speculative PLAIN copy on the side stream, beside everything below (overlap 1:
  // right after k_prepare, one workgroup per page; 2: after the def levels' front end, beside
  // their emit, a full grid)
  auto fork_spec = [&](uint32_t gx) -> int {
    HIPCHK(hipStreamWaitEvent(ctx->side, sl.fork, 0), "stream wait");
    HIPCHK(pqg_launch_plain_spec(b, blob_len, d_pages, ni, d_chunks, tlp[TL_PSPEC], ntl[TL_PSPEC], gx, ctx->side),
           "speculative plain");
    HIPCHK(hipEventRecord(sl.join, ctx->side), "event");
    return PQG_OK;
  };
  const bool late_fork = spec && ctx->overlap == 2 && any_def;
  if (spec && !late_fork) {
    HIPCHK(hipEventRecord(sl.fork, s), "event");
    if (const int e = fork_spec(1u)) return e;
  }
  if (ctx->timing) hipEventRecord(ev[1], s);
  // the value-offset scan runs in the def stream's last kernel when no rep stream follows it
  const bool fused_scan = np && any_def && !any_rep;
  if (np && any_def) {
    HIPCHK(pqg_launch_levels(b, blob_len, d_pages, ni, d_chunks, 0, def_w, sl.tile_page, sl.rt[K_DEF],
                             sl.lt(K_DEF, tstride[K_DEF]), s, ctx->timing ? &ev[6] : nullptr, fused_scan ? 1 : 0,
                             late_fork ? sl.fork : nullptr),
           "def levels");
    if (late_fork) {
      const uint64_t gx = (spec_max + 64ull * 256ull - 1) / (64ull * 256ull) + 1;  // 4 x 16 bytes per lane
      if (const int e = fork_spec((uint32_t)(gx > 4096 ? 4096 : gx))) return e;
    }
    sl.kl = ctx->timing;
  }
  if (np && any_rep)
    HIPCHK(pqg_launch_levels(b, blob_len, d_pages, ni, d_chunks, 1, rep_w, sl.tile_page, sl.rt[K_REP],
                             sl.lt(K_REP, tstride[K_REP]), s, nullptr, 0, nullptr),
           "rep levels");
  if (ctx->timing) hipEventRecord(ev[2], s);
  if (np && !fused_scan) HIPCHK(pqg_launch_scan(d_pages, ni, d_chunks, s), "scan");
  if (ctx->timing) hipEventRecord(ev[3], s);
  ctx->values_kernel = 0;
  ctx->paths = 0;
  if (np) {
    const RunTables& rd = sl.rt[K_DICT];
    if (any_badict)
      HIPCHK(pqg_launch_ba_dict_prep(b, blob_len, d_pages, d_chunks, (int)nc, sl.dsrc, sl.dlen, s),
             "byte-array dictionary");
    if (nlvdict) ctx->paths |= PQG_PATH_DICT_LEVEL;
    if (ntl[TL_W4] + ntl[TL_W8]) ctx->paths |= PQG_PATH_DICT_WINDOW;
    if (ntl[TL_D1] + ntl[TL_D4] + ntl[TL_D8] + ntl[TL_D12]) ctx->paths |= PQG_PATH_DICT_TILES;
    if (any_ba) ctx->paths |= PQG_PATH_BYTES | (any_dba ? PQG_PATH_DELTA_BYTES : 0u);
    if (any_plain) ctx->paths |= PQG_PATH_PLAIN;
    if (delta_es) ctx->paths |= PQG_PATH_DELTA;
    if (any_rbool) ctx->paths |= PQG_PATH_RLE_BOOL;
    if (nlvdict)  // every dictionary chunk the level path takes, fixed-width and byte-array, in one pass
      HIPCHK(pqg_launch_lv(b, blob_len, d_pages, ni, d_chunks, SS_DICT, 0u, sl.dsrc, sl.dlen, sl.vsrc, sl.vlen, rd,
                           sl.lt(K_DICT, 64), s),
             "dictionary indices");
    if (ntl[TL_DALL] || ntl[TL_BADICT])  // the general path's index pass, both kinds together
      HIPCHK(pqg_launch_run_index(b, blob_len, d_pages, ni, d_chunks, SS_DICT, rd, s), "dictionary index pass");
    if (lv_es || fixed_gen) {
      ctx->values_kernel = PQG_RLE_DICTIONARY;
      const uint32_t* dl[4] = {tlp[TL_D1], tlp[TL_D4], tlp[TL_D8], tlp[TL_D12]};
      const uint32_t dn[4] = {ntl[TL_D1], ntl[TL_D4], ntl[TL_D8], ntl[TL_D12]};
      const uint32_t* wl[2] = {tlp[TL_W4], tlp[TL_W8]};
      const uint32_t wn[2] = {ntl[TL_W4], ntl[TL_W8]};
      HIPCHK(pqg_launch_dict(b, blob_len, d_pages, ni, d_chunks, sl.tile_page, lv_es, dl, dn, tlp[TL_DALL],
                             ntl[TL_DALL], wl, wn, sl.didx, rd, s, ctx->timing ? &ev[8] : nullptr),
             "dict");
      sl.kv = ctx->timing;
    }
    if (any_badict)
      HIPCHK(pqg_launch_badict_general(b, blob_len, d_pages, ni, d_chunks, sl.tile_page, tlp[TL_BADICT],
                                       ntl[TL_BADICT], rd, sl.dsrc, sl.dlen, sl.vsrc, sl.vlen, ba_lv ? 1 : 0, s),
             "byte-array dictionary indices");
    if (any_ba) {
      if (!ctx->values_kernel) ctx->values_kernel = any_dba ? PQG_DELTA_BYTE_ARRAY : PQG_PLAIN;
      HIPCHK(pqg_launch_bytes(b, blob_len, d_pages, ni, d_chunks, sl.tile_page, tlp[TL_BA], ntl[TL_BA], any_dba, ba_lv,
                              sl.vsrc, sl.vlen, sl.vpre, sl.dsrc, sl.dlen, sl.tsum, sl.vaux, sl.dtile, tlp[TL_BLEN],
                              ntl[TL_BLEN], bl_maxtiles, sl.blbuf, total_tiles, s),
             "byte arrays");
    }
    if (any_plain || any_pbool) {
      if (any_plain) ctx->values_kernel = PQG_PLAIN;
      if (ctx->timing && any_plain) hipEventRecord(ev[8], s);
      HIPCHK(pqg_launch_plain(b, blob_len, d_pages, d_chunks, sl.tile_page, tlp[TL_PLAIN], ntl[TL_PLAIN], plain_max,
                              tlp[TL_PBOOL], ntl[TL_PBOOL], s),
             "plain");
      if (ctx->timing && any_plain) hipEventRecord(ev[9], s);
      sl.kv = ctx->timing && any_plain;
    }
    if (delta_es) {
      ctx->values_kernel = PQG_DELTA_BINARY_PACKED;
      HIPCHK(pqg_launch_delta_tiled(b, blob_len, d_pages, ni, d_chunks, total_tiles, sl.tile_page, sl.dt, delta_es, s,
                                    ctx->timing ? &ev[8] : nullptr),
             "delta");
      sl.kv = ctx->timing;
    }
    if (any_rbool) {
      if (!ctx->values_kernel) ctx->values_kernel = PQG_RLE;
      HIPCHK(pqg_launch_rle_bool(b, blob_len, d_pages, ni, d_chunks, sl.tile_page, tlp[TL_BOOL], ntl[TL_BOOL],
                                 sl.rt[K_BOOL], sl.lt(K_BOOL, 64), s),
             "rle bool");
    }
  }
  if (spec) {  // join, then the chunks the offset scan flagged copied again
    HIPCHK(hipStreamWaitEvent(s, sl.join, 0), "stream wait");
    HIPCHK(pqg_launch_plain_fix(b, blob_len, d_pages, d_chunks, tlp[TL_PSPEC], ntl[TL_PSPEC], s), "plain fix-up");
  }
  if (ctx->timing) hipEventRecord(ev[4], s);
  if (nc)
    HIPCHK(hipMemcpyAsync(sl.h_res, d_chunks, (size_t)nc * sizeof(ChunkWork), hipMemcpyDeviceToHost, s),
           "D2H results");
  HIPCHK(hipEventRecord(ev[5], s), "event");
  sl.used = true;
  sl.pending = true;
  sl.seq = ++ctx->seq;
  sl.call = ctx->calls++;
  return PQG_OK;
}

extern "C" {

int pqg_decode_chunk(pqg_ctx* ctx, const pqg_column* col, const uint8_t* blob, uint64_t blob_len,
                     const pqg_page* pages, uint32_t npages, pqg_output* out, void* stream) {
  if (!ctx || !col || !out || (npages && !pages)) return PQG_ERR_INVALID;
  return decode_batch(ctx, 1, col, blob, blob_len, &pages, &npages, out, (hipStream_t)stream);
}

int pqg_decode_chunks(pqg_ctx* ctx, uint32_t nchunks, const pqg_column* cols, const uint8_t* blob, uint64_t blob_len,
                      const pqg_page* const* pages, const uint32_t* npages, pqg_output* outs, void* stream) {
  return decode_batch(ctx, nchunks, cols, blob, blob_len, pages, npages, outs, (hipStream_t)stream);
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

int pqg_sync_detail(pqg_ctx* ctx, int* bad_call, int* bad_chunk, int* bad_page) {
  if (!ctx) return PQG_ERR_INVALID;
  if (bad_call) *bad_call = -1;
  if (bad_chunk) *bad_chunk = -1;
  if (bad_page) *bad_page = -1;
  Slot* order[2] = {&ctx->slot[ctx->cur ^ 1], &ctx->slot[ctx->cur]};
  if (order[0]->pending && order[1]->pending && order[0]->seq > order[1]->seq) std::swap(order[0], order[1]);
  if (!order[0]->pending && !order[1]->pending && !ctx->held_status) {
    ctx->calls = 0;
    return set_err(ctx, PQG_ERR_INVALID, "no decode pending");
  }
  // every pending decode is delivered, in issue order; the first failure is reported
  int st = ctx->held_status, call = ctx->held_call, chunk = ctx->held_chunk, page = ctx->held_page;
  std::string msg = ctx->held_msg;
  ctx->held_status = 0;
  ctx->held_call = ctx->held_chunk = ctx->held_page = -1;
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
    int ch, pg;
    std::string m;
    const int c = sl->call;
    const int s2 = finish_slot(*sl, &ch, &pg, m);
    if (s2 && !st) {
      st = s2;
      call = c;
      chunk = ch;
      page = pg;
      msg = m;
    }
  }
  ctx->calls = 0;
  if (herr != hipSuccess) return hip_fail(ctx, herr, "hipEventSynchronize");
  ctx->msg = msg;
  if (st) {
    if (bad_call) *bad_call = call;
    if (bad_chunk) *bad_chunk = chunk;
    if (bad_page) *bad_page = page;
  }
  return st;
}

int pqg_sync(pqg_ctx* ctx, int* first_bad_page) { return pqg_sync_detail(ctx, nullptr, nullptr, first_bad_page); }

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

int pqg_ctx_last_paths(pqg_ctx* ctx, uint32_t* mask) {
  if (!ctx || !mask) return PQG_ERR_INVALID;
  *mask = ctx->paths;
  return PQG_OK;
}

// Diagnostics: raw copy of the debug buffer (PQG_DIAG builds; u64 words).
int pqg_debug_read(pqg_ctx* ctx, uint64_t* out, size_t n) {
  if (!ctx || !ctx->dbgbuf || !out || n * 8 > ctx->dbg_cap) return PQG_ERR_INVALID;
  return hipMemcpy(out, ctx->dbgbuf, n * 8, hipMemcpyDeviceToHost) == hipSuccess ? PQG_OK : PQG_ERR_HIP;
}

// Diagnostics: average per-wave phase cycles of the last decode (PQG_DIAG builds).
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
