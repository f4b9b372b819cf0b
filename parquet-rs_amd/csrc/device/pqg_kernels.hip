// pqg_kernels.hip — CDNA4 (gfx950) kernels for the parquet-rs page-decode hot path.
//
//   k_prepare        page layout: level streams + value section per page
//                    (column/reader.rs:269-380, levels.rs:191-233)
//   k_run_index, k_tile_desc, k_texpand_*  the general RLE/bit-packing hybrid decoder
//                    (rle.rs:398-487, levels.rs:249-271): dictionary indices, and the level /
//                    boolean streams the level path hands back
//   k_scan_values    dense value offsets per page (column/reader.rs:252-253)
//   k_texpand_dict   RLE_DICTIONARY indices -> dictionary gather (rle.rs:437-487,
//                    decoding.rs:256-315)
//   k_plain_copy     PLAIN fixed-width values (decoding.rs:138-186, 228-247)
//   k_plain_bool     PLAIN booleans (decoding.rs:188-204)
//
// All work is integer/byte movement bound by HBM: no MFMA. The general RLE/bit-packing hybrid
// decoder (index pass + grid-wide expand pass) is in pqg_runs.hpp / pqg_texpand.hpp; level
// streams and RLE booleans take the fast path of pqg_levels.hip first.
#include "pqg_texpand.hpp"

namespace pqg {



// ------------------------------------------------------------------------------ prepare

__device__ inline uint32_t rd_u32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__device__ inline int type_size(int t, int tl) {
  switch (t) {
    case T_BOOLEAN: return 1;
    case T_INT32: return 4;
    case T_INT64: return 8;
    case T_INT96: return 12;
    case T_FLOAT: return 4;
    case T_DOUBLE: return 8;
    case T_FLBA: return tl;
    default: return 0;
  }
}

// One v1 level stream (levels.rs:191-211). `start` is the BufferPtr start of the slice
// within the page; returns bytes consumed or -1 (panic).
__device__ inline int64_t v1_level_stream(const uint8_t* page, uint32_t nbytes, uint32_t start,
                                          int enc, int bw, uint32_t nvals, uint32_t& off,
                                          uint32_t& len, uint8_t& kind) {
  uint32_t slice_len = nbytes - start;
  if (enc == E_RLE) {
    if (slice_len < 4) return -1;
    int32_t sz = (int32_t)rd_u32(page + start);
    if (sz < 0 || 4ull + (uint64_t)(uint32_t)sz > slice_len) return -1;
    off = start + 4;
    len = (uint32_t)sz;
    kind = LK_RLE;
    return 4 + (int64_t)sz;
  }
  if (enc == E_BIT_PACKED) {
    uint64_t num_bytes = ((uint64_t)nvals * (uint64_t)bw + 7) / 8;
    uint32_t data_size = (uint32_t)(num_bytes < slice_len ? num_bytes : slice_len);
    // data.range(data.start(), data_size): the start is applied twice
    if ((uint64_t)start + data_size > slice_len) return -1;
    off = start + start;
    len = data_size;
    kind = LK_BIT_PACKED;
    return data_size;
  }
  return -1;  // LevelDecoder::v1 panics on other encodings (levels.rs:170)
}

// Thread 0 of k_prepare: page p's layout (level streams, value section) into pages[p] and out.
__device__ inline void prepare_page(const uint8_t* __restrict__ blob, uint64_t blob_len, PageWork* __restrict__ pages,
                                    int p, const ColumnParams& cp, ChunkResult* res, const PrepInit& ini,
                                    PageWork& out) {
  PageWork pw = pages[p];
  const int32_t host_status = pw.status;  // set by the host for pages the reference rejects
  pw.rep_kind = pw.def_kind = LK_NONE;
  pw.rep_off = pw.rep_bytes = pw.def_off = pw.def_bytes = 0;
  pw.nonnull = 0;
  pw.nbytes_out = 0;
  int32_t err = 0;
  if (host_status) {
    pages[p].nonnull = 0;
    out = pw;  // (status set: not probed)
    return;
  }
  if (pw.base + pw.nbytes > blob_len || pw.nbytes > 0x7FFFFFF0u) err = ST_INVALID_ARG;
  const uint8_t* page = blob + pw.base;
  if (!err && pw.page_type == P_DATA) {
    uint32_t start = 0;
    if (cp.max_rep > 0) {
      int64_t tb = v1_level_stream(page, pw.nbytes, start, pw.rep_encoding, cp.rep_bit_width,
                                   pw.num_values, pw.rep_off, pw.rep_bytes, pw.rep_kind);
      if (tb < 0) err = ST_PANIC;
      else start += (uint32_t)tb;
    }
    if (!err && cp.max_def > 0) {
      int64_t tb = v1_level_stream(page, pw.nbytes, start, pw.def_encoding, cp.def_bit_width,
                                   pw.num_values, pw.def_off, pw.def_bytes, pw.def_kind);
      if (tb < 0) err = ST_PANIC;
      else start += (uint32_t)tb;
    }
    pw.val_off = start;
    pw.val_bytes = pw.nbytes - start;
  } else if (!err && pw.page_type == P_DATA_V2) {
    uint32_t off = 0;
    if (cp.max_rep > 0) {  // set_data_range(rep_levels_byte_len), column/reader.rs:341-351
      if ((uint64_t)pw.rep_len > pw.nbytes) err = ST_PANIC;
      pw.rep_off = 0;
      pw.rep_bytes = pw.rep_len;
      pw.rep_kind = LK_RLE;
      off += pw.rep_len;
    }
    if (!err && cp.max_def > 0) {
      if ((uint64_t)off + pw.def_len > pw.nbytes) err = ST_PANIC;
      pw.def_off = off;
      pw.def_bytes = pw.def_len;
      pw.def_kind = LK_RLE;
      off += pw.def_len;
    }
    if (!err && off > pw.nbytes) err = ST_PANIC;
    pw.val_off = off;
    pw.val_bytes = err ? 0 : pw.nbytes - off;
  } else if (!err && pw.page_type == P_DICTIONARY) {
    pw.val_off = 0;
    pw.val_bytes = pw.nbytes;
  }
  // Values each page must yield: def == max_def count when levels are read (filled by
  // k_rle_levels), else the page's level count (column/reader.rs:212-226).
  bool data = pw.page_type == P_DATA || pw.page_type == P_DATA_V2;
  if (data && !(cp.max_def > 0 && cp.want_def)) pw.nonnull = pw.num_values;
  if (!err && p == ini.dict_page && ini.dict_es > 0) {  // DictDecoder::set_dict (was k_dict_check)
    if (pw.encoding != E_PLAIN && pw.encoding != E_PLAIN_DICTIONARY) err = ST_NYI;
    else if ((uint64_t)pw.num_values * (uint64_t)ini.dict_es > pw.nbytes) err = ST_EOF;
  }
  pw.status = err;
  pages[p] = pw;
  out = pw;
  if (err) atomicMin((unsigned long long*)&res->bad, ((unsigned long long)(uint32_t)p << 32) | (uint32_t)err);
}

// One wave per page: the lanes fill the page's tile -> page entries (a dictionary column's
// single data page has thousands), lane 0 the rest.
__global__ void __launch_bounds__(64) k_prepare(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                PageWork* __restrict__ pages, int npages, ColumnParams cp,
                                                uint32_t* __restrict__ tile_page, ChunkResult* res, PrepInit ini) {
  const int p = blockIdx.x;
  if (p >= npages) return;
  {
    const uint32_t t0 = pages[p].ltile0, nt = pages[p].ntiles;
    for (uint32_t k = threadIdx.x; k < nt; k += 64) tile_page[t0 + k] = (uint32_t)p;
  }
  __shared__ PageWork pw_s;
  if (threadIdx.x == 0) {
    prepare_page(blob, blob_len, pages, p, cp, res, ini, pw_s);
    if (p == 0)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (ini.word[i]) *ini.word[i] = ini.val[i];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (ini.pzero[i]) ini.pzero[i][p] = 0;
    if (ini.dense_zero) ini.dense_zero[p] = 0;
  }
  __syncthreads();
  // density probes of the level streams just located (wave-uniform from here)
  for (int k = 0; k < 2; ++k) {
    uint32_t* dn = k == 0 ? ini.dense_def : ini.dense_rep;
    if (!dn) continue;
    const PageWork& pw = pw_s;
    const bool data = pw.page_type == P_DATA || pw.page_type == P_DATA_V2;
    const int kind = k == 0 ? pw.def_kind : pw.rep_kind;
    const uint32_t slen = k == 0 ? pw.def_bytes : pw.rep_bytes;
    const uint32_t w = (uint32_t)(k == 0 ? cp.def_bit_width : cp.rep_bit_width);
    uint32_t dense = 0;
    if (data && pw.status == 0 && kind == LK_RLE && w >= 1 && w <= 16 && pw.num_values && slen >= PROBE_SPAN + 64u)
      dense = lv_probe_dense(blob, blob_len, pw.base + (k == 0 ? pw.def_off : pw.rep_off), w);
    if (threadIdx.x == 0) dn[p] = dense;
  }
}

// ------------------------------------------------------------------------------ hybrid streams

// Index pass over stream `sel` of every page (one wave per page), pqg_runs.hpp.
__global__ void __launch_bounds__(64) k_run_index(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                  PageWork* pages, ColumnParams cp, int sel,
                                                  int dict_page, RunTables rt, ChunkResult* res,
                                                  int bailed_only = 0) {
  __shared__ IndexSmem sm;
  const int p = blockIdx.x;
  if (bailed_only ? rt.pflag[p] != PF_BAIL : (*rt.nfall == 0 || pf_level_path(rt.pflag[p]))) return;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  Stream s;
  if (!get_stream(blob, pw, sel, cp, s)) return;
  if (sel == SS_DICT) {
    if (dict_page < 0) {  // "Decoder for dict should have been set"
      if (threadIdx.x == 0) report(pages, res, p, ST_PANIC);
      return;
    }
    if (pages[dict_page].status != 0) return;
  }
  const int32_t st = run_index(blob, blob_len, s, rt.ck + pw.ltile0,
                              rt.runs + (uint64_t)pw.ltile0 * RUN_CAPT, rt.nruns + pw.ltile0, sm,
                              (cp.debug & 32) && cp.dbgbuf ? cp.dbgbuf + 2 * p : nullptr);
  if (st && threadIdx.x == 0) report(pages, res, p, st);
}


// Quarter-tile descriptors of stream `sel` (one thread per quarter), read by the wave expand
// kernels.
__global__ void __launch_bounds__(WG) k_quarter_desc(const uint8_t* __restrict__ blob, const PageWork* pages,
                                                     const uint32_t* __restrict__ tile_page,
                                                     uint32_t ntiles, RunTables rt, ColumnParams cp,
                                                     int sel, int dict_page) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= ntiles * 4) return;
  rt.desc[i] = quarter_desc(blob, pages, tile_page, rt, cp, sel, dict_page, i >> 2, i & 3);
}

// Tile descriptors of stream `sel` (one thread per tile), read by the tile expand kernels.
__global__ void __launch_bounds__(WG) k_tile_desc(const uint8_t* __restrict__ blob, const PageWork* pages,
                                                  const uint32_t* __restrict__ tile_page,
                                                  uint32_t ntiles, RunTables rt, ColumnParams cp,
                                                  int sel, int dict_page) {
  const uint32_t t = blockIdx.x * WG + threadIdx.x;
  if (t >= ntiles || *rt.nfall == 0) return;
  rt.desc[t] = quarter_desc(blob, pages, tile_page, rt, cp, sel, dict_page, t, 0, RUN_TILE);
}

// Tile expand of a level stream (which: SS_DEF / SS_REP), pqg_texpand.hpp, persistent grid.
// Def levels also count the values read_batch will ask for: each wave writes its count of the
// tile to qcount[4t + wave] (k_page_counts sums them per page).
struct LevelsMaker {
  int16_t* out;
  int16_t maxl;
  bool count;
  uint32_t* qcount;
  __device__ TxLevels make(const QDesc& d) { return TxLevels{out + d.out, maxl, count, 0u}; }
  const uint32_t* pflag;
  __device__ void done(const QDesc& d, uint32_t t, TxLevels& em) {
    if (!count || (!d.qhi && pf_level_path(pflag[d.page]))) return;  // the level path wrote these counts
    const uint32_t nn = wave_sum_u32(em.nonnull);
    if ((threadIdx.x & 63) == 0) qcount[4 * t + (threadIdx.x >> 6)] = nn;
  }
};

// Level streams the level path handed back (PF_BAIL: malformed input, unusual header forms), one
// workgroup per page: wave 0 walks the page's header chain (run_index: every reference check,
// per-tile checkpoints and records), then the workgroup expands the page's tiles one after the
// other and sums the page's def levels == max_def (its non-null count). One launch in place of
// index pass + tile descriptors + tile expand + page counts: the level path leaves these streams
// to it only on unusual input, so the latency of a serial page matters less than three launches
// on every decode.
struct LevelsPageMaker {
  int16_t* out;
  int16_t maxl;
  bool count;
  uint32_t acc;  // this thread's outputs == maxl
  __device__ TxLevels make(const QDesc& d) { return TxLevels{out + d.out, maxl, count, 0u}; }
  __device__ void done(const QDesc&, uint32_t, TxLevels& em) { acc += em.nonnull; }
};

__device__ inline void lv_fallback_page(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                        PageWork* pages, const uint32_t* __restrict__ tile_page,
                                        ColumnParams cp, int sel, RunTables rt, ChunkResult* res,
                                        int16_t* __restrict__ out) {
  __shared__ IndexSmem ism;
  __shared__ TileSmem sm;
  __shared__ int32_t st_s;
  __shared__ uint64_t red[WG / 64];
  const int p = blockIdx.x;
  if (rt.pflag[p] != PF_BAIL) return;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  Stream s;
  if (!get_stream(blob, pw, sel, cp, s)) return;
  if (threadIdx.x < 64) {
    const int32_t st = run_index(blob, blob_len, s, rt.ck + pw.ltile0, rt.runs + (uint64_t)pw.ltile0 * RUN_CAPT,
                                 rt.nruns + pw.ltile0, ism);
    if (threadIdx.x == 0) {
      st_s = st;
      if (st) report(pages, res, p, st);
    }
  }
  __syncthreads();
  if (st_s) return;
  LevelsPageMaker mk{out, sel == SS_DEF ? cp.max_def : cp.max_rep, sel == SS_DEF, 0u};
  for (uint32_t t = pw.ltile0; t < pw.ltile0 + pw.ntiles; ++t) {
    if (threadIdx.x == 0) rt.desc[t] = quarter_desc(blob, pages, tile_page, rt, cp, sel, -1, t, 0, RUN_TILE);
    __syncthreads();  // (the descriptor is read by every thread of the workgroup)
    tile_one(blob, blob_len, rt.desc, t, rt.runs, sm, mk);
    __syncthreads();  // sm is refilled by the next tile
  }
  if (sel == SS_DEF) {
    const uint64_t nn = block_sum_u64(mk.acc, red);
    if (threadIdx.x == 0) pages[p].nonnull = nn;
  }
}

__device__ inline void scan_values(PageWork* pages, int npages, ChunkResult* res, int es, uint64_t cap_bytes);

// scan_es >= 0 (a def stream, no rep stream after it): the grid's last workgroup also runs
// k_scan_values (the non-null counts are final), one launch fewer per chunk.
__global__ void __launch_bounds__(WG) k_lv_fallback(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                    PageWork* pages, const uint32_t* __restrict__ tile_page,
                                                    ColumnParams cp, int sel, RunTables rt, ChunkResult* res,
                                                    int16_t* __restrict__ out, uint32_t* ctr, int scan_es,
                                                    uint64_t scan_cap) {
  lv_fallback_page(blob, blob_len, pages, tile_page, cp, sel, rt, res, out);
  if (scan_es >= 0 && last_workgroup(ctr)) scan_values(pages, (int)gridDim.x, res, scan_es, scan_cap);
}

// Tile expand of RLE_DICTIONARY indices with the dictionary gather.
template <int ES>
struct DictMaker {
  const uint8_t* dict;
  uint32_t ndict;
  bool aligned;
  uint8_t* out;
  PageWork* pages;
  ChunkResult* res;
  __device__ TxDict<ES> make(const QDesc& d) {
    return TxDict<ES>{dict, ndict, aligned, out + d.out * (uint64_t)ES, 0};
  }
  __device__ void done(const QDesc& d, uint32_t, TxDict<ES>& em) {
    const uint64_t bad = __ballot(em.err != 0);
    if (bad && (threadIdx.x & 63) == 0) report(pages, res, (int)d.page, ST_PANIC);
  }
};

#define PQG_TEXPAND_DICT(NAME, ATTR)                                                                  \
  template <int ES>                                                                                   \
  __global__ void ATTR __launch_bounds__(WG) NAME(const uint8_t* __restrict__ blob, uint64_t blob_len, \
                                                  uint32_t ntiles, PageWork* pages, RunTables rt,     \
                                                  int dict_page, uint8_t* __restrict__ out,           \
                                                  ChunkResult* res) {                                 \
    __shared__ TileSmem sm;                                                                         \
    if (dict_page < 0) return;                                                                      \
    const PageWork& dp = pages[dict_page];                                                          \
    DictMaker<ES> mk{blob + dp.base, dp.num_values, ((dp.base % (ES == 12 ? 4 : ES)) == 0),   \
                           out, pages, res};                                                        \
    if (*rt.nfall == 0) return;                                                                     \
    if (blockIdx.x < ntiles) tile_one(blob, blob_len, rt.desc, blockIdx.x, rt.runs, sm, mk);       \
  }
PQG_TEXPAND_DICT(k_texpand_dict, )

// Dictionary index streams the level path handed back, when they are expected to be rare (the
// dictionary's index width is within the level path's limit): one workgroup per page, index walk
// then the page's tiles with the gather, as k_lv_fallback does for levels.
template <int ES>
__global__ void __launch_bounds__(WG) k_dict_fallback(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                      PageWork* pages, const uint32_t* __restrict__ tile_page,
                                                      ColumnParams cp, int dict_page, RunTables rt,
                                                      uint8_t* __restrict__ out, ChunkResult* res) {
  __shared__ IndexSmem ism;
  __shared__ TileSmem sm;
  __shared__ int32_t st_s;
  const int p = blockIdx.x;
  if (rt.pflag[p] != PF_BAIL) return;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  Stream s;
  if (!get_stream(blob, pw, SS_DICT, cp, s)) return;
  if (dict_page < 0) {  // "Decoder for dict should have been set"
    if (threadIdx.x == 0) report(pages, res, p, ST_PANIC);
    return;
  }
  if (pages[dict_page].status != 0) return;
  if (threadIdx.x < 64) {
    const int32_t st = run_index(blob, blob_len, s, rt.ck + pw.ltile0, rt.runs + (uint64_t)pw.ltile0 * RUN_CAPT,
                                 rt.nruns + pw.ltile0, ism);
    if (threadIdx.x == 0) {
      st_s = st;
      if (st) report(pages, res, p, st);
    }
  }
  __syncthreads();
  if (st_s) return;
  const PageWork& dp = pages[dict_page];
  DictMaker<ES> mk{blob + dp.base, dp.num_values, ((dp.base % (ES == 12 ? 4 : ES)) == 0), out, pages, res};
  for (uint32_t t = pw.ltile0; t < pw.ltile0 + pw.ntiles; ++t) {
    if (threadIdx.x == 0) rt.desc[t] = quarter_desc(blob, pages, tile_page, rt, cp, SS_DICT, dict_page, t, 0, RUN_TILE);
    __syncthreads();
    tile_one(blob, blob_len, rt.desc, t, rt.runs, sm, mk);
    __syncthreads();
  }
}

// Tile expand of RLE booleans (data page v2 values).
struct BoolMaker {
  uint8_t* out;
  __device__ TxBool make(const QDesc& d) { return TxBool{out + d.out}; }
  __device__ void done(const QDesc&, uint32_t, TxBool&) {}
};

__global__ void __launch_bounds__(WG) k_texpand_bool(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                     uint32_t ntiles, RunTables rt, uint8_t* __restrict__ out) {
  __shared__ TileSmem sm;
  if (*rt.nfall == 0) return;
  BoolMaker mk{out};
  if (blockIdx.x < ntiles) tile_one(blob, blob_len, rt.desc, blockIdx.x, rt.runs, sm, mk);
}

static inline dim3 tx_grid(uint32_t ntiles) { return dim3(ntiles); }  // one tile per workgroup

// Per-page sum of the quarter-tile counts -> pages[p].nonnull (field 0) / nbytes_out (1).
__global__ void __launch_bounds__(WG) k_page_counts(PageWork* pages, const uint32_t* __restrict__ qcount,
                                                    const uint32_t* __restrict__ pflag,
                                                    const uint32_t* __restrict__ nfall, int field) {
  __shared__ uint64_t red[WG / 64];
  if (*nfall == 0) return;  // every stream done by the level path, which set the counts
  const int p = blockIdx.x;
  const PageWork& pw = pages[p];
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  if (pf_level_path(pflag[p])) return;
  const uint32_t q0 = pw.ltile0 * 4u, nq = pw.ntiles * 4u;
  uint64_t s = 0;
  for (uint32_t i = threadIdx.x; i < nq; i += WG) s += qcount[q0 + i];
  const uint64_t t = block_sum_u64(s, red);
  if (threadIdx.x == 0) {
    if (field == 0) pages[p].nonnull = t;
    else pages[p].nbytes_out = t;
  }
}

// ------------------------------------------------------------------------------ scan

// Exclusive scan of per-page value counts -> value_out (single workgroup).
__device__ inline void scan_values(PageWork* pages, int npages, ChunkResult* res, int es, uint64_t cap_bytes) {
  __shared__ uint64_t wsum[WG / 64];
  __shared__ uint64_t carry_s;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < npages; base += WG) {
    int p = base + threadIdx.x;
    uint64_t x = 0;
    if (p < npages) {
      int t = pages[p].page_type;
      if (t == P_DATA || t == P_DATA_V2) x = pages[p].nonnull;
    }
    // inclusive wave scan
    uint64_t s = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      uint64_t y = __shfl_up(s, off, 64);
      if ((threadIdx.x & 63) >= (unsigned)off) s += y;
    }
    if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = s;
    __syncthreads();
    uint64_t pre = carry_s;
    for (int k = 0; k < (int)(threadIdx.x >> 6); ++k) pre += wsum[k];
    if (p < npages) {
      pages[p].value_out = pre + s - x;
      if (es > 0 && x > 0 && (pre + s) * (uint64_t)es > cap_bytes && pages[p].status == 0)
        report(pages, res, p, ST_CAPACITY);
    }
    __syncthreads();
    if (threadIdx.x == WG - 1) carry_s = pre + s;
    __syncthreads();
  }
  if (threadIdx.x == 0) res->total_values = carry_s;
}

__global__ void __launch_bounds__(WG) k_scan_values(PageWork* pages, int npages, ChunkResult* res, int es,
                                                    uint64_t cap_bytes) {
  scan_values(pages, npages, res, es, cap_bytes);
}

// ------------------------------------------------------------------------------ dictionary

// ------------------------------------------------------------------------------ PLAIN

// Copies each page's `nonnull * es` value bytes to out + value_out * es. grid.y = page,
// grid.x strides 16-byte output chunks. Source alignment is arbitrary (the value section
// follows the level streams): dword loads + v_alignbyte; the destination is chunked on
// 16-byte boundaries of the output so stores are dwordx4 except at page edges.
__global__ void __launch_bounds__(WG) k_plain_copy(const uint8_t* __restrict__ blob,
                                                   uint64_t blob_len, PageWork* pages, int es,
                                                   int enc_filter, uint8_t* __restrict__ out,
                                                   ChunkResult* res) {
  const int p = blockIdx.y;
  const PageWork& pwr = pages[p];
  if (pwr.status != 0) return;
  if (pwr.page_type != P_DATA && pwr.page_type != P_DATA_V2) return;
  if (pwr.encoding != enc_filter) return;
  const uint64_t nbytes = pwr.nonnull * (uint64_t)es;
  if (nbytes > pwr.val_bytes) {  // eof_err!("Not enough bytes to decode")
    if (blockIdx.x == 0 && threadIdx.x == 0) report(pages, res, p, ST_EOF);
    return;
  }
  const uint64_t src = pwr.base + pwr.val_off;
  const uint64_t dst = pwr.value_out * (uint64_t)es;
  const uint64_t dend = dst + nbytes;
  const uint64_t c0 = dst & ~15ull;
  for (uint64_t c = c0 + ((uint64_t)blockIdx.x * WG + threadIdx.x) * 16ull; c < dend;
       c += (uint64_t)gridDim.x * WG * 16ull) {
    const uint64_t lo = c < dst ? dst : c;
    const uint64_t hi = (c + 16 < dend) ? c + 16 : dend;
    if (lo == c && hi == c + 16) {
      const uint64_t s = src + (c - dst);
      const uint64_t sal = s & ~3ull;
      const uint32_t sh = (uint32_t)(s - sal);
      uint32_t w[5];
      if (sal + 20 <= blob_len) {
        const uint32_t* sp = reinterpret_cast<const uint32_t*>(blob + sal);
#pragma unroll
        for (int k = 0; k < 5; ++k) w[k] = __builtin_nontemporal_load(sp + k);
      } else {
#pragma unroll
        for (int k = 0; k < 5; ++k)
          w[k] = gbyte(blob, blob_len, sal + 4 * k) | (gbyte(blob, blob_len, sal + 4 * k + 1) << 8) |
                 (gbyte(blob, blob_len, sal + 4 * k + 2) << 16) |
                 (gbyte(blob, blob_len, sal + 4 * k + 3) << 24);
      }
      uint4 v;
      v.x = __builtin_amdgcn_alignbyte(w[1], w[0], sh);
      v.y = __builtin_amdgcn_alignbyte(w[2], w[1], sh);
      v.z = __builtin_amdgcn_alignbyte(w[3], w[2], sh);
      v.w = __builtin_amdgcn_alignbyte(w[4], w[3], sh);
      *reinterpret_cast<uint4*>(out + c) = v;
    } else {
      for (uint64_t b = lo; b < hi; ++b) out[b] = blob[src + (b - dst)];
    }
  }
}

// PLAIN booleans: LSB-first bits from the value section, one byte (0/1) per value.
__global__ void __launch_bounds__(WG) k_plain_bool(const uint8_t* __restrict__ blob,
                                                   PageWork* pages, uint8_t* __restrict__ out,
                                                   ChunkResult* res) {
  const int p = blockIdx.y;
  const PageWork& pw = pages[p];
  if (pw.status != 0) return;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  if (pw.encoding != E_PLAIN) return;
  const uint64_t n = pw.nonnull;
  if ((n + 7) / 8 > pw.val_bytes && n > (uint64_t)pw.val_bytes * 8) {
    if (blockIdx.x == 0 && threadIdx.x == 0) report(pages, res, p, ST_EOF);
    return;
  }
  const uint8_t* src = blob + pw.base + pw.val_off;
  for (uint64_t k = (uint64_t)blockIdx.x * WG + threadIdx.x; k * 8 < n;
       k += (uint64_t)gridDim.x * WG) {
    uint32_t byte = src[k];
    for (int j = 0; j < 8; ++j) {
      uint64_t i = k * 8 + j;
      if (i < n) out[pw.value_out + i] = (byte >> j) & 1u;
    }
  }
}

// ------------------------------------------------------------------------------ launchers

extern "C" {

hipError_t pqg_launch_lv(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages,
                         ColumnParams cp, int sel, int dict_page, int es, RunTables rt, LevelTables lt, void* out,
                         ChunkResult* res, hipStream_t s);

hipError_t pqg_launch_prepare(const uint8_t* blob, uint64_t blob_len, PageWork* pages,
                              int npages, ColumnParams cp, uint32_t* tile_page, ChunkResult* res,
                              PrepInit ini, hipStream_t s) {
  hipLaunchKernelGGL(k_prepare, dim3(npages), dim3(64), 0, s, blob, blob_len, pages, npages, cp, tile_page, res, ini);
  return hipGetLastError();
}

hipError_t pqg_launch_run_index(const uint8_t* blob, uint64_t blob_len, PageWork* pages,
                                int npages, ColumnParams cp, int sel, int dict_page, RunTables rt,
                                ChunkResult* res, hipStream_t s) {
  hipLaunchKernelGGL(k_run_index, dim3(npages), dim3(64), 0, s, blob, blob_len, pages, cp, sel,
                     dict_page, rt, res);
  return hipGetLastError();
}

hipError_t pqg_launch_tile_desc(const uint8_t* blob, PageWork* pages, uint32_t ntiles,
                                const uint32_t* tile_page, RunTables rt, ColumnParams cp, int sel,
                                int dict_page, hipStream_t s) {
  if (ntiles)
    hipLaunchKernelGGL(k_quarter_desc, dim3((ntiles * 4 + WG - 1) / WG), dim3(WG), 0, s, blob, pages, tile_page,
                       ntiles, rt, cp, sel, dict_page);
  return hipGetLastError();
}

hipError_t pqg_launch_page_counts(PageWork* pages, int npages, RunTables rt, int field, hipStream_t s) {
  hipLaunchKernelGGL(k_page_counts, dim3(npages), dim3(WG), 0, s, pages, rt.qcount, rt.pflag, rt.nfall, field);
  return hipGetLastError();
}

// Level stream `which` (0 def, 1 rep): the window-parallel level path (levels + per-page non-null
// counts, pqg_levels.hip), then the general hybrid decoder for the streams it hands back
// (k_run_index walks only those; the tiled kernels exit at once when there are none).
hipError_t pqg_launch_levels(const uint8_t* blob, uint64_t blob_len, PageWork* pages,
                             int npages, uint32_t ntiles, ColumnParams cp, int which,
                             const uint32_t* tile_page, RunTables rt, LevelTables lt, int16_t* out,
                             ChunkResult* res, hipStream_t s, hipEvent_t* kev, int scan_es, uint64_t scan_cap) {
  const int sel = which ? SS_REP : SS_DEF;
  if (kev) (void)hipEventRecord(kev[0], s);
  hipError_t e = pqg_launch_lv(blob, blob_len, pages, npages, cp, sel, -1, 0, rt, lt, out, res, s);
  if (kev) (void)hipEventRecord(kev[1], s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_lv_fallback, dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, tile_page, cp, sel, rt, res,
                     out, lt.ctr + 1, scan_es, scan_cap);
  return hipGetLastError();
}

hipError_t pqg_launch_scan(PageWork* pages, int npages, ChunkResult* res, int es,
                           uint64_t cap_bytes, hipStream_t s) {
  hipLaunchKernelGGL(k_scan_values, dim3(1), dim3(WG), 0, s, pages, npages, res, es, cap_bytes);
  return hipGetLastError();
}

// RLE_DICTIONARY values. 4- and 8-byte values take the hybrid-stream path (pqg_levels.hip: segment
// walks, then a gather per output); its pages the general decoder takes back (dense or malformed
// streams, indices wider than 16 bits), and other value sizes, take the index pass and tiled
// expand.
hipError_t pqg_launch_dict(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages,
                           uint32_t ntiles, ColumnParams cp, int dict_page, int es,
                           const uint32_t* tile_page, RunTables rt, LevelTables lt, uint8_t* out,
                           ChunkResult* res, hipStream_t s, hipEvent_t* kev, int small_dict) {
  // (the dictionary page's checks ran in k_prepare)
  bool lvpath = es == 4 || es == 8;
#ifdef PQG_DIAG
  if (cp.debug & 256) lvpath = false;
#endif
  if (kev) (void)hipEventRecord(kev[0], s);
  if (lvpath) {
    const hipError_t e = pqg_launch_lv(blob, blob_len, pages, npages, cp, SS_DICT, dict_page, es, rt, lt, out, res, s);
    if (e != hipSuccess) return e;
    if (small_dict) {  // the level path takes (nearly) every page: its rare leftovers in one launch
      if (es == 8)
        hipLaunchKernelGGL((k_dict_fallback<8>), dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, tile_page, cp,
                           dict_page, rt, out, res);
      else
        hipLaunchKernelGGL((k_dict_fallback<4>), dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, tile_page, cp,
                           dict_page, rt, out, res);
      if (kev) (void)hipEventRecord(kev[1], s);
      return hipGetLastError();
    }
  }
  hipLaunchKernelGGL(k_run_index, dim3(npages), dim3(64), 0, s, blob, blob_len, pages, cp, SS_DICT,
                     dict_page, rt, res, lvpath ? 1 : 0);
  if (!ntiles) {
    if (kev) (void)hipEventRecord(kev[1], s);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_tile_desc, dim3((ntiles + WG - 1) / WG), dim3(WG), 0, s, blob, pages, tile_page,
                     ntiles, rt, cp, (int)SS_DICT, dict_page);
  const dim3 g = tx_grid(ntiles);
  switch (es) {
    case 1: hipLaunchKernelGGL((k_texpand_dict<1>), g, dim3(WG), 0, s, blob, blob_len, ntiles, pages, rt, dict_page, out, res); break;
    case 4: hipLaunchKernelGGL((k_texpand_dict<4>), g, dim3(WG), 0, s, blob, blob_len, ntiles, pages, rt, dict_page, out, res); break;
    case 8: hipLaunchKernelGGL((k_texpand_dict<8>), g, dim3(WG), 0, s, blob, blob_len, ntiles, pages, rt, dict_page, out, res); break;
    case 12: hipLaunchKernelGGL((k_texpand_dict<12>), g, dim3(WG), 0, s, blob, blob_len, ntiles, pages, rt, dict_page, out, res); break;
    default: return hipErrorInvalidValue;
  }
  if (kev) (void)hipEventRecord(kev[1], s);
  return hipGetLastError();
}

hipError_t pqg_launch_plain_copy(const uint8_t* blob, uint64_t blob_len, PageWork* pages,
                                 int npages, int es, int enc, uint64_t max_page_bytes,
                                 uint8_t* out, ChunkResult* res, hipStream_t s) {
  uint64_t chunks = (max_page_bytes + 16 * WG - 1) / (16 * WG) + 1;
  if (chunks > 4096) chunks = 4096;
  hipLaunchKernelGGL(k_plain_copy, dim3((unsigned)chunks, npages), dim3(WG), 0, s, blob,
                     blob_len, pages, es, enc, out, res);
  return hipGetLastError();
}

hipError_t pqg_launch_plain_bool(const uint8_t* blob, PageWork* pages, int npages,
                                 uint64_t max_page_values, uint8_t* out, ChunkResult* res,
                                 hipStream_t s) {
  uint64_t chunks = (max_page_values + 8 * WG - 1) / (8 * WG) + 1;
  if (chunks > 4096) chunks = 4096;
  hipLaunchKernelGGL(k_plain_bool, dim3((unsigned)chunks, npages), dim3(WG), 0, s, blob, pages,
                     out, res);
  return hipGetLastError();
}

// RLE booleans (data page v2 values, RleValueDecoder<bool>): the level path (one byte per value)
// with the general hybrid decoder for the streams it hands back.
hipError_t pqg_launch_rle_bool(const uint8_t* blob, uint64_t blob_len, PageWork* pages,
                               int npages, uint32_t ntiles, ColumnParams cp,
                               const uint32_t* tile_page, RunTables rt, LevelTables lt, uint8_t* out,
                               ChunkResult* res, hipStream_t s) {
  hipError_t e = pqg_launch_lv(blob, blob_len, pages, npages, cp, SS_BOOL, -1, 0, rt, lt, out, res, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_run_index, dim3(npages), dim3(64), 0, s, blob, blob_len, pages, cp, SS_BOOL,
                     -1, rt, res, 1);
  if (ntiles) {
    hipLaunchKernelGGL(k_tile_desc, dim3((ntiles + WG - 1) / WG), dim3(WG), 0, s, blob, pages, tile_page,
                       ntiles, rt, cp, (int)SS_BOOL, -1);
    hipLaunchKernelGGL(k_texpand_bool, tx_grid(ntiles), dim3(WG), 0, s, blob, blob_len, ntiles, rt, out);
  }
  return hipGetLastError();
}


}  // extern "C"

// ------------------------------------------------------------------------------ spacing
// Record assembly on the device: the layout TypedTripletIter builds batch by batch
// (record/triplet.rs:300-318), over a whole decoded chunk. Slot i of `spaced` receives dense
// value k(i) = the number of levels before i with def == max_def when def[i] == max_def, zero
// bytes otherwise. Tiles of SP_T levels: counts, one exclusive scan, scatter.
constexpr uint32_t SP_VPT = 16;
constexpr uint32_t SP_T = SP_VPT * WG;

__global__ void __launch_bounds__(WG) k_space_count(const int16_t* __restrict__ def, uint64_t n, int16_t max_def,
                                                    uint64_t* __restrict__ tcount) {
  __shared__ uint64_t red[WG / 64];
  const uint64_t i0 = (uint64_t)blockIdx.x * SP_T + (uint64_t)threadIdx.x * SP_VPT;
  uint64_t c = 0;
#pragma unroll
  for (uint32_t k = 0; k < SP_VPT; ++k) c += (i0 + k < n && def[i0 + k] == max_def) ? 1u : 0u;
  const uint64_t t = block_sum_u64(c, red);
  if (threadIdx.x == 0) tcount[blockIdx.x] = t;
}

__global__ void __launch_bounds__(WG) k_space_scan(uint64_t* __restrict__ tcount, uint32_t ntiles) {
  __shared__ uint64_t wsum[WG / 64];
  __shared__ uint64_t carry_s;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (uint32_t b = 0; b < ntiles; b += WG) {
    const uint32_t t = b + threadIdx.x;
    const uint64_t x = t < ntiles ? tcount[t] : 0;
    uint64_t incl = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(incl, d, 64);
      if ((threadIdx.x & 63) >= (unsigned)d) incl += y;
    }
    if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint64_t pre = carry_s;
    for (int k = 0; k < (int)(threadIdx.x >> 6); ++k) pre += wsum[k];
    if (t < ntiles) tcount[t] = pre + incl - x;
    __syncthreads();
    if (threadIdx.x == WG - 1) carry_s = pre + incl;
    __syncthreads();
  }
}

template <int ES>
__global__ void __launch_bounds__(WG) k_space_scatter(const int16_t* __restrict__ def, uint64_t n, int16_t max_def,
                                                      const uint8_t* __restrict__ values,
                                                      const uint64_t* __restrict__ tbase,
                                                      uint8_t* __restrict__ spaced) {
  __shared__ uint64_t wsum[WG / 64];
  const uint64_t i0 = (uint64_t)blockIdx.x * SP_T + (uint64_t)threadIdx.x * SP_VPT;
  uint32_t m = 0;  // max_def flags of this thread's levels
#pragma unroll
  for (uint32_t k = 0; k < SP_VPT; ++k) m |= (i0 + k < n && def[i0 + k] == max_def ? 1u : 0u) << k;
  const uint64_t c = (uint64_t)__builtin_popcount(m);
  uint64_t incl = c;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d, 64);
    if ((threadIdx.x & 63) >= (unsigned)d) incl += y;
  }
  if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
  __syncthreads();
  uint64_t k = tbase[blockIdx.x] + incl - c;
  for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) k += wsum[w];
#pragma unroll
  for (uint32_t q = 0; q < SP_VPT; ++q) {
    const uint64_t i = i0 + q;
    if (i >= n) break;
    uint8_t* o = spaced + i * ES;
    if ((m >> q) & 1u) {
      const uint8_t* v = values + k * ES;
      if constexpr (ES == 1) *o = *v;
      else if constexpr (ES == 4) *reinterpret_cast<uint32_t*>(o) = *reinterpret_cast<const uint32_t*>(v);
      else if constexpr (ES == 8) *reinterpret_cast<uint64_t*>(o) = *reinterpret_cast<const uint64_t*>(v);
      else
        for (int b = 0; b < ES; b += 4) *reinterpret_cast<uint32_t*>(o + b) = *reinterpret_cast<const uint32_t*>(v + b);
      ++k;
    } else {
      for (int b = 0; b < ES; ++b) o[b] = 0;
    }
  }
}

extern "C" {

// Tiles (SP_T levels each) pqg_launch_space needs `tiles` entries for: the host sizes its buffer
// from this, not from a copy of the constant.
uint64_t pqg_space_tiles(uint64_t n) { return (n + SP_T - 1) / SP_T; }

hipError_t pqg_launch_space(const int16_t* def, uint64_t n, int16_t max_def, const void* values, int es,
                            uint64_t* tiles, void* spaced, hipStream_t s) {
  if (n == 0) return hipSuccess;
  const uint32_t nt = (uint32_t)((n + SP_T - 1) / SP_T);
  hipLaunchKernelGGL(k_space_count, dim3(nt), dim3(WG), 0, s, def, n, max_def, tiles);
  hipLaunchKernelGGL(k_space_scan, dim3(1), dim3(WG), 0, s, tiles, nt);
  const uint8_t* v = (const uint8_t*)values;
  uint8_t* o = (uint8_t*)spaced;
  switch (es) {
    case 1: hipLaunchKernelGGL(k_space_scatter<1>, dim3(nt), dim3(WG), 0, s, def, n, max_def, v, tiles, o); break;
    case 4: hipLaunchKernelGGL(k_space_scatter<4>, dim3(nt), dim3(WG), 0, s, def, n, max_def, v, tiles, o); break;
    case 8: hipLaunchKernelGGL(k_space_scatter<8>, dim3(nt), dim3(WG), 0, s, def, n, max_def, v, tiles, o); break;
    case 12: hipLaunchKernelGGL(k_space_scatter<12>, dim3(nt), dim3(WG), 0, s, def, n, max_def, v, tiles, o); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // extern "C"

}  // namespace pqg
