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
// A decode covers a batch of column chunks (pqg_decode_chunks; one for pqg_decode_chunk): every
// kernel runs once over the pages of all of them, each page taking its column parameters,
// dictionary and output buffers from its chunk (ChunkWork, pqg_internal.hpp). Kernels over tiles
// of one kind of page take a host-built list of those tiles (tl, ntl) instead of a grid over
// every tile of the batch.
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
                                    int p, ChunkWork* chunks, PageWork& out) {
  PageWork pw = pages[p];
  ChunkWork& ck = chunks[pw.chunk];
  const ColumnParams& cp = ck.cp;
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
  // Values each page must yield: def == max_def count when levels are read (filled by the level
  // path), else the page's level count (column/reader.rs:212-226).
  bool data = pw.page_type == P_DATA || pw.page_type == P_DATA_V2;
  if (data && !(cp.max_def > 0 && cp.want_def)) pw.nonnull = pw.num_values;
  pw.spec_n = (!err && data && ck.spec && pw.encoding == E_PLAIN && ck.es > 0) ? pw.val_bytes / (uint32_t)ck.es : 0;
  if (!err && p == ck.dict_page && ck.dict_es > 0) {  // DictDecoder::set_dict (decoding.rs:282-288)
    if (pw.encoding != E_PLAIN && pw.encoding != E_PLAIN_DICTIONARY) err = ST_NYI;
    else if ((uint64_t)pw.num_values * (uint64_t)ck.dict_es > pw.nbytes) err = ST_EOF;
  }
  pw.status = err;
  pages[p] = pw;
  out = pw;
  if (err)
    atomicMin((unsigned long long*)&ck.res.bad,
              ((unsigned long long)((uint32_t)p - ck.first_page) << 32) | (uint32_t)err);
}

// One wave per page: the lanes fill the page's tile -> page entries (a dictionary column's
// single data page has thousands), lane 0 the rest.
__global__ void __launch_bounds__(64) k_prepare(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                PageWork* __restrict__ pages, int npages, ChunkWork* chunks,
                                                uint32_t* __restrict__ tile_page, PrepInit ini) {
  const int p = blockIdx.x;
  if (p >= npages) return;
  {
    const uint32_t t0 = pages[p].ltile0, nt = pages[p].ntiles;
    for (uint32_t k = threadIdx.x; k < nt; k += 64) tile_page[t0 + k] = (uint32_t)p;
  }
  __shared__ PageWork pw_s;
  if (threadIdx.x == 0) {
    prepare_page(blob, blob_len, pages, p, chunks, pw_s);
    if (p == 0)
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (ini.word[i]) *ini.word[i] = ini.val[i];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      if (ini.pzero[i]) ini.pzero[i][p] = 0;
    if (ini.dense_zero) ini.dense_zero[p] = 0;
  }
  __syncthreads();
  // density probes of the level streams just located (wave-uniform from here)
  const ColumnParams& cp = pcp(chunks, pw_s);
  for (int k = 0; k < 2; ++k) {
    uint32_t* dn = k == 0 ? ini.dense_def : ini.dense_rep;
    if (!dn) continue;
    const PageWork& pw = pw_s;
    const bool data = pw.page_type == P_DATA || pw.page_type == P_DATA_V2;
    const int kind = k == 0 ? pw.def_kind : pw.rep_kind;
    const uint32_t slen = k == 0 ? pw.def_bytes : pw.rep_bytes;
    const uint32_t w = (uint32_t)(k == 0 ? cp.def_bit_width : cp.rep_bit_width);
    const bool want = k == 0 ? cp.want_def : cp.want_rep;
    uint32_t dense = 0;
    if (want && data && pw.status == 0 && kind == LK_RLE && w >= 1 && w <= 16 && pw.num_values &&
        slen >= PROBE_SPAN + 64u)
      dense = lv_probe_dense(blob, blob_len, pw.base + (k == 0 ? pw.def_off : pw.rep_off), w);
    if (threadIdx.x == 0) dn[p] = dense;
  }
}

// ------------------------------------------------------------------------------ hybrid streams

// Index pass over stream `sel` of every page (one wave per page), pqg_runs.hpp.
__global__ void __launch_bounds__(64) k_run_index(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                  PageWork* pages, ChunkWork* chunks, int sel, RunTables rt,
                                                  int bailed_only = 0) {
  __shared__ IndexSmem sm;
  const int p = blockIdx.x;
  if (bailed_only ? rt.pflag[p] != PF_BAIL : (*rt.nfall == 0 || pf_level_path(rt.pflag[p]))) return;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  const ChunkWork& ck = chunks[pw.chunk];
  if (!bailed_only && sel == SS_DICT && ck.lvdict) return;  // the level path's chunk (its leftovers: k_*_fallback)
  Stream s;
  if (!get_stream(blob, pw, sel, ck.cp, s)) return;
  if (sel == SS_DICT) {
    if (ck.dict_page < 0) {  // "Decoder for dict should have been set"
      if (threadIdx.x == 0) report(pages, chunks, p, ST_PANIC);
      return;
    }
    if (!dict_usable(pages, ck)) return;
  }
  const int32_t st = run_index(blob, blob_len, s, rt.ck + pw.ltile0,
                              rt.runs + (uint64_t)pw.ltile0 * RUN_CAPT, rt.nruns + pw.ltile0, sm,
                              (ck.cp.debug & 32) && ck.cp.dbgbuf ? ck.cp.dbgbuf + 2 * p : nullptr);
  if (st && threadIdx.x == 0) report(pages, chunks, p, st);
}

// Quarter-tile descriptors of stream `sel` over the listed tiles (one thread per quarter; desc
// and its count slot at 4 t + q), read by the wave expand kernels.
__global__ void __launch_bounds__(WG) k_quarter_desc(const uint8_t* __restrict__ blob, const PageWork* pages,
                                                     const ChunkWork* chunks, const uint32_t* __restrict__ tile_page,
                                                     const uint32_t* __restrict__ tl, uint32_t ntl, RunTables rt,
                                                     int sel) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= ntl * 4) return;
  const uint32_t t = tl[i >> 2];
  rt.desc[4 * t + (i & 3)] = quarter_desc(blob, pages, chunks, tile_page, rt, sel, t, i & 3);
}

// Tile descriptors of stream `sel` over the listed tiles (one thread per tile), read by the tile
// expand kernels.
__global__ void __launch_bounds__(WG) k_tile_desc(const uint8_t* __restrict__ blob, const PageWork* pages,
                                                  const ChunkWork* chunks, const uint32_t* __restrict__ tile_page,
                                                  const uint32_t* __restrict__ tl, uint32_t ntl, RunTables rt,
                                                  int sel) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= ntl || *rt.nfall == 0) return;
  const uint32_t t = tl[i];
  rt.desc[t] = quarter_desc(blob, pages, chunks, tile_page, rt, sel, t, 0, RUN_TILE);
}

// Level streams the level path handed back (PF_BAIL: malformed input, unusual header forms), one
// workgroup per page: wave 0 walks the page's header chain (run_index: every reference check,
// per-tile checkpoints and records), then the workgroup expands the page's tiles one after the
// other and sums the page's def levels == max_def (its non-null count). One launch in place of
// index pass + tile descriptors + tile expand + page counts: the level path leaves these streams
// to it only on unusual input, so the latency of a serial page matters less than three launches
// on every decode.
struct LevelsPageMaker {
  gptr<int16_t> out;
  int16_t maxl;
  bool count;
  uint32_t acc;  // this thread's outputs == maxl
  __device__ TxLevels make(const QDesc& d) { return TxLevels{out + d.out, maxl, count, 0u}; }
  __device__ void done(const QDesc&, uint32_t, TxLevels& em) { acc += em.nonnull; }
};

__device__ inline void lv_fallback_page(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                        PageWork* pages, ChunkWork* chunks, const uint32_t* __restrict__ tile_page,
                                        int sel, RunTables rt, int p) {
  __shared__ IndexSmem ism;
  __shared__ TileSmem sm;
  __shared__ int32_t st_s;
  __shared__ uint64_t red[WG / 64];
  if (rt.pflag[p] != PF_BAIL) return;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  const ChunkWork& ck = chunks[pw.chunk];
  Stream s;
  if (!get_stream(blob, pw, sel, ck.cp, s)) return;
  if (threadIdx.x < 64) {
    const int32_t st = run_index(blob, blob_len, s, rt.ck + pw.ltile0, rt.runs + (uint64_t)pw.ltile0 * RUN_CAPT,
                                 rt.nruns + pw.ltile0, ism);
    if (threadIdx.x == 0) {
      st_s = st;
      if (st) report(pages, chunks, p, st);
    }
  }
  __syncthreads();
  if (st_s) return;
  LevelsPageMaker mk{gp(sel == SS_DEF ? ck.def_out : ck.rep_out), sel == SS_DEF ? ck.cp.max_def : ck.cp.max_rep,
                     sel == SS_DEF, 0u};
  for (uint32_t t = pw.ltile0; t < pw.ltile0 + pw.ntiles; ++t) {
    if (threadIdx.x == 0) rt.desc[t] = quarter_desc(blob, pages, chunks, tile_page, rt, sel, t, 0, RUN_TILE);
    __syncthreads();  // (the descriptor is read by every thread of the workgroup)
    tile_one(blob, blob_len, rt.desc, t, rt.runs, sm, mk);
    __syncthreads();  // sm is refilled by the next tile
  }
  if (sel == SS_DEF) {
    const uint64_t nn = block_sum_u64(mk.acc, red);
    if (threadIdx.x == 0) pages[p].nonnull = nn;
  }
}

__device__ inline void scan_values(PageWork* pages, ChunkWork* chunks, int npages);

#ifndef PQG_LF_GRID
#define PQG_LF_GRID 256
#endif
constexpr int LF_GRID = PQG_LF_GRID;  // k_lv_fallback workgroups at most

// scan != 0 (a def stream, no rep stream after it): the grid's last workgroup also runs
// k_scan_values (the non-null counts are final), one launch fewer per decode.
__global__ void __launch_bounds__(WG) k_lv_fallback(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                    PageWork* pages, ChunkWork* chunks,
                                                    const uint32_t* __restrict__ tile_page, int sel, RunTables rt,
                                                    uint32_t* ctr, int scan, int npages) {
  // a grid of at most LF_GRID workgroups strides over the pages (handed-back pages are rare: a
  // workgroup per page made the launch itself cost ~10 us more)
  for (int p = (int)blockIdx.x; p < npages; p += (int)gridDim.x) {
    lv_fallback_page(blob, blob_len, pages, chunks, tile_page, sel, rt, p);
    __syncthreads();  // (the page's shared state before the next page's)
  }
  if (scan && last_workgroup(ctr)) scan_values(pages, chunks, npages);
}

// Tile expand of RLE_DICTIONARY indices with the dictionary gather: the tile's page names its
// chunk, whose dictionary page and value buffer the emitter takes.
template <int ES>
struct DictMaker {
  const uint8_t* blob;
  PageWork* pages;
  ChunkWork* chunks;
  __device__ TxDict<ES> make(const QDesc& d) {
    if (!d.qhi) return TxDict<ES>{nullptr, 0u, false, nullptr, 0};
    const ChunkWork& ck = chunks[pages[d.page].chunk];
    const PageWork& dp = pages[ck.dict_page];  // (quarter_desc gives work only with a valid dictionary)
    return TxDict<ES>{blob + dp.base, dp.num_values, ((dp.base % (ES == 12 ? 4 : ES)) == 0),
                      gp(ck.val_out) + d.out * (uint64_t)ES, 0};
  }
  __device__ void done(const QDesc& d, uint32_t, TxDict<ES>& em) {
    const uint64_t bad = __ballot(em.err != 0);
    if (bad && (threadIdx.x & 63) == 0) report(pages, chunks, (int)d.page, ST_PANIC);
  }
};

// One tile of the list per workgroup (the list holds the tiles of the chunks whose value size is ES).
template <int ES>
__global__ void __launch_bounds__(WG) k_texpand_dict(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                     const uint32_t* __restrict__ tl, PageWork* pages,
                                                     ChunkWork* chunks, RunTables rt) {
  __shared__ TileSmem sm;
  if (*rt.nfall == 0) return;
  DictMaker<ES> mk{blob, pages, chunks};
  tile_one(blob, blob_len, rt.desc, tl[blockIdx.x], rt.runs, sm, mk);
}

// ---- dictionaries of at most 65536 entries of 4 or 8 bytes, too large for the level path's
// LDS copy. A random gather served from L2 costs one L2 request per value, and the request rate,
// not HBM, bounds it (k_texpand_dict<8> at 64K entries: 4.45 ms for 1e9 values). Instead the
// tile expand keeps each tile's indices (16-bit, one RUN_TILE slot per listed tile), and
// k_dict_win streams the dictionary through LDS in 128 KiB windows: a workgroup of 1024 threads
// takes 8 tiles (32 values per thread, in registers), fills window after window of their
// dictionary by LDS-DMA (no registers held by the fill) and gathers the indices that fall in
// each; L2 serves whole lines of the dictionary (D x ES bytes per 32768 values) instead of one
// request per value (tools/ubench/win_ubench.hip: 2.7 ms against 4.5 ms for the L2 gather).
struct DictIdxMaker {
  PageWork* pages;
  ChunkWork* chunks;
  uint16_t* idx;  // the list's slots
  uint32_t p;     // the tile's position in the list (its slot)
  __device__ TxDictIdx make(const QDesc& d) {
    if (!d.qhi) return TxDictIdx{gptr<uint16_t>(nullptr), 0u, 0u, 0};
    const ChunkWork& ck = chunks[pages[d.page].chunk];
    return TxDictIdx{gp(idx) + (uint64_t)p * RUN_TILE, d.qlo, pages[ck.dict_page].num_values, 0};
  }
  __device__ void done(const QDesc& d, uint32_t, TxDictIdx& em) {
    const uint64_t bad = __ballot(em.err != 0);
    if (bad && (threadIdx.x & 63) == 0) report(pages, chunks, (int)d.page, ST_PANIC);
  }
};

// Tiles k_dict_win decodes itself (their run records fit its record region). The others -- more
// run records than DF_RC, or than the index pass keeps (re-walk), or stream offsets past 2^28
// bytes -- have their indices kept in the tile's slot by k_texpand_didx first.
constexpr uint32_t DF_RC = 128;                      // run records per tile
constexpr uint32_t DF_TR = 2 * (DF_RC + 2) + 64 + 32;  // record region words: starts, info, blk, blk2
static_assert(DF_RC <= 128, "one record per thread of a tile");
static_assert(DF_TR % 4 == 0 && (2 * (DF_RC + 2)) % 4 == 0, "16-byte block descriptors");

__device__ inline bool df_easy(const QDesc& d) {
  return d.qhi && d.rec != RUN_REWALK && !tx_wide(d) && tx_nrec(d) <= DF_RC;
}

// A payload word (4-aligned offset a of n readable bytes; bytes past them read as zero).
__device__ __forceinline__ uint32_t dw_word(const uint8_t* p, uint64_t n, uint64_t a) {
  if (a + 4 <= n) return *reinterpret_cast<const uint32_t*>(p + a);
  uint32_t v = 0;
  for (uint32_t k = 0; k < 4; ++k)
    if (a + k < n) v |= (uint32_t)p[a + k] << (8 * k);
  return v;
}

// The list's tiles k_dict_win does not decode itself (none at the benchmark's shape), appended
// to a compact list: *cnt entries of the list from hl (one thread per list entry, one atomic per
// wave).
__global__ void __launch_bounds__(WG) k_didx_mark(const uint32_t* __restrict__ tl, uint32_t ntl, RunTables rt,
                                                  uint32_t* cnt, uint32_t* hl) {
  if (*rt.nfall == 0) return;
  const uint32_t pi = blockIdx.x * WG + threadIdx.x, lane = threadIdx.x & (WAVE - 1);
  const bool h = pi < ntl && !df_easy(rt.desc[tl[pi]]);
  const uint64_t m = __ballot(h);
  if (!m) return;
  const int first = __builtin_ctzll(m);
  uint32_t base = 0;
  if ((int)lane == first) base = atomicAdd(cnt, (uint32_t)__builtin_popcountll(m));
  base = __shfl(base, first);
  if (h) hl[base + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull))] = pi;
}

// Index expand of the marked tiles into their slots: the grid strides over the compact list, one
// tile per workgroup at a time, so a list of many hard tiles (short runs: sorted or low-cardinality
// data) is spread over the whole grid.
__global__ void __launch_bounds__(WG) k_texpand_didx(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                     const uint32_t* __restrict__ tl, PageWork* pages,
                                                     ChunkWork* chunks, RunTables rt, const uint32_t* cnt,
                                                     const uint32_t* hl, uint16_t* idx) {
  __shared__ TileSmem sm;
  if (*rt.nfall == 0) return;
  const uint32_t nh = *cnt;
  for (uint32_t k = blockIdx.x; k < nh; k += gridDim.x) {
    const uint32_t p = hl[k];
    DictIdxMaker mk{pages, chunks, idx, p};
    tile_one(blob, blob_len, rt.desc, tl[p], rt.runs, sm, mk);
    __syncthreads();
  }
}

constexpr int DW_NT = 1024;                         // k_dict_win threads
#ifndef PQG_DW_GRID
#define PQG_DW_GRID 256u                            // k_dict_win workgroups (the CUs)
#endif
constexpr int DW_TPW = DW_NT / 128;                 // tiles per workgroup (128 threads x 32 values)
constexpr uint32_t DW_BYTES = 128u << 10;           // window bytes
constexpr uint32_t DW_LDS = DW_BYTES + 1024u;       // + the shift of an unaligned dictionary
constexpr uint32_t DW_CH = DW_LDS / 16u;            // 16-byte LDS-DMA chunks per fill
constexpr int DW_F = (int)((DW_CH + DW_NT - 1) / DW_NT);

template <int ES>
__global__ void __launch_bounds__(DW_NT) k_dict_win(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                    const uint32_t* __restrict__ tl, uint32_t ntl,
                                                    PageWork* __restrict__ pages, ChunkWork* __restrict__ chunks,
                                                    RunTables rt, const uint16_t* __restrict__ idx) {
  using T = typename std::conditional<ES == 8, uint64_t, uint32_t>::type;
  constexpr uint32_t WIN = DW_BYTES / ES;  // entries per window
  __shared__ uint4 win[DW_CH + 1];         // (+1: the unaligned reads' third word)
  __shared__ uint4 trec[DW_TPW][DF_TR / 4];  // per tile: run records and block descriptors
  __shared__ int32_t dkey[DW_TPW];
  if (*rt.nfall == 0) return;
  const uint32_t tid = threadIdx.x, q = tid >> 7, lt = tid & 127u;
#ifdef PQG_DIAG
  // diagnostics (PQG_DEBUG bit 4096, tools/diag/diag_dict.py): thread 0's s_memtime cycles per
  // phase -- stage, block descriptors, index decode, window fills (issue to the barrier after the
  // wait), gathers, stores
  const bool dst = tid == 0 && (chunks[0].cp.debug & 4096) && chunks[0].cp.dbgbuf;
  uint64_t dt_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, dt0 = __builtin_amdgcn_s_memtime();
#define DW_STAMP(k)                                   \
  if (dst) {                                          \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(); \
    dt_[k] += t1 - dt0;                               \
    dt0 = t1;                                         \
  }
#else
#define DW_STAMP(k)
#endif
  // persistent: the workgroup takes batches of DW_TPW tiles in turn; the window left in LDS by one
  // batch (res_key / res_w) is the next batch's first, its windows visited in reverse order every
  // other batch (snake), so one fill in nw is saved per batch
  const uint32_t nbt = (ntl + DW_TPW - 1) / DW_TPW;
  int32_t res_key = -1;
  uint32_t res_w = 0xFFFFFFFFu, it = 0;
#pragma unroll 1
  for (uint32_t bt = blockIdx.x; bt < nbt; bt += gridDim.x, ++it) {
  const uint32_t p = bt * DW_TPW + q;
  __syncthreads();  // (the previous batch's reads of dkey and the record regions are done)
  const QDesc d = p < ntl ? rt.desc[tl[p]] : QDesc{};
  const uint32_t qlo = d.qlo, qhi = d.qhi;
  uint64_t obase = 0;
  int32_t key = -1;
  uint32_t D0 = 0;
  if (qhi) {
    const ChunkWork& ck = chunks[pages[d.page].chunk];
    key = ck.dict_page;
    D0 = pages[key].num_values;
    obase = reinterpret_cast<uint64_t>(ck.val_out) + (d.out + qlo) * (uint64_t)ES;
  }
  if (lt == 0) dkey[q] = key;
  // the thread's 32 values: 16 pairs, pair s at tile outputs qlo + 2 (128 s + lt) + {0, 1} (each
  // store instruction of a wave one contiguous run of 64 pairs); rem: the tile's outputs from the
  // thread's first pair on
  const int32_t rem = (int32_t)(qhi - qlo) - (int32_t)(2u * lt);
  uint32_t ix[16];
  const bool easy = df_easy(d);
  // ---- an easy tile's indices are decoded here (rle.rs:437-487): its run records go to the
  // tile's record region in LDS; each thread then loads its pairs' payload words straight from
  // the stream (a pair is 2w <= 32 bits: a wave's lanes read consecutive words), issued while the
  // first window's LDS-DMA fill is in flight. Bit offsets count from A0 (the payload's first byte,
  // aligned down to 16).
  uint32_t* rs = reinterpret_cast<uint32_t*>(trec[q]);  // run starts (page-relative outputs)
  uint32_t* ri = rs + DF_RC + 2;                        // run info (payload offset, or R_RLE | value)
  const uint32_t nr = tx_nrec(d);
  const uint64_t A0 = ((d.bhi ? d.S + d.blo : d.S) & ~15ull);
  const uint32_t sb32 = (uint32_t)(A0 - d.S);
  if (easy) {
    if (d.kind == LK_BIT_PACKED) {  // one header-less run from output 0
      if (lt == 0) {
        rs[0] = 0;
        ri[0] = 0;
      }
    } else if (lt < nr) {  // (nr <= DF_RC = 128: one record per thread)
      const uint2 r = rt.runs[d.rec + lt];
      rs[lt] = r.x;
      ri[lt] = r.y;
    }
    if (lt == 0) rs[nr] = rs[nr + 1] = qhi;
  }
  __syncthreads();  // (every wave: the tiles of one workgroup may differ in kind)
  DW_STAMP(0)
  // per 256-output block k of an easy tile (pair s of every thread lies in block s), found once
  // by thread k: the run holding its first output (A) and the run after it (B), as block-relative
  // ends and, for a bit-packed run, the bit offset of the block's first output from A0 (the pair
  // at block output r then starts at bit base + r w); an RLE run's value instead
  uint4* blk = reinterpret_cast<uint4*>(ri + DF_RC + 2);  // (end A, base A, end B, base B)
  uint32_t* blk2 = reinterpret_cast<uint32_t*>(blk + 16);  // (RLE flags, run A)
  if (easy && lt < 16) {
    const uint32_t o = qlo + 256u * lt;
    uint32_t a = 0;
#pragma unroll
    for (uint32_t step = DF_RC / 2; step; step >>= 1)
      if (a + step < nr && rs[a + step] <= o) a += step;
    const bool two = a + 1 < nr;
    const uint32_t ia = ri[a], ib = two ? ri[a + 1] : 0u, w = d.w;
    const uint32_t ba = ia & R_RLE ? ia & 0x7FFFFFFFu : (ia - sb32) * 8u + (o - rs[a]) * w;
    const uint32_t bb = ib & R_RLE ? ib & 0x7FFFFFFFu : (ib - sb32) * 8u - (rs[a + 1] - o) * w;  // (mod 2^32)
    blk[lt] = make_uint4(rs[a + 1] - o, ba, rs[a + 2] - o, bb);  // (rs[nr] = rs[nr + 1] = qhi)
    blk2[2 * lt] = (ia & R_RLE ? 1u : 0u) | (two && (ib & R_RLE) ? 2u : 0u);
    blk2[2 * lt + 1] = a;
  }
  __syncthreads();
  DW_STAMP(1)
  // the index decode, run once, right after the first window's fill is issued
  auto decode = [&]() {
    if (easy) {
      const uint8_t* pay = blob + A0;
      const uint64_t plen = blob_len - A0;  // (A0 < blob_len: inside the stream)
      const uint32_t w = d.w, wm = w >= 32 ? 0xFFFFFFFFu : ((1u << w) - 1u);
      const uint32_t r = 2u * lt, rw = r * w;  // the thread's pair in every block
      bool bad = false;
      // fast pass: each pair inside one of its block's two runs (w <= 16: both values in one
      // 32-bit window) -- a bit offset, or an RLE run's value; the rest marked for the slow pass
      uint32_t q[16], slow = 0, rle = 0, dead = 0;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const uint4 b = blk[s];
        const uint32_t fl = blk2[2 * s];
        const bool inA = r + 1 < b.x, inB = r >= b.x && r + 1 < b.z;
        q[s] = inA ? b.y : b.w;
        const bool dd = s * 256 >= rem, sl = !dd && !((inA || inB) && w <= 16);  // (selects, no branches)
        dead |= (uint32_t)dd << s;
        slow |= (uint32_t)sl << s;
        rle |= (uint32_t)((fl & (inA ? 1u : 2u)) != 0u) << s;
      }
      uint32_t lo[16], hi[16];
      if (d.S + d.bhi + 8u <= blob_len) {  // (the tile's wave-uniform common case: no load near the blob's end)
        const uint32_t* pw32 = reinterpret_cast<const uint32_t*>(pay);
#pragma unroll
        for (int s = 0; s < 16; ++s) {  // (every load in flight at once; RLE, slow and dead pairs load nothing)
          lo[s] = hi[s] = 0u;
          if (!(((rle | slow | dead) >> s) & 1u)) {
            const uint32_t wi = (q[s] + rw) >> 5;
            lo[s] = pw32[wi];
            hi[s] = pw32[wi + 1];
          }
        }
      } else {
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          lo[s] = hi[s] = 0u;
          if (!(((rle | slow | dead) >> s) & 1u)) {
            const uint32_t wi = (q[s] + rw) >> 5;
            lo[s] = dw_word(pay, plen, 4ull * wi);
            hi[s] = dw_word(pay, plen, 4ull * wi + 4u);
          }
        }
      }
      // dict[idx] out of bounds: the reference panics (rle.rs:455,470); the tile's last output
      // has no second value
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const uint32_t x = __builtin_amdgcn_alignbit(hi[s], lo[s], (q[s] + rw) & 31u);
        uint32_t v0 = (rle >> s) & 1u ? q[s] : x & wm;
        uint32_t v1 = (rle >> s) & 1u ? q[s] : (x >> w) & wm;
        if (((dead | slow) >> s) & 1u) v0 = v1 = 0;
        if (s * 256 + 1 >= rem) v1 = 0;
        bad |= v0 >= D0 || v1 >= D0;
        ix[s] = (v0 & 0xFFFFu) | (v1 << 16);
      }
      // slow pass (a pair across a run boundary, a block past its first two runs, w > 16): value
      // by value from the block's first run on
      if (slow) {
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          if (!((slow >> s) & 1u)) continue;
          const uint32_t o0 = qlo + 256u * (uint32_t)s + r;
          uint32_t a = blk2[2 * s + 1], st = rs[a], inf = ri[a], nx = rs[a + 1];
          uint32_t v2[2] = {0u, 0u};
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const uint32_t o = o0 + (uint32_t)j;
#pragma unroll 1
            while (nx <= o && a + 1 < nr) {
              ++a;
              st = nx;
              inf = ri[a];
              nx = rs[a + 1];
            }
            if (inf & R_RLE) {
              v2[j] = inf & 0x7FFFFFFFu;
            } else {
              const uint32_t bit = (inf - sb32) * 8u + (o - st) * w;
              const uint32_t wi = bit >> 5;
              v2[j] = __builtin_amdgcn_alignbit(dw_word(pay, plen, 4ull * wi + 4u), dw_word(pay, plen, 4ull * wi),
                                                bit & 31u) & wm;
            }
          }
          if (s * 256 + 1 >= rem) v2[1] = 0;
          bad |= v2[0] >= D0 || v2[1] >= D0;
          ix[s] = (v2[0] & 0xFFFFu) | (v2[1] << 16);
        }
      }
      const uint64_t bm = __ballot(bad);
      if (bm && (tid & 63u) == (uint32_t)__builtin_ctzll(bm)) report(pages, chunks, (int)d.page, ST_PANIC);
    } else {
      const uint32_t* ip = reinterpret_cast<const uint32_t*>(idx + (uint64_t)p * RUN_TILE) + lt;
#pragma unroll
      for (int s = 0; s < 16; ++s) ix[s] = s * 256 < rem ? ip[s * 128] : 0u;
    }
  };
  // a window fill by LDS-DMA (no registers held): chunks c < lim, inside the window's bytes and
  // the blob
  auto fill_lim = [&](uint64_t dbase, uint32_t D, uint32_t w0) -> uint32_t {
    const uint64_t a = dbase + (uint64_t)w0 * ES, a0 = a & ~15ull;
    const uint32_t nb = (uint32_t)(a - a0) + (D - w0 < WIN ? D - w0 : WIN) * (uint32_t)ES;
    const uint64_t bl = blob_len > a0 ? (blob_len - a0) / 16u : 0u;
    return (uint32_t)min(min((uint64_t)DW_CH, (uint64_t)(nb + 15u) / 16u), bl);
  };
  auto fill = [&](uint64_t dbase, uint32_t D, uint32_t w0) {
    const uint64_t a0 = (dbase + (uint64_t)w0 * ES) & ~15ull;
    const uint32_t lim = fill_lim(dbase, D, w0);
    const uint8_t* src = blob + a0 + (uint64_t)tid * 16u;
#pragma unroll 1  // (unrolled, the fill's addresses and M0 values took registers the values need)
    for (int f = 0; f < DW_F; ++f) {
      const uint32_t c = (uint32_t)f * DW_NT + tid;
      if (c < lim)
        __builtin_amdgcn_global_load_lds(
            (const __attribute__((address_space(1))) void*)(src + (uint64_t)f * DW_NT * 16u),
            (__attribute__((address_space(3))) void*)((__attribute__((address_space(3))) uint8_t*)win +
                                                       ((uint32_t)f * DW_NT + (tid & ~63u)) * 16u),
            16, 0, 0);
    }
  };
  // the first window (the first distinct dictionary's, in the loop's order) is filled while the
  // indices are decoded, unless it is the one left in LDS
  const bool rev = (it & 1u) != 0;
  int32_t k1 = -1;
  for (int qq = 0; qq < DW_TPW && k1 < 0; ++qq) k1 = dkey[qq];
  bool prefilled = false;
  if (k1 >= 0) {
    const uint32_t D1 = pages[k1].num_values, nw1 = (D1 + WIN - 1) / WIN;
    const uint32_t wf = rev ? nw1 - 1u : 0u;
    if (!(k1 == res_key && wf == res_w)) {
      fill(pages[k1].base, D1, wf * WIN);
      prefilled = true;
    }
  }
  decode();
  T x[16][2];
#pragma unroll
  for (int s = 0; s < 16; ++s) x[s][0] = x[s][1] = 0;
  DW_STAMP(2)
  for (int qq = 0; qq < DW_TPW; ++qq) {  // each distinct dictionary of the 8 tiles (uniform)
    const int32_t kq = dkey[qq];
    bool seen = kq < 0;
    for (int r = 0; r < qq; ++r) seen |= dkey[r] == kq;
    if (seen) continue;
    const uint64_t dbase = pages[kq].base;
    const uint32_t D = pages[kq].num_values, nw = (D + WIN - 1) / WIN;
    const bool mine = key == kq;
    for (uint32_t wk = 0; wk < nw; ++wk) {
      const uint32_t wi = rev ? nw - 1u - wk : wk, w0 = wi * WIN;
      const uint64_t a = dbase + (uint64_t)w0 * ES, a0 = a & ~15ull;
      const uint32_t sh = (uint32_t)(a - a0);  // the window's first entry lands at LDS byte sh
      if (!(kq == res_key && wi == res_w)) {  // (uniform) not the window already in LDS
      if (prefilled) {
        prefilled = false;  // (the fill issued before the decode)
      } else {
        __syncthreads();  // (the previous window's gathers are done)
        fill(dbase, D, w0);
      }
      // every wave's LDS-DMA fill must have landed before any wave reads the window: each wave
      // waits for its own (vmcnt(0), explicit: the barrier alone does not promise it), then the
      // barrier orders the waves. 0x0F70 is vmcnt(0) in the gfx9 (gfx950) encoding; the guard
      // below fails the build for a target whose encoding differs
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "k_dict_win: the s_waitcnt immediate 0x0F70 (vmcnt(0)) is the gfx9 encoding"
#endif
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __syncthreads();
      DW_STAMP(3)
      if (sh) {  // a dictionary at an odd offset: the window moved down by sh bytes, in place
        const uint32_t k0 = sh >> 2, bs = sh & 3u, lim = fill_lim(dbase, D, w0);
#pragma unroll 1
        for (int f = 0; f < DW_F; ++f) {
          const uint32_t c = (uint32_t)f * DW_NT + tid;
          const uint32_t cc = c < DW_CH ? c : DW_CH - 1u;  // (LDS reads in bounds; results unused)
          const uint4 a4 = win[cc], b4 = win[cc + 1];
          const uint32_t v0 = a4.x, v1 = a4.y, v2 = a4.z, v3 = a4.w, v4 = b4.x, v5 = b4.y, v6 = b4.z, v7 = b4.w;
          __syncthreads();  // (every chunk read before any is rewritten)
          if (c < lim) {
            // words k0 .. k0 + 4 of the 8 hold the chunk's 16 bytes from byte sh on
            const uint32_t w0_ = k0 == 0 ? v0 : k0 == 1 ? v1 : k0 == 2 ? v2 : v3;
            const uint32_t w1_ = k0 == 0 ? v1 : k0 == 1 ? v2 : k0 == 2 ? v3 : v4;
            const uint32_t w2_ = k0 == 0 ? v2 : k0 == 1 ? v3 : k0 == 2 ? v4 : v5;
            const uint32_t w3_ = k0 == 0 ? v3 : k0 == 1 ? v4 : k0 == 2 ? v5 : v6;
            const uint32_t w4_ = k0 == 0 ? v4 : k0 == 1 ? v5 : k0 == 2 ? v6 : v7;
            win[c] = bs ? make_uint4(__builtin_amdgcn_alignbyte(w1_, w0_, bs), __builtin_amdgcn_alignbyte(w2_, w1_, bs),
                                     __builtin_amdgcn_alignbyte(w3_, w2_, bs), __builtin_amdgcn_alignbyte(w4_, w3_, bs))
                        : make_uint4(w0_, w1_, w2_, w3_);
          }
          __syncthreads();
        }
      }
      res_key = kq;
      res_w = wi;
      }  // (not resident)
      if (mine) {
        const T* wt = reinterpret_cast<const T*>(win);
#pragma unroll
        for (int s = 0; s < 16; ++s)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            const uint32_t r = (j ? ix[s] >> 16 : ix[s] & 0xFFFFu) - w0;
            if (r < WIN) x[s][j] = wt[r];
          }
      }
      DW_STAMP(4)
    }
  }
  gptr<uint8_t> o = reinterpret_cast<gptr<uint8_t>>(obase) + (uint64_t)lt * 2u * ES;
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    gptr<uint8_t> os = o + s * 256 * ES;
    if (s * 256 + 2 <= rem) {
      if constexpr (ES == 8)
        gst16(os, make_uint4((uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32)));
      else
        *reinterpret_cast<gptr<uint64_t>>(os) = (uint64_t)x[s][0] | ((uint64_t)x[s][1] << 32);
    } else if (s * 256 < rem) {
      *reinterpret_cast<gptr<T>>(os) = x[s][0];
    }
  }
  DW_STAMP(5)
  }  // batches
#ifdef PQG_DIAG
  if (dst) {
    dt_[7] = it;  // batches of this workgroup
    uint64_t* d = chunks[0].cp.dbgbuf + 8ull * blockIdx.x;
    for (int i = 0; i < 8; ++i) d[i] = dt_[i];
  }
#endif
#undef DW_STAMP
}

// Dictionary index streams the level path handed back, when they are expected to be rare (the
// dictionary's index width is within the level path's limit): one workgroup per page of a chunk
// of ES-byte values, index walk then the page's tiles with the gather, as k_lv_fallback does for
// levels.
template <int ES>
__global__ void __launch_bounds__(WG) k_dict_fallback(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                      PageWork* pages, ChunkWork* chunks,
                                                      const uint32_t* __restrict__ tile_page, RunTables rt) {
  __shared__ IndexSmem ism;
  __shared__ TileSmem sm;
  __shared__ int32_t st_s;
  const int p = blockIdx.x;
  if (rt.pflag[p] != PF_BAIL) return;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  const ChunkWork& ck = chunks[pw.chunk];
  if (ck.es != ES) return;
  Stream s;
  if (!get_stream(blob, pw, SS_DICT, ck.cp, s)) return;
  if (ck.dict_page < 0) {  // "Decoder for dict should have been set"
    if (threadIdx.x == 0) report(pages, chunks, p, ST_PANIC);
    return;
  }
  if (!dict_usable(pages, ck)) return;
  if (threadIdx.x < 64) {
    const int32_t st = run_index(blob, blob_len, s, rt.ck + pw.ltile0, rt.runs + (uint64_t)pw.ltile0 * RUN_CAPT,
                                 rt.nruns + pw.ltile0, ism);
    if (threadIdx.x == 0) {
      st_s = st;
      if (st) report(pages, chunks, p, st);
    }
  }
  __syncthreads();
  if (st_s) return;
  DictMaker<ES> mk{blob, pages, chunks};
  for (uint32_t t = pw.ltile0; t < pw.ltile0 + pw.ntiles; ++t) {
    if (threadIdx.x == 0) rt.desc[t] = quarter_desc(blob, pages, chunks, tile_page, rt, SS_DICT, t, 0, RUN_TILE);
    __syncthreads();
    tile_one(blob, blob_len, rt.desc, t, rt.runs, sm, mk);
    __syncthreads();
  }
}

// Tile expand of RLE booleans (data page v2 values) over the listed tiles.
struct BoolMaker {
  PageWork* pages;
  ChunkWork* chunks;
  __device__ TxBool make(const QDesc& d) {
    return TxBool{d.qhi ? gp(chunks[pages[d.page].chunk].val_out) + d.out : gptr<uint8_t>(nullptr)};
  }
  __device__ void done(const QDesc&, uint32_t, TxBool&) {}
};

__global__ void __launch_bounds__(WG) k_texpand_bool(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                     const uint32_t* __restrict__ tl, PageWork* pages,
                                                     ChunkWork* chunks, RunTables rt) {
  __shared__ TileSmem sm;
  if (*rt.nfall == 0) return;
  BoolMaker mk{pages, chunks};
  tile_one(blob, blob_len, rt.desc, tl[blockIdx.x], rt.runs, sm, mk);
}

// Per-page sum of the quarter-tile byte counts -> pages[p].nbytes_out, for the dictionary pages
// of the byte-array chunks the general decoder expanded (k_wexpand_badict).
__global__ void __launch_bounds__(WG) k_page_counts(PageWork* pages, const ChunkWork* chunks,
                                                    const uint32_t* __restrict__ qcount,
                                                    const uint32_t* __restrict__ pflag,
                                                    const uint32_t* __restrict__ nfall) {
  __shared__ uint64_t red[WG / 64];
  if (*nfall == 0) return;  // every stream done by the level path, which set the counts
  const int p = blockIdx.x;
  const PageWork& pw = pages[p];
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  if (pw.encoding != E_RLE_DICTIONARY) return;
  const ChunkWork& ck = chunks[pw.chunk];
  if (ck.es != 0 || ck.lvdict) return;  // (the level path's chunks: counted by their emit or fallback)
  if (pf_level_path(pflag[p])) return;
  const uint32_t q0 = pw.ltile0 * 4u, nq = pw.ntiles * 4u;
  uint64_t s = 0;
  for (uint32_t i = threadIdx.x; i < nq; i += WG) s += qcount[q0 + i];
  const uint64_t t = block_sum_u64(s, red);
  if (threadIdx.x == 0) pages[p].nbytes_out = t;
}

// ------------------------------------------------------------------------------ scan

// Value offsets per page, chunk by chunk (exclusive scan of the data pages' non-null counts,
// restarted at each chunk's first page), each chunk's total and its capacity check (single
// workgroup).
__device__ inline void scan_values(PageWork* pages, ChunkWork* chunks, int npages) {
  seg_scan_pages(
      pages, chunks, npages,
      [&](int p) -> uint64_t {
        const int t = pages[p].page_type;
        return (t == P_DATA || t == P_DATA_V2) ? pages[p].nonnull : 0ull;
      },
      [&](int p, uint64_t excl, uint64_t incl) {
        ChunkWork& ck = chunks[pages[p].chunk];
        pages[p].value_out = excl;
        // a speculative PLAIN copy at the wrong offset or count: the chunk is copied again (mode 2)
        if (ck.spec && (pages[p].page_type == P_DATA || pages[p].page_type == P_DATA_V2) &&
            pages[p].encoding == E_PLAIN && (pages[p].spec_out != excl || pages[p].spec_n != incl - excl))
          atomicOr(&ck.spec_bad, 1u);
        const uint64_t es = (uint64_t)ck.es;
        if (es > 0 && incl > excl && incl * es > ck.val_cap && pages[p].status == 0) report(pages, chunks, p, ST_CAPACITY);
        if ((uint32_t)p == ck.first_page + ck.npages - 1u) ck.res.total_values = incl;
      });
}

__global__ void __launch_bounds__(WG) k_scan_values(PageWork* pages, ChunkWork* chunks, int npages) {
  scan_values(pages, chunks, npages);
}

// Speculative value offsets of the PLAIN pages of ChunkWork::spec chunks: the exclusive prefix of
// the value sections' value counts, chunk by chunk (single workgroup, right after k_prepare).
__global__ void __launch_bounds__(WG) k_spec_scan(PageWork* pages, ChunkWork* chunks, int npages) {
  seg_scan_pages(
      pages, chunks, npages, [&](int p) -> uint64_t { return pages[p].spec_n; },
      [&](int p, uint64_t excl, uint64_t) { pages[p].spec_out = excl; });
}

// ------------------------------------------------------------------------------ PLAIN

// PLAIN fixed-width values: grid.y over the listed pages (PLAIN pages of fixed-width chunks),
// grid.x over 16-byte chunks of a page's output: the page's `nonnull * es` value bytes go to its
// chunk's values + value_out * es. Source alignment is arbitrary (the value section follows the
// level streams): dword loads + v_alignbyte; the destination is chunked on 16-byte boundaries of
// the output so stores are dwordx4 except at page edges.
//
// mode 0: at the page's value offset (after the level decode and the offset scan);
// mode 1 (speculative, ChunkWork::spec chunks, on a side stream beside the level decode): the
//   value section's values (spec_n) at the offsets their counts give (spec_out), so the copy does
//   not wait for the def levels; the offset scan flags the chunk when a page's count or offset
//   turns out different (ChunkWork::spec_bad);
// mode 2: the pages of flagged chunks again, as mode 0.
#ifndef PQG_PC_U
#define PQG_PC_U 2
#endif
constexpr uint32_t PC_U = PQG_PC_U;  // 16-byte chunks per lane in flight (k_plain_copy)

__global__ void __launch_bounds__(WG) k_plain_copy(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                   PageWork* pages, ChunkWork* chunks,
                                                   const uint32_t* __restrict__ pl, int mode) {
  const uint32_t p = pl[blockIdx.y];
  const PageWork& pwr = pages[p];
  if (pwr.status != 0) return;
  const ChunkWork& ck = chunks[pwr.chunk];
  if (mode == 2 && !ck.spec_bad) return;
  const uint64_t es = (uint64_t)ck.es;
  const gptr<uint8_t> __restrict__ out = gp(ck.val_out);
  const uint64_t nv = mode == 1 ? pwr.spec_n : pwr.nonnull;
  const uint64_t nbytes = nv * es;
  if (nbytes > pwr.val_bytes) {  // eof_err!("Not enough bytes to decode")
    if (blockIdx.x == 0 && threadIdx.x == 0) report(pages, chunks, (int)p, ST_EOF);
    return;
  }
  const uint64_t src = pwr.base + pwr.val_off;
  const uint64_t dst = (mode == 1 ? pwr.spec_out : pwr.value_out) * es;
  if (mode == 1 && dst + nbytes > ck.val_cap) return;  // (the offset scan flags it: copied again)
  const uint64_t dend = dst + nbytes;
  const uint64_t c0 = dst & ~15ull;
  // PC_U chunks per lane per step (WG * 16 bytes apart: each wave-instruction stays contiguous),
  // their loads all issued before the stores. A chunk's 16 source bytes start sh bytes into an
  // aligned 16-byte source chunk (the same sh for every chunk of the page): each lane loads its
  // aligned chunk with one 16-byte load and takes the next one from the lane above (DPP wave
  // shift; lane 63 loads it), then v_alignbyte picks the 16 bytes.
  const uint64_t stepb = (uint64_t)WG * 16ull;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t sh = (uint32_t)((src - dst) & 15u), q4 = sh >> 2, r8 = (sh & 3u);
  const uint64_t wbase = c0 + (uint64_t)(threadIdx.x >> 6) * 1024u;  // (wave-uniform: the loop below is too)
  for (uint64_t cw = wbase + (uint64_t)blockIdx.x * stepb * PC_U; cw < dend; cw += (uint64_t)gridDim.x * stepb * PC_U) {
    uint4 v[PC_U];
    bool full[PC_U];
    uint4 A[PC_U], N[PC_U];
#pragma unroll
    for (uint32_t u = 0; u < PC_U; ++u) {
      const uint64_t c = cw + u * stepb + lane * 16u;
      full[u] = c >= dst && c + 16 <= dend;
      const uint64_t a = src + (c - dst) - sh;  // aligned source chunk (wraps below the blob: guarded)
      if (a + 16 <= blob_len) {
        const pqg_u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const pqg_u32x4*>(blob + a));
        A[u] = make_uint4(t[0], t[1], t[2], t[3]);
      } else {
        A[u] = gload_u128_tail(blob, blob_len, a);
      }
      if (lane == 63u && sh) N[u] = a + 32 <= blob_len ? *reinterpret_cast<const uint4*>(blob + a + 16)
                                                       : gload_u128_tail(blob, blob_len, a + 16);
    }
#pragma unroll
    for (uint32_t u = 0; u < PC_U; ++u) {
      if (sh == 0) {
        v[u] = A[u];
        continue;
      }
      uint4 n;  // lane + 1's aligned chunk (DPP wave_shl:1)
      n.x = (uint32_t)__builtin_amdgcn_update_dpp((int)N[u].x, (int)A[u].x, 0x130, 0xf, 0xf, false);
      n.y = (uint32_t)__builtin_amdgcn_update_dpp((int)N[u].y, (int)A[u].y, 0x130, 0xf, 0xf, false);
      n.z = (uint32_t)__builtin_amdgcn_update_dpp((int)N[u].z, (int)A[u].z, 0x130, 0xf, 0xf, false);
      n.w = (uint32_t)__builtin_amdgcn_update_dpp((int)N[u].w, (int)A[u].w, 0x130, 0xf, 0xf, false);
      const uint32_t w[8] = {A[u].x, A[u].y, A[u].z, A[u].w, n.x, n.y, n.z, n.w};
      uint32_t o[4];
      switch (q4) {  // (wave-uniform)
        case 0:
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = __builtin_amdgcn_alignbyte(w[j + 1], w[j], r8);
          break;
        case 1:
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = __builtin_amdgcn_alignbyte(w[j + 2], w[j + 1], r8);
          break;
        case 2:
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = __builtin_amdgcn_alignbyte(w[j + 3], w[j + 2], r8);
          break;
        default:
#pragma unroll
          for (int j = 0; j < 4; ++j) o[j] = __builtin_amdgcn_alignbyte(w[j + 4], w[j + 3], r8);
          break;
      }
      v[u] = make_uint4(o[0], o[1], o[2], o[3]);
    }
#pragma unroll
    for (uint32_t u = 0; u < PC_U; ++u) {
      const uint64_t c = cw + u * stepb + lane * 16u;
      if (full[u]) {
        gst16(out + c, v[u]);
      } else if (c < dend) {  // a chunk shared with a neighbouring page: its bytes only
        const uint64_t lo = c < dst ? dst : c;
        const uint64_t hi = (c + 16 < dend) ? c + 16 : dend;
        for (uint64_t b = lo; b < hi; ++b) out[b] = blob[src + (b - dst)];
      }
    }
  }
}

// PLAIN booleans (decoding.rs:188-204 via BitReader::get_batch::<bool>): LSB-first bits of the
// value section, one byte (0/1) per value, one workgroup per listed tile; every 16-byte chunk of
// the output (aligned on the chunk's buffer) from the 16 bits at its values' bit offset.
__global__ void __launch_bounds__(WG) k_plain_bool(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                   PageWork* pages, ChunkWork* chunks,
                                                   const uint32_t* __restrict__ tile_page,
                                                   const uint32_t* __restrict__ tl) {
  const uint32_t gt = tl[blockIdx.x], p = tile_page[gt];
  const PageWork& pw = pages[p];
  if (pw.status != 0) return;
  const ChunkWork& ck = chunks[pw.chunk];
  const gptr<uint8_t> __restrict__ out = gp(ck.val_out);
  const uint64_t n = pw.nonnull;
  if ((n + 7) / 8 > pw.val_bytes && n > (uint64_t)pw.val_bytes * 8) {
    if (threadIdx.x == 0 && gt == pw.ltile0) report(pages, chunks, (int)p, ST_EOF);
    return;
  }
  const uint64_t v0 = (uint64_t)(gt - pw.ltile0) * RUN_TILE;
  if (v0 >= n) return;
  const uint64_t v1 = v0 + RUN_TILE < n ? v0 + RUN_TILE : n;
  const uint64_t src = pw.base + pw.val_off;
  const uint64_t dst = pw.value_out;
  const uint64_t lo_b = dst + v0, hi_b = dst + v1;
  for (uint64_t c = (lo_b & ~15ull) + (uint64_t)threadIdx.x * 16ull; c < hi_b; c += (uint64_t)WG * 16ull) {
    const uint64_t lo = c < lo_b ? lo_b : c;
    const uint64_t hi = (c + 16 < hi_b) ? c + 16 : hi_b;
    if (lo == c && hi == c + 16) {
      const uint64_t vi = c - dst;  // value (bit) index of the chunk's first output
      const uint64_t a = src + (vi >> 3);
      const uint32_t x = (gbyte(blob, blob_len, a) | (gbyte(blob, blob_len, a + 1) << 8) |
                          (gbyte(blob, blob_len, a + 2) << 16)) >> (vi & 7u);
      uint32_t d[4];
#pragma unroll
      for (uint32_t t = 0; t < 4; ++t) d[t] = (((x >> (4u * t)) & 15u) * 0x204081u) & 0x01010101u;
      gst16(out + c, make_uint4(d[0], d[1], d[2], d[3]));
    } else {
      for (uint64_t b = lo; b < hi; ++b) {
        const uint64_t vi = b - dst;
        out[b] = (uint8_t)((blob[src + (vi >> 3)] >> (vi & 7u)) & 1u);
      }
    }
  }
}

// ------------------------------------------------------------------------------ launchers

extern "C" {

hipError_t pqg_launch_lv(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages, ChunkWork* chunks,
                         int sel, uint32_t widths, const uint64_t* dsrc, const uint32_t* dlen, uint64_t* vsrc,
                         uint32_t* vlen, RunTables rt, LevelTables lt, hipStream_t s, hipEvent_t front = nullptr);

hipError_t pqg_launch_prepare(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages,
                              ChunkWork* chunks, uint32_t* tile_page, PrepInit ini, hipStream_t s) {
  hipLaunchKernelGGL(k_prepare, dim3(npages), dim3(64), 0, s, blob, blob_len, pages, npages, chunks, tile_page, ini);
  return hipGetLastError();
}

hipError_t pqg_launch_run_index(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages,
                                ChunkWork* chunks, int sel, RunTables rt, hipStream_t s) {
  hipLaunchKernelGGL(k_run_index, dim3(npages), dim3(64), 0, s, blob, blob_len, pages, chunks, sel, rt, 0);
  return hipGetLastError();
}

hipError_t pqg_launch_quarter_desc(const uint8_t* blob, PageWork* pages, ChunkWork* chunks, const uint32_t* tile_page,
                                   const uint32_t* tl, uint32_t ntl, RunTables rt, int sel, hipStream_t s) {
  if (ntl)
    hipLaunchKernelGGL(k_quarter_desc, dim3((ntl * 4 + WG - 1) / WG), dim3(WG), 0, s, blob, pages, chunks, tile_page,
                       tl, ntl, rt, sel);
  return hipGetLastError();
}

hipError_t pqg_launch_page_counts(PageWork* pages, int npages, ChunkWork* chunks, RunTables rt, hipStream_t s) {
  hipLaunchKernelGGL(k_page_counts, dim3(npages), dim3(WG), 0, s, pages, chunks, rt.qcount, rt.pflag, rt.nfall);
  return hipGetLastError();
}

// Level stream `which` (0 def, 1 rep) of every chunk that reads it: the window-parallel level path
// (levels + per-page non-null counts, pqg_levels.hip), then the general hybrid decoder for the
// streams it hands back (one workgroup per handed-back page; the others exit at once). `widths`:
// bit mask of the streams' bit widths (1 << w). scan: the value-offset scan runs in that last
// kernel's last workgroup. front: recorded after the front end (plan .. compact), when given.
hipError_t pqg_launch_levels(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages, ChunkWork* chunks,
                             int which, uint32_t widths, const uint32_t* tile_page, RunTables rt, LevelTables lt,
                             hipStream_t s, hipEvent_t* kev, int scan, hipEvent_t front) {
  const int sel = which ? SS_REP : SS_DEF;
  if (kev) (void)hipEventRecord(kev[0], s);
  hipError_t e = pqg_launch_lv(blob, blob_len, pages, npages, chunks, sel, widths, nullptr, nullptr, nullptr, nullptr,
                               rt, lt, s, front);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_lv_fallback, dim3(npages < LF_GRID ? npages : LF_GRID), dim3(WG), 0, s, blob, blob_len, pages,
                     chunks, tile_page, sel, rt, lt.ctr + 1, scan, npages);
  if (kev) (void)hipEventRecord(kev[1], s);
  return hipGetLastError();
}

hipError_t pqg_launch_scan(PageWork* pages, int npages, ChunkWork* chunks, hipStream_t s) {
  hipLaunchKernelGGL(k_scan_values, dim3(1), dim3(WG), 0, s, pages, chunks, npages);
  return hipGetLastError();
}

// RLE_DICTIONARY values of fixed-width chunks. Chunks of 4- and 8-byte values with a dictionary of
// at most 2^dict_maxw entries take the hybrid-stream path (pqg_launch_lv with SS_DICT, launched by
// the host for every dictionary chunk on it), their rare leftovers one workgroup per page here
// (lv_es: bit mask of those value sizes). The other chunks' pages (larger dictionaries: wider
// indices, gathers served from L2; other value sizes) take the tiled expand over the listed
// tiles (tl_all: every such tile; tl[i] / ntl[i]: those of value size 1, 4, 8, 12), their index
// pass (pqg_launch_run_index with SS_DICT) having run before.
hipError_t pqg_launch_dict(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages, ChunkWork* chunks,
                           const uint32_t* tile_page, uint32_t lv_es, const uint32_t* const* tl,
                           const uint32_t* ntl, const uint32_t* tl_all, uint32_t ntl_all,
                           const uint32_t* const* wl, const uint32_t* wn, uint16_t* didx, RunTables rt,
                           hipStream_t s, hipEvent_t* kev) {
  // (the dictionary pages' checks ran in k_prepare)
  if (kev) (void)hipEventRecord(kev[0], s);
  if (lv_es & 8)
    hipLaunchKernelGGL((k_dict_fallback<8>), dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, chunks, tile_page, rt);
  if (lv_es & 4)
    hipLaunchKernelGGL((k_dict_fallback<4>), dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, chunks, tile_page, rt);
  if (ntl_all) {
    hipLaunchKernelGGL(k_tile_desc, dim3((ntl_all + WG - 1) / WG), dim3(WG), 0, s, blob, pages, chunks, tile_page,
                       tl_all, ntl_all, rt, (int)SS_DICT);
    if (ntl[0]) hipLaunchKernelGGL((k_texpand_dict<1>), dim3(ntl[0]), dim3(WG), 0, s, blob, blob_len, tl[0], pages, chunks, rt);
    if (ntl[1]) hipLaunchKernelGGL((k_texpand_dict<4>), dim3(ntl[1]), dim3(WG), 0, s, blob, blob_len, tl[1], pages, chunks, rt);
    if (ntl[2]) hipLaunchKernelGGL((k_texpand_dict<8>), dim3(ntl[2]), dim3(WG), 0, s, blob, blob_len, tl[2], pages, chunks, rt);
    if (ntl[3]) hipLaunchKernelGGL((k_texpand_dict<12>), dim3(ntl[3]), dim3(WG), 0, s, blob, blob_len, tl[3], pages, chunks, rt);
    // windowed gathers (wl[0] / wl[1]: tiles of 4- / 8-byte values, slots of didx in that order)
    uint16_t* slot = didx;
    if (wn[0] + wn[1]) (void)hipMemsetAsync(rt.hard, 0, 2 * sizeof(uint32_t), s);
    uint32_t* hl = rt.hard + 2;
    for (int k = 0; k < 2; ++k) {
      if (!wn[k]) continue;
      // the tiles k_dict_win does not decode itself (none at the benchmark's shape): marked, then
      // expanded by a grid striding over them
      hipLaunchKernelGGL(k_didx_mark, dim3((wn[k] + WG - 1) / WG), dim3(WG), 0, s, wl[k], wn[k], rt, rt.hard + k, hl);
      hipLaunchKernelGGL(k_texpand_didx, dim3(wn[k] < 1024u ? wn[k] : 1024u), dim3(WG), 0, s, blob, blob_len, wl[k],
                         pages, chunks, rt, rt.hard + k, hl, slot);
      hl += wn[k];
      // persistent workgroups (one per CU: the window takes the LDS), batches of DW_TPW tiles in turn
      const uint32_t nbt = (wn[k] + DW_TPW - 1) / DW_TPW;
      const dim3 g(nbt < PQG_DW_GRID ? nbt : PQG_DW_GRID);
      if (k == 0)
        hipLaunchKernelGGL((k_dict_win<4>), g, dim3(DW_NT), 0, s, blob, blob_len, wl[k], wn[k], pages, chunks, rt, slot);
      else
        hipLaunchKernelGGL((k_dict_win<8>), g, dim3(DW_NT), 0, s, blob, blob_len, wl[k], wn[k], pages, chunks, rt, slot);
      slot += (uint64_t)wn[k] * RUN_TILE;
    }
  }
  if (kev) (void)hipEventRecord(kev[1], s);
  return hipGetLastError();
}

// PLAIN values: fixed-width over the listed pages (pl, npl; max_bytes: the largest of them) and
// booleans over the listed tiles (tlb, ntlb).
hipError_t pqg_launch_plain(const uint8_t* blob, uint64_t blob_len, PageWork* pages, ChunkWork* chunks,
                            const uint32_t* tile_page, const uint32_t* pl, uint32_t npl, uint64_t max_bytes,
                            const uint32_t* tlb, uint32_t ntlb, hipStream_t s) {
  if (npl) {
    // PC_U x 16 bytes per lane (k_plain_copy): more, shorter workgroups copy faster (2 or 4
    // iterations per workgroup measured 1.30 -> 1.33-1.41 ms for 8 GB; 2 chunks per lane instead
    // of 4: 1.257 -> 1.248 ms, 8: 1.32 ms)
    uint64_t nch = (max_bytes + 16ull * PC_U * WG - 1) / (16ull * PC_U * WG) + 1;
    if (nch > 4096) nch = 4096;
    hipLaunchKernelGGL(k_plain_copy, dim3((unsigned)nch, npl), dim3(WG), 0, s, blob, blob_len, pages, chunks, pl, 0);
  }
  if (ntlb)
    hipLaunchKernelGGL(k_plain_bool, dim3(ntlb), dim3(WG), 0, s, blob, blob_len, pages, chunks, tile_page, tlb);
  return hipGetLastError();
}

// The speculative PLAIN copy of ChunkWork::spec chunks (pages pl, npl): offsets scan + copy on
// `side` (mode 1), launched after k_prepare; the re-copy of flagged chunks (mode 2) on `s` once the
// offset scan has run there and the side stream's copy is joined.
hipError_t pqg_launch_plain_spec(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages,
                                 ChunkWork* chunks, const uint32_t* pl, uint32_t npl, uint32_t gx,
                                 hipStream_t side) {
  hipLaunchKernelGGL(k_spec_scan, dim3(1), dim3(WG), 0, side, pages, chunks, npages);
  // gx workgroups per page: the copy holds a few workgroups per CU and leaves the rest of the
  // chip to the level decode it runs beside (a full-size grid takes every CU and the level
  // kernels wait for it)
  hipLaunchKernelGGL(k_plain_copy, dim3(gx, npl), dim3(WG), 0, side, blob, blob_len, pages, chunks, pl, 1);
  return hipGetLastError();
}

hipError_t pqg_launch_plain_fix(const uint8_t* blob, uint64_t blob_len, PageWork* pages, ChunkWork* chunks,
                                const uint32_t* pl, uint32_t npl, hipStream_t s) {
  hipLaunchKernelGGL(k_plain_copy, dim3(8, npl), dim3(WG), 0, s, blob, blob_len, pages, chunks, pl, 2);
  return hipGetLastError();
}

// RLE booleans (data page v2 values, RleValueDecoder<bool>): the level path (one byte per value)
// with the general hybrid decoder for the streams it hands back, over the listed tiles (the tiles
// of the pages of RLE-encoded BOOLEAN chunks).
hipError_t pqg_launch_rle_bool(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages, ChunkWork* chunks,
                               const uint32_t* tile_page, const uint32_t* tl, uint32_t ntl, RunTables rt,
                               LevelTables lt, hipStream_t s) {
  hipError_t e = pqg_launch_lv(blob, blob_len, pages, npages, chunks, SS_BOOL, 2u, nullptr, nullptr, nullptr, nullptr,
                               rt, lt, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_run_index, dim3(npages), dim3(64), 0, s, blob, blob_len, pages, chunks, (int)SS_BOOL, rt, 1);
  if (ntl) {
    hipLaunchKernelGGL(k_tile_desc, dim3((ntl + WG - 1) / WG), dim3(WG), 0, s, blob, pages, chunks, tile_page, tl, ntl,
                       rt, (int)SS_BOOL);
    hipLaunchKernelGGL(k_texpand_bool, dim3(ntl), dim3(WG), 0, s, blob, blob_len, tl, pages, chunks, rt);
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
