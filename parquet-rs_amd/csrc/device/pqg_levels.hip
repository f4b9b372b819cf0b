// pqg_levels.hip — level streams (def / rep levels) and RLE boolean values: the
// RLE/bit-packing hybrid (RleDecoder::reload / get_batch, rle.rs:352-434, 490-508;
// LevelDecoder::get, levels.rs:249-271), decoded window-parallel.
//
// Run headers sit at data-dependent offsets: where a header starts depends on every header
// before it. Instead of walking that chain once per page, every 1 KiB window of every stream is
// solved independently for ALL the places the chain could enter it:
//
//   k_lv_plan    windows per page stream (exclusive scan), eligibility of each stream.
//   k_lv_win     one wave per window: every byte position of the window is parsed as if a header
//                started there (next header offset, output count), then pointer jumping (ten
//                rounds of J[i] = J[J[i]], C[i] += C[J[i]]) gives, for every position, where its
//                chain leaves the window and how many outputs it produces on the way. The
//                answers for the positions a chain can enter at (the first 64 * w bytes: a
//                header plus at most 63 bit-packed groups) go to a table.
//   k_lv_stitch  one wave per page: follows the window tables from offset 0 (one lookup per
//                window) to each window's true entry and first output.
//   k_lv_emit    one wave per window: pointer jumping again, now marking the positions
//                reachable from the true entry (the window's true headers); they are parsed in
//                parallel, a wave scan places their runs, and the window's outputs are written:
//                int16 levels (column/reader.rs:162-163) or one byte per boolean, 16-byte
//                stores (element stores for the groups shared with a neighbouring window). Def
//                streams add their count of outputs == max_def (the non-null count read_batch
//                uses, column/reader.rs:212-226) to the page.
//
// Streams off the common path (a header form the fast parse does not take, a stream that ends
// before its outputs, truncated payload, an RLE value wider than sw, an entry past the table)
// go to the general decoder (pqg_runs.hpp / pqg_texpand.hpp), which reproduces every reference
// error. Work is proportional to stream bytes, not to the number of headers, and no page waits
// on a serial walk longer than one table lookup per 1 KiB.
#include "pqg_runs.hpp"

namespace pqg {

constexpr uint32_t LV_WIN = 1024;                  // stream bytes per window (one wave)
constexpr uint32_t LV_PPL = LV_WIN / WAVE;         // positions per lane (16)
constexpr uint32_t LV_STG = LV_WIN + 48;           // staged bytes (+ alignment slack, read-ahead)
constexpr uint32_t LV_STG_CH = LV_STG / 16;        // 16-byte chunks (67)
constexpr uint32_t LV_RCAP = LV_WIN;               // runs per window
constexpr uint32_t LV_ROUNDS = 10;                 // 2^10 = LV_WIN: chains of any length
constexpr uint32_t LV_SERIAL = 64;                 // k_lv_emit: windows with at most this many
                                                   // true headers are walked by one lane
constexpr uint32_t LV_BM = 16384;                  // one-bit outputs per bitmap chunk
constexpr uint32_t LV_NONE = 0xFFFFFFFFu;          // window not on the true chain
// jump-table values >= LV_WIN are terminal: the chain leaves the window at W0 + value, or
constexpr uint32_t LV_J_FAR = 0xFFFDu;             //   leaves it beyond W0 + 0xFFFC,
constexpr uint32_t LV_J_END = 0xFFFEu;             //   reaches the end of the stream,
constexpr uint32_t LV_J_DEAD = 0xFFFFu;            //   meets a header the fast parse refuses

// Bit widths the window path takes: levels up to 16 bits (RLE values of <= 2 bytes).
__device__ inline bool lv_width_ok(uint32_t w) { return w >= 1 && w <= 16; }

// Entry offsets a window table keeps: a chain enters a window at most one hop past its start,
// and a hop is a <= 4-byte header plus <= 63 groups of w bytes or a <= 2-byte value.
__device__ __host__ inline uint32_t lv_ent(uint32_t w) {
  return w == 1 ? 64u : w == 2 ? 128u : w <= 4 ? 256u : w <= 8 ? 512u : 1024u;
}

// Wave-private LDS of the window kernels. Lane l owns positions j * 64 + l (j < 16), so the
// wave's accesses to its own entries are consecutive (conflict-free).
struct LvWave {
  uint32_t stage[LV_STG / 4];
  union {
    uint2 JC[LV_WIN];       // jump table: (next position | terminal code, outputs on the way)
    struct {
      uint32_t rstart[LV_RCAP + 1];  // k_lv_emit, after the jumps: run list
      uint32_t rinfo[LV_RCAP];
    } runs;
  };
  union {
    uint8_t R[LV_WIN];           // k_lv_emit: 1 = position reachable from the true entry
    uint32_t bm[LV_BM / 32];     // k_lv_emit, one-bit outputs: a chunk of them as a bitmap
  };
};

struct LvSmem {
  LvWave wv[WG / WAVE];
};

// Inclusive scan of x over the wave's lanes with DPP row shifts and broadcasts (no LDS).
__device__ inline uint32_t wave_incl_scan_u32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS accesses have completed
  __builtin_amdgcn_wave_barrier();
}

// Header at stream position p (stage byte index rel), general form: varints of <= 4 bytes,
// <= 2 value bytes. False for anything else, including a header or RLE value that runs past
// the stream end.
__device__ inline bool lv_parse(const uint32_t* st, uint32_t rel, uint32_t p, uint32_t slen,
                                uint32_t w, uint32_t vb, uint32_t& nxt, uint32_t& cnt,
                                uint32_t& val, bool& bp) {
  if (p >= slen) return false;
  const uint64_t x = lload_u64(st, rel);
  const uint32_t lo = (uint32_t)x;
  uint32_t h, hl;
  if (!(lo & 0x80u)) {
    h = lo & 0x7Fu;
    hl = 1;
  } else {
    const uint32_t t = ~lo & 0x80808080u;
    if (!t) return false;  // varint longer than 4 bytes: not the writer's form
    hl = ((uint32_t)__builtin_ctz(t) >> 3) + 1u;
    const uint32_t y = lo & 0x7F7F7F7Fu;
    h = (y & 0x7Fu) | ((y >> 1) & 0x3F80u) | ((y >> 2) & 0x1FC000u) | ((y >> 3) & 0xFE00000u);
    if (hl < 4) h &= (1u << (7 * hl)) - 1u;
  }
  if (hl > slen - p) return false;
  if (h & 1u) {
    bp = true;
    const uint32_t g = h >> 1;
    cnt = g * 8u;
    val = p + hl;
    const uint64_t nx = (uint64_t)p + hl + (uint64_t)g * w;
    nxt = nx > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)nx;
  } else {
    bp = false;
    cnt = h >> 1;
    if (vb > slen - p - hl) return false;
    const uint32_t v = (uint32_t)(x >> (8 * hl));
    val = vb == 1 ? (v & 0xFFu) : (v & 0xFFFFu);
    nxt = p + hl + vb;
  }
  return true;
}

// Header at stream position p for the window kernels: branch-free for varints of 1-4 bytes
// (run lengths < 2^27; every header the reference writer emits, rle.rs:167-178), reading a
// third dword only for an RLE value past the first 4 bytes. Longer varints, and headers
// running past the stream end, return false (dead): a true chain that meets one goes to the
// general decoder.
__device__ inline bool lv_parse4(const uint32_t* st, uint32_t rel, uint32_t p, uint32_t slen,
                                 uint32_t w, uint32_t vb, uint32_t& nxt, uint32_t& cnt,
                                 uint32_t& val, bool& bp) {
  const uint32_t wi = rel >> 2, sh = (rel & 3u) * 8u;
  const uint32_t d1 = st[wi + 1];
  const uint32_t x = __builtin_amdgcn_alignbit(d1, st[wi], sh);  // bytes p .. p+3
  const uint32_t c0 = (x >> 7) & 1u, c1 = (x >> 15) & 1u, c2 = (x >> 23) & 1u, c3 = x >> 31;
  const uint32_t c01 = c0 & c1, c012 = c01 & c2;
  const uint32_t hl = 1u + c0 + c01 + c012;
  const uint32_t h = (x & 0x7Fu) | (c0 ? ((x >> 1) & 0x3F80u) : 0u) | (c01 ? ((x >> 2) & 0x1FC000u) : 0u) |
                     (c012 ? ((x >> 3) & 0xFE00000u) : 0u);
  bp = (h & 1u) != 0;
  const uint32_t g = h >> 1;
  cnt = bp ? g * 8u : g;
  uint32_t v = 0;
  if (!bp) {
    const uint32_t vm = vb == 1 ? 0xFFu : 0xFFFFu;
    if (hl + vb <= 4u) {
      v = (x >> (8u * hl)) & vm;
    } else {
      const uint32_t y = __builtin_amdgcn_alignbit(st[wi + 2], d1, sh);  // bytes p+4 .. p+7
      v = (uint32_t)((((uint64_t)y << 32) | x) >> (8u * hl)) & vm;
    }
  }
  val = bp ? p + hl : v;
  const uint32_t len = bp ? hl + g * w : hl + vb;  // g < 2^27, w <= 16: < 2^32
  nxt = p + len;
  return !(c012 & c3) && p < slen && len <= slen - p;
}

// A window's stream: the page stream `sel`, its window k (stage origin, bytes).
struct LvWin {
  Stream s;
  uint32_t p;      // page
  uint32_t k;      // window of the page
  uint32_t W0;     // stream offset of the window
  uint32_t sb;     // stage byte of stream offset W0
};

// Stage stream bytes [W0, W0 + LV_WIN + 32) (16-byte aligned loads, guarded at the blob end).
__device__ inline void lv_stage(const uint8_t* __restrict__ blob, uint64_t blob_len, const LvWin& x,
                                uint32_t* stage, uint32_t& sb) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t A = (x.s.S + x.W0) & ~15ull;
  sb = (uint32_t)(x.s.S + x.W0 - A);
#pragma unroll
  for (uint32_t c = lane; c < LV_STG_CH; c += WAVE) {
    const uint64_t a = A + (uint64_t)c * 16u;
    const uint4 v = a + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
    reinterpret_cast<uint4*>(stage)[c] = v;
  }
  wave_lds_sync();
}

// Page and window of global window index g (wbase: exclusive scan of windows per page).
__device__ inline uint32_t lv_page_of(const uint32_t* __restrict__ wbase, uint32_t npages, uint32_t g) {
  uint32_t lo = 0, hi = npages;  // last page with wbase[p] <= g
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (wbase[mid] <= g) lo = mid;
    else hi = mid;
  }
  return lo;
}

__device__ inline bool lv_stream(const uint8_t* blob, const PageWork& pw, int sel, const ColumnParams& cp,
                                 Stream& s) {
  return get_stream(blob, pw, sel, cp, s) && pw.status == 0 && !s.err && s.kind == LK_RLE &&
         lv_width_ok((uint32_t)s.w);
}

// Hand page p to the general decoder (once).
__device__ inline void lv_bail(RunTables& rt, uint32_t p) {
  if (atomicCAS(&rt.pflag[p], PF_PAGE, PF_BAIL) == PF_PAGE) atomicAdd(rt.nfall, 1u);
}

// Own positions' first hop (window-relative next offset, terminal codes >= LV_WIN) and output
// count. Position i = j * 64 + lane.
__device__ inline void lv_first_hops(const uint32_t* stage, uint32_t sb, uint32_t W0, uint32_t slen,
                                     uint32_t w, uint32_t vb, uint32_t (&jv)[LV_PPL],
                                     uint32_t (&cv)[LV_PPL]) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (uint32_t j = 0; j < LV_PPL; ++j) {
    const uint32_t i = j * WAVE + lane;
    const uint32_t q = W0 + i;
    uint32_t nx, c = 0, v;
    bool bp;
    uint32_t jj;
    if (q >= slen) {
      jj = LV_J_END;
    } else if (!lv_parse4(stage, i + sb, q, slen, w, vb, nx, c, v, bp)) {
      jj = LV_J_DEAD;
      c = 0;
    } else {
      const uint32_t d = nx - W0;
      jj = (d < 0xFFFDu ? d : LV_J_FAR) | 0x10000u;  // one header on the way (hop count << 16)
    }
    jv[j] = jj;
    cv[j] = c;
  }
}

// ------------------------------------------------------------------------------ k_lv_plan
// One workgroup: per page the stream's windows (exclusive scan into wbase), and the page flag:
// PF_PAGE (level path) or PF_BAIL (general decoder). Def streams start their count at 0.
__global__ void __launch_bounds__(WG) k_lv_plan(const uint8_t* __restrict__ blob, PageWork* pages, int npages,
                                                ColumnParams cp, int sel, RunTables rt, LevelTables lt) {
  __shared__ uint32_t wsum[WG / 64];
  __shared__ uint32_t carry_s;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < npages; base += WG) {
    const int p = base + (int)threadIdx.x;
    uint32_t nw = 0;
    if (p < npages) {
      const PageWork& pw = pages[p];
      Stream s;
      uint32_t flag = 0;
      if (get_stream(blob, pw, sel, cp, s)) {
        if (lv_stream(blob, pw, sel, cp, s) && (s.n == 0 || s.slen > 0)) {
          flag = PF_PAGE;
          nw = s.n ? (s.slen + LV_WIN - 1) / LV_WIN : 0u;
          if (sel == SS_DEF) pages[p].nonnull = 0;
        } else {
          flag = PF_BAIL;
          atomicAdd(rt.nfall, 1u);
        }
      }
      rt.pflag[p] = flag;
    }
    uint32_t incl = nw;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(incl, d, 64);
      if ((threadIdx.x & 63) >= (unsigned)d) incl += y;
    }
    if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint32_t pre = carry_s;
    for (int k = 0; k < (int)(threadIdx.x >> 6); ++k) pre += wsum[k];
    if (p < npages) lt.wbase[p] = pre + incl - nw;
    __syncthreads();
    if (threadIdx.x == WG - 1) carry_s = pre + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) lt.wbase[npages] = carry_s;
}

// ------------------------------------------------------------------------------ k_lv_win
__global__ void __launch_bounds__(WG) k_lv_win(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                               const PageWork* __restrict__ pages, int npages,
                                               ColumnParams cp, int sel, RunTables rt, LevelTables lt) {
  __shared__ LvSmem sm;
  const uint32_t wid = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  LvWave& W = sm.wv[wid];
  const uint32_t total = lt.wbase[npages];
  for (uint32_t g = blockIdx.x * (WG / WAVE) + wid; g < total; g += gridDim.x * (WG / WAVE)) {
    LvWin x;
    x.p = lv_page_of(lt.wbase, (uint32_t)npages, g);
    const PageWork& pw = pages[x.p];
    if (rt.pflag[x.p] != PF_PAGE || !lv_stream(blob, pw, sel, cp, x.s)) continue;
    x.k = g - lt.wbase[x.p];
    x.W0 = x.k * LV_WIN;
    const uint32_t w = (uint32_t)x.s.w, vb = (w + 7u) >> 3, slen = x.s.slen;
    lv_stage(blob, blob_len, x, W.stage, x.sb);
    uint32_t jv[LV_PPL], cv[LV_PPL];
    lv_first_hops(W.stage, x.sb, x.W0, slen, w, vb, jv, cv);
#pragma unroll
    for (uint32_t j = 0; j < LV_PPL; ++j) W.JC[j * WAVE + lane] = make_uint2(jv[j], cv[j]);
    wave_lds_sync();
    // pointer jumping: after round r, jv[j] is 2^(r+1) hops on (or terminal) and cv[j] the
    // outputs along the way (saturating); the high half of jv counts the headers passed (also
    // saturating). Stops once every chain has left the window.
#pragma unroll 1
    for (uint32_t r = 0; r < LV_ROUNDS; ++r) {
      bool live = false;
#pragma unroll
      for (uint32_t j = 0; j < LV_PPL; ++j) live |= (jv[j] & 0xFFFFu) < LV_WIN;
      if (!__any(live)) break;
      uint2 nx[LV_PPL];
#pragma unroll
      for (uint32_t j = 0; j < LV_PPL; ++j) {
        const uint32_t t = jv[j] & 0xFFFFu;
        nx[j] = t < LV_WIN ? W.JC[t] : make_uint2(t, 0u);
      }
      wave_lds_sync();
#pragma unroll
      for (uint32_t j = 0; j < LV_PPL; ++j) {
        const uint32_t s2 = cv[j] + nx[j].y;
        cv[j] = s2 < cv[j] ? 0xFFFFFFFFu : s2;
        const uint32_t hs = (jv[j] >> 16) + (nx[j].x >> 16);
        jv[j] = (nx[j].x & 0xFFFFu) | ((hs < 0xFFFFu ? hs : 0xFFFFu) << 16);
        W.JC[j * WAVE + lane] = make_uint2(jv[j], cv[j]);
      }
      wave_lds_sync();
    }
    // table of the entry offsets: (exit offset from W0 or terminal code | headers << 16, outputs)
    const uint32_t ent = lv_ent(w);
    uint2* tab = lt.tab + (uint64_t)g * ent;
#pragma unroll
    for (uint32_t j = 0; j < LV_PPL; ++j) {
      const uint32_t i = j * WAVE + lane;
      if (i < ent) tab[i] = make_uint2(jv[j], cv[j]);
    }
  }
}

// ------------------------------------------------------------------------------ k_lv_stitch
// One wave per page: the true entry and first output of every window of the page.
__global__ void __launch_bounds__(WG) k_lv_stitch(const uint8_t* __restrict__ blob, const PageWork* __restrict__ pages,
                                                  int npages, ColumnParams cp, int sel, RunTables rt,
                                                  LevelTables lt) {
  const uint32_t p = blockIdx.x * (WG / WAVE) + (threadIdx.x >> 6), lane = threadIdx.x & 63u;
  if (p >= (uint32_t)npages || rt.pflag[p] != PF_PAGE) return;
  const PageWork& pw = pages[p];
  Stream s;
  if (!lv_stream(blob, pw, sel, cp, s)) return;
  const uint32_t k0 = lt.wbase[p], nw = lt.wbase[p + 1] - k0;
  for (uint32_t k = lane; k < nw; k += WAVE) lt.win[k0 + k] = make_uint2(LV_NONE, 0u);
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0): the NONE marks land before the walk's writes
  __builtin_amdgcn_wave_barrier();
  if (lane != 0 || nw == 0) return;
  const uint32_t ent = lv_ent((uint32_t)s.w), n = s.n;
  uint32_t e = 0;
  uint64_t acc = 0;
  bool ok = false;
  while (true) {
    if (e >= s.slen) break;  // the stream ends before n outputs
    const uint32_t kk = e / LV_WIN, idx = e - kk * LV_WIN;
    if (kk >= nw || idx >= ent) break;  // an entry past the table (foreign long runs)
    const uint2 t = lt.tab[(uint64_t)(k0 + kk) * ent + idx];
    lt.win[k0 + kk] = make_uint2(idx | (t.x & 0xFFFF0000u), (uint32_t)acc);  // entry | headers << 16
    acc += t.y;
    if (acc >= n) {
      ok = true;
      break;
    }
    const uint32_t jt = t.x & 0xFFFFu;
    if (jt >= LV_J_FAR || t.y == 0xFFFFFFFFu) break;  // far / end / dead, or a saturated count
    e = kk * LV_WIN + jt;
  }
  if (!ok) lv_bail(rt, p);
}

// ------------------------------------------------------------------------------ k_lv_emit

// 64-bit little-endian window of stream bytes at stream offset q: staged or from global memory.
__device__ inline uint64_t lv_bytes8(const uint32_t* stage, const uint8_t* __restrict__ blob,
                                     uint64_t blob_len, uint64_t S, uint32_t W0, uint32_t sb,
                                     uint32_t q) {
  const uint32_t r = q - W0 + sb;
  if (q >= W0 && r + 12 <= LV_STG) return lload_u64(stage, r);
  return gload_u64(blob, blob_len, S + q);
}

__device__ inline uint32_t wave_sum_u32_(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
  return v;
}

// Outputs [o, e) (page-relative, e - o <= 32) of run `info` starting at output `start`, w = 1:
// bit j = output o + j.
__device__ inline uint32_t lv_run_bits1(const LvWave& W, const uint8_t* __restrict__ blob, uint64_t blob_len,
                                        const LvWin& x, uint32_t start, uint32_t info, uint32_t o, uint32_t e) {
  const uint32_t nb = e - o;
  const uint32_t m = nb >= 32 ? 0xFFFFFFFFu : (1u << nb) - 1u;
  if (info & R_RLE) return (info & 1u) ? m : 0u;
  const uint64_t bit = (uint64_t)info * 8ull + (o - start);
  return (uint32_t)(lv_bytes8(W.stage, blob, blob_len, x.s.S, x.W0, x.sb, (uint32_t)(bit >> 3)) >> (bit & 7u)) & m;
}

// OUT = 2: int16 levels; OUT = 1: one byte per boolean.
template <int OUT>
__global__ void __launch_bounds__(WG) k_lv_emit(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                PageWork* pages, int npages, ColumnParams cp, int sel,
                                                RunTables rt, LevelTables lt, uint8_t* __restrict__ out) {
  __shared__ LvSmem sm;
  const uint32_t wid = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  LvWave& W = sm.wv[wid];
  const uint32_t total = lt.wbase[npages];
  const bool count = sel == SS_DEF;
  const uint32_t maxl = sel == SS_DEF ? (uint32_t)cp.max_def : (uint32_t)cp.max_rep;
  constexpr uint32_t G = 16u / OUT;  // outputs per 16-byte store
  for (uint32_t g = blockIdx.x * (WG / WAVE) + wid; g < total; g += gridDim.x * (WG / WAVE)) {
    LvWin x;
    x.p = lv_page_of(lt.wbase, (uint32_t)npages, g);
    const PageWork& pw = pages[x.p];
    if (rt.pflag[x.p] != PF_PAGE || !lv_stream(blob, pw, sel, cp, x.s)) continue;
    const uint2 wi = lt.win[g];
    if (wi.x == LV_NONE) continue;  // no true header in this window
    x.k = g - lt.wbase[x.p];
    x.W0 = x.k * LV_WIN;
    const uint32_t w = (uint32_t)x.s.w, vb = (w + 7u) >> 3, slen = x.s.slen, n = x.s.n;
    const uint32_t wm = w >= 32 ? 0xFFFFFFFFu : (1u << w) - 1u;
    const uint32_t e0 = wi.x & 0xFFFFu, nh = wi.x >> 16;  // entry, true headers (saturated)
    const uint32_t base = wi.y;
    lv_stage(blob, blob_len, x, W.stage, x.sb);
    uint32_t R = 0;  // runs placed (wave-uniform)
    uint64_t T = 0;  // outputs of those runs (wave-uniform)
    bool bad = false;
    if (nh <= LV_SERIAL) {
      // sparse window: one lane follows the chain from the entry
      if (lane == 0) {
        uint32_t q = x.W0 + e0, nr = 0;
        uint64_t acc = base;
        while (q < x.W0 + LV_WIN && q < slen && acc < n) {
          uint32_t nx, c, v;
          bool bp;
          if (!lv_parse4(W.stage, q - x.W0 + x.sb, q, slen, w, vb, nx, c, v, bp)) {
            bad = true;  // a true header the window path does not take, before n outputs
            break;
          }
          W.runs.rstart[nr] = acc < 0xFFFFFFFFull ? (uint32_t)acc : 0xFFFFFFFFu;
          W.runs.rinfo[nr] = bp ? v : (R_RLE | v);
          bad |= c && !(bp ? ((uint64_t)v * 8ull + (uint64_t)min((uint64_t)c, n - acc) * w <= (uint64_t)slen * 8ull)
                           : (v >> w) == 0);
          ++nr;
          acc += c;
          q = nx;
        }
        R = nr;
        T = acc - base;
      }
      R = (uint32_t)__shfl((int)R, 0, 64);
      T = __shfl(T, 0, 64);
    } else {
      // dense window: pointer jumping marks the positions reachable from the entry
      uint32_t jv[LV_PPL], cv[LV_PPL];
      lv_first_hops(W.stage, x.sb, x.W0, slen, w, vb, jv, cv);
#pragma unroll
      for (uint32_t j = 0; j < LV_PPL; ++j) {
        jv[j] &= 0xFFFFu;
        W.JC[j * WAVE + lane] = make_uint2(jv[j], 0u);
      }
      reinterpret_cast<uint4*>(W.R)[lane] = make_uint4(0u, 0u, 0u, 0u);
      wave_lds_sync();
      if (lane == 0) W.R[e0] = 1;
      wave_lds_sync();
#pragma unroll 1
      for (uint32_t r = 0; r < LV_ROUNDS; ++r) {
        bool live = false;
#pragma unroll
        for (uint32_t j = 0; j < LV_PPL; ++j) live |= jv[j] < LV_WIN;
        if (!__any(live)) break;
        uint32_t rb = 0, nj[LV_PPL];
#pragma unroll
        for (uint32_t j = 0; j < LV_PPL; ++j) {
          rb |= (uint32_t)W.R[j * WAVE + lane] << j;
          nj[j] = jv[j] < LV_WIN ? W.JC[jv[j]].x : jv[j];
        }
        wave_lds_sync();
#pragma unroll
        for (uint32_t j = 0; j < LV_PPL; ++j) {
          if (((rb >> j) & 1u) && jv[j] < LV_WIN) W.R[jv[j]] = 1;  // idempotent: no atomics needed
          jv[j] = nj[j];
          W.JC[j * WAVE + lane].x = jv[j];
        }
        wave_lds_sync();
      }
      // the true headers, in stream order (j-major, then lane): parse, count, place
      uint32_t mine = 0;
#pragma unroll
      for (uint32_t j = 0; j < LV_PPL; ++j) mine |= (uint32_t)W.R[j * WAVE + lane] << j;
      wave_lds_sync();  // the jump table's space now holds the run list
#pragma unroll 1
      for (uint32_t j = 0; j < LV_PPL; ++j) {
        const uint32_t i = j * WAVE + lane;
        uint32_t nx, c = 0, v = 0;
        bool bp = false, hdr = (mine >> j) & 1u, dead = false;
        if (hdr && !lv_parse4(W.stage, i + x.sb, x.W0 + i, slen, w, vb, nx, c, v, bp)) {
          dead = true;  // a true header the window path does not take: fatal unless n comes first
          hdr = false;
        }
        if (!hdr) c = 0;
        const uint64_t hb = __ballot(hdr);
        const uint64_t db = __ballot(dead);
        if (!hb && !db) continue;  // no true header in this row
        // inclusive counts over the lanes: runs by popcount, outputs by a DPP scan (32-bit while
        // every count is below 2^25, else a 64-bit shuffle scan)
        const uint32_t ir = (uint32_t)__builtin_popcountll(hb & ((2ull << lane) - 1ull));
        uint64_t ic;
        if (!__ballot(c >= (1u << 25))) {
          ic = wave_incl_scan_u32(c);
        } else {
          ic = c;
#pragma unroll
          for (int d = 1; d < 64; d <<= 1) {
            const uint64_t b = __shfl_up(ic, d, 64);
            if (lane >= (uint32_t)d) ic += b;
          }
        }
        const uint64_t acc = (uint64_t)base + T + ic - c;
        if (hdr) {
          const uint32_t k = R + ir - 1u;
          W.runs.rstart[k] = acc < 0xFFFFFFFFull ? (uint32_t)acc : 0xFFFFFFFFu;
          W.runs.rinfo[k] = bp ? v : (R_RLE | v);
          // what the reader consumes must be decodable: payload inside the stream, an RLE
          // value that fits the bit width
          bad |= acc < n && c && !(bp ? ((uint64_t)v * 8ull + (uint64_t)min((uint64_t)c, n - acc) * w <= (uint64_t)slen * 8ull)
                                      : (v >> w) == 0);
        }
        bad |= dead && acc < n;
        R += (uint32_t)__builtin_popcountll(hb);
        T += __shfl(ic, 63, 64);
        if (db) break;  // nothing after a dead header is on the chain
      }
    }
    if (__ballot(bad)) {
      if (lane == 0) lv_bail(rt, x.p);
      continue;
    }
    if (lane == 0) W.runs.rstart[R] = 0xFFFFFFFFu;
    wave_lds_sync();
    // outputs [base, min(base + T, n)) of the page
    const uint64_t endo = (uint64_t)base + T < n ? (uint64_t)base + T : (uint64_t)n;
    if (endo <= base || R == 0) continue;
#ifdef PQG_DIAG
    if (cp.debug & 128) continue;  // diagnostics: index work only, no output
#endif
    const uint64_t go = x.s.out;  // global index of the page's output 0
    uint32_t cnt = 0;
    if (w == 1) {
      // one-bit outputs: chunks of LV_BM outputs (aligned on global groups of G) go through an
      // LDS bitmap, filled run by run (lane r: runs r, r + 64, ...), then stored 16 bytes at a time
      const uint64_t G0 = (go + base) & ~(uint64_t)(G - 1);
#pragma unroll 1
      for (uint64_t c0 = G0; c0 < go + endo; c0 += LV_BM) {
        const uint64_t c1 = c0 + LV_BM < go + endo ? c0 + LV_BM : go + endo;
        const uint32_t plo = (uint32_t)((c0 > go + base ? c0 : go + base) - go);  // page-relative
        const uint32_t phi = (uint32_t)(c1 - go);
        const uint32_t pc0 = (uint32_t)(c0 - go);  // page-relative output of bitmap bit 0 (may wrap)
#pragma unroll
        for (uint32_t t = 0; t < LV_BM / 32 / WAVE; ++t) W.bm[t * WAVE + lane] = 0;
        wave_lds_sync();
        for (uint32_t r0 = 0; r0 < R; r0 += WAVE) {
          const uint32_t r = r0 + lane;
          uint32_t st = 0, inf = 0, o = 0, e = 0;
          if (r < R) {
            st = W.runs.rstart[r];
            inf = W.runs.rinfo[r];
            const uint32_t en = W.runs.rstart[r + 1];
            o = st > plo ? st : plo;
            e = en < phi ? en : phi;
          }
          const bool lng = e > o && e - o > 1024u;  // long runs: the whole wave, below
          if (!lng) {
            while (o < e) {  // one bitmap word at a time
              const uint32_t b = o - pc0;
              const uint32_t we = (b | 31u) + 1u + pc0;  // page output after this word
              const uint32_t oe = we < e ? we : e;
              const uint32_t bits = lv_run_bits1(W, blob, blob_len, x, st, inf, o, oe);
              if (bits) atomicOr(&W.bm[b >> 5], bits << (b & 31u));
              o = oe;
            }
          }
          for (uint64_t lb = __ballot(lng); lb; lb &= lb - 1) {
            const int L = __builtin_ctzll(lb);
            const uint32_t lst = (uint32_t)__shfl((int)st, L, 64), linf = (uint32_t)__shfl((int)inf, L, 64);
            const uint32_t lo_ = (uint32_t)__shfl((int)o, L, 64), le = (uint32_t)__shfl((int)e, L, 64);
            const uint32_t b0 = (lo_ - pc0) >> 5, b1 = (le - pc0 + 31u) >> 5;
            for (uint32_t wd = b0 + lane; wd < b1; wd += WAVE) {
              const uint32_t wo0 = pc0 + wd * 32u;
              const uint32_t wo = wo0 > lo_ && wd == b0 ? lo_ : (wd == b0 ? lo_ : wo0);
              const uint32_t we = wo0 + 32u < le ? wo0 + 32u : le;
              const uint32_t bits = lv_run_bits1(W, blob, blob_len, x, lst, linf, wo, we);
              if (bits) atomicOr(&W.bm[wd], bits << ((wo - pc0) & 31u));
            }
          }
        }
        wave_lds_sync();
        const uint32_t ngr = (uint32_t)((c1 - c0 + G - 1) / G);
        for (uint32_t k = lane; k < ngr; k += WAVE) {
          const uint64_t gl = c0 + (uint64_t)k * G;
          const uint32_t bits = (W.bm[(k * G) >> 5] >> ((k * G) & 31u)) & ((1u << G) - 1u);
          if (count) cnt += __builtin_popcount(bits);
          if (gl >= go + base && gl + G <= go + endo) {
            uint4 v;
            if (OUT == 2) {
              uint32_t q[4];
#pragma unroll
              for (uint32_t t = 0; t < 4; ++t) q[t] = ((bits >> (2 * t)) & 1u) | (((bits >> (2 * t + 1)) & 1u) << 16);
              v = make_uint4(q[0], q[1], q[2], q[3]);
            } else {
              uint32_t q[4];
#pragma unroll
              for (uint32_t t = 0; t < 4; ++t) {
                const uint32_t y = bits >> (4 * t);
                q[t] = (y & 1u) | (((y >> 1) & 1u) << 8) | (((y >> 2) & 1u) << 16) | (((y >> 3) & 1u) << 24);
              }
              v = make_uint4(q[0], q[1], q[2], q[3]);
            }
            *reinterpret_cast<uint4*>(out + gl * OUT) = v;
          } else {  // a group shared with a neighbouring window: only this window's outputs
#pragma unroll
            for (uint32_t j = 0; j < G; ++j) {
              const uint64_t gi = gl + j;
              if (gi >= go + base && gi < go + endo) {
                if (OUT == 2) reinterpret_cast<int16_t*>(out)[gi] = (int16_t)((bits >> j) & 1u);
                else out[gi] = (uint8_t)((bits >> j) & 1u);
              }
            }
          }
        }
        wave_lds_sync();
      }
    } else {
      // wider levels: groups of G outputs, each from the runs covering it
      const uint64_t k0 = (go + base) / G, k1 = (go + endo + G - 1) / G;
      uint32_t lgn = 1;
      while (lgn * 2 <= R) lgn *= 2;
      uint32_t a = 0;
#pragma unroll 1
      for (uint64_t k = k0 + lane; k < k1; k += WAVE) {
        const uint64_t gl = k * G;
        const uint32_t olo = (uint32_t)((gl > go + base ? gl : go + base) - go);
        const uint32_t ohi = (uint32_t)((gl + G < go + endo ? gl + G : go + endo) - go);
        const uint32_t f0 = (uint32_t)(gl - go);  // page-relative index of field 0 (may wrap)
        for (uint32_t st = lgn; st; st >>= 1)
          if (a + st < R && W.runs.rstart[a + st] <= olo) a += st;
        uint32_t f[G];
#pragma unroll
        for (uint32_t j = 0; j < G; ++j) f[j] = 0;
        uint32_t b = a, o = olo;
        while (o < ohi) {
          const uint32_t st = W.runs.rstart[b], nst = W.runs.rstart[b + 1], inf = W.runs.rinfo[b];
          const uint32_t be = nst < ohi ? nst : ohi;
          for (; o < be; ++o) {
            uint32_t v;
            if (inf & R_RLE) {
              v = inf & 0x7FFFFFFFu;
            } else {
              const uint64_t bit = (uint64_t)inf * 8ull + (uint64_t)(o - st) * w;
              v = (uint32_t)(lv_bytes8(W.stage, blob, blob_len, x.s.S, x.W0, x.sb, (uint32_t)(bit >> 3)) >> (bit & 7u)) & wm;
            }
#pragma unroll
            for (uint32_t j = 0; j < G; ++j)
              if (o - f0 == j) f[j] = v;
            if (count) cnt += v == maxl ? 1u : 0u;
          }
          ++b;
        }
        if (ohi - olo == G) {
          uint4 v;
          if (OUT == 2) {
            v = make_uint4((f[0] & 0xFFFFu) | (f[1] << 16), (f[2] & 0xFFFFu) | (f[3] << 16),
                           (f[4] & 0xFFFFu) | (f[5] << 16), (f[6] & 0xFFFFu) | (f[7] << 16));
          } else {
            uint32_t q[4];
#pragma unroll
            for (uint32_t t = 0; t < 4; ++t)
              q[t] = (f[4 * t] & 0xFFu) | ((f[4 * t + 1] & 0xFFu) << 8) | ((f[4 * t + 2] & 0xFFu) << 16) |
                     ((f[4 * t + 3] & 0xFFu) << 24);
            v = make_uint4(q[0], q[1], q[2], q[3]);
          }
          *reinterpret_cast<uint4*>(out + gl * OUT) = v;
        } else {
#pragma unroll
          for (uint32_t j = 0; j < G; ++j) {
            const uint32_t oo = f0 + j;
            if (oo >= olo && oo < ohi) {
              if (OUT == 2) reinterpret_cast<int16_t*>(out)[gl + j] = (int16_t)f[j];
              else out[gl + j] = (uint8_t)f[j];
            }
          }
        }
      }
    }
    if (count) {
      cnt = wave_sum_u32_(cnt);
      if (lane == 0 && cnt) atomicAdd((unsigned long long*)&pages[x.p].nonnull, (unsigned long long)cnt);
    }
  }
}

extern "C" {

// Level path of stream `sel` (def / rep levels: int16 out; RLE booleans: bytes out): plan,
// window tables, stitch, emit (+ def counts). 2048 workgroups (4 windows each) sweep the
// windows of every page.
hipError_t pqg_launch_lv(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages,
                         ColumnParams cp, int sel, RunTables rt, LevelTables lt, void* out, hipStream_t s) {
  if (npages <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_lv_plan, dim3(1), dim3(WG), 0, s, blob, pages, npages, cp, sel, rt, lt);
  const uint32_t wgrid = 256u * 8u;
  hipLaunchKernelGGL(k_lv_win, dim3(wgrid), dim3(WG), 0, s, blob, blob_len, pages, npages, cp, sel, rt, lt);
  hipLaunchKernelGGL(k_lv_stitch, dim3((npages + 3) / 4), dim3(WG), 0, s, blob, pages, npages, cp, sel, rt, lt);
  if (sel == SS_BOOL)
    hipLaunchKernelGGL(k_lv_emit<1>, dim3(wgrid), dim3(WG), 0, s, blob, blob_len, pages, npages, cp, sel, rt, lt,
                       (uint8_t*)out);
  else
    hipLaunchKernelGGL(k_lv_emit<2>, dim3(wgrid), dim3(WG), 0, s, blob, blob_len, pages, npages, cp, sel, rt, lt,
                       (uint8_t*)out);
  return hipGetLastError();
}

}  // extern "C"

}  // namespace pqg
