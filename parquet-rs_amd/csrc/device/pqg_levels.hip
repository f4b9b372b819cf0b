// pqg_levels.hip — level streams (def / rep levels) and RLE boolean values: the
// RLE/bit-packing hybrid (RleDecoder::reload / get_batch, rle.rs:352-434, 490-508;
// LevelDecoder::get, levels.rs:249-271), decoded on the GPU without a per-output serial loop.
//
// Run headers sit at data-dependent offsets: where a header starts depends on every header
// before it. Two ways to find them, chosen per page by the page itself:
//
//   k_lv_plan    windows (1 KiB of stream) per page (exclusive scan), eligibility of each stream.
//   k_lv_walk    one wave per page walks the header chain: a scalar hop loop follows up to 64
//                headers in an LDS-staged 4 KiB region (one LDS read and a few scalar ops per
//                one-byte header), then the 64 lanes parse those headers together, check them,
//                prefix-sum their output counts and write run records (first output, RLE value or
//                payload offset) plus, per window, the index of its first run. Sparse streams
//                (bit-packed runs of tens of bytes: random levels) finish here in a few hundred
//                microseconds for the whole chunk. A page whose 64-header batches span less than
//                1 KiB is dense (short RLE runs) and goes to the window path instead.
//   window path, for the dense pages (k_lv_plan2 compacts their windows):
//     k_lv_win   one wave per window: every byte position of the window is parsed as if a header
//                started there (next header offset, output count), then pointer jumping (ten
//                rounds of J[i] = J[J[i]], C[i] += C[J[i]]) gives, for every position, where its
//                chain leaves the window and how many outputs it produces on the way. The
//                answers for the positions a chain can enter at (the first 64 * w bytes: a
//                header plus at most 63 bit-packed groups) go to a table.
//     k_lv_stitch one workgroup per page: follows the window tables from offset 0 (one lookup per
//                window, the tables streamed through LDS) to each window's true entry and first
//                output.
//     k_lv_emit  one wave per window: pointer jumping again, now marking the positions reachable
//                from the true entry (the window's true headers), which are parsed in parallel
//                and placed by a wave scan into the window's run list.
//   k_lv_emit_walk  one wave per window of the walked pages: loads the window's run records.
//
// Both emits then write the window's outputs from its run list: int16 levels
// (column/reader.rs:162-163) or one byte per boolean, 16-byte stores (element stores for the
// groups shared with a neighbouring window); one-bit streams one 32-output word per lane. Def
// streams add their count of outputs == max_def (the non-null count read_batch uses,
// column/reader.rs:212-226) to the page.
//
// Streams off the common path (a header form the fast parse does not take, a stream that ends
// before its outputs, truncated payload, an RLE value wider than the bit width) go to the
// general decoder (pqg_runs.hpp / pqg_texpand.hpp), which reproduces every reference error.
#include "pqg_runs.hpp"

namespace pqg {

constexpr uint32_t LV_WIN = 1024;                  // stream bytes per window (one wave)
constexpr uint32_t LV_PPL = LV_WIN / WAVE;         // positions per lane (16)
#ifndef PQG_LV_STG_EXTRA
#define PQG_LV_STG_EXTRA 48
#endif
constexpr uint32_t LV_STG = LV_WIN + PQG_LV_STG_EXTRA;  // window path: staged bytes (+ alignment, read-ahead)
constexpr uint32_t LV_STG_CH = LV_STG / 16;             // 16-byte chunks
static_assert(LV_STG % 16 == 0 && LV_STG_CH <= 2 * 64, "two chunks per lane at most");
constexpr uint32_t LV_RCAP = LV_WIN;               // runs per window
constexpr uint32_t LV_ROUNDS = 10;                 // 2^10 = LV_WIN: chains of any length
constexpr uint32_t LV_SERIAL = 64;                 // k_lv_emit: windows with at most this many
                                                   // true headers are walked by one lane
constexpr uint32_t LV_NONE = 0xFFFFFFFFu;          // window not on the true chain
// jump-table values >= LV_WIN are terminal: the chain leaves the window at W0 + value, or
constexpr uint32_t LV_J_FAR = 0xFFFDu;             //   leaves it beyond W0 + 0xFFFC,
constexpr uint32_t LV_J_END = 0xFFFEu;             //   reaches the end of the stream,
constexpr uint32_t LV_J_DEAD = 0xFFFFu;            //   meets a header the fast parse refuses

// page walker (k_lv_walk) and the emit of walked pages (k_lv_emit_walk)
constexpr uint32_t LW_REG = 3072 - 128;            // stream bytes whose headers one region holds
constexpr uint32_t LW_CH = 3;                      // 16-byte loads per lane per region
constexpr uint32_t LW_STG = LW_CH * 16 * WAVE;     // staged bytes (region + alignment + read-ahead)
constexpr uint32_t LW_SPAN = 1024;                 // 64 headers within fewer bytes: a dense page
constexpr uint32_t LW_RPW = 256;                   // runs per window k_lv_emit_walk takes (the span
                                                   // rule keeps walked windows at <= 192)
constexpr uint32_t LW_REC = 64;                    // run records per window (+ 2 windows per page)
constexpr uint32_t LE_STG = LV_WIN + 64 * 16 + 64; // k_lv_emit_walk: staged bytes (runs of w <= 16
                                                   // whose header is in the window)

// Bit widths the level path takes: levels up to 16 bits (RLE values of <= 2 bytes).
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
    uint16_t J16[LV_WIN];   // k_lv_emit: the positions alone (16-bit: a quarter of the LDS traffic)
    struct {
      uint32_t rstart[LV_RCAP + 1];  // k_lv_emit, after the jumps: run list
      uint32_t rinfo[LV_RCAP];
    } runs;
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

// Inclusive scan of output counts (32-bit DPP while every count is below 2^25, else 64-bit).
__device__ inline uint64_t wave_incl_scan_cnt(uint32_t c) {
  if (!__ballot(c >= (1u << 25))) return wave_incl_scan_u32(c);
  uint64_t ic = c;
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t b = __shfl_up(ic, d, 64);
    if (lane >= (uint32_t)d) ic += b;
  }
  return ic;
}

// The same for 64-bit counts.
__device__ inline uint64_t wave_incl_scan_cnt64(uint64_t c) {
  if (!__ballot(c >= (1ull << 25))) return wave_incl_scan_u32((uint32_t)c);
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t b = __shfl_up(c, d, 64);
    if (lane >= (uint32_t)d) c += b;
  }
  return c;
}

__device__ inline void wave_lds_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS accesses have completed
  __builtin_amdgcn_wave_barrier();
}

// Header at stream position p from its bytes x (p .. p+3) and y (p+4 .. p+7).
__device__ inline bool lv_parse_xy(uint32_t x, uint32_t y, uint32_t p, uint32_t slen, uint32_t w, uint32_t vb,
                                   uint32_t& nxt, uint32_t& cnt, uint32_t& val, bool& bp) {
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
    v = (uint32_t)((((uint64_t)y << 32) | x) >> (8u * hl)) & vm;
  }
  val = bp ? p + hl : v;
  const uint32_t len = bp ? hl + g * w : hl + vb;  // g < 2^27, w <= 16: < 2^32
  nxt = p + len;
  return !(c012 & c3) && p < slen && len <= slen - p;
}

// Header at stream position p (stage byte index rel): branch-free for varints of 1-4 bytes (run
// lengths < 2^27; every header the reference writer emits, rle.rs:167-178), reading a third
// dword only for an RLE value past the first 4 bytes. Longer varints, and headers or RLE values
// running past the stream end, return false (dead): a true chain that meets one goes to the
// general decoder.
__device__ inline bool lv_parse4(const uint32_t* st, uint32_t rel, uint32_t p, uint32_t slen,
                                 uint32_t w, uint32_t vb, uint32_t& nxt, uint32_t& cnt,
                                 uint32_t& val, bool& bp) {
  const uint32_t wi = rel >> 2, sh = (rel & 3u) * 8u;
  const uint32_t d1 = st[wi + 1];
  const uint32_t x = __builtin_amdgcn_alignbit(d1, st[wi], sh);  // bytes p .. p+3
  // the third dword only for an RLE value past byte 3
  const bool far = (x & 1u) == 0u && 1u + ((x >> 7) & 1u) + ((x >> 7) & (x >> 15) & 1u) +
                                         ((x >> 7) & (x >> 15) & (x >> 23) & 1u) + vb > 4u;
  const uint32_t y = far ? __builtin_amdgcn_alignbit(st[wi + 2], d1, sh) : 0u;
  return lv_parse_xy(x, y, p, slen, w, vb, nxt, cnt, val, bp);
}

// What the reader consumes of a run must be decodable: the bit-packed payload of its first
// min(c, n - acc) outputs inside the stream, an RLE value that fits the bit width.
__device__ inline bool lv_run_ok(bool bp, uint32_t v, uint32_t c, uint64_t acc, uint32_t n, uint32_t slen,
                                 uint32_t w) {
  if (!c || acc >= n) return true;
  return bp ? (uint64_t)v * 8ull + (uint64_t)min((uint64_t)c, (uint64_t)n - acc) * w <= (uint64_t)slen * 8ull
            : (v >> w) == 0;
}

// A window's stream: the page stream `sel`, its window k (stage origin, bytes).
struct LvWin {
  Stream s;
  uint32_t p;      // page
  uint32_t k;      // window of the page
  uint32_t W0;     // stream offset of the window
  uint32_t sb;     // stage byte of stream offset W0
  uint32_t cap;    // staged bytes
};

// Stage nch 16-byte chunks from stream offset W0 (aligned down; guarded at the blob end).
__device__ inline void lv_stage(const uint8_t* __restrict__ blob, uint64_t blob_len, LvWin& x,
                                uint32_t* stage, uint32_t nch) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t A = (x.s.S + x.W0) & ~15ull;
  x.sb = (uint32_t)(x.s.S + x.W0 - A);
  x.cap = nch * 16u;
  for (uint32_t c = lane; c < nch; c += WAVE) {
    const uint64_t a = A + (uint64_t)c * 16u;
    const uint4 v = a + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
    reinterpret_cast<uint4*>(stage)[c] = v;
  }
  wave_lds_sync();
}

// Page and window of global window index g (wbase: exclusive scan of windows per page; pages
// without windows share their offset with the next page, which this finds).
__device__ inline uint32_t lv_page_of(const uint32_t* __restrict__ wbase, uint32_t npages, uint32_t g) {
  uint32_t lo = 0, hi = npages;  // last page with wbase[p] <= g
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (wbase[mid] <= g) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Streams this path takes (wide streams: k_lv_bound's wide mode finds their segment starts).
// Dictionary indices of the chunks the host gave this path (ChunkWork::lvdict: a dictionary of
// at most 2^dict_maxw entries), up to dict_maxw bits: wider indices into 4- / 8-byte values (a
// large dictionary, its gathers served from L2) expand faster through the general decoder's tiles.
__device__ inline bool lv_stream(const uint8_t* blob, const PageWork& pw, int sel, const ChunkWork* chunks,
                                 Stream& s) {
  const ChunkWork& ck = chunks[pw.chunk];
  return get_stream(blob, pw, sel, ck.cp, s) && pw.status == 0 && !s.err && s.kind == LK_RLE &&
         lv_width_ok((uint32_t)s.w) && (sel != SS_DICT || (ck.lvdict && (uint32_t)s.w <= ck.cp.dict_maxw));
}

// Hand page p to the general decoder (once).
__device__ inline void lv_bail(RunTables& rt, uint32_t p, uint32_t from) {
  if (atomicCAS(&rt.pflag[p], from, PF_BAIL) == from) atomicAdd(rt.nfall, 1u);
}
// The same, recording in diagnostic builds where (lt.bail, PQG_DEBUG 512): 1 segment scan,
// 2 stitch, 4 emit: a chain walk or run check, 5 emit: a run of the bitmap writes, 6 / 7
// walked-page emit.
#ifdef PQG_DIAG
#define LV_BAIL(rt, lt, p, from, site)                               \
  do {                                                               \
    if ((lt).bail) atomicCAS(&(lt).bail[p], 0u, (uint32_t)(site));  \
    lv_bail(rt, p, from);                                            \
  } while (0)
#else
#define LV_BAIL(rt, lt, p, from, site) lv_bail(rt, p, from)
#endif

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

// Exclusive scan of per-page window counts over one workgroup (pages in order).
template <class F>
__device__ inline void lv_scan_windows(int npages, uint32_t* wbase, F nwin_of) {
  __shared__ uint32_t wsum[WG / 64];
  __shared__ uint32_t carry_s;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < npages; base += WG) {
    const int p = base + (int)threadIdx.x;
    const uint32_t nw = p < npages ? nwin_of(p) : 0u;
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
    if (p < npages) wbase[p] = pre + incl - nw;
    __syncthreads();
    if (threadIdx.x == WG - 1) carry_s = pre + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) wbase[npages] = carry_s;
}

// ------------------------------------------------------------------------------ k_lv_probe
// One wave per page of an RLE boolean stream: the density probe (pqg_runs.hpp lv_probe_dense);
// the def / rep streams are probed by k_prepare, dictionary indices (no window path) never.
__global__ void __launch_bounds__(WG) k_lv_probe(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                 const PageWork* __restrict__ pages, int npages,
                                                 const ChunkWork* chunks, int sel, LevelTables lt) {
  const uint32_t wid = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63u;  // (uniform: scalar readlane indices)
  const uint32_t p = blockIdx.x * (WG / WAVE) + wid;
  if (p >= (uint32_t)npages) return;
  Stream st;
  uint32_t dense = 0;
  if (lv_stream(blob, pages[p], sel, chunks, st) && st.n && st.slen >= LW_SPAN + 64u)
    dense = lv_probe_dense(blob, blob_len, st.S, rfl((uint32_t)st.w));
  if (lane == 0) lt.dense[p] = dense;
}

// ------------------------------------------------------------------------------ k_lv_plan
// One workgroup: per page the stream's windows (exclusive scan into wbase), and the page flag:
// PF_PAGE (level path) or PF_BAIL (general decoder); 0 for pages without the stream and, for
// dictionary indices, pages of chunks the general decoder takes (ChunkWork::lvdict 0). Def
// streams start their count at 0.
__device__ inline bool lv_nodict(const PageWork* pages, const ChunkWork& ck, int sel) {
  // dictionary indices without a usable dictionary: the general decoder reports it
  return sel == SS_DICT && !dict_usable(pages, ck);
}

// Dense def / rep streams of bit width 1 (int16 outputs) take the chunk walks of pqg_lvd1.hpp.
#ifndef PQG_D1
#define PQG_D1 1
#endif
// Dense one-bit pages with at most PQG_D1_LPB16 / 16 levels per stream byte (mostly bit-packed:
// 6.7 at p_null 0.1) take the chunk walks; denser-in-levels streams (8.5 at p_null 0.05, config 5)
// carry long RLE runs whose fills one thread of k_d1_emit writes alone, and stay on the window
// path (config 5: 1.22 ms of D1 kernels per step against 0.94 on the window path).
#ifndef PQG_D1_LPB16
#define PQG_D1_LPB16 120
#endif
__device__ inline bool lv_d1_page(const LevelTables& lt, int p, const Stream& s, int sel) {
  return PQG_D1 && lt.dense[p] && s.w == 1 && (sel == SS_DEF || sel == SS_REP) && s.n && s.slen &&
         (uint64_t)s.n * 16u <= (uint64_t)s.slen * PQG_D1_LPB16;
}

__global__ void __launch_bounds__(WG) k_lv_plan(const uint8_t* __restrict__ blob, PageWork* pages, int npages,
                                                const ChunkWork* chunks, int sel, RunTables rt, LevelTables lt) {
  // one thread per page: flag, window and segment counts (into wbase / sbase, scanned in place
  // by the last workgroup; a single workgroup paid the pages' dependent loads four at a time)
  const int p = (int)(blockIdx.x * WG + threadIdx.x);
  if (p < npages) {
    const PageWork& pw = pages[p];
    const ChunkWork& ck = chunks[pw.chunk];
    const bool nodict = lv_nodict(pages, ck, sel);
    Stream s;
    uint32_t flag = 0, nw = 0, ns = 0;
    if (get_stream(blob, pw, sel, ck.cp, s) && (sel != SS_DICT || ck.lvdict)) {
      if (!nodict && lv_stream(blob, pw, sel, chunks, s) && (s.n == 0 || s.slen > 0)) {
        flag = PF_PAGE;
        nw = s.n ? (s.slen + LV_WIN - 1) / LV_WIN : 0u;
        if (sel == SS_DEF) pages[p].nonnull = 0;
        if (lv_d1_page(lt, p, s, sel)) {  // dense one-bit levels: the chunk walks (pqg_lvd1.hpp)
          flag = PF_D1;
          ns = (s.slen + LW_SEGW * LV_WIN - 1) / (LW_SEGW * LV_WIN);
        } else if (!lt.dense[p] && s.n && s.slen) {
          const uint32_t sw = lw_segw((uint32_t)s.w);
          ns = ((s.slen + LV_WIN - 1) / LV_WIN + sw - 1) / sw;
        }
      } else {
        flag = PF_BAIL;
        atomicAdd(rt.nfall, 1u);
      }
    }
    rt.pflag[p] = flag;
    lt.wbase[p] = nw;
    lt.sbase[p] = ns;
  }
  if (last_workgroup(lt.ctr + 2)) {
    lv_scan_windows(npages, lt.wbase, [&](int q) -> uint32_t { return lt.wbase[q]; });
    lv_scan_windows(npages, lt.sbase, [&](int q) -> uint32_t { return lt.sbase[q]; });
  }
}

// One workgroup: windows of the pages the walker left to the window path (wbase2).
__device__ inline void lv_plan2_scan(int npages, RunTables rt, LevelTables lt) {
  lv_scan_windows(npages, lt.wbase2, [&](int p) -> uint32_t {
    return rt.pflag[p] == PF_PAGE ? lt.wbase[p + 1] - lt.wbase[p] : 0u;
  });
}

// ------------------------------------------------------------------------------ sparse streams
// A page stream is cut into segments of lw_segw(w) windows, each walked by its own wave: the
// chain of a sparse stream enters segment j somewhere in its first window, and chains entering
// a window at different offsets meet within a few headers. k_lv_bound finds, for segment j's
// first window, where every chain entering it leaves it; when they all leave at one offset
// (X_j), the true chain passes there whatever its entry. Segment j's walk starts at X_j and stops
// when it lands exactly on X_m, a later segment's start (one it jumps over was not on the true
// chain, and it walks on to the next); the page scan follows the walks from offset 0 and places
// their runs. A dense stream hands the page to the window path.

// LvSeg::status
constexpr uint32_t LS_LANDED = 1;    // reached X_next
constexpr uint32_t LS_END = 2;       // reached the end of the stream
constexpr uint32_t LS_DEAD = 3;      // met a header the fast parse refuses (not recorded)
constexpr uint32_t LS_TRUNC = 4;     // last recorded run: bit-packed payload past the stream end
constexpr uint32_t LS_BADVAL = 5;    // last recorded run: RLE value wider than the bit width
constexpr uint32_t LS_DENSE = 6;     // 64 headers within fewer than LW_SPAN bytes, or too many runs
constexpr uint32_t LS_NOSTART = 7;   // the first window has no exit to start from
constexpr uint32_t LV_BX_NONE = 0xFFFFFFFFu, LV_BX_AMBIG = 0xFFFFFFFEu;

// Pointer jumping over the staged window x (see k_lv_win): jv/cv for the lane's positions.
__device__ inline void lv_jump(LvWave& W, const LvWin& x, uint32_t (&jv)[LV_PPL], uint32_t (&cv)[LV_PPL]) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = (uint32_t)x.s.w, vb = (w + 7u) >> 3;
  lv_first_hops(W.stage, x.sb, x.W0, x.s.slen, w, vb, jv, cv);
#pragma unroll
  for (uint32_t j = 0; j < LV_PPL; ++j) W.JC[j * WAVE + lane] = make_uint2(jv[j], cv[j]);
  wave_lds_sync();
  // after round r, jv[j] is 2^(r+1) hops on (or terminal) and cv[j] the outputs along the way
  // (saturating); the high half of jv counts the headers passed (also saturating). Stops once
  // every chain has left the window.
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
}

// Segment s of the level streams: page, segment of the page; false unless the page is still
// on the level path's sparse candidates.
__device__ inline bool lv_seg_of(const uint8_t* blob, const PageWork* pages, uint32_t npages, const ChunkWork* chunks,
                                 int sel, const RunTables& rt, const LevelTables& lt, uint32_t s, uint32_t& p,
                                 uint32_t& j, Stream& st) {
  p = lv_page_of(lt.sbase, npages, s);
  j = s - lt.sbase[p];
  return rt.pflag[p] == PF_PAGE && lv_stream(blob, pages[p], sel, chunks, st);
}

// ------------------------------------------------------------------------------ k_lv_bound
// One wave per segment j >= 1: a start for its walk (bexit). The chains entering the segment's
// first window at offsets [0, ent) are walked by their own lanes over two windows (chains keep
// meeting; capped at LB_HOPS headers: a dense stream is the window path's anyway); among the
// exits one hop of the writer's form can reach past them (a <= 2-byte header and <= 64 groups:
// rle.rs:48-50), the one most chains share is taken — chains entering on payload bytes that do
// not meet the true chain mostly jump far away. The walk of the segment before verifies the
// choice by landing on it exactly.
// Wide streams (w > 4: dictionary indices, mostly bit-packed runs of 1 + 63w bytes) give chains
// entering at different offsets little chance to meet: there every hop of a chain must be of the
// writer's form (a one-byte header of <= 63 groups, or an RLE value that fits w bits) and the
// chains are walked over LB_SPANW bytes (~8 headers at w = 16), so that a chain entering on
// payload bytes rarely survives (~1/4 per hop) and the true chain's exit is the one left.
constexpr uint32_t LB_SPAN = 2 * LV_WIN;         // bytes walked from the segment start
constexpr uint32_t LB_SPANW = 8 * LV_WIN;        // the same for wide streams
constexpr uint32_t LB_STG = LB_SPANW + 64;       // staged bytes
constexpr uint32_t LB_HOPS = 128;                // headers per chain at most
constexpr uint32_t LB_BINS = 8 + 64 * 16;        // exits one writer-form hop can reach past the span
constexpr uint32_t LB_PER = 7;                   // wide streams: full bit-packed runs in a row that
                                                 // place the true chain

__global__ void __launch_bounds__(WG) k_lv_bound(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                 const PageWork* __restrict__ pages, int npages,
                                                 const ChunkWork* chunks, int sel, RunTables rt, LevelTables lt) {
  __shared__ uint32_t stg[WG / WAVE][LB_STG / 4];
  __shared__ uint32_t hist_s[WG / WAVE][LB_BINS];
  const uint32_t wid = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  uint32_t* st = stg[wid];
  uint32_t* hist = hist_s[wid];
  const uint32_t total = lt.sbase[npages];
  for (uint32_t s = blockIdx.x * (WG / WAVE) + wid; s < total; s += gridDim.x * (WG / WAVE)) {
    LvWin x;
    uint32_t j;
    if (!lv_seg_of(blob, pages, (uint32_t)npages, chunks, sel, rt, lt, s, x.p, j, x.s) || j == 0) continue;
    x.k = j * lw_segw((uint32_t)x.s.w);
    x.W0 = x.k * LV_WIN;
    const uint32_t w = (uint32_t)x.s.w, vb = (w + 7u) >> 3, slen = x.s.slen;
    const bool wide = w >= 4;
    const uint32_t span = min(wide ? LB_SPANW : LB_SPAN, slen - x.W0);  // walked bytes (the stream may end first)
    lv_stage(blob, blob_len, x, st, (span + 64u) / 16u);
    const uint32_t ent = lv_ent(w);
    const uint32_t near = span + 8u + 64u * w;
    if (wide) {
      // the writer's full bit-packed runs (header 0x7F, then 63 groups: P bytes apart): an offset
      // of the first period whose next LB_PER headers all are is on the true chain (a chain of
      // payload bytes matching LB_PER times has odds 2^-8 each)
      const uint32_t P = 1u + 63u * w;
      uint32_t hit = 0xFFFFFFFFu;
      if ((LB_PER - 1u) * P + P + 1u <= span) {
        for (uint32_t q0 = 0; q0 < P && hit == 0xFFFFFFFFu; q0 += WAVE) {
          const uint32_t o = q0 + lane;
          bool all = o < P;
          for (uint32_t h = 0; h < LB_PER && all; ++h) {
            const uint32_t r = o + h * P + x.sb;
            all = ((st[r >> 2] >> (8u * (r & 3u))) & 0xFFu) == 0x7Fu;
          }
          hit = wave_min_u32(all ? o : 0xFFFFFFFFu);
        }
      }
      if (hit != 0xFFFFFFFFu) {
        if (lane == 0) lt.bexit[s] = x.W0 + hit;
        wave_lds_sync();  // the stage is refilled by the next segment
        continue;
      }
    }
    uint32_t ex[LV_PPL];
#pragma unroll
    for (uint32_t q = 0; q < LV_PPL; ++q) {
      ex[q] = 0xFFFFFFFFu;
      if (q * WAVE >= ent) continue;
      uint32_t o = q * WAVE + lane;
      bool ok = o < ent;
      for (uint32_t h = 0; h < LB_HOPS && __any(ok && o < span); ++h) {
        if (ok && o < span) {
          uint32_t nx, c, v;
          bool bp;
          ok = lv_parse4(st, o + x.sb, x.W0 + o, slen, w, vb, nx, c, v, bp);
          const uint32_t o2 = nx - x.W0;
          // a hop out of the first window must be one of the writer's form as well
          if (o < LV_WIN && o2 >= LV_WIN + 8u + 64u * w) ok = false;
          if (wide && (bp ? c > 504u : (v >> w) != 0u)) ok = false;
          o = o2;
        }
      }
      if (ok && o >= span && o < near) ex[q] = o;
    }
    // histogram of the exits (LDS), then its arg-max: most chains, then the lowest exit
    const uint32_t nb = near - span;
    for (uint32_t i = lane; i < nb; i += WAVE) hist[i] = 0;
    wave_lds_sync();
#pragma unroll
    for (uint32_t q = 0; q < LV_PPL; ++q)
      if (ex[q] != 0xFFFFFFFFu) atomicAdd(&hist[ex[q] - span], 1u);
    wave_lds_sync();
    uint32_t best = 0xFFFFFFFFu, bestn = 0;
    for (uint32_t i = lane; i < nb; i += WAVE) {
      const uint32_t c = hist[i];
      if (c > bestn) {
        bestn = c;
        best = span + i;
      }
    }
    const uint32_t top = wave_max_u32(bestn);
    const uint32_t pick = wave_min_u32(bestn == top ? best : 0xFFFFFFFFu);
    if (lane == 0) lt.bexit[s] = top == 0 ? LV_BX_NONE : x.W0 + pick;
    wave_lds_sync();  // the stage is refilled by the next segment
  }
}

// Follows one-byte headers through the hop-length table: while addr < alim and k < 64, the
// u16 at LDS address addr is the step to the next header's entry (0: not a one-byte header,
// stop, with lane k of posv already holding addr — harmless, the caller overwrites or ignores
// lanes >= k); lane k of posv records addr. Ten scalar instructions and one LDS byte read per header: the walk is bound by
// the CU's scalar issue rate, shared by every wave walking on it.
__device__ inline void lv_hops(uint32_t& addr, uint32_t alim, uint32_t& k, uint32_t& posv) {
  uint32_t len, vt, va;
  const uint32_t vlane = threadIdx.x & 63u;
  asm volatile(
      "1:\n\t"
      "s_cmp_ge_u32 %[addr], %[alim]\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_cmp_eq_u32 %[k], 64\n\t"
      "s_cbranch_scc1 2f\n\t"
      "v_mov_b32 %[va], %[addr]\n\t"
      "ds_read_u16 %[vt], %[va]\n\t"
      "v_cmp_eq_u32 vcc, %[k], %[vlane]\n\t"
      "v_cndmask_b32 %[posv], %[posv], %[va], vcc\n\t"
      "s_waitcnt lgkmcnt(0)\n\t"
      "v_readfirstlane_b32 %[len], %[vt]\n\t"
      "s_cmp_eq_u32 %[len], 0\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_add_u32 %[addr], %[addr], %[len]\n\t"
      "s_add_u32 %[k], %[k], 1\n\t"
      "s_branch 1b\n"
      "2:"
      : [addr] "+s"(addr), [k] "+s"(k), [posv] "+v"(posv), [len] "=&s"(len), [vt] "=&v"(vt), [va] "=&v"(va)
      : [alim] "s"(alim), [vlane] "v"(vlane)
      : "scc", "vcc", "memory");
}

// ------------------------------------------------------------------------------ k_lv_segwalk
// One wave per segment: walks the chain from X_j (segment 0: offset 0) to X_m, the next segment
// start with a common exit. A scalar hop loop follows up to 64 headers in an LDS-staged region
// (header bytes read from VGPRs: one v_readlane per one-byte header), then the 64 lanes parse
// those headers together, check them and record their runs (output offset within the segment,
// RLE value or payload offset) and header offsets.
__global__ void __launch_bounds__(WG) k_lv_segwalk(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                   const PageWork* __restrict__ pages, int npages,
                                                   const ChunkWork* chunks, int sel, RunTables rt, LevelTables lt) {
  __shared__ uint32_t stg[WG / WAVE][LW_STG / 4];
  __shared__ uint4 lent_s[WG / WAVE][LW_STG / 8];  // per staged byte (u16): 2 * hop length of a one-byte header
  const uint32_t wid = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  // LDS address of this wave's hop-length table
  const uint32_t lb = rfl((uint32_t)(uintptr_t)(__attribute__((address_space(3))) const uint4*)lent_s[wid]);
  const uint32_t total = lt.sbase[npages];
  for (uint32_t sidx = blockIdx.x * (WG / WAVE) + wid; sidx < total; sidx += gridDim.x * (WG / WAVE)) {
  uint32_t p, j;
  Stream s;
  if (!lv_seg_of(blob, pages, (uint32_t)npages, chunks, sel, rt, lt, sidx, p, j, s)) continue;
  LvSeg& sg = lt.seg[sidx];
  const uint32_t s0 = lt.sbase[p], nseg = lt.sbase[p + 1] - s0;
  const uint32_t start = j == 0 ? 0u : lt.bexit[sidx];
  if (start >= LV_BX_AMBIG) {
    if (lane == 0) sg.status = LS_NOSTART;
    continue;
  }
  // the next segment start the walk must land on (a start it jumps over was not on the true
  // chain: the walk goes on to the following one, and the segment is left off the page's chain)
  uint32_t stop = 0xFFFFFFFFu, m = j;
  auto next_stop = [&]() {
    stop = 0xFFFFFFFFu;
    for (++m; m < nseg; ++m) {
      const uint32_t b = lt.bexit[s0 + m];
      if (b < LV_BX_AMBIG) {
        stop = b;
        break;
      }
    }
  };
  next_stop();
  uint32_t* st = stg[wid];
  const uint32_t slen = s.slen, w = (uint32_t)s.w, vb = (w + 7u) >> 3;
  const bool ffw = w >= 4;  // fast-forward over full bit-packed runs (>= 253 bytes each)
  uint2* rec = lt.srec + (uint64_t)sidx * LW_SCAP;
  uint32_t* pos = lt.spos + (uint64_t)sidx * LW_SCAP;
  uint32_t cur = start, nr = 0, loaded = 0xFFFFFFFFu, sb = 0, lastpos = 0xFFFFFFFFu, status = 0, tv = 0, tc = 0;
  uint64_t acc = 0;
  uint4 pf[LW_CH];
#ifdef PQG_DIAG
  // diagnostics (PQG_DEBUG bit 7): per segment s_memtime cycles in region installs, hop loops,
  // batches, and the headers walked
  const ColumnParams& cp = pcp(chunks, pages[p]);
  const bool stamps = (cp.debug & 128) && cp.dbgbuf;
  uint64_t t0 = stamps ? __builtin_amdgcn_s_memtime() : 0, t_reg = 0, t_hop = 0, t_bat = 0, nhops = 0;
#define LW_STAMP(acc)                                      \
  if (stamps) {                                            \
    const uint64_t t1 = __builtin_amdgcn_s_memtime();      \
    acc += t1 - t0;                                        \
    t0 = t1;                                               \
  }
#else
#define LW_STAMP(acc)
#endif
  auto fetch = [&](uint32_t r) {  // region r's bytes into registers
    const uint64_t A = (s.S + (uint64_t)r * LW_REG) & ~15ull;
#pragma unroll
    for (uint32_t q = 0; q < LW_CH; ++q) {
      const uint64_t a = A + (uint64_t)(q * WAVE + lane) * 16u;
      pf[q] = a + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
    }
  };
  const uint32_t nreg = (slen + LW_REG - 1) / LW_REG;
  uint32_t fetched = cur / LW_REG;
  fetch(fetched);
  while (true) {
    if (cur == stop) {
      status = LS_LANDED;
      break;
    }
    if (cur > stop) {
      next_stop();
      continue;
    }
    if (cur >= slen) {
      status = LS_END;
      break;
    }
    uint32_t k = 0, posv = 0;
    const uint32_t c0 = cur;
    bool dead = false;
    if (ffw) {
      // wide streams: the writer's full bit-packed runs (header 0x7F, P bytes each) in one step —
      // lane l reads the header byte P * l past cur; the matching prefix is the chain's next
      // headers (each 0x7F header puts the next one exactly P bytes on)
      const uint32_t P = 1u + 63u * w;
      const uint32_t lim = min(slen, stop);
      const uint32_t q = cur + lane * P;
      const bool hit = q < lim && blob[s.S + q] == 0x7Fu;
      const uint64_t m = __ballot(hit);
      const uint32_t run = ~m ? (uint32_t)__builtin_ctzll(~m) : 64u;
      if (run >= 2u) {
        k = run;
        posv = q;
        cur = rfl(cur + run * P);
      }
    }
    const uint32_t r = cur / LW_REG;
    if (k == 0 && r != loaded) {
      if (r != fetched) fetch(r);
#pragma unroll
      for (uint32_t q = 0; q < LW_CH; ++q) {
        reinterpret_cast<uint4*>(st)[q * WAVE + lane] = pf[q];
        // twice the hop lengths of one-byte headers (byte offsets of the u16 table), 0 for any
        // other first byte: the hop loop then costs one LDS read per header
        uint32_t lw[8];
        const uint32_t src[4] = {pf[q].x, pf[q].y, pf[q].z, pf[q].w};
#pragma unroll
        for (uint32_t t = 0; t < 8; ++t) {
          const uint32_t b0 = (src[t >> 1] >> (16u * (t & 1u))) & 0xFFu, b1 = (src[t >> 1] >> (16u * (t & 1u) + 8u)) & 0xFFu;
          const uint32_t l0 = (b0 & 0x80u) ? 0u : 2u + ((b0 & 1u) ? (b0 >> 1) * w : vb) * 2u;
          const uint32_t l1 = (b1 & 0x80u) ? 0u : 2u + ((b1 & 1u) ? (b1 >> 1) * w : vb) * 2u;
          lw[t] = l0 | (l1 << 16);
        }
        lent_s[wid][2 * (q * WAVE + lane)] = make_uint4(lw[0], lw[1], lw[2], lw[3]);
        lent_s[wid][2 * (q * WAVE + lane) + 1] = make_uint4(lw[4], lw[5], lw[6], lw[7]);
      }
      sb = (uint32_t)(s.S + (uint64_t)r * LW_REG - ((s.S + (uint64_t)r * LW_REG) & ~15ull));
      loaded = r;
      wave_lds_sync();
      if (r + 1 < nreg) {  // the next region's loads fly while this one is walked
        fetch(r + 1);
        fetched = r + 1;
      }
      LW_STAMP(t_reg);
    }
    const uint32_t rb = rfl(r * LW_REG);
    const bool ffb = k != 0;  // this batch came from the fast-forward
    if (!ffb) {
      const uint32_t lim = rfl(min(min(rb + LW_REG, slen), stop));
      // hop loop (wave-uniform): up to 64 headers. One-byte headers take lv_hops (scalar loop
      // over the hop-length table, positions as LDS addresses of their table entries); any other
      // header the general parse.
      const uint32_t ab = rfl(lb + 2u * (sb - rb));  // LDS address of stream offset 0's entry (mod 2^32)
      uint32_t addr = ab + 2u * cur;
      const uint32_t alim = ab + 2u * lim;
      while (true) {
        lv_hops(addr, alim, k, posv);
        if (addr >= alim || k == 64u) break;
        const uint32_t q = (addr - ab) >> 1;  // stream offset of a header whose hop is not in the table
        uint32_t nxt, v, cnt;
        bool bp;
        const bool ok = lv_parse4(st, q - rb + sb, q, slen, w, vb, nxt, cnt, v, bp);
        if (!rfl(ok ? 1u : 0u)) {
          dead = true;
          break;
        }
        posv = lane == k ? addr : posv;
        ++k;
        addr += 2u * (rfl(nxt) - q);
      }
      cur = (addr - ab) >> 1;
      posv = (posv - ab) >> 1;
    }
    LW_STAMP(t_hop);
#ifdef PQG_DIAG
    nhops += k;
#endif
    if (k) {
      // batch: lane l parses header l, checks it and records its run
      const bool act = lane < k;
      uint32_t nx, c = 0, v = 0;
      bool bp = false, okp = true;
      if (act) {
        if (ffb) {  // a full bit-packed run
          c = 504u;
          v = posv + 1u;
          bp = true;
        } else {
          okp = lv_parse4(st, posv - rb + sb, posv, slen, w, vb, nx, c, v, bp);
        }
      }
      const uint64_t ic = wave_incl_scan_cnt(act ? c : 0u);
      const uint64_t accb = acc + ic - (act ? c : 0u);
      if ((k == 64u && cur - c0 < LW_SPAN) || nr + k > LW_SCAP) {
        status = LS_DENSE;
        break;
      }
      // the first run whose payload runs past the stream end, or whose RLE value does not fit
      const bool trunc = act && c && bp && (uint64_t)v * 8ull + (uint64_t)c * w > (uint64_t)slen * 8ull;
      const bool badv = act && !bp && (!okp || (c && (v >> w) != 0));  // (or its value past the end)
      const uint64_t bb = __ballot(trunc || badv);
      const uint32_t kk = bb ? (uint32_t)__builtin_ctzll(bb) + 1u : k;  // runs kept
      if (lane < kk) {
        rec[nr + lane] = make_uint2(accb < 0xFFFFFFFFull ? (uint32_t)accb : 0xFFFFFFFFu, bp ? v : (R_RLE | v));
        pos[nr + lane] = posv;
      }
      lastpos = rfl((uint32_t)__shfl((int)posv, (int)kk - 1, 64));
      nr += kk;
      const uint64_t bt = __shfl(ic, (int)kk - 1, 64);
      acc += ((uint64_t)rfl((uint32_t)(bt >> 32)) << 32) | rfl((uint32_t)bt);  // through run kk - 1
      if (bb) {
        const uint32_t L = kk - 1u;
        status = rfl((uint32_t)__shfl((int)(trunc ? LS_TRUNC : LS_BADVAL), (int)L, 64));
        tv = rfl((uint32_t)__shfl((int)v, (int)L, 64));
        tc = rfl((uint32_t)__shfl((int)c, (int)L, 64));
        break;
      }
    }
    LW_STAMP(t_bat);
    if (dead) {
      status = LS_DEAD;
      break;
    }
  }
#ifdef PQG_DIAG
  if (stamps && lane == 0) {
    uint64_t* d = cp.dbgbuf + 4ull * sidx;
    d[0] = t_reg;
    d[1] = t_hop;
    d[2] = t_bat;
    d[3] = nhops;
  }
#endif
#undef LW_STAMP
  if (lane == 0) {
    sg.out = acc;
    sg.runs = nr;
    sg.status = status;
    sg.next = m;
    sg.lastpos = lastpos;
    sg.tv = tv;
    sg.tc = tc;
  }
  wave_lds_sync();  // the stage is refilled by the next segment
  }
}

// ------------------------------------------------------------------------------ k_lv_segscan
// One workgroup per page: follows the segment walks from offset 0, places them (first run, first
// output), finds the run holding output n - 1, and decides the page: walked (PF_WALK), window
// path (PF_PAGE stays) or general decoder (PF_BAIL). The common case — every walk landed on the
// next segment's start — is a workgroup scan of the segments' output and run counts; anything
// else (a start that was not on the true chain, a walk that ended early) is followed by one lane.

// The last segment J of the chain (outputs acc before it reach n): keep its runs up to the one
// holding output n - 1. Returns the verdict (0 walked, 1 window path, 2 general decoder).
__device__ inline uint32_t lv_seg_last(LvSeg& sg, const uint2* rec, uint64_t acc, uint32_t runs, uint32_t n,
                                       uint32_t w, uint32_t slen, uint32_t cap) {
  uint32_t lo = 0, hi = sg.runs;  // runs [0, sg.runs) start at acc + rec[i].x (ascending)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (acc + rec[mid].x < n) lo = mid;
    else hi = mid;
  }
  const uint32_t keep = lo + 1;
  if (keep == sg.runs && (sg.status == LS_TRUNC || sg.status == LS_BADVAL)) {
    const uint64_t before = acc + rec[lo].x;
    const uint64_t need = sg.status == LS_TRUNC ? (uint64_t)sg.tv * 8ull + min((uint64_t)sg.tc, n - before) * w : 0;
    if (sg.status == LS_BADVAL || need > (uint64_t)slen * 8ull) return 2;
  }
  if (runs + keep + 1u > cap) return 1;
  sg.keep = keep;
  sg.flags = 3;
  return 0;
}

__device__ inline uint32_t lv_segscan_serial(LvSeg* seg, const uint2* srec, uint32_t nseg, uint32_t n, uint32_t w,
                                             uint32_t slen, uint32_t cap) {
  uint64_t acc = 0;
  uint32_t runs = 0, prevpos = 0xFFFFFFFFu, j = 0;
  while (true) {
    LvSeg& sg = seg[j];
    if (sg.status == LS_NOSTART) return 1;
    sg.base_out = acc;
    sg.base_run = runs;
    sg.prevpos = prevpos;
    if (acc + sg.out >= n) return lv_seg_last(sg, srec + (uint64_t)j * LW_SCAP, acc, runs, n, w, slen, cap);
    acc += sg.out;
    runs += sg.runs;
    sg.keep = sg.runs;
    sg.flags = 1;
    if (sg.runs) prevpos = sg.lastpos;
    if (sg.status == LS_LANDED) {
      j = sg.next;
      continue;
    }
    return sg.status == LS_DENSE ? 1 : 2;  // else: the stream ends or breaks before n
  }
}

__device__ inline void lv_segscan_page(const uint8_t* __restrict__ blob, const PageWork* __restrict__ pages,
                                       int npages, const ChunkWork* chunks, int sel, RunTables rt, LevelTables lt,
                                       uint32_t p) {
  __shared__ uint64_t wout[WG / WAVE];
  __shared__ uint32_t wrun[WG / WAVE], wlast[WG / WAVE], wmin[WG / WAVE];
  __shared__ uint64_t c_out;
  __shared__ uint32_t c_run, c_pos, J_s, broken_s, verdict_s;
  const uint32_t tid = threadIdx.x, wid = tid >> 6, lane = tid & 63u;
  if (p >= (uint32_t)npages || rt.pflag[p] != PF_PAGE) return;
  Stream s;
  if (!lv_stream(blob, pages[p], sel, chunks, s)) return;
  if (lt.dense[p]) return;  // the window path's (k_lv_probe)
  const uint32_t n = s.n, w = (uint32_t)s.w;
  const uint32_t s0 = lt.sbase[p], nseg = lt.sbase[p + 1] - s0;
  LvSeg* seg = lt.seg + s0;
  if (n == 0 || nseg == 0) {  // nothing to read: no windows, no runs
    if (tid == 0) {
      lt.wfirst[lt.wbase[p] + p] = 0;
      rt.pflag[p] = PF_WALK;
    }
    return;
  }
  const uint32_t cap = LW_REC * (lt.wbase[p + 1] - lt.wbase[p] + 2u);
  for (uint32_t q = tid; q < nseg; q += WG) seg[q].flags = 0;  // (the tables outlive a decode)
  if (tid == 0) {
    c_out = 0;
    c_run = 0;
    c_pos = 0xFFFFFFFFu;
    J_s = 0xFFFFFFFFu;
    broken_s = 0;
  }
  __syncthreads();
  // placement assuming the chain visits every segment in order; J = the first segment whose
  // outputs reach n; the assumption holds when every segment before J landed on its successor
  for (uint32_t c = 0; c < nseg; c += WG) {
    const uint32_t j = c + tid;
    const bool in = j < nseg;
    uint64_t o = 0;
    uint32_t r = 0, st = 0, nx = 0, lp = 0;
    if (in) {
      const LvSeg& sg = seg[j];
      o = sg.out;
      r = sg.runs;
      st = sg.status;
      nx = sg.next;
      lp = sg.lastpos;
    }
    // inclusive scans over the workgroup: outputs, runs, last header of a non-empty segment
    uint64_t io = o;
    uint32_t ir = r, il = r ? j : 0xFFFFFFFFu;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t yo = __shfl_up(io, d, 64);
      const uint32_t yr = __shfl_up(ir, d, 64);
      const uint32_t yl = __shfl_up(il, d, 64);
      if (lane >= (uint32_t)d) {
        io += yo;
        ir += yr;
        il = il == 0xFFFFFFFFu ? yl : il;
      }
    }
    if (lane == 63) {
      wout[wid] = io;
      wrun[wid] = ir;
      wlast[wid] = il;
    }
    __syncthreads();
    uint64_t bo = c_out;
    uint32_t br = c_run, bl = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < wid; ++k) {
      bo += wout[k];
      br += wrun[k];
      if (wlast[k] != 0xFFFFFFFFu) bl = wlast[k];
    }
    const uint64_t base_out = bo + io - o;
    const uint32_t base_run = br + ir - r;
    // last non-empty segment before j: within the wave (exclusive), earlier waves, earlier chunks
    uint32_t ex = (uint32_t)__shfl_up((int)il, 1, 64);
    if (lane == 0) ex = 0xFFFFFFFFu;
    const uint32_t lastj = ex != 0xFFFFFFFFu ? ex : bl;
    const uint32_t prevpos = lastj != 0xFFFFFFFFu ? seg[lastj].lastpos : c_pos;
    const bool hit = in && base_out + o >= n;
    const uint32_t jm = wave_min_u32(hit ? j : 0xFFFFFFFFu);
    if (lane == 0) wmin[wid] = jm;
    __syncthreads();
    uint32_t J = 0xFFFFFFFFu;
    for (uint32_t k = 0; k < WG / WAVE; ++k) J = min(J, wmin[k]);
    if (in && j <= J) {
      LvSeg& sg = seg[j];
      sg.base_out = base_out;
      sg.base_run = base_run;
      sg.prevpos = prevpos;
      const bool ok = st != LS_NOSTART && (j == J || (st == LS_LANDED && nx == j + 1));
      if (!ok) atomicOr(&broken_s, 1u);
      if (j < J) {
        sg.keep = r;
        sg.flags = 1;
      }
    }
    (void)lp;
    __syncthreads();
    if (tid == WG - 1) {  // carries into the next chunk
      c_out = bo + io;
      c_run = br + ir;
      const uint32_t lj = il != 0xFFFFFFFFu ? il : bl;
      if (lj != 0xFFFFFFFFu) c_pos = seg[lj].lastpos;
      J_s = J;
    }
    __syncthreads();
    if (J_s != 0xFFFFFFFFu || broken_s) break;
  }
  if (tid == 0) {
    uint32_t verdict;
    const uint32_t J = J_s;
    if (broken_s || J == 0xFFFFFFFFu) {
      for (uint32_t q = 0; q < nseg; ++q) seg[q].flags = 0;
      verdict = lv_segscan_serial(seg, lt.srec + (uint64_t)s0 * LW_SCAP, nseg, n, w, s.slen, cap);
    } else {
      LvSeg& sg = seg[J];
      verdict = lv_seg_last(sg, lt.srec + (uint64_t)(s0 + J) * LW_SCAP, sg.base_out, sg.base_run, n, w, s.slen, cap);
    }
    if (verdict == 1 && sel == SS_DICT) verdict = 2;  // no window path for dictionary indices
    verdict_s = verdict;
    if (verdict == 0) rt.pflag[p] = PF_WALK;
    else if (verdict == 2) LV_BAIL(rt, lt, p, PF_PAGE, 1);
  }
  __syncthreads();
  if (verdict_s != 0)
    for (uint32_t q = tid; q < nseg; q += WG) seg[q].flags = 0;
}

// The grid's last workgroup also runs k_lv_plan2's scan (the windows of the pages left to the
// window path), one launch fewer per level stream.
__global__ void __launch_bounds__(WG) k_lv_segscan(const uint8_t* __restrict__ blob, const PageWork* __restrict__ pages,
                                                   int npages, const ChunkWork* chunks, int sel, RunTables rt,
                                                   LevelTables lt) {
  for (uint32_t p = blockIdx.x; p < (uint32_t)npages; p += gridDim.x) {
    lv_segscan_page(blob, pages, npages, chunks, sel, rt, lt, p);
    __syncthreads();  // (the page's shared state before the next page's)
  }
  if (last_workgroup(lt.ctr + 0)) lv_plan2_scan(npages, rt, lt);
}

// ------------------------------------------------------------------------------ k_lv_compact
// One wave per segment on a walked page's chain: its runs to the page's run list (first outputs
// made page-relative), the first run of every window whose start lies before one of its headers,
// and after the page's last run a sentinel and the windows past it.
__global__ void __launch_bounds__(WG) k_lv_compact(int npages, RunTables rt, LevelTables lt) {
  const uint32_t wid = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  const uint32_t total = lt.sbase[npages];
  for (uint32_t sidx = blockIdx.x * (WG / WAVE) + wid; sidx < total; sidx += gridDim.x * (WG / WAVE)) {
  const uint32_t p = lv_page_of(lt.sbase, (uint32_t)npages, sidx);
  if (rt.pflag[p] != PF_WALK) continue;
  const LvSeg& sg = lt.seg[sidx];
  if (!(sg.flags & 1u)) continue;
  const uint32_t k0 = lt.wbase[p], nwin = lt.wbase[p + 1] - k0;
  uint32_t* wf = lt.wfirst + k0 + p;
  uint2* rec = lt.rec + (uint64_t)LW_REC * (k0 + 2ull * p);
  const uint2* sr = lt.srec + (uint64_t)sidx * LW_SCAP;
  const uint32_t* sp = lt.spos + (uint64_t)sidx * LW_SCAP;
  const uint32_t K = sg.keep, br = sg.base_run;
  const uint64_t bo = sg.base_out;
  for (uint32_t i = lane; i < K; i += WAVE) {
    const uint2 r = sr[i];
    const uint64_t o = bo + r.x;
    rec[br + i] = make_uint2(o < 0xFFFFFFFFull ? (uint32_t)o : 0xFFFFFFFFu, r.y);
    const uint32_t q = sp[i];
    const uint32_t prev = i ? sp[i - 1] : sg.prevpos;
    const uint32_t wlo = prev == 0xFFFFFFFFu ? 0u : prev / LV_WIN + 1u;
    for (uint32_t kw = wlo; kw <= q / LV_WIN; ++kw) wf[kw] = br + i;
  }
  if (sg.flags & 2u) {
    const uint64_t o = bo + (K < sg.runs ? (uint64_t)sr[K].x : sg.out);
    if (lane == 0) rec[br + K] = make_uint2(o < 0xFFFFFFFFull ? (uint32_t)o : 0xFFFFFFFFu, 0u);  // sentinel
    const uint32_t wlo = K ? sp[K - 1] / LV_WIN + 1u : (sg.prevpos == 0xFFFFFFFFu ? 0u : sg.prevpos / LV_WIN + 1u);
    for (uint32_t kw = wlo + lane; kw <= nwin; kw += WAVE) wf[kw] = br + K;
  }
  }
}

// ------------------------------------------------------------------------------ segment tables
// Dense windows (k_lv_win for w = 1, k_lv_emit): lane l takes the 16 positions [16 l, 16 l + 16)
// of the staged window (a segment) and parses each as a header; a backward pass over the segment
// gives, per position, where its chain leaves the segment (window-relative, or a terminal code),
// the outputs on the way (saturating) and the headers it passes (a 16-bit mask), in
// W.JC[t * 64 + l] for position 16 l + t. A chain then crosses a window in at most 64 lookups.
constexpr uint32_t LV_SEG = LV_WIN / WAVE;

__device__ inline void lv_seg_build(LvWave& W, const LvWin& x, uint32_t (&pc)[LV_SEG], uint32_t (&pv)[LV_SEG],
                                    uint32_t& bpm) {
  constexpr uint32_t SEG = LV_SEG;
  const uint32_t lane = threadIdx.x & 63u, i0 = lane * SEG;
  const uint32_t w = (uint32_t)x.s.w, vb = (w + 7u) >> 3, slen = x.s.slen;
  uint32_t a[SEG / 4 + 2];  // segment bytes 0 .. 23, dword-aligned on the segment
  {
    const uint32_t d0 = (x.sb >> 2) + i0 / 4u, sh = (x.sb & 3u) * 8u;
    uint32_t d[SEG / 4 + 3];
#pragma unroll
    for (uint32_t k = 0; k < SEG / 4 + 3; ++k) d[k] = W.stage[d0 + k];
#pragma unroll
    for (uint32_t k = 0; k < SEG / 4 + 2; ++k) a[k] = __builtin_amdgcn_alignbit(d[k + 1], d[k], sh);
  }
  uint32_t pn[SEG];
  bpm = 0;
#pragma unroll
  for (uint32_t t = 0; t < SEG; ++t) {
    const uint32_t q = x.W0 + i0 + t;
    const uint32_t xx = t & 3u ? __builtin_amdgcn_alignbit(a[t / 4 + 1], a[t / 4], 8u * (t & 3u)) : a[t / 4];
    const uint32_t yy = t & 3u ? __builtin_amdgcn_alignbit(a[t / 4 + 2], a[t / 4 + 1], 8u * (t & 3u)) : a[t / 4 + 1];
    uint32_t nx, c = 0, v = 0;
    bool bp = false;
    if (q >= slen) {
      pn[t] = LV_J_END;
    } else if (!lv_parse_xy(xx, yy, q, slen, w, vb, nx, c, v, bp)) {
      pn[t] = LV_J_DEAD;
      c = 0;
    } else {
      const uint32_t dd = nx - x.W0;
      pn[t] = dd < 0xFFFDu ? dd : LV_J_FAR;
    }
    pc[t] = c;
    pv[t] = v;
    bpm |= (uint32_t)bp << t;
  }
  // backward pass: entry (t * 64 + lane) = (exit | headers mask << 16, outputs)
#pragma unroll
  for (int t = SEG - 1; t >= 0; --t) {
    const uint32_t nt = pn[t];
    uint32_t ex = nt, m = nt < LV_J_END ? 1u << t : 0u, c = pc[t];  // (END / DEAD: no header)
    if (nt < i0 + SEG) {                                             // lands in this segment
      const uint2 r = W.JC[(nt - i0) * WAVE + lane];
      ex = r.x & 0xFFFFu;
      m |= r.x >> 16;
      const uint32_t s2 = c + r.y;
      c = s2 < c ? 0xFFFFFFFFu : s2;
    }
    W.JC[t * WAVE + lane] = make_uint2(ex | (m << 16), c);
  }
  wave_lds_sync();
}

// Speculative parallel walk of the chain from window position e0 over the segment tables: lane s
// guesses the chain's first position in segment s (q; valid: one lies in the segment) by walking
// at most LV_SPK segments — from e0 for the lanes up to LV_SPK segments past e0's, else from the
// first byte of segment s - LV_SPK (chains entering at different positions mostly meet within a
// few headers) — and r = its table entry, c its outputs, inc the inclusive sum of c over the
// lanes. The guesses are checked: each one's exit is the next valid lane's guess (leaving the
// window: there is none), for the lanes whose outputs start below lim (the walk's stop). A chain
// that never meets the true one (payload bytes parsed in another phase) makes its lane's guess
// wrong: then every lane walks again from the guess of the valid lane before it, up to LV_SPR
// rounds (a wrong guess between right ones is put right by one). When the check passes, the
// valid guesses are the chain (by induction from e0's segment, whose guess is e0), found with
// ~LV_SPK dependent table reads instead of one per segment. Returns false if it never passes.
#ifndef PQG_LV_SPK
#define PQG_LV_SPK 4
#endif
constexpr uint32_t LV_SPK = PQG_LV_SPK;  // segments walked per guess
#ifndef PQG_LV_SPEND
#define PQG_LV_SPEND 1
#endif
#ifndef PQG_LV_SPR
#define PQG_LV_SPR 4
#endif
constexpr uint32_t LV_SPR = PQG_LV_SPR;  // repair rounds
#ifndef PQG_LV_K2
#define PQG_LV_K2 4
#endif
constexpr uint32_t LV_K2 = PQG_LV_K2;  // window path: segments walked before the second chain (0: none)

__device__ inline bool lv_spec_chain(const LvWave& W, uint32_t e0, uint64_t lim, uint32_t& q, bool& valid, uint2& r,
                                     uint64_t& inc) {
  const uint32_t lane = threadIdx.x & 63u, lo = lane * LV_SEG;
  q = lane <= e0 / LV_SEG + LV_SPK ? e0 : lo - LV_SPK * LV_SEG;
#pragma unroll 1
  for (uint32_t round = 0;; ++round) {
#pragma unroll
    for (uint32_t it = 0; it < LV_SPK; ++it)
      if (q < lo) q = W.JC[(q % LV_SEG) * WAVE + q / LV_SEG].x & 0xFFFFu;  // (exits and codes >= LV_WIN stop)
    valid = q >= lo && q < lo + LV_SEG;
    r = valid ? W.JC[(q - lo) * WAVE + lane] : make_uint2(LV_J_END, 0u);
    const uint64_t vm = __ballot(valid);
    const uint64_t after = lane == 63u ? 0ull : vm & (~0ull << (lane + 1u));
    const uint32_t nxt = after ? (uint32_t)__builtin_ctzll(after) : 64u;
    const uint32_t gn = (uint32_t)__shfl((int)q, (int)(nxt & 63u), 64);
    const uint32_t xq = r.x & 0xFFFFu;
    const bool okl = xq < LV_WIN ? nxt < 64u && gn == xq : nxt == 64u;
    const uint32_t c = valid ? r.y : 0u;
    inc = wave_incl_scan_cnt(c);
    const uint64_t bad = __ballot(valid && inc - c < lim && inc < lim && !okl);
    if (!bad) return true;
#if PQG_LV_SPEND
    // the lanes up to the first bad one are verified; if that one leaves the window (or ends the
    // stream) the chain ends there and the guesses after it are off it (repairing them would take
    // a round per lane)
    const uint32_t b = (uint32_t)__builtin_ctzll(bad);
    if ((uint32_t)__shfl((int)xq, (int)b, 64) >= LV_WIN) {
      if (lane > b) {
        valid = false;
        r = make_uint2(LV_J_END, 0u);
      }
      inc = wave_incl_scan_cnt(valid ? r.y : 0u);
      return true;
    }
#endif
    if (round == LV_SPR) return false;
    // repair: from the guess of the valid lane before this one (e0 for the lanes before any)
    const uint64_t before = vm & ((1ull << lane) - 1ull);
    const int pv = before ? 63 - __builtin_clzll(before) : 0;
    const uint32_t gp = (uint32_t)__shfl((int)q, pv, 64);
    q = before ? gp : e0;
  }
}

// Output buffer of stream `sel` of a chunk: def / rep levels, RLE booleans.
__device__ inline uint8_t* lv_out(const ChunkWork& ck, int sel) {
  return sel == SS_DEF ? (uint8_t*)ck.def_out : sel == SS_REP ? (uint8_t*)ck.rep_out : ck.val_out;
}

// Max level of stream `sel` (the def count's test, column/reader.rs:212-226).
__device__ inline uint32_t lv_maxl(const ChunkWork& ck, int sel) {
  return sel == SS_DEF ? (uint32_t)ck.cp.max_def : sel == SS_REP ? (uint32_t)ck.cp.max_rep : 1u;
}

// A wave's contiguous range [g0, g1) of the dense pages' windows (wbase2): the page is found once
// and then advanced with the window, its stream parsed once per page (a grid-stride loop paid a
// binary search and the page's dependent loads per window).
struct LvDense {
  uint32_t g0, g1, pb, pend, wb;
  bool ok;
  uint8_t* out;   // the page's output buffer and max level (k_lv_emit), read once per page: a load
  uint32_t maxl;  // issued after a window's stores waits for them to complete (one vmcnt)
  __device__ inline void page(const uint8_t* blob, const PageWork* pages, const ChunkWork* chunks, int sel,
                              const RunTables& rt, const LevelTables& lt, LvWin& x) {
    pend = lt.wbase2[x.p + 1];
    wb = lt.wbase[x.p];
    ok = pend > pb && rt.pflag[x.p] == PF_PAGE && lv_stream(blob, pages[x.p], sel, chunks, x.s);
    const ChunkWork& ck = chunks[pages[x.p].chunk];
    out = lv_out(ck, sel);
    maxl = lv_maxl(ck, sel);
  }
  __device__ inline bool begin(const uint8_t* blob, const PageWork* pages, int npages, const ChunkWork* chunks, int sel,
                               const RunTables& rt, const LevelTables& lt, LvWin& x) {
    const uint32_t total = lt.wbase2[npages];
    const uint32_t nwv = gridDim.x * (WG / WAVE), gw = blockIdx.x * (WG / WAVE) + rfl(threadIdx.x >> 6);
    const uint32_t per = (total + nwv - 1u) / nwv;
    g0 = gw * per;
    g1 = min(total, g0 + per);
    if (g0 >= g1) return false;
    x.p = lv_page_of(lt.wbase2, (uint32_t)npages, g0);
    pb = lt.wbase2[x.p];
    page(blob, pages, chunks, sel, rt, lt, x);
    return true;
  }
  // window g2 (>= the last one asked): x.p / x.k / x.s set; false for a page off the window path
  __device__ inline bool at(const uint8_t* blob, const PageWork* pages, const ChunkWork* chunks, int sel,
                            const RunTables& rt, const LevelTables& lt, LvWin& x, uint32_t& g2) {
    while (g2 >= pend) {
      ++x.p;
      pb = pend;
      page(blob, pages, chunks, sel, rt, lt, x);
    }
    if (!ok) {
      g2 = pend - 1u;
      return false;
    }
    x.k = g2 - pb;
    return true;
  }
};

// The next window's staged bytes, loaded into registers while the current window is processed
// (window kernels: one global round trip per window otherwise stands between two windows).
struct LvPf {
  uint4 a, b;
  uint2 wi;  // k_lv_emit: the window's stitch result (lt.win), with its bytes
  uint64_t A;
  uint32_t p, k;
  bool ok;
  __device__ inline void issue(const uint8_t* __restrict__ blob, uint64_t blob_len, const LvWin& x, uint32_t k2,
                               const uint2* wsrc = nullptr) {
    if (wsrc) wi = wsrc[k2];
    const uint32_t lane = threadIdx.x & 63u;
    A = (x.s.S + (uint64_t)k2 * LV_WIN) & ~15ull;
    const uint64_t a0 = A + lane * 16u, a1 = A + (WAVE + lane) * 16u;
    a = a0 + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + a0) : gload_u128_tail(blob, blob_len, a0);
    b = lane + WAVE < LV_STG_CH ? (a1 + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + a1)
                                                       : gload_u128_tail(blob, blob_len, a1))
                                : make_uint4(0u, 0u, 0u, 0u);
    p = x.p;
    k = k2;
    ok = true;
  }
  // window x's stage: from the registers when they hold it, else loaded now
  __device__ inline void stage(const uint8_t* __restrict__ blob, uint64_t blob_len, LvWin& x, uint32_t* st) {
    if (!(ok && p == x.p && k == x.k)) {
      lv_stage(blob, blob_len, x, st, LV_STG_CH);
      return;
    }
    const uint32_t lane = threadIdx.x & 63u;
    x.sb = (uint32_t)(x.s.S + x.W0 - A);
    x.cap = LV_STG_CH * 16u;
    reinterpret_cast<uint4*>(st)[lane] = a;
    if (lane + WAVE < LV_STG_CH) reinterpret_cast<uint4*>(st)[WAVE + lane] = b;
    ok = false;
    wave_lds_sync();
  }
};

// ------------------------------------------------------------------------------ k_lv_win
// Window path: windows g2 of the dense pages (wbase2); g = the page's window in wbase terms.
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(4))) k_lv_win(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                               const PageWork* __restrict__ pages, int npages,
                                               const ChunkWork* chunks, int sel, RunTables rt, LevelTables lt) {
  __shared__ LvSmem sm;
  const uint32_t wid = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  LvWave& W = sm.wv[wid];
  LvDense D;
  LvWin x;
  LvPf pf;
  pf.ok = false;
  if (!D.begin(blob, pages, npages, chunks, sel, rt, lt, x)) return;
#ifdef PQG_DIAG
  // diagnostics (PQG_DEBUG bit 2048, bit width 1): per wave s_memtime cycles in the stage wait, the
  // segment tables, the chain from 0 and the entry walks, the reference choice (and second chain),
  // the table writes; the windows, and those that needed a second chain
  const bool wst = (chunks[0].cp.debug & 2048) && chunks[0].cp.dbgbuf;
  uint64_t wt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, wt0 = 0;
#define LWN_STAMP(k)                                  \
  if (wst) {                                          \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(); \
    wt[k] += t1 - wt0;                                \
    wt0 = t1;                                         \
  }
#else
#define LWN_STAMP(k)
#endif
  for (uint32_t g2 = D.g0; g2 < D.g1; ++g2) {
    if (!D.at(blob, pages, chunks, sel, rt, lt, x, g2)) continue;
#ifdef PQG_DIAG
    if (wst) wt0 = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t g = D.wb + x.k;
    x.W0 = x.k * LV_WIN;
    const uint32_t w = (uint32_t)x.s.w;
    pf.stage(blob, blob_len, x, W.stage);
    if (g2 + 1 < D.g1 && g2 + 1 < D.pend) pf.issue(blob, blob_len, x, x.k + 1);
    LWN_STAMP(0)
    // table of the entry offsets: (exit offset from W0 or terminal code | headers << 16, outputs)
    const uint32_t ent = lv_ent(w);
    uint2* tab = lt.tab + (uint64_t)g * lt.tstride;
    if (w == 1) {  // 64 entry offsets: lane e follows entry e across the segments
      uint32_t pc[LV_SEG], pv[LV_SEG], bpm;
      lv_seg_build(W, x, pc, pv, bpm);
      LWN_STAMP(1)
      uint32_t e = lane, c = 0, me = 0xFFFFu;
      // the chain from position 0, speculatively (lv_spec_chain); each entry's chain is then
      // followed only until it meets it (me: where), the rest from the chain's per-segment suffix
      // sums
      uint32_t q;
      bool valid;
      uint2 r;
      uint64_t ci;
      const bool spec = lv_spec_chain(W, 0u, ~0ull, q, valid, r, ci);
      uint32_t* sp = W.stage;  // (staged bytes no longer needed): chain position, output suffixes
      uint32_t exitc = LV_J_END;
      if (spec) {
        const uint32_t cc = valid ? r.y : 0u;
        const uint64_t ctot = __shfl(ci, 63, 64);
        const uint64_t vm = __ballot(valid);
        exitc = (uint32_t)__shfl((int)(r.x & 0xFFFFu), 63 - __builtin_clzll(vm), 64);  // (lane 0 is valid)
        const uint64_t cs = ctot - ci + cc;
        sp[lane] = valid ? q : LV_NONE;
        sp[128 + lane] = cs > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cs;
        wave_lds_sync();
      }
      // entries still off the chain after LV_K2 segments are mostly on one other chain (when
      // position 0 is inside a run's values its chain soon ends: 21% of the windows at p_null
      // 0.1): that chain too is built speculatively, from the first such entry, and they meet it
      // instead of walking every segment of the window
      uint32_t exit2 = LV_J_END, hops = 0, m2 = 0xFFFFu;  // m2: where the second chain meets the first
      uint32_t ref2 = 0;  // the second chain's headers in this lane's segment
      bool two = false;
#pragma unroll 1
      while (__any(e < LV_WIN)) {
        if (e < LV_WIN) {
          const uint32_t sg = e / LV_SEG;
          uint32_t dc;
          if (spec && sp[sg] == e) {  // on the chain from 0: its rest
            me = me == 0xFFFFu ? e : me;
            dc = sp[128 + sg];
            e = exitc;
          } else if (two && sp[64 + sg] == e) {  // on the second chain: its rest
            me = me == 0xFFFFu ? m2 : me;
            dc = sp[192 + sg];
            e = exit2;
          } else {
            const uint2 t = W.JC[(e % LV_SEG) * WAVE + sg];
            dc = t.y;
            e = t.x & 0xFFFFu;
          }
          const uint32_t s2 = c + dc;
          c = s2 < c ? 0xFFFFFFFFu : s2;
        }
        if (++hops == LV_K2 && spec) {
          const uint64_t un = __ballot(e < LV_WIN);
          if (un) {
            const uint32_t f = (uint32_t)__builtin_ctzll(un);  // (from that entry: the whole chain)
            uint32_t q2;
            bool v2;
            uint2 r2;
            uint64_t ci2;
            if (lv_spec_chain(W, f, ~0ull, q2, v2, r2, ci2)) {
              const uint32_t cc = v2 ? r2.y : 0u;
              const uint64_t ctot = __shfl(ci2, 63, 64);
              const uint64_t vm = __ballot(v2);
              exit2 = (uint32_t)__shfl((int)(r2.x & 0xFFFFu), 63 - __builtin_clzll(vm), 64);
              const uint64_t cs = ctot - ci2 + cc;
              sp[64 + lane] = v2 ? q2 : LV_NONE;
              ref2 = v2 ? r2.x >> 16 : 0u;
              sp[192 + lane] = cs > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cs;
              const uint64_t mg = __ballot(v2 && sp[lane] == q2);
              m2 = mg ? (uint32_t)__builtin_amdgcn_readlane((int)q2, (int)__builtin_ctzll(mg)) : 0xFFFFu;
              wave_lds_sync();
              two = true;
            }
          }
        }
      }
      LWN_STAMP(2)
      // the reference chain of the window's emit (k_lv_emit: the true chain's headers are its
      // headers from where the true entry's chain meets it, and the few before): the chain most
      // entries leave the window by (the chain from 0 when entry 0 is one of them), so that the
      // true entry, whichever it is, almost always meets it inside the window
      uint32_t bx = 0, bn = 0, bl = 0;
      for (uint64_t rem = ~0ull; rem;) {
        const uint32_t ld = (uint32_t)__builtin_ctzll(rem);
        const uint32_t xv = (uint32_t)__builtin_amdgcn_readlane((int)e, (int)ld);
        const uint64_t m = __ballot(e == xv);
        const uint32_t nm = (uint32_t)__builtin_popcountll(m);
        if (nm > bn) {
          bn = nm;
          bx = xv;
          bl = ld;
        }
        rem &= ~m;
      }
      uint16_t ref = (uint16_t)(spec && valid ? (r.x >> 16) : 0u);
      const uint32_t e0x = (uint32_t)__builtin_amdgcn_readlane((int)e, 0);
      if (!spec) me = 0xFFFFu;
      if (spec && e0x != bx) {  // another chain leaves by the majority exit: it is the reference
        uint32_t sb = 64;       // (the second chain's positions when it is that chain)
        bool rk = true;
        me = 0xFFFFu;
        if (two && exit2 == bx) {
          ref = (uint16_t)ref2;
        } else {
          wave_lds_sync();  // (every read of sp is done)
          sb = 0;
          ref = 0;
          rk = lv_spec_chain(W, bl, ~0ull, q, valid, r, ci);
          if (rk) {
            sp[lane] = valid ? q : LV_NONE;
            ref = (uint16_t)(valid ? (r.x >> 16) : 0u);
            wave_lds_sync();
          }
        }
        if (rk) {  // where the entries that leave by it meet it (those that do not never do)
          uint32_t f = lane;
#pragma unroll 1
          while (__any(f < LV_WIN && me == 0xFFFFu && e == bx)) {
            if (f < LV_WIN && me == 0xFFFFu && e == bx) {
              const uint32_t sg = f / LV_SEG;
              if (sp[sb + sg] == f) me = f;
              else f = W.JC[(f % LV_SEG) * WAVE + sg].x & 0xFFFFu;
            }
          }
        }
      }
#ifdef PQG_DIAG
      if (wst) wt[6] += spec && e0x != bx ? 1u : 0u;
      // entry-walk steps, windows whose chain from 0 failed, those with a second chain
      if (wst) wt[7] += hops + (!spec ? (1ull << 24) : 0ull) + (two ? (1ull << 44) : 0ull);
#endif
      LWN_STAMP(3)
      lt.bmp[(uint64_t)g * WAVE + lane] = ref;
      tab[lane] = make_uint2(e | (me << 16), c);
      wave_lds_sync();  // the next window's stage and table
      LWN_STAMP(4)
#ifdef PQG_DIAG
      if (wst) wt[5] += 1;
#endif
      continue;
    }
    uint32_t jv[LV_PPL], cv[LV_PPL];
    lv_jump(W, x, jv, cv);
#pragma unroll
    for (uint32_t j = 0; j < LV_PPL; ++j) {
      const uint32_t i = j * WAVE + lane;
      if (i < ent) tab[i] = make_uint2(jv[j], cv[j]);
    }
  }
#ifdef PQG_DIAG
  if (wst && lane == 0) {
    uint64_t* d = chunks[0].cp.dbgbuf + 8ull * (blockIdx.x * (WG / WAVE) + wid);
    for (int i = 0; i < 8; ++i) d[i] = wt[i];
  }
#endif
#undef LWN_STAMP
}

// ------------------------------------------------------------------------------ k_lv_stitch
// One 1024-thread workgroup per dense page: the true entry and first output of every window of
// the page, i.e. the chain of window tables followed from offset 0. The tables come through LDS
// in chunks of SC_ENT entries (the next chunk's loads in flight in registers meanwhile); within
// a chunk every wave composes the tables of its m windows for all entry offsets at once (one
// lane per entry: m LDS lookups), one wave then follows the chunk's wave compositions and every
// wave walks its windows from its true entry, writing them. With at most 128 entry offsets per
// window (bit widths 1 and 2) those two serial walks read the compositions and tables from
// VGPRs (v_readlane: a few cycles per step instead of an LDS round trip). A chain that leaves
// the composable form (a hop past the next window, a terminal code, a saturated count) before n
// outputs is followed window by window by one lane, as the tables give it.
constexpr uint32_t SC_ENT = 6144;   // table entries staged per chunk (48 KiB)
constexpr uint32_t SC_FENT = 2048;  // composition entries (16 KiB)
constexpr uint32_t SC_WG = 1024;
constexpr uint32_t SC_NW = SC_WG / WAVE;
constexpr uint32_t SC_MMAX = 6;     // windows per wave with readlane walks (EPL 1: 96 / 16)
constexpr uint32_t SC_SPEC = 0x80000000u;  // composition left the composable form

__device__ inline bool lv_stitch_serial(const uint2* __restrict__ tab, uint2* win, uint32_t nw, uint32_t ent,
                                        uint32_t stride, uint32_t n, uint32_t slen) {
  uint32_t cur = 0, e = 0;
  uint64_t acc = 0;
  while (cur < nw) {
    const uint2 t = tab[(uint64_t)cur * stride + e];
    win[cur] = make_uint2(e | (t.x & 0xFFFF0000u), (uint32_t)acc);  // entry | headers << 16
    acc += t.y;
    if (acc >= n) return true;
    const uint32_t jt = t.x & 0xFFFFu;
    if (jt >= LV_J_FAR || t.y == 0xFFFFFFFFu) return false;  // far / end / dead, or a saturated count
    const uint32_t q = cur * LV_WIN + jt;
    cur = q / LV_WIN;
    e = q - cur * LV_WIN;
    if (q >= slen || cur >= nw || e >= ent) return false;  // the stream ends before n outputs, or an
  }                                                         // entry past the table (foreign long runs)
  return false;
}

// Lane e of an EPL-VGPR "table" (entry e = j * 64 + lane in VGPR j), e wave-uniform.
template <uint32_t EPL>
__device__ inline uint32_t sc_rl(const uint32_t (&v)[EPL], uint32_t e) {
  if (EPL == 1) return (uint32_t)__builtin_amdgcn_readlane((int)v[0], (int)(e & 63u));
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)v[0], (int)(e & 63u));
  const uint32_t b = (uint32_t)__builtin_amdgcn_readlane((int)v[EPL - 1], (int)(e & 63u));
  return e >= 64u ? b : a;
}

template <uint32_t EPL>  // entries per lane (ent / 64): 1, 2 (readlane walks: streams of bit width 1 / 2) or
                        // 0 (any ent, LDS walks: wider streams)
__global__ void __launch_bounds__(SC_WG) k_lv_stitch(const uint8_t* __restrict__ blob, const PageWork* __restrict__ pages,
                                                     int npages, const ChunkWork* chunks, int sel, RunTables rt,
                                                     LevelTables lt) {
  __shared__ uint2 tb[SC_ENT];
  __shared__ uint2 F[SC_FENT];  // per composing wave and entry offset: (exit entry | SC_SPEC, outputs)
  __shared__ uint32_t went[SC_NW];
  __shared__ uint64_t wacc[SC_NW];
  __shared__ uint64_t acc_s;
  __shared__ uint32_t e_s, ok_s, serial_s, nv_s;
  const uint32_t p = blockIdx.x, tid = threadIdx.x, wid = tid >> 6, lane = tid & 63u;
  if (p >= (uint32_t)npages || rt.pflag[p] != PF_PAGE) return;
  const PageWork& pw = pages[p];
  Stream s;
  if (!lv_stream(blob, pw, sel, chunks, s)) return;
  if (EPL == 1 ? s.w != 1 : EPL == 2 ? s.w != 2 : s.w <= 2) return;  // another launch's width
  const uint32_t k0 = lt.wbase[p], nw = lt.wbase[p + 1] - k0;
  uint2* win = lt.win + k0;
  for (uint32_t k = tid; k < nw; k += SC_WG) win[k] = make_uint2(LV_NONE, 0u);
  if (nw == 0) return;
  const uint32_t ent = EPL ? EPL * WAVE : lv_ent((uint32_t)s.w), n = s.n, slen = s.slen;
  const uint32_t CW = SC_ENT / ent;                        // windows per chunk
  const uint32_t amax = min(SC_NW, SC_FENT / ent);         // composing waves at most
  const uint32_t m = (CW + amax - 1) / amax;               // windows per wave
  const uint32_t A = (CW + m - 1) / m;                     // composing waves
  const uint32_t nch = (nw + CW - 1) / CW;
  const uint32_t ts = lt.tstride;  // table row stride (>= ent; rows of ent entries are staged)
  const uint32_t lge = 31u - __builtin_clz(ent);  // (ent: a power of two)
  const uint2* tab = lt.tab + (uint64_t)k0 * ts;
  constexpr uint32_t PF = SC_ENT / SC_WG;
  uint2 pf[PF];
  auto fetch = [&](uint32_t c) {
    const uint32_t cnt = min(CW, nw - c * CW) * ent;
    const uint2* src = tab + (uint64_t)c * CW * ts;
#pragma unroll
    for (uint32_t i = 0; i < PF; ++i) {
      const uint32_t idx = tid + i * SC_WG;
      pf[i] = idx < cnt ? src[(uint64_t)(idx >> lge) * ts + (idx & (ent - 1u))] : make_uint2(LV_J_DEAD, 0u);
    }
  };
  fetch(0);
  if (tid == 0) {
    acc_s = 0;
    e_s = 0;
    ok_s = serial_s = 0;
  }
  __syncthreads();  // (also orders the NONE marks before the window writes)
  for (uint32_t c = 0; c < nch; ++c) {
    const uint32_t cnt = min(CW, nw - c * CW), cw0 = c * CW;
#pragma unroll
    for (uint32_t i = 0; i < PF; ++i) tb[tid + i * SC_WG] = pf[i];
    __syncthreads();
    if (c + 1 < nch) fetch(c + 1);  // in flight while this chunk is composed and walked
    // compositions: wave v over windows [v * m, v * m + m) of the chunk, every entry offset
    const uint32_t wlo = wid * m, whi = min(cnt, wlo + m);
    if (wid < A && wlo < cnt) {
      for (uint32_t e = lane; e < ent; e += WAVE) {
        uint32_t ce = e, out = 0, spec = 0;
        for (uint32_t k = wlo; k < whi; ++k) {
          const uint2 t = tb[k * ent + ce];
          const uint32_t o2 = out + t.y;
          out = o2 < out ? 0xFFFFFFFFu : o2;
          const uint32_t jt = t.x & 0xFFFFu;
          const uint32_t kn = cw0 + k + 1u;  // the page window the hop lands in, if composable
          if (t.y == 0xFFFFFFFFu || jt < LV_WIN || jt >= 2u * LV_WIN || jt - LV_WIN >= ent || kn >= nw ||
              kn * LV_WIN + (jt - LV_WIN) >= slen) {
            spec = SC_SPEC;
            break;
          }
          ce = jt - LV_WIN;
        }
        F[wid * ent + e] = make_uint2(ce | spec, out);
      }
    }
    __syncthreads();
    // the chunk's chain over the wave compositions
    if (EPL) {
      if (wid == 0) {
        constexpr uint32_t E = EPL ? EPL : 1;
        uint32_t fx[SC_NW][E], fy[SC_NW][E];
#pragma unroll
        for (uint32_t v = 0; v < SC_NW; ++v)
#pragma unroll
          for (uint32_t j = 0; j < E; ++j) {
            const uint2 f = v < A ? F[v * ent + j * WAVE + lane] : make_uint2(0u, 0u);
            fx[v][j] = f.x;
            fy[v][j] = f.y;
          }
        uint32_t e = rfl(e_s), nv = 0, ok = 0, ser = 0;
        uint64_t acc = acc_s;
#pragma unroll
        for (uint32_t v = 0; v < SC_NW; ++v) {
          if (v < A && v * m < cnt && !ok && !ser) {
            if (lane == v) {
              went[v] = e;
              wacc[v] = acc;
            }
            nv = v + 1;
            const uint32_t x = sc_rl<E>(fx[v], e), y = sc_rl<E>(fy[v], e);
            acc += y;
            if (acc >= n) ok = 1;
            else if (x & SC_SPEC) ser = 1;  // not composable before n: one lane follows the tables
            else e = x;
          }
        }
        if (lane == 0) {
          e_s = e;
          acc_s = acc;
          ok_s = ok;
          serial_s = ser;
          nv_s = ser ? 0u : nv;
        }
      }
    } else if (tid == 0) {
      uint32_t e = e_s, nv = 0;
      uint64_t acc = acc_s;
      for (uint32_t v = 0; v < A && v * m < cnt; ++v) {
        went[v] = e;
        wacc[v] = acc;
        nv = v + 1;
        const uint2 f = F[v * ent + e];
        acc += f.y;
        if (acc >= n) {
          ok_s = 1;
          break;
        }
        if (f.x & SC_SPEC) {
          serial_s = 1;
          break;
        }
        e = f.x;
      }
      e_s = e;
      acc_s = acc;
      nv_s = serial_s ? 0u : nv;
    }
    __syncthreads();
    // every wave on the chain walks its windows from its true entry
    if (wid < nv_s) {
      if (EPL) {
        constexpr uint32_t E = EPL ? EPL : 1;
        uint32_t tx[SC_MMAX][E], ty[SC_MMAX][E];
#pragma unroll
        for (uint32_t k = 0; k < SC_MMAX; ++k)
#pragma unroll
          for (uint32_t j = 0; j < E; ++j) {
            const uint2 t = wlo + k < whi ? tb[(wlo + k) * ent + j * WAVE + lane] : make_uint2(0u, 0u);
            tx[k][j] = t.x;
            ty[k][j] = t.y;
          }
        uint32_t e = rfl(went[wid]);
        uint64_t acc = wacc[wid];
        bool done = false;
#pragma unroll
        for (uint32_t k = 0; k < SC_MMAX; ++k) {
          if (wlo + k < whi && !done) {
            const uint32_t x = sc_rl<E>(tx[k], e), y = sc_rl<E>(ty[k], e);
            if (lane == 0) win[cw0 + wlo + k] = make_uint2(e | (x & 0xFFFF0000u), (uint32_t)acc);
            acc += y;
            if (acc >= n) done = true;
            e = (x & 0xFFFFu) - LV_WIN;
          }
        }
      } else if (lane == 0) {
        uint32_t e = went[wid];
        uint64_t acc = wacc[wid];
        for (uint32_t k = wlo; k < whi; ++k) {
          const uint2 t = tb[k * ent + e];
          win[cw0 + k] = make_uint2(e | (t.x & 0xFFFF0000u), (uint32_t)acc);
          acc += t.y;
          if (acc >= n) break;
          e = (t.x & 0xFFFFu) - LV_WIN;
        }
      }
    }
    __syncthreads();
    if (ok_s || serial_s) break;
  }
  if (tid == 0) {
    bool ok = ok_s != 0;
    if (serial_s) ok = lv_stitch_serial(tab, win, nw, ent, ts, n, slen);
    if (!ok) LV_BAIL(rt, lt, p, PF_PAGE, 2);
  }
}

// ------------------------------------------------------------------------------ output writers

// 64-bit little-endian window of stream bytes at stream offset q: staged or from global memory.
__device__ inline uint64_t lv_bytes8(const uint32_t* stage, const uint8_t* __restrict__ blob,
                                     uint64_t blob_len, const LvWin& x, uint32_t q) {
  const uint32_t r = q - x.W0 + x.sb;
  if (q >= x.W0 && r + 12 <= x.cap) return lload_u64(stage, r);
  return gload_u64(blob, blob_len, x.s.S + q);
}

#ifndef PQG_LV_BMW
#define PQG_LV_BMW 1  // payload bits by aligned stage dword pairs (0: unaligned 8-byte reads, A/B runs)
#endif

// 32 bits of the stream from bit `bit` (stream-relative): an aligned dword pair of the stage and
// one funnel shift when staged, else from global memory.
__device__ inline uint32_t lv_bits32(const uint32_t* stage, const uint8_t* __restrict__ blob, uint64_t blob_len,
                                     const LvWin& x, uint64_t bit) {
  const uint32_t q = (uint32_t)(bit >> 3);
  if (PQG_LV_BMW && q >= x.W0) {
    const uint64_t B = bit - (uint64_t)x.W0 * 8u + (uint64_t)x.sb * 8u;  // (stage bit)
    if ((B >> 3) + 8u <= x.cap) {
      const uint32_t b = (uint32_t)B;
      return __builtin_amdgcn_alignbit(stage[(b >> 5) + 1u], stage[b >> 5], b & 31u);
    }
  }
  return (uint32_t)(lv_bytes8(stage, blob, blob_len, x, q) >> (bit & 7u));
}

__device__ inline uint32_t wave_sum_u32_(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
  return v;
}

// Outputs [o, e) (page-relative, e - o <= 32) of run `info` starting at output `start`, w = 1:
// bit j = output o + j.
__device__ inline uint32_t lv_run_bits1(const uint32_t* stage, const uint8_t* __restrict__ blob, uint64_t blob_len,
                                        const LvWin& x, uint32_t start, uint32_t info, uint32_t o, uint32_t e) {
  const uint32_t nb = e - o;
  const uint32_t m = nb >= 32 ? 0xFFFFFFFFu : (1u << nb) - 1u;
  if (info & R_RLE) return (info & 1u) ? m : 0u;
  const uint64_t bit = (uint64_t)info * 8ull + (o - start);
  return lv_bits32(stage, blob, blob_len, x, bit) & m;
}

// Run list in LDS: runs [0, R), rstart[R] = 0xFFFFFFFF; the window writes page outputs
// [base, endo) (base = rstart[0]).
struct LvRuns {
  const uint32_t* rstart;
  const uint32_t* rinfo;
  uint32_t R;
};

// One-bit outputs. Each step the wave builds 64 consecutive 32-output words (aligned on the
// global output index), one per lane, from the runs covering them; then the words are
// redistributed (ds_bpermute) so that every store instruction covers one contiguous 1 KiB:
// lane l stores outputs [8l, 8l + 8) (int16) or [16l, 16l + 16) (bytes) of each KiB. Chunks
// shared with a neighbouring window are stored element by element, inside [base, endo) only.
// Returns this lane's count of 1s.
template <int OUT>
__device__ inline uint32_t lv_write1(const LvRuns& rl, const uint32_t* stage, const uint8_t* __restrict__ blob,
                                     uint64_t blob_len, const LvWin& x, uint32_t base, uint32_t endo,
                                     gptr<uint8_t> __restrict__ out) {
  constexpr uint32_t V = 16u / OUT;        // outputs per 16-byte chunk
  constexpr uint32_t NQ = 64u * 32u / (V * 64u);  // store instructions per step (4 / 2)
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t go = x.s.out;  // global index of the page's output 0
  const uint64_t lo = go + base, hi = go + endo;
  if (rl.R == 1 && (rl.rinfo[0] & R_RLE)) {  // one RLE run (a page of equal levels): a fill
    const uint32_t bit = rl.rinfo[0] & 1u;
    const uint32_t d = OUT == 2 ? bit * 0x00010001u : bit * 0x01010101u;
    const uint4 v = make_uint4(d, d, d, d);
    uint64_t c0 = (lo + V - 1) / V, c1 = hi / V;  // whole 16-byte chunks inside [lo, hi)
    if (c1 < c0) c1 = c0;
#pragma unroll 4
    for (uint64_t c = c0 + lane; c < c1; c += WAVE) gst16(out + c * 16u, v);
    // the edges (fewer than V outputs each), element by element
    const uint64_t h1 = c0 * V < hi ? c0 * V : hi, t0 = c1 * V > h1 ? c1 * V : h1;
    const uint64_t gi = lane < V ? lo + lane : t0 + (lane - V);
    if ((lane < V && gi < h1) || (lane >= V && lane < 2 * V && gi < hi)) {
      if (OUT == 2) reinterpret_cast<gptr<int16_t>>(out)[gi] = (int16_t)bit;
      else out[gi] = (uint8_t)bit;
    }
    return lane == 0 ? bit * (uint32_t)(hi - lo) : 0u;
  }
  const uint64_t A0 = lo & ~31ull;
  const uint32_t nwords = (uint32_t)((hi - A0 + 31u) >> 5);
  uint32_t lgn = 1;
  while (lgn * 2u <= rl.R) lgn *= 2u;
  uint32_t cnt = 0;
#pragma unroll 1
  for (uint32_t w0 = 0; w0 < nwords; w0 += WAVE) {
    const uint32_t wd = w0 + lane;
    const uint64_t ga = A0 + (uint64_t)wd * 32u;
    uint32_t bits = 0;
    if (wd < nwords) {
      const uint32_t pa = (uint32_t)(ga - go);  // page-relative output of bit 0 (may wrap)
      const uint32_t olo = ga >= lo ? pa : base;
      const uint32_t ohi = ga + 32u <= hi ? pa + 32u : endo;
      uint32_t b = 0;  // last run starting at or before olo
      for (uint32_t sp = lgn; sp; sp >>= 1)
        if (b + sp < rl.R && rl.rstart[b + sp] <= olo) b += sp;
      for (uint32_t o = olo; o < ohi; ++b) {
        const uint32_t nst = rl.rstart[b + 1];
        const uint32_t e = nst < ohi ? nst : ohi;
        if (e > o) bits |= lv_run_bits1(stage, blob, blob_len, x, rl.rstart[b], rl.rinfo[b], o, e) << (o - pa);
        o = e > o ? e : o;
      }
      cnt += __builtin_popcount(bits);
    }
    const uint64_t gb = A0 + (uint64_t)w0 * 32u;  // global output of this step's bit 0
#pragma unroll
    for (uint32_t q = 0; q < NQ; ++q) {
      const uint32_t per = 32u / V;  // chunks per word
      const uint32_t wv = (uint32_t)__shfl((int)bits, (int)(q * (WAVE / per) + lane / per), 64);
      const uint32_t cb = (wv >> (V * (lane % per))) & ((1u << V) - 1u);
      const uint64_t gc = gb + (uint64_t)(q * WAVE + lane) * V;  // the chunk's first output
      if (gc >= hi || gc + V <= lo) continue;
      if (gc >= lo && gc + V <= hi) {
        uint32_t d[4];
#pragma unroll
        for (uint32_t t = 0; t < 4; ++t)
          d[t] = OUT == 2 ? (((cb >> (2u * t)) & 3u) * 0x8001u) & 0x10001u
                          : (((cb >> (4u * t)) & 15u) * 0x204081u) & 0x01010101u;
        gst16(out + gc * OUT, make_uint4(d[0], d[1], d[2], d[3]));
      } else {
        for (uint32_t j = 0; j < V; ++j) {
          const uint64_t gi = gc + j;
          if (gi >= lo && gi < hi) {
            if (OUT == 2) reinterpret_cast<gptr<int16_t>>(out)[gi] = (int16_t)((cb >> j) & 1u);
            else out[gi] = (uint8_t)((cb >> j) & 1u);
          }
        }
      }
    }
  }
  return cnt;
}

// Bit width 1, a dense window whose true headers are known per segment (lane l: the mask mym of
// positions [16 l, 16 l + 16), its first output oa): the lane parses its own headers once and ORs
// their bits into a bitmap of the window's outputs in LDS (the jump table's space: 32-output
// words aligned on the global output index; a word two lanes share is merged by the OR), then
// the wave stores the bitmap expanded, one contiguous KiB per store instruction. The run list
// (lv_write1: a binary search and a walk over the runs per word) is not built at all. Taken when
// the words fit and no lane generates more than LV_BM_SPAN outputs (a long RLE run: word by
// word on one lane); returns false, nothing stored, at a run the window path does not take.
constexpr uint32_t LV_BM_WORDS = LV_WIN * 2;  // bitmap words (the jump table's 8 KiB)
constexpr uint32_t LV_BM_SPAN = 2048;         // outputs one lane generates at most
#ifndef PQG_LV_BM
#define PQG_LV_BM 1  // (0: every dense window through the run list, for A/B runs)
#endif

__device__ inline bool lv_bm_fits(const LvWin& x, uint32_t base, uint64_t endo, uint64_t span) {
  if (!PQG_LV_BM) return false;
  const uint64_t lo = x.s.out + base, hi = x.s.out + endo;
  return !__ballot(span > LV_BM_SPAN) && ((hi - (lo & ~31ull) + 31u) >> 5) <= LV_BM_WORDS;
}

// The window's bitmap: outputs [lo, hi) of the page at bits (global output - A0) of words
// bm[0, nw), A0 = lo rounded down to 32.
struct LvBm {
  uint64_t A0;
  uint32_t ra, rb, nw;  // [lo, hi) - A0; words
  __device__ LvBm(const LvWin& x, uint32_t base, uint32_t endo) {
    const uint64_t lo = x.s.out + base;
    A0 = lo & ~31ull;
    ra = (uint32_t)(lo - A0);
    rb = ra + (endo - base);
    nw = (rb + 31u) >> 5;
  }
};

// Generation: each lane ORs its own runs' bits (outputs from oa, page-relative) into the bitmap.
// Returns the lane's count of 1s, or 0xFFFFFFFF for the whole wave at a run the window path does
// not take.
__device__ inline uint32_t lv_bm_gen(const uint32_t* stage, uint32_t* bm, const uint8_t* __restrict__ blob,
                                     uint64_t blob_len, const LvWin& x, const LvBm& B, uint32_t mym, uint64_t oa,
                                     uint32_t n) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t slen = x.s.slen, i0 = lane * LV_SEG;
  wave_lds_sync();  // (the jump table / prefix list is read)
  for (uint32_t i = lane; i < B.nw; i += WAVE) bm[i] = 0u;
  wave_lds_sync();
  bool bad = false;
  uint32_t cw = 0xFFFFFFFFu, cb = 0, cnt = 0;
  uint32_t rs = B.ra + (uint32_t)(oa - (B.A0 + B.ra - x.s.out));  // the lane's first output, bitmap-relative
#pragma unroll 1
  for (uint32_t m = mym; m; m &= m - 1u) {
    const uint32_t t = (uint32_t)__builtin_ctz(m);
    uint32_t nx, c, v;
    bool bp;
    lv_parse4(stage, i0 + t + x.sb, x.W0 + i0 + t, slen, 1u, 1u, nx, c, v, bp);  // (a true header: parses)
    bad |= !lv_run_ok(bp, v, c, oa, n, slen, 1u);
    const uint32_t e = (uint64_t)rs + c < B.rb ? rs + c : B.rb;
#pragma unroll 1
    for (uint32_t q = rs; q < e;) {
      const uint32_t wi = q >> 5, bpos = q & 31u;
      const uint32_t take = e - q < 32u - bpos ? e - q : 32u - bpos;
      const uint32_t mk = take >= 32u ? 0xFFFFFFFFu : (1u << take) - 1u;
      uint32_t bits;
      if (bp) {
        const uint32_t d = q - rs;
        // (32-bit stage arithmetic here: the generic lv_bits32 measured 7% slower in this loop)
        const uint32_t B = (v - x.W0 + x.sb) * 8u + d;  // (the payload's stage bit)
        if (PQG_LV_BMW && v >= x.W0 && (B >> 3) + 8u <= x.cap)
          bits = __builtin_amdgcn_alignbit(stage[(B >> 5) + 1u], stage[B >> 5], B & 31u) & mk;
        else
          bits = (uint32_t)(lv_bytes8(stage, blob, blob_len, x, v + (d >> 3)) >> (d & 7u)) & mk;
      } else {
        bits = (v & 1u) ? mk : 0u;
      }
      if (wi != cw) {
        if (cb) atomicOr(&bm[cw], cb);
        cnt += (uint32_t)__builtin_popcount(cb);
        cw = wi;
        cb = 0;
      }
      cb |= bits << bpos;
      q += take;
    }
    oa += c;
    rs = (uint64_t)rs + c < B.rb ? rs + c : B.rb;
  }
  if (cb) atomicOr(&bm[cw], cb);
  cnt += (uint32_t)__builtin_popcount(cb);
  return __ballot(bad) ? 0xFFFFFFFFu : cnt;
}

// Stores: the bitmap expanded, one contiguous KiB per store instruction (chunks shared with a
// neighbouring window element by element), and the page's def count.
template <int OUT>
__device__ inline void lv_bm_store(const uint32_t* bm, const LvWin& x, const LvBm& B, uint32_t cnt, int sel,
                                   PageWork* pages, gptr<uint8_t> __restrict__ out) {
  constexpr uint32_t V = 16u / OUT;  // outputs per 16-byte chunk
  const uint32_t lane = threadIdx.x & 63u;
  wave_lds_sync();
  gptr<uint8_t> ob = out + B.A0 * OUT;
  // chunks [c0, c1) lie inside [ra, rb); chunk ka (holding ra) and kb (holding rb - 1) may not
  const uint32_t c0 = (B.ra + V - 1u) / V, c1 = B.rb / V, ka = B.ra / V, kb = (B.rb - 1u) / V;
#pragma unroll 2
  for (uint32_t k = c0 + lane; k < c1; k += WAVE) {
    const uint32_t cbits = (bm[k * V / 32u] >> ((k * V) & 31u)) & ((1u << V) - 1u);
    uint32_t d[4];
#pragma unroll
    for (uint32_t t = 0; t < 4; ++t)
      d[t] = OUT == 2 ? (((cbits >> (2u * t)) & 3u) * 0x8001u) & 0x10001u
                      : (((cbits >> (4u * t)) & 15u) * 0x204081u) & 0x01010101u;
    gst16(ob + k * 16u, make_uint4(d[0], d[1], d[2], d[3]));
  }
  const bool ea = lane == 0 && c0 > ka, eb = lane == 1 && c1 <= kb && !(kb == ka && c0 > ka);
  if (ea || eb) {
    const uint32_t kk = ea ? ka : kb;
    for (uint32_t j = 0; j < V; ++j) {
      const uint32_t r = kk * V + j;
      if (r >= B.ra && r < B.rb) {
        const uint32_t b = (bm[r >> 5] >> (r & 31u)) & 1u;
        if (OUT == 2) reinterpret_cast<gptr<int16_t>>(ob)[r] = (int16_t)b;
        else ob[r] = (uint8_t)b;
      }
    }
  }
  if (sel == SS_DEF) {
    cnt = wave_sum_u32_(cnt);
    if (lane == 0 && cnt) atomicAdd((unsigned long long*)&pages[x.p].nonnull, (unsigned long long)cnt);
  }
}

// Wider levels: groups of G outputs (one 16-byte store), each from the runs covering it.
// Returns this lane's count of outputs == maxl.
template <int OUT>
__device__ inline uint32_t lv_write_wide(const LvRuns& rl, const uint32_t* stage, const uint8_t* __restrict__ blob,
                                         uint64_t blob_len, const LvWin& x, uint32_t base, uint32_t endo,
                                         uint32_t maxl, bool count, gptr<uint8_t> __restrict__ out) {
  constexpr uint32_t G = 16u / OUT;  // outputs per 16-byte store
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = (uint32_t)x.s.w, wm = (1u << w) - 1u;
  const uint64_t go = x.s.out;
  const uint64_t k0 = (go + base) / G, k1 = (go + endo + G - 1) / G;
  uint32_t lgn = 1;
  while (lgn * 2u <= rl.R) lgn *= 2u;
  uint32_t a = 0, cnt = 0;
#pragma unroll 1
  for (uint64_t k = k0 + lane; k < k1; k += WAVE) {
    const uint64_t gl = k * G;
    const uint32_t olo = (uint32_t)((gl > go + base ? gl : go + base) - go);
    const uint32_t ohi = (uint32_t)((gl + G < go + endo ? gl + G : go + endo) - go);
    const uint32_t f0 = (uint32_t)(gl - go);  // page-relative index of field 0 (may wrap)
    for (uint32_t sp = lgn; sp; sp >>= 1)
      if (a + sp < rl.R && rl.rstart[a + sp] <= olo) a += sp;
    uint32_t f[G];
#pragma unroll
    for (uint32_t j = 0; j < G; ++j) f[j] = 0;
    uint32_t b = a, o = olo;
    while (o < ohi) {
      const uint32_t st = rl.rstart[b], nst = rl.rstart[b + 1], inf = rl.rinfo[b];
      const uint32_t be = nst < ohi ? nst : ohi;
      for (; o < be; ++o) {
        uint32_t v;
        if (inf & R_RLE) {
          v = inf & 0x7FFFFFFFu;
        } else {
          const uint64_t bit = (uint64_t)inf * 8ull + (uint64_t)(o - st) * w;
          v = lv_bits32(stage, blob, blob_len, x, bit) & wm;
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
      gst16(out + gl * OUT, v);
    } else {
#pragma unroll
      for (uint32_t j = 0; j < G; ++j) {
        const uint32_t oo = f0 + j;
        if (oo >= olo && oo < ohi) {
          if (OUT == 2) reinterpret_cast<gptr<int16_t>>(out)[gl + j] = (int16_t)f[j];
          else out[gl + j] = (uint8_t)f[j];
        }
      }
    }
  }
  return cnt;
}

// Outputs of one window from its run list (into out, the page's chunk buffer), and the def count.
template <int OUT>
__device__ inline void lv_write(const LvRuns& rl, const uint32_t* stage, const uint8_t* __restrict__ blob,
                                uint64_t blob_len, const LvWin& x, uint32_t base, uint32_t endo, int sel,
                                uint32_t maxl, PageWork* pages, gptr<uint8_t> __restrict__ out) {
  const bool count = sel == SS_DEF;
  uint32_t cnt = x.s.w == 1 ? lv_write1<OUT>(rl, stage, blob, blob_len, x, base, endo, out)
                            : lv_write_wide<OUT>(rl, stage, blob, blob_len, x, base, endo, maxl, count, out);
  if (count) {
    cnt = wave_sum_u32_(cnt);
    if ((threadIdx.x & 63u) == 0 && cnt) atomicAdd((unsigned long long*)&pages[x.p].nonnull, (unsigned long long)cnt);
  }
}

// RLE_DICTIONARY values (get_batch_with_dict, rle.rs:437-487): each output's index, from its
// run, gathers its value from the PLAIN dictionary page; groups of 16 / ES outputs, one 16-byte
// store each (element stores for the groups shared with a neighbouring window). Returns nonzero
// when an index is out of the dictionary (the reference panics).
template <int ES, bool LDSD>
__device__ __forceinline__ uint32_t lv_write_dict(const LvRuns& rl, const uint32_t* stage, const uint8_t* __restrict__ blob,
                                         uint64_t blob_len, const LvWin& x, uint32_t base, uint32_t endo,
                                         const uint8_t* __restrict__ dict, uint32_t ndict, bool aligned,
                                         const uint32_t* ldict, gptr<uint8_t> __restrict__ out) {
  using T = typename std::conditional<ES == 8, uint64_t, uint32_t>::type;
  constexpr uint32_t V = 16u / ES;  // outputs per 16-byte store
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = (uint32_t)x.s.w, wm = (1u << w) - 1u;
  const uint64_t go = x.s.out;
  const uint64_t lo = go + base, hi = go + endo;
  const uint64_t k0 = lo / V, k1 = (hi + V - 1) / V;
  uint32_t lgn = 1;
  while (lgn * 2u <= rl.R) lgn *= 2u;
  // U groups per lane per step: their indices first, then every gather, then the stores (the
  // gathers of a step are in flight together)
  constexpr uint32_t U = LDSD ? 2 : (ES == 8 ? 8 : 4);  // (LDS gathers: 2 keep the emit at 80 VGPRs)
  uint32_t a = 0, bad = 0;
#pragma unroll 1
  for (uint64_t kb = k0 + lane; kb < k1; kb += (uint64_t)WAVE * U) {
    uint32_t id[U][V], msk[U];
    bool full[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint64_t k = kb + (uint64_t)u * WAVE;
      msk[u] = 0;
      full[u] = false;
      if (k >= k1) continue;
      const uint64_t gl = k * V;
      const uint32_t olo = (uint32_t)((gl > lo ? gl : lo) - go);
      const uint32_t ohi = (uint32_t)((gl + V < hi ? gl + V : hi) - go);
      const uint32_t f0 = (uint32_t)(gl - go);  // page-relative index of field 0 (may wrap)
      full[u] = ohi - olo == V;
      for (uint32_t sp = lgn; sp; sp >>= 1)
        if (a + sp < rl.R && rl.rstart[a + sp] <= olo) a += sp;
      uint32_t b = a;
#pragma unroll
      for (uint32_t j = 0; j < V; ++j) {
        id[u][j] = 0;
        const uint32_t o = f0 + j;
        if (o < olo || o >= ohi) continue;
        while (rl.rstart[b + 1] <= o) ++b;
        const uint32_t inf = rl.rinfo[b];
        uint32_t idx;
        if (inf & R_RLE) {
          idx = inf & 0x7FFFFFFFu;
        } else {
          const uint64_t bit = (uint64_t)inf * 8ull + (uint64_t)(o - rl.rstart[b]) * w;
          idx = lv_bits32(stage, blob, blob_len, x, bit) & wm;
        }
        if (idx >= ndict) {
          bad = 1;
        } else {
          id[u][j] = idx;
          msk[u] |= 1u << j;
        }
      }
    }
    T f[U][V];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u)
#pragma unroll
      for (uint32_t j = 0; j < V; ++j) {
        T t = 0;
        if ((msk[u] >> j) & 1u) {
          if constexpr (LDSD) {  // the dictionary in LDS (LvDictOut::page): no global load to wait for
            if constexpr (ES == 8)
              t = (uint64_t)ldict[2 * id[u][j]] | ((uint64_t)ldict[2 * id[u][j] + 1] << 32);
            else
              t = ldict[id[u][j]];
          } else if (aligned) {
            t = reinterpret_cast<const T*>(dict)[id[u][j]];
          } else {
            const uint8_t* pv = dict + (uint64_t)id[u][j] * ES;
#pragma unroll
            for (int q = 0; q < ES; ++q) t |= (T)pv[q] << (8 * q);
          }
        }
        f[u][j] = t;
      }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint64_t gl = (kb + (uint64_t)u * WAVE) * V;
      if (full[u]) {
        uint4 v;
        if constexpr (ES == 8)
          v = make_uint4((uint32_t)f[u][0], (uint32_t)(f[u][0] >> 32), (uint32_t)f[u][1], (uint32_t)(f[u][1] >> 32));
        else
          v = make_uint4(f[u][0], f[u][1], f[u][2], f[u][3]);
        gst16(out + gl * ES, v);
      } else {
#pragma unroll
        for (uint32_t j = 0; j < V; ++j)
          if ((msk[u] >> j) & 1u) reinterpret_cast<gptr<T>>(out)[gl + j] = f[u][j];
      }
    }
  }
  return bad;
}

// lv_write_dict for windows of long runs (average >= 64 outputs, random indices give bit-packed
// runs of 504), the dictionary in LDS: run by run, the wave's lanes take the run's whole 16-byte
// groups, each read with one 8-byte stage load (V indices of w <= 8 bits) and V LDS gathers (RLE
// runs: one gather, the same 16 bytes stored); no per-output run search. The groups a run
// boundary or the window's ends cut (at most R + 1) then go one per lane, output by output.
template <int ES>
__device__ __forceinline__ uint32_t lv_write_dict_runs(const LvRuns& rl, const uint32_t* stage, const uint8_t* __restrict__ blob,
                                              uint64_t blob_len, const LvWin& x, uint32_t base, uint32_t endo,
                                              uint32_t ndict, const uint32_t* ldict, gptr<uint8_t> __restrict__ out) {
  using T = typename std::conditional<ES == 8, uint64_t, uint32_t>::type;
  constexpr uint32_t V = 16u / ES;
  constexpr uint32_t U = 4;  // (80 VGPRs for the kernel with the U = 2 of lv_write_dict: 6 waves per SIMD)
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t w = (uint32_t)x.s.w, wm = (1u << w) - 1u;
  const uint64_t go = x.s.out;
  uint32_t bad = 0;
  auto gather = [&](uint32_t idx) -> T {
    if constexpr (ES == 8) return (uint64_t)ldict[2 * idx] | ((uint64_t)ldict[2 * idx + 1] << 32);
    else return ldict[idx];
  };
  auto pack = [&](const T* f) -> uint4 {
    if constexpr (ES == 8)
      return make_uint4((uint32_t)f[0], (uint32_t)(f[0] >> 32), (uint32_t)f[1], (uint32_t)(f[1] >> 32));
    else
      return make_uint4(f[0], f[1], f[2], f[3]);
  };
#pragma unroll 1
  for (uint32_t b = 0; b < rl.R; ++b) {  // (wave-uniform)
    const uint32_t rs = rl.rstart[b], re = rl.rstart[b + 1], inf = rl.rinfo[b];
    const uint32_t st = rs > base ? rs : base, en = re < endo ? re : endo;
    if (st >= en) continue;
    const uint64_t g0 = (go + st + V - 1) / V, g1 = (go + en) / V;  // groups inside [st, en)
    if (g0 >= g1) continue;
    if (inf & R_RLE) {
      const uint32_t idx = inf & 0x7FFFFFFFu;
      bad |= idx >= ndict ? 1u : 0u;
      T f[V];
#pragma unroll
      for (uint32_t j = 0; j < V; ++j) f[j] = idx < ndict ? gather(idx) : (T)0;
      const uint4 v = pack(f);
      for (uint64_t k = g0 + lane; k < g1; k += WAVE) gst16(out + k * 16u, v);
      continue;
    }
    const uint64_t bit0 = (uint64_t)inf * 8ull;
#pragma unroll 1
    for (uint64_t kb = g0 + lane; kb < g1; kb += (uint64_t)WAVE * U) {
      T f[U][V];
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint64_t k = kb + (uint64_t)u * WAVE;
        if (k >= g1) continue;
        const uint32_t o = (uint32_t)(k * V - go);  // page-relative first output of the group
        const uint64_t bit = bit0 + (uint64_t)(o - rs) * w;
        const uint64_t x8 = lv_bytes8(stage, blob, blob_len, x, (uint32_t)(bit >> 3)) >> (bit & 7u);
#pragma unroll
        for (uint32_t j = 0; j < V; ++j) {
          const uint32_t idx = (uint32_t)(x8 >> (j * w)) & wm;
          bad |= idx >= ndict ? 1u : 0u;
          f[u][j] = idx < ndict ? gather(idx) : (T)0;
        }
      }
#pragma unroll
      for (uint32_t u = 0; u < U; ++u) {
        const uint64_t k = kb + (uint64_t)u * WAVE;
        if (k < g1) gst16(out + k * 16u, pack(f[u]));
      }
    }
  }
  // cut groups: the one holding each boundary q (base, every inner run start, endo) not on a
  // group edge; consecutive boundaries in one group take it once
  uint32_t lgn = 1;
  while (lgn * 2u <= rl.R) lgn *= 2u;
  auto qpos = [&](uint32_t c) -> uint64_t {  // boundary c in global outputs (c = 0: base, R: endo)
    const uint32_t p = c == 0 ? base : c >= rl.R ? endo : rl.rstart[c];
    return go + (p < base ? base : p > endo ? endo : p);
  };
#pragma unroll 1
  for (uint32_t c0 = 0; c0 <= rl.R; c0 += WAVE) {
    const uint32_t c = c0 + lane;
    if (c > rl.R) continue;
    const uint64_t q = qpos(c);
    if (q % V == 0) continue;
    const uint64_t k = q / V;
    if (c > 0) {
      const uint64_t qp = qpos(c - 1);
      if (qp % V != 0 && qp / V == k) continue;  // (taken by the previous boundary's lane)
    }
    uint32_t a = 0;
#pragma unroll 1
    for (uint32_t j = 0; j < V; ++j) {
      const uint64_t gl = k * V + j;
      if (gl < go + base || gl >= go + endo) continue;
      const uint32_t o = (uint32_t)(gl - go);
      for (uint32_t sp = lgn; sp; sp >>= 1)
        if (a + sp < rl.R && rl.rstart[a + sp] <= o) a += sp;
      const uint32_t inf = rl.rinfo[a];
      uint32_t idx;
      if (inf & R_RLE) {
        idx = inf & 0x7FFFFFFFu;
      } else {
        const uint64_t bit = (uint64_t)inf * 8ull + (uint64_t)(o - rl.rstart[a]) * w;
        idx = lv_bits32(stage, blob, blob_len, x, bit) & wm;
      }
      bad |= idx >= ndict ? 1u : 0u;
      reinterpret_cast<gptr<T>>(out)[gl] = idx < ndict ? gather(idx) : (T)0;
    }
  }
  return bad;
}

// What the walked-page emit writes: levels / booleans, or dictionary values. page() takes the
// per-page state (the chunk's buffer and parameters) when the emit moves to another page, so
// that a window's writes start without a dependent load.
template <int OUT>
struct LvLevelOut {
  static constexpr bool PIPE = true;  // k_lv_emit_walk prefetches the next window (registers to spare)
  uint8_t* out;
  uint32_t maxl;
  static constexpr uint32_t XW = 1;  // per-wave LDS words it uses (none)
  __device__ void page(const ChunkWork& ck, const PageWork*, const uint8_t*, int sel, uint32_t*) {
    out = lv_out(ck, sel);
    maxl = lv_maxl(ck, sel);
  }
  __device__ void operator()(const LvRuns& rl, const uint32_t* stage, const uint8_t* blob, uint64_t blob_len,
                             const LvWin& x, uint32_t base, uint32_t endo, int sel, const ChunkWork*,
                             PageWork* pages, const uint32_t*) const {
    lv_write<OUT>(rl, stage, blob, blob_len, x, base, endo, sel, maxl, pages, gp(out));
  }
};

// BYTE_ARRAY / FLBA dictionary indices (decoding.rs:256-315 over the entries k_ba_dict_prep
// decoded): per output the entry's index, in the value-length slot (the byte-array scan and copy,
// pqg_bytes.hip BaSrc, take the entry's address and length from there), and the page's byte total.
// Scratch slots: the chunk's scr_base (values) and dscr_base (dictionary entries) on.
// Run by run (wave-uniform): an RLE run's slots are one index; a bit-packed run's outputs go in
// groups of 4 on 4-aligned slots, one 8-byte stage read and one 16-byte store per group (indices
// of w <= 14 bits; wider ones one read per output), the groups a run boundary cuts output by
// output.
__device__ __forceinline__ void lv_write_badict(const LvRuns& rl, const uint32_t* stage, const uint8_t* blob, uint64_t blob_len,
                                       const LvWin& x, uint32_t base, uint32_t endo, const ChunkWork& ck,
                                       PageWork* pages, ChunkWork* chunks, const uint64_t* __restrict__ dsrc0,
                                       const uint32_t* __restrict__ dlen0, uint64_t* __restrict__ vsrc0,
                                       uint32_t* __restrict__ vlen0, const uint32_t* ldlen) {
  (void)dsrc0;
  (void)vsrc0;
  gptr<const uint32_t> dlen = gp(dlen0 + ck.dscr_base);
  gptr<uint32_t> vlen = gp(vlen0 + ck.scr_base);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t ndict = pages[ck.dict_page].num_values;
  const uint32_t w = (uint32_t)x.s.w, wm = (1u << w) - 1u;
  const uint64_t go = x.s.out;
  (void)dlen;
  (void)ldlen;
  uint32_t bad = 0;
#pragma unroll 1
  for (uint32_t b = 0; b < rl.R; ++b) {
    const uint32_t rs = rl.rstart[b], re = rl.rstart[b + 1], inf = rl.rinfo[b];
    const uint32_t st = rs > base ? rs : base, en = re < endo ? re : endo;
    if (st >= en) continue;
    if (inf & R_RLE) {
      const uint32_t idx = inf & 0x7FFFFFFFu;
      bad |= idx >= ndict ? 1u : 0u;
      for (uint32_t o = st + lane; o < en; o += WAVE) vlen[go + o] = idx;
      continue;
    }
    const uint64_t bit0 = (uint64_t)inf * 8ull;
    auto one = [&](uint32_t o) -> uint32_t {  // the index of output o of this run
      const uint64_t bit = bit0 + (uint64_t)(o - rs) * w;
      return lv_bits32(stage, blob, blob_len, x, bit) & wm;
    };
    const uint64_t k0 = (go + st + 3u) / 4u, k1 = (go + en) / 4u;  // 4-aligned groups inside [st, en)
#pragma unroll 1
    for (uint64_t k = k0 + lane; k < k1; k += WAVE) {
      const uint32_t o = (uint32_t)(k * 4u - go);
      uint32_t id[4];
      if (w <= 14u) {
        const uint64_t bit = bit0 + (uint64_t)(o - rs) * w;
        const uint64_t x8 = lv_bytes8(stage, blob, blob_len, x, (uint32_t)(bit >> 3)) >> (bit & 7u);
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) id[j] = (uint32_t)(x8 >> (j * w)) & wm;
      } else {
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) id[j] = one(o + j);
      }
#pragma unroll
      for (uint32_t j = 0; j < 4; ++j) bad |= id[j] >= ndict ? 1u : 0u;
      gst16(reinterpret_cast<gptr<uint8_t>>(vlen + k * 4u), make_uint4(id[0], id[1], id[2], id[3]));
    }
    // the cut groups: outputs [st, 4 k0 - go) and [4 k1 - go, en) (at most 3 each), or the whole
    // run when no group lies inside it
    const uint32_t h1 = k0 < k1 ? (uint32_t)(k0 * 4u - go) : en, t0 = k0 < k1 ? (uint32_t)(k1 * 4u - go) : en;
    const uint32_t nh = h1 - st, nt = en - t0;
    for (uint32_t j = lane; j < nh + nt; j += WAVE) {
      const uint32_t o = j < nh ? st + j : t0 + (j - nh);
      const uint32_t idx = one(o);
      bad |= idx >= ndict ? 1u : 0u;
      vlen[go + o] = idx;
    }
  }
  // the page's bytes: the sum of its tiles' (k_ba_tsum, from the indices written here)
  if (lane == 0) pages[x.p].tile_bytes = 1u;
  if (__ballot(bad) && lane == 0) report(pages, chunks, (int)x.p, ST_PANIC);
}

// Dictionary indices of every chunk on this path (ChunkWork::lvdict), by the chunk's value type:
// 4- / 8-byte values gathered from its PLAIN dictionary page (k_prepare checked it), byte arrays
// as entry addresses and lengths.
//
// The dictionary itself (<= 2 KiB: 4- / 8-byte values) or, for byte arrays, its entries' lengths
// (<= 512 entries) are copied into the wave's LDS words at each page change, so that the gathers
// are LDS reads: on CDNA the vector memory counter covers loads and stores in issue order, and a
// wave waiting for a global gather would wait for every store it issued before it as well.
struct LvDictOut {
  static constexpr bool PIPE = false;  // (its gathers hold the registers the prefetch would take: measured slower, 1.61 -> 1.68 ms)
#ifndef PQG_DICT_XW
#define PQG_DICT_XW 512
#endif
  static constexpr uint32_t XW = PQG_DICT_XW;  // per-wave LDS words: the dictionary, or its entry lengths
  const uint64_t* dsrc;
  const uint32_t* dlen;
  uint64_t* vsrc;
  uint32_t* vlen;
  const ChunkWork* ck;  // the current page's chunk, value size, buffer and dictionary (page())
  uint8_t* val_out;
  const uint8_t* dict;
  uint32_t ndict;
  int es;
  bool lds;  // the page's dictionary (or entry lengths) is in the wave's LDS words
  __device__ __forceinline__ void page(const ChunkWork& c, const PageWork* pages, const uint8_t* blob, int, uint32_t* xw) {
    ck = &c;
    es = c.es;
    val_out = c.val_out;
    const PageWork& dp = pages[c.dict_page];
    dict = blob + dp.base;
    ndict = dp.num_values;
    const uint32_t lane = threadIdx.x & 63u;
    if (es == 4 || es == 8) {
      const uint32_t nw = ndict * (uint32_t)es / 4u;  // (k_prepare checked the page holds them)
      lds = nw <= XW;
      if (lds)
        for (uint32_t i = lane; i < nw; i += WAVE)
          xw[i] = (uint32_t)dict[4 * i] | ((uint32_t)dict[4 * i + 1] << 8) | ((uint32_t)dict[4 * i + 2] << 16) |
                  ((uint32_t)dict[4 * i + 3] << 24);
    } else {
      lds = ndict <= XW;
      if (lds)
        for (uint32_t i = lane; i < ndict; i += WAVE) xw[i] = gp(dlen)[c.dscr_base + i];
    }
    wave_lds_sync();
  }
  __device__ __forceinline__ void operator()(const LvRuns& rl, const uint32_t* stage, const uint8_t* blob,
                                             uint64_t blob_len, const LvWin& x, uint32_t base, uint32_t endo, int,
                                             const ChunkWork* chunks, PageWork* pages, const uint32_t* xw) const {
    if (es == 0) {
      lv_write_badict(rl, stage, blob, blob_len, x, base, endo, *ck, pages, const_cast<ChunkWork*>(chunks), dsrc, dlen,
                      vsrc, vlen, lds ? xw : nullptr);
      return;
    }
    uint32_t bad;
    if ((uint64_t)(endo - base) >= 64ull * rl.R && x.s.w <= 8) {  // long runs: run by run
      bad = es == 8 ? lv_write_dict_runs<8>(rl, stage, blob, blob_len, x, base, endo, ndict, xw, gp(val_out))
                    : lv_write_dict_runs<4>(rl, stage, blob, blob_len, x, base, endo, ndict, xw, gp(val_out));
    } else if (!lds) {  // (the host puts only dictionaries of <= 2^8 entries on this path: they fit)
      bad = 0;
      if ((threadIdx.x & 63u) == 0) report(pages, const_cast<ChunkWork*>(chunks), (int)x.p, ST_INVALID_ARG);
    } else {
      bad = es == 8 ? lv_write_dict<8, true>(rl, stage, blob, blob_len, x, base, endo, dict, ndict, true, xw, gp(val_out))
                    : lv_write_dict<4, true>(rl, stage, blob, blob_len, x, base, endo, dict, ndict, true, xw, gp(val_out));
    }
    if (__ballot(bad) && (threadIdx.x & 63u) == 0) report(pages, const_cast<ChunkWork*>(chunks), (int)x.p, ST_PANIC);
  }
};

// Bit width 1, the true entry's chain meets the window's reference chain at `me`: the window's
// true headers are the reference chain's (k_lv_win's mask per segment, refm) from the meeting
// point on, plus the entry's own headers before it, which one lane walks into per-segment masks
// (pm: 65 LDS words). Sets the lane's header mask (mym), its segment's outputs (so), their place
// (myacc) and the window's total (T); false (wave-uniform) when the walk does not land on the
// meeting point (a table k_lv_win made wrong: the caller takes the chain walk instead).
__device__ inline bool lv_ref_headers(const uint32_t* stage, uint32_t* pm, const LvWin& x, uint32_t e0, uint32_t me,
                                      uint32_t refm, uint32_t& mym, uint64_t& so, uint64_t& myacc, uint64_t& T) {
  constexpr uint32_t SEG = LV_SEG;
  const uint32_t lane = threadIdx.x & 63u, i0 = lane * SEG, slen = x.s.slen;
  pm[lane] = 0u;
  wave_lds_sync();
  if (lane == 0) {
    uint32_t qq = e0;
    while (qq < me) {  // (every hop advances: at most LV_WIN + 64 of them)
      uint32_t nx, c, v;
      bool bp;
      if (!lv_parse4(stage, qq + x.sb, x.W0 + qq, slen, 1u, 1u, nx, c, v, bp)) break;
      pm[qq / SEG] |= 1u << (qq % SEG);
      qq = nx - x.W0;
    }
    pm[64] = qq == me ? 1u : 0u;
  }
  wave_lds_sync();
  if (!pm[64]) return false;
  mym = (i0 + SEG <= me ? 0u : i0 >= me ? refm : refm & (0xFFFFu << (me - i0))) | pm[lane];
  // outputs of this segment's true headers, then their place: a lane scan
  so = 0;
#pragma unroll 1
  for (uint32_t m = mym; m; m &= m - 1u) {
    const uint32_t t = (uint32_t)__builtin_ctz(m);
    uint32_t nx, c, v;
    bool bp;
    lv_parse4(stage, i0 + t + x.sb, x.W0 + i0 + t, slen, 1u, 1u, nx, c, v, bp);  // (chain headers parse)
    so += c;
  }
  const uint64_t si = wave_incl_scan_cnt64(so);
  myacc = si - so;
  T = __shfl(si, 63, 64);
  return true;
}

// ------------------------------------------------------------------------------ k_lv_emit
// Window path: windows g2 of the dense pages.
template <int OUT>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(4))) k_lv_emit(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                PageWork* pages, int npages, const ChunkWork* chunks, int sel,
                                                RunTables rt, LevelTables lt) {
  __shared__ LvSmem sm;
  const uint32_t wid = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  LvWave& W = sm.wv[wid];
  LvDense D;
  LvWin x;
  LvPf pf;
  pf.ok = false;
  if (!D.begin(blob, pages, npages, chunks, sel, rt, lt, x)) return;
#ifdef PQG_DIAG
  // diagnostics (PQG_DEBUG bit 256): per wave s_memtime cycles in the window's staging wait,
  // chain / run placement, bitmap generation and output stores, and the windows written
  const bool stamps = (chunks[0].cp.debug & 256) && chunks[0].cp.dbgbuf;
  uint64_t ts0 = 0, tacc[4] = {0, 0, 0, 0}, tn = 0, tmiss = 0, tw0 = 0, tspec = 0, nspec = 0;
#define LE_STAMP(k)                                   \
  if (stamps) {                                       \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(); \
    tacc[k] += t1 - ts0;                              \
    ts0 = t1;                                         \
  }
#else
#define LE_STAMP(k)
#endif
  for (uint32_t g2 = D.g0; g2 < D.g1; ++g2) {
#ifdef PQG_DIAG
    if (stamps) tw0 = ts0 = __builtin_amdgcn_s_memtime();
#endif
    if (!D.at(blob, pages, chunks, sel, rt, lt, x, g2)) continue;
    const uint2 wi = pf.ok && pf.p == x.p && pf.k == x.k ? pf.wi : lt.win[D.wb + x.k];
    if (wi.x == LV_NONE) {  // no true header in this window
      pf.ok = false;
      if (g2 + 1 < D.g1 && g2 + 1 < D.pend) pf.issue(blob, blob_len, x, x.k + 1, lt.win + D.wb);
      continue;
    }
    x.W0 = x.k * LV_WIN;
    const uint32_t w = (uint32_t)x.s.w, vb = (w + 7u) >> 3, slen = x.s.slen, n = x.s.n;
    // entry; bit width 1: where the entry's chain meets the window's reference chain (0xFFFF:
    // not inside the window), else the true headers (saturated)
    const uint32_t e0 = wi.x & 0xFFFFu, nh = wi.x >> 16;
    const uint32_t base = wi.y;
    // bit width 1, the entry's chain meets the reference chain: that chain's headers (k_lv_win's
    // bitmap, one 16-bit mask per segment) from the meeting point on
    const bool viaref = w == 1 && nh != 0xFFFFu;
    const uint32_t refm = viaref ? (uint32_t)lt.bmp[(uint64_t)(D.wb + x.k) * WAVE + lane] : 0u;
    pf.stage(blob, blob_len, x, W.stage);
    if (g2 + 1 < D.g1 && g2 + 1 < D.pend) pf.issue(blob, blob_len, x, x.k + 1, lt.win + D.wb);
#ifdef PQG_DIAG
    if (stamps && viaref) asm volatile("" ::"v"(refm));  // (the bitmap's load has landed)
#endif
    LE_STAMP(0)
    uint32_t R = 0;  // runs placed (wave-uniform)
    uint64_t T = 0;  // outputs of those runs (wave-uniform)
    bool bad = false;
    // bit width 1: this segment's true headers and first output (window-relative); bm: written
    // from those by lv_bm_gen / lv_bm_store, no run list placed (wave-uniform)
    uint32_t mym = 0;
    uint64_t myacc = 0;
    bool bm = false;
    bool placed = false;  // (wave-uniform) the window's true headers found
    if (viaref) {
      const uint32_t i0 = lane * LV_SEG;
      uint64_t so = 0;
      // (pm: the run list's space, written after the masks are read)
      if (lv_ref_headers(W.stage, W.runs.rinfo, x, e0, nh, refm, mym, so, myacc, T)) {
        placed = true;
        bm = lv_bm_fits(x, base, (uint64_t)base + T < n ? (uint64_t)base + T : (uint64_t)n, so);
        wave_lds_sync();  // (the prefix masks are read)
        if (!bm) {
          const uint32_t nh_l = (uint32_t)__builtin_popcount(mym);
          const uint32_t rb = wave_incl_scan_u32(nh_l) - nh_l;
          uint32_t k = rb;
          uint64_t oa = (uint64_t)base + myacc;
#pragma unroll 1
          for (uint32_t m = mym; m; m &= m - 1u) {
            const uint32_t t = (uint32_t)__builtin_ctz(m);
            uint32_t nx, c, v;
            bool bp;
            lv_parse4(W.stage, i0 + t + x.sb, x.W0 + i0 + t, slen, w, vb, nx, c, v, bp);
            W.runs.rstart[k] = oa < 0xFFFFFFFFull ? (uint32_t)oa : 0xFFFFFFFFu;
            W.runs.rinfo[k] = bp ? v : (R_RLE | v);
            bad |= !lv_run_ok(bp, v, c, oa, n, slen, w);
            ++k;
            oa += c;
          }
          R = (uint32_t)__shfl((int)(rb + nh_l), 63, 64);
        }
      } else {
        wave_lds_sync();
      }
    }
    if (placed) {
      // (the true headers came from the reference chain)
    } else if (w != 1 && nh <= LV_SERIAL) {
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
          bad |= !lv_run_ok(bp, v, c, acc, n, slen, w);
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
      // dense window: lane l takes the 16 positions [16 l, 16 l + 16) (a segment). Every
      // position is parsed as a header; a backward pass over the segment gives, per position,
      // where its chain leaves the segment, the outputs on the way and the headers it passes
      // (a mask); then one walk from the entry, one table lookup per segment, finds the true
      // headers of every segment and the output each segment starts at.
      constexpr uint32_t SEG = LV_SEG;
      uint32_t pc[SEG], pv[SEG], bpm;
      lv_seg_build(W, x, pc, pv, bpm);
      // the walk from the entry (wave-uniform): segment s's true headers and first output
      const uint64_t lim = (uint64_t)n - base;
      uint32_t e = e0, mys = 0;
      uint64_t acc = 0;
      {  // speculatively in parallel (lv_spec_chain): the segments the walk visits are the chain's
         // segments before the one whose outputs reach lim
        uint32_t q;
        bool valid;
        uint2 r;
        uint64_t inc;
        if (lv_spec_chain(W, e0, lim, q, valid, r, inc)) {
          const uint64_t P = inc - (valid ? r.y : 0u);
          const bool vis = valid && P < lim;
          mym = vis ? r.x >> 16 : 0u;
          myacc = P;
          mys = vis ? r.y : 0u;
          const uint64_t vsm = __ballot(vis);
          const int last = vsm ? 63 - __builtin_clzll(vsm) : 0;
          acc = vsm ? __shfl(inc, last, 64) : 0ull;
          e = vsm ? (uint32_t)__shfl((int)(r.x & 0xFFFFu), last, 64) : LV_WIN;
          e = e < LV_WIN ? LV_WIN : e;  // (a chain past lim: not walked on; e matters only below lim)
        }
      }
#pragma unroll 1
      while (e < LV_WIN) {
        const uint32_t sg = e / SEG;
        const uint2 r = W.JC[(e % SEG) * WAVE + sg];
        const uint32_t rx = rfl(r.x), ry = rfl(r.y);
        if (lane == sg) {
          mym = rx >> 16;
          myacc = acc;
          mys = ry;
        }
        acc += ry;
        if (acc >= lim) break;
        e = rx & 0xFFFFu;
      }
      // a dead header, or the stream's end, before n outputs
      bad = acc < lim && (e == LV_J_DEAD || e == LV_J_END);
      T = acc;
      bm = w == 1 && !__ballot(bad) && lv_bm_fits(x, base, (uint64_t)base + T < n ? (uint64_t)base + T : (uint64_t)n, mys);
      wave_lds_sync();  // the table's space now holds the run list
      if (!bm) {
        const uint32_t nh_l = (uint32_t)__builtin_popcount(mym);
        const uint32_t rb = wave_incl_scan_u32(nh_l) - nh_l;
        uint32_t k = rb;
        uint64_t oa = (uint64_t)base + myacc;
        // the segment's true headers parsed again from the stage (keeping the segment build's 32
        // per-position registers live through the walk spilled them)
        const uint32_t i0 = lane * SEG;
  #pragma unroll 1
        for (uint32_t m = mym; m; m &= m - 1u) {
          const uint32_t t = (uint32_t)__builtin_ctz(m);
          uint32_t nx, c, v;
          bool bp;
          lv_parse4(W.stage, i0 + t + x.sb, x.W0 + i0 + t, slen, w, vb, nx, c, v, bp);  // (a true header: parses)
          W.runs.rstart[k] = oa < 0xFFFFFFFFull ? (uint32_t)oa : 0xFFFFFFFFu;
          W.runs.rinfo[k] = bp ? v : (R_RLE | v);
          bad |= !lv_run_ok(bp, v, c, oa, n, slen, w);
          ++k;
          oa += c;
        }
        R = (uint32_t)__shfl((int)(rb + nh_l), 63, 64);
      }
    }
    if (__ballot(bad)) {
      if (lane == 0) LV_BAIL(rt, lt, x.p, PF_PAGE, 4);
#ifdef PQG_DIAG
      // (the first failing window of the page: its index + 1, stitch entry, first output)
      if (lt.bail && lane == 0 && atomicCAS(&lt.bail[npages + 4 * x.p], 0u, x.k + 1u) == 0u) {
        lt.bail[npages + 4 * x.p + 1] = wi.x;
        lt.bail[npages + 4 * x.p + 2] = wi.y;
      }
#endif
      continue;
    }
    // outputs [base, min(base + T, n)) of the page
    const uint64_t endo = (uint64_t)base + T < n ? (uint64_t)base + T : (uint64_t)n;
    if (bm) {
      LE_STAMP(1)
      if (endo > base) {
        const LvBm B(x, base, (uint32_t)endo);
        const uint32_t cnt = lv_bm_gen(W.stage, reinterpret_cast<uint32_t*>(W.JC), blob, blob_len, x, B, mym,
                                       (uint64_t)base + myacc, n);
        LE_STAMP(2)
        if (cnt == 0xFFFFFFFFu) {
          if (lane == 0) LV_BAIL(rt, lt, x.p, PF_PAGE, 5);
        } else {
          lv_bm_store<OUT>(reinterpret_cast<const uint32_t*>(W.JC), x, B, cnt, sel, pages, gp(D.out));
        }
      }
    } else {
      if (lane == 0) W.runs.rstart[R] = 0xFFFFFFFFu;
      wave_lds_sync();
      if (endo <= base || R == 0) continue;
      LE_STAMP(1)
      LE_STAMP(2)
      lv_write<OUT>(LvRuns{W.runs.rstart, W.runs.rinfo, R}, W.stage, blob, blob_len, x, base, (uint32_t)endo, sel,
                    D.maxl, pages, gp(D.out));
    }
    wave_lds_sync();  // the run list / bitmap and stage are refilled by the next window
    LE_STAMP(3)
#ifdef PQG_DIAG
    tn += 1ull | (viaref ? 1ull << 20 : 0ull) | (bm ? 1ull << 40 : 0ull);  // windows | via the reference | bitmap
    tmiss += viaref && !placed ? 1u : 0u;  // the entry's chain missed the meeting point
    if (stamps && !placed) {  // windows through the segment tables: their whole time
      tspec += ts0 - tw0;
      ++nspec;
    }
#endif
  }
#ifdef PQG_DIAG
  if (stamps && lane == 0) {
    const uint32_t gw = blockIdx.x * (WG / WAVE) + wid;
    uint64_t* d = chunks[0].cp.dbgbuf + 8ull * gw;
    d[0] = tacc[0];
    d[1] = tacc[1];
    d[2] = tacc[2];
    d[3] = tacc[3];
    d[4] = tn;
    d[5] = tmiss;
    d[6] = tspec;
    d[7] = nspec;
  }
#endif
#undef LE_STAMP
}

// ------------------------------------------------------------------------------ k_lv_emit_walk
// Windows of the walked pages: each wave takes a contiguous range of windows (one page lookup,
// then the page advances with the window), loads each window's run records and staged payload
// and writes its outputs. Software-pipelined: while window g's outputs are written, window
// g + 1's records and payload (same page) are in flight in registers and window g + 2's run
// bounds are read, so a window's three dependent loads (run bounds, records, payload) overlap
// the previous window's stores.
constexpr uint32_t LE_RPL = (LW_RPW + 1 + WAVE - 1) / WAVE;  // record registers per lane (5)
constexpr uint32_t LE_SPL = (LE_STG / 16 + WAVE - 1) / WAVE;  // stage registers per lane (3)
// the level emits on a 4x grid (k_lv_emit_walk<LvLevelOut<2>>: p_null 0.5 0.469 -> 0.452 ms, p_null
// 0 0.383 -> 0.363; 16x 0.476 / 0.361, 32x 0.618 / 0.366)
#ifndef PQG_EW_GRIDX
#define PQG_EW_GRIDX 4
#endif
#ifndef PQG_LE_SMAX
#define PQG_LE_SMAX 16
#endif
constexpr uint32_t LE_SMAX = PQG_LE_SMAX;                     // waves per window at most
constexpr uint32_t LE_SLICE = 16384;                          // outputs per slice at least

// The unpipelined writers (dictionary values) take up to LE_UNIT consecutive windows of a page as
// one unit (their run records are contiguous, at most LW_RPW runs in all): one chain of dependent
// loads (bounds, records, payload) per unit instead of per window.
#ifndef PQG_LE_UNIT
#define PQG_LE_UNIT 2
#endif
constexpr uint32_t LE_UNIT = PQG_LE_UNIT;
constexpr uint32_t LE_STG_U = LE_UNIT * LV_WIN + 64 * 16 + 64;

template <uint32_t STG>
struct LeWaveT {
  uint32_t stage[STG / 4];
  uint32_t rstart[LW_RPW + 1];
  uint32_t rinfo[LW_RPW];
  uint32_t endn;
};
using LeWave = LeWaveT<LE_STG>;

// One window's loads in flight: its run records [fr, fr + R] and staged payload.
struct LeLoad {
  uint2 r[LE_RPL];
  uint4 st[LE_SPL];
  uint32_t k, R, nch, sb;
  bool ok;  // loads issued (a window of the same walked page with runs, R <= LW_RPW)
};

__device__ inline uint32_t le_nch(uint32_t w, uint32_t nwin = 1, uint32_t stg = LE_STG) {
  const uint32_t n = (nwin * LV_WIN + 16u + 64u * w + 16u) / 16u + 1u;
  return n > stg / 16 ? stg / 16 : n;
}

__device__ inline void le_issue(const uint8_t* __restrict__ blob, uint64_t blob_len, const uint2* rc, uint32_t R,
                                uint64_t S, uint32_t k, uint32_t w, LeLoad& f) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (uint32_t j = 0; j < LE_RPL; ++j) {
    const uint32_t i = lane + j * WAVE;
    f.r[j] = i <= R ? rc[i] : make_uint2(0u, 0u);
  }
  const uint64_t A = (S + (uint64_t)k * LV_WIN) & ~15ull;
  f.sb = (uint32_t)(S + (uint64_t)k * LV_WIN - A);
  f.nch = le_nch(w);
#pragma unroll
  for (uint32_t c = 0; c < LE_SPL; ++c) {
    const uint32_t ci = lane + c * WAVE;
    const uint64_t a = A + (uint64_t)ci * 16u;
    f.st[c] = ci >= f.nch ? make_uint4(0u, 0u, 0u, 0u)
              : a + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
  }
  f.k = k;
  f.R = R;
  f.ok = true;
}

template <class WaveT>
__device__ inline void le_install(const LeLoad& f, WaveT& E) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (uint32_t j = 0; j < LE_RPL; ++j) {
    const uint32_t i = lane + j * WAVE;
    if (i < f.R) {
      E.rstart[i] = f.r[j].x;
      E.rinfo[i] = f.r[j].y;
    } else if (i == f.R) {
      E.rstart[i] = 0xFFFFFFFFu;
      E.rinfo[i] = f.r[j].y;
      E.endn = f.r[j].x;  // first output of the next window's first run (or the total)
    }
  }
#pragma unroll
  for (uint32_t c = 0; c < LE_SPL; ++c) {
    const uint32_t ci = lane + c * WAVE;
    if (ci < f.nch) reinterpret_cast<uint4*>(E.stage)[ci] = f.st[c];
  }
  wave_lds_sync();
}

template <class Writer>
__global__ void __launch_bounds__(WG) k_lv_emit_walk(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                     PageWork* pages, int npages, const ChunkWork* chunks,
                                                     int sel, RunTables rt, LevelTables lt, Writer wr) {
  using WaveT = LeWaveT<Writer::PIPE ? LE_STG : LE_STG_U>;
  __shared__ WaveT sm[WG / WAVE];
  __shared__ uint32_t smx[WG / WAVE][Writer::XW];
  const uint32_t wid = rfl(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  WaveT& E = sm[wid];
  uint32_t* xw = smx[wid];
  const uint32_t total = lt.wbase[npages];
  const uint32_t nwv = gridDim.x * (WG / WAVE), gw = blockIdx.x * (WG / WAVE) + wid;
  // fewer windows than waves (short streams of long runs: 2^20 levels in one RLE run per page):
  // S waves per window, each writing a slice of its outputs; else contiguous window ranges
  const uint32_t S = total && total < nwv ? min(nwv / total, LE_SMAX) : 1u, slice = gw % S;
  const uint32_t per = S > 1 ? 1u : (total + nwv - 1u) / nwv;
  const uint32_t g0 = S > 1 ? gw / S : gw * per, g1 = min(total, g0 + per);
  if (g0 >= g1) return;
  uint32_t p = lv_page_of(lt.wbase, (uint32_t)npages, g0);
  uint32_t wb = lt.wbase[p], pend = lt.wbase[p + 1];
  LvWin x;
  // outputs [base, endo) of a window -> this wave's slice, its inner bounds on 64-output edges of
  // the chunk's buffer (whole 16-byte stores on both sides)
  auto cut = [&](uint32_t& base, uint32_t& endo) {
    if (S == 1) return;
    const uint64_t lo = x.s.out + base, T = endo - base;
    const uint32_t Se = (uint32_t)min((uint64_t)S, (T + LE_SLICE - 1) / LE_SLICE);  // slices of >= LE_SLICE outputs
    auto bnd = [&](uint32_t i) -> uint32_t {
      if (i == 0) return base;
      if (i >= Se) return endo;
      const uint64_t a = (lo + T * i / Se) & ~63ull;
      return a <= lo ? base : (uint32_t)(a - x.s.out);
    };
    const uint32_t b0 = bnd(slice), b1 = bnd(slice + 1);
    base = b0;
    endo = b1;
  };
  x.p = p;
  bool walked = rt.pflag[p] == PF_WALK && lv_stream(blob, pages[p], sel, chunks, x.s);
  if (walked) wr.page(chunks[pages[p].chunk], pages, blob, sel, xw);
  LeLoad nf;  // the next window's loads, issued while the current one is written
  nf.ok = false;
#ifdef PQG_DIAG
  // diagnostics (PQG_DEBUG bit 1024, unpipelined writers): per wave s_memtime cycles in the run
  // bounds + records, the payload staging and the writes by value size (0: byte arrays, 4, 8),
  // then the units and outputs written
  const bool wst = !Writer::PIPE && (chunks[0].cp.debug & 1024) && chunks[0].cp.dbgbuf;
  uint64_t wt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, wt0 = 0;
#define LW_STAMP(k)                                   \
  if (wst) {                                          \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(); \
    wt[k] += t1 - wt0;                                \
    wt0 = t1;                                         \
  }
#else
#define LW_STAMP(k)
#endif
  uint32_t nb0 = 0, nb1 = 0, nbk = 0;  // run bounds (wfirst) of window nbk of the page, read ahead
  bool nbv = false;
  for (uint32_t g = g0; g < g1; ++g) {
    while (g >= pend) {  // next page (pages without windows are passed over)
      ++p;
      wb = pend;
      pend = lt.wbase[p + 1];
      x.p = p;
      walked = pend > wb && rt.pflag[p] == PF_WALK && lv_stream(blob, pages[p], sel, chunks, x.s);
      if (walked) wr.page(chunks[pages[p].chunk], pages, blob, sel, xw);
      nf.ok = false;
      nbv = false;
    }
    if (!walked) {
      g = pend - 1u;
      continue;
    }
    x.k = g - wb;
    const uint32_t* wf = lt.wfirst + wb + p;
    const uint2* recp = lt.rec + (uint64_t)LW_REC * (wb + 2ull * p);
    const uint32_t w = (uint32_t)x.s.w;
    if constexpr (!Writer::PIPE) {  // a unit of windows at a time: records and payload straight to LDS
#ifdef PQG_DIAG
      if (wst) wt0 = __builtin_amdgcn_s_memtime();
#endif
      // the unit: windows [x.k, x.k + nu) of this page with at most LW_RPW runs in all (lane i
      // reads the run bound of window x.k + i)
      const uint32_t lim = S > 1 ? 1u : min(LE_UNIT, min(g1, pend) - g);
      const uint32_t fi = lane <= lim ? wf[x.k + lane] : 0u;
      const uint32_t fr = rfl(fi);
      const uint64_t fit = __ballot(lane >= 1 && lane <= lim && fi - fr <= LW_RPW);
      const uint32_t nu = fit & 2ull ? (uint32_t)__builtin_ctzll(~(fit >> 1)) : 1u;  // leading windows that fit
      const uint32_t fe = (uint32_t)__shfl((int)fi, (int)nu, 64);
      g += nu - 1u;  // (the loop's ++g moves past the unit)
      if (fr == fe) continue;
      const uint32_t R = fe - fr;
      if (R > LW_RPW) {
        if (lane == 0) LV_BAIL(rt, lt, p, PF_WALK, 6);
        continue;
      }
      const uint2* rc = recp + fr;
      const uint32_t endn = rc[R].x;
      for (uint32_t i = lane; i <= R; i += WAVE) {
        const uint2 r = rc[i];
        E.rstart[i] = i < R ? r.x : 0xFFFFFFFFu;
        E.rinfo[i] = r.y;
      }
      x.W0 = x.k * LV_WIN;
      LW_STAMP(0)
      lv_stage(blob, blob_len, x, E.stage, le_nch(w, nu, LE_STG_U));  // ends with a wave LDS sync (run list too)
      LW_STAMP(1)
      uint32_t base = E.rstart[0];
      uint32_t endo = endn < x.s.n ? endn : x.s.n;
      if (endo > base) cut(base, endo);
      if (endo > base) wr(LvRuns{E.rstart, E.rinfo, R}, E.stage, blob, blob_len, x, base, endo, sel, chunks, pages, xw);
      wave_lds_sync();
#ifdef PQG_DIAG
      if (wst) {
        const uint32_t es = chunks[pages[p].chunk].es;
        LW_STAMP(es == 8 ? 4 : es == 4 ? 3 : 2)
        wt[5] += 1;
        const uint64_t no = endo > base ? endo - base : 0u;
        if (es) wt[6] += es == 8 ? no << 32 : no;  // (4-byte outputs low, 8-byte high)
        else wt[7] += no;
      }
#endif
      continue;
    }
    bool have = nf.ok && nf.k == x.k;
    uint32_t R;
    if (have) {
      R = nf.R;
    } else {
      const uint32_t fr = wf[x.k], fe = wf[x.k + 1];
      if (fr == fe) continue;  // no header starts in this window
      R = fe - fr;
      if (R > LW_RPW) {  // more runs than the run list holds (not from the walker's span rule)
        if (lane == 0) LV_BAIL(rt, lt, p, PF_WALK, 7);
        continue;
      }
      le_issue(blob, blob_len, recp + fr, R, x.s.S, x.k, w, nf);
    }
    le_install(nf, E);  // (waits for its loads)
    nf.ok = false;
    // the next window of this page: issue its loads now (its run bounds were read one window ago)
    if (Writer::PIPE && g + 1 < g1 && g + 1 < pend) {
      uint32_t fr2, fe2;
      if (nbv && nbk == x.k + 1) {
        fr2 = nb0;
        fe2 = nb1;
      } else {
        fr2 = wf[x.k + 1];
        fe2 = wf[x.k + 2];
      }
      if (fe2 > fr2 && fe2 - fr2 <= LW_RPW) le_issue(blob, blob_len, recp + fr2, fe2 - fr2, x.s.S, x.k + 1, w, nf);
      nbv = false;
      if (g + 2 < g1 && g + 2 < pend) {  // and the bounds of the one after
        nb0 = wf[x.k + 2];
        nb1 = wf[x.k + 3];
        nbk = x.k + 2;
        nbv = true;
      }
    } else {
      nbv = false;
    }
    x.W0 = x.k * LV_WIN;
    x.sb = 0;
    x.cap = 0;
    {
      const uint64_t A = (x.s.S + x.W0) & ~15ull;
      x.sb = (uint32_t)(x.s.S + x.W0 - A);
      x.cap = le_nch(w) * 16u;
    }
    uint32_t base = E.rstart[0];
    const uint32_t endn = E.endn;
    uint32_t endo = endn < x.s.n ? endn : x.s.n;
    if (endo > base) cut(base, endo);
    if (endo > base) wr(LvRuns{E.rstart, E.rinfo, R}, E.stage, blob, blob_len, x, base, endo, sel, chunks, pages, xw);
    wave_lds_sync();  // the run list and stage are refilled by the next window
  }
#ifdef PQG_DIAG
  if (wst && lane == 0) {
    uint64_t* d = chunks[0].cp.dbgbuf + 8ull * gw;
    for (int i = 0; i < 8; ++i) d[i] = wt[i];
  }
#endif
#undef LW_STAMP
}

#include "pqg_lvd1.hpp"

// Plan, segment starts and walks, page scan, run compaction: every page of stream `sel` ends
// walked (PF_WALK, its run list built), dense (PF_PAGE) or handed back (PF_BAIL).
static void lv_front(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages, const ChunkWork* chunks,
                     int sel, RunTables rt, LevelTables lt, uint32_t wgrid, hipStream_t s) {
  if (sel == SS_BOOL)  // (def / rep: k_prepare probed them; dictionary indices: cleared there)
    hipLaunchKernelGGL(k_lv_probe, dim3((npages + WG / WAVE - 1) / (WG / WAVE)), dim3(WG), 0, s, blob, blob_len,
                       pages, npages, chunks, sel, lt);
  hipLaunchKernelGGL(k_lv_plan, dim3((npages + WG - 1) / WG), dim3(WG), 0, s, blob, pages, npages, chunks, sel, rt, lt);
  hipLaunchKernelGGL(k_lv_bound, dim3(wgrid), dim3(WG), 0, s, blob, blob_len, pages, npages, chunks, sel, rt, lt);
  hipLaunchKernelGGL(k_lv_segwalk, dim3(wgrid), dim3(WG), 0, s, blob, blob_len, pages, npages, chunks, sel, rt, lt);
#ifndef PQG_SS_GRID
#define PQG_SS_GRID 512
#endif
  hipLaunchKernelGGL(k_lv_segscan, dim3(npages < PQG_SS_GRID ? npages : PQG_SS_GRID), dim3(WG), 0, s, blob, pages, npages,
                     chunks, sel, rt, lt);
  hipLaunchKernelGGL(k_lv_compact, dim3(wgrid), dim3(WG), 0, s, npages, rt, lt);
}

extern "C" {

// Hybrid-stream path of stream `sel` over every chunk of the decode: plan, segment starts and
// walks, page scan, run compaction, window path for the dense pages, emits. Def / rep levels:
// int16 out (+ def counts); RLE booleans: bytes out; dictionary indices (SS_DICT, the chunks with
// ChunkWork::lvdict): 4- / 8-byte dictionary values, or byte-array entry addresses and lengths
// (scratch dsrc/dlen -> vsrc/vlen). widths: bit mask (1 << w) of the level streams' bit widths.
hipError_t pqg_launch_lv(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages, ChunkWork* chunks,
                         int sel, uint32_t widths, const uint64_t* dsrc, const uint32_t* dlen, uint64_t* vsrc,
                         uint32_t* vlen, RunTables rt, LevelTables lt, hipStream_t s, hipEvent_t front) {
  if (npages <= 0) return hipSuccess;
  const uint32_t wgrid = 256u * 8u;
  lv_front(blob, blob_len, pages, npages, chunks, sel, rt, lt, wgrid, s);
  if (front) (void)hipEventRecord(front, s);
  if (sel == SS_DICT) {  // (dense dictionary streams went to the general decoder)
    // short window ranges (one or two two-window units per wave on config 5): the waves' costs
    // differ by value kind and index width (1.6x) and the hardware's workgroup dispatch evens
    // them out, better than a cost-weighted split (k_lv_emit_walk<LvDictOut> on config 5: 2048
    // workgroups 0.98-0.99 ms, cost-weighted 0.96, 4096 0.89-0.91, 8192 0.84, 16384 0.83, 32768
    // 0.79-0.80, 65536 0.76-0.77, 120 K 0.87); one per 16 KiB of the batch up to 65536
#ifndef PQG_LD_GRID
#define PQG_LD_GRID 65536
#endif
    const uint32_t ldgrid = (uint32_t)std::min<uint64_t>(PQG_LD_GRID, std::max<uint64_t>(wgrid, blob_len >> 14));
    hipLaunchKernelGGL(k_lv_emit_walk<LvDictOut>, dim3(ldgrid), dim3(WG), 0, s, blob, blob_len, pages, npages, chunks,
                       sel, rt, lt, LvDictOut{dsrc, dlen, vsrc, vlen});
    return hipGetLastError();
  }
  // (k_lv_plan2's scan ran in k_lv_segscan's last workgroup)
  if (PQG_D1 && (sel == SS_DEF || sel == SS_REP) && (widths & 2u)) lv_launch_d1(blob, blob_len, pages, npages, chunks, sel, rt, lt, s);
// window table and window emit kernels on 4x grids (round 5, kernel times: config 5 k_lv_win
// 0.286 -> 0.267 ms, k_lv_emit 0.536 -> 0.515; config 2 at p_null 0.1 0.401 -> 0.386 and 0.698 ->
// 0.679; 2x about half of that)
#ifndef PQG_LW_GRIDX
#define PQG_LW_GRIDX 4
#endif
  hipLaunchKernelGGL(k_lv_win, dim3(wgrid * PQG_LW_GRIDX), dim3(WG), 0, s, blob, blob_len, pages, npages, chunks, sel, rt,
                     lt);
  // window tables of 64 / 128 entry offsets (bit width 1 / 2) take the readlane walks
  if (widths & 2u)
    hipLaunchKernelGGL(k_lv_stitch<1>, dim3(npages), dim3(SC_WG), 0, s, blob, pages, npages, chunks, sel, rt, lt);
  if (widths & 4u)
    hipLaunchKernelGGL(k_lv_stitch<2>, dim3(npages), dim3(SC_WG), 0, s, blob, pages, npages, chunks, sel, rt, lt);
  if (widths & ~7u)
    hipLaunchKernelGGL(k_lv_stitch<0>, dim3(npages), dim3(SC_WG), 0, s, blob, pages, npages, chunks, sel, rt, lt);
  if (sel == SS_BOOL) {
    hipLaunchKernelGGL(k_lv_emit<1>, dim3(wgrid), dim3(WG), 0, s, blob, blob_len, pages, npages, chunks, sel, rt, lt);
    hipLaunchKernelGGL(k_lv_emit_walk<LvLevelOut<1>>, dim3(wgrid), dim3(WG), 0, s, blob, blob_len, pages, npages,
                       chunks, sel, rt, lt, LvLevelOut<1>{});
  } else {
#ifndef PQG_LE_GRIDX
#define PQG_LE_GRIDX 4
#endif
    hipLaunchKernelGGL(k_lv_emit<2>, dim3(wgrid * PQG_LE_GRIDX), dim3(WG), 0, s, blob, blob_len, pages, npages, chunks, sel,
                       rt, lt);
    hipLaunchKernelGGL(k_lv_emit_walk<LvLevelOut<2>>, dim3(wgrid * PQG_EW_GRIDX), dim3(WG), 0, s, blob, blob_len, pages, npages,
                       chunks, sel, rt, lt, LvLevelOut<2>{});
  }
  return hipGetLastError();
}

}  // extern "C"

}  // namespace pqg
