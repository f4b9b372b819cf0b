// pqg_lvd1.hpp — one-bit level streams of dense pages (def / rep levels of max level 1: config
// 2's def levels and every config-5 column's), included by pqg_levels.hip. RleDecoder::get_batch
// over the RLE/bit-packing hybrid (rle.rs:398-434, 490-508; LevelDecoder::get, levels.rs:249-271)
// with w = 1: a header is a varint, an RLE run one value byte, a bit-packed run of g groups g
// payload bytes whose bit j is output j (LSB first, bit_util.rs:456-528).
//
// The stream is cut into 16 KiB segments, a segment into 256 chunks of 64 bytes, one thread per
// chunk. A thread walks the header chain through its chunk from a guessed first header (the exit
// of a walk through the 64 bytes before the chunk: chains entering anywhere meet the true one
// within a few headers). The guesses are then checked against the chunk before (its chain's exit
// must be this chunk's first header) and the chunks whose guess was wrong walk again from the
// right entry until no exit changes (lv_spec_chain's idea at chunk granularity). Every walk is
// exact; only the number of rounds depends on the data.
//
//   k_d1_tab     per segment: the chain R from chunk 0's guess, each chunk's walk of it (exit,
//                outputs, header mask: kept for the emit) and, for the 64 offsets a chain can
//                enter the segment at (one hop is at most a 1-byte header and 63 groups, or a
//                longer header of an RLE run), where the chain leaves the segment and its outputs
//                on the way: a lane per entry walks until it lands on a header of R, whose output
//                suffix sums give the rest.
//   k_d1_stitch  per page: follows the segment tables from offset 0: each segment's true entry
//                and first output (one LDS lookup per segment).
//   k_d1_emit    per segment: R's walks taken over (the true entry is R's, or its chain joins R
//                within a few headers: only those chunks walk again), each chunk's first output by
//                a workgroup scan, then every thread writes its outputs' bits into an LDS bitmap of
//                the segment (a word at a time: a register accumulator over its runs' payload bits
//                and RLE fills) and the workgroup stores it expanded to int16, one contiguous
//                4 KiB per store instruction, counting the 1s (the def count).
//
// Pages whose true chain meets a header the fast parse refuses, runs past the stream end before
// n outputs, an RLE value above 1, or enters a segment past its first 64 bytes (runs longer than
// the writer's 63 groups) are handed to the general decoder (lv_bail, PF_D1 -> PF_BAIL), which
// reproduces every reference error.
#pragma once
// (included inside namespace pqg)

#ifndef PQG_D1
#define PQG_D1 1  // (0: dense one-bit pages on the window path, for A/B runs)
#endif
constexpr uint32_t D1_SEG = LW_SEGW * LV_WIN;  // 16 KiB: a segment of k_lv_plan's sbase
constexpr uint32_t D1_CH = 64;                 // stream bytes per chunk (one thread)
constexpr uint32_t D1_NCH = D1_SEG / D1_CH;    // 256 chunks = threads per workgroup
constexpr uint32_t D1_PRE = 64;                // k_d1_tab: bytes staged before the segment (chunk 0's guess)
constexpr uint32_t D1_STB = D1_PRE + D1_SEG + 128 + 16;  // staged bytes (+ payload read-ahead, alignment)
constexpr uint32_t D1_STW = D1_STB / 4;
constexpr uint32_t D1_DEAD = 0xFFFFFFFFu;      // a chain that met a header the fast parse refuses
constexpr uint32_t D1_UNKNOWN = 0xFFFFFFFEu;   // table: an entry whose chain was not followed to its end
constexpr uint32_t D1_NONE = 0xFFFFFFFFu;      // segment not on the true chain
constexpr uint32_t D1_ENT = 64;                // entry offsets per segment table
constexpr uint32_t D1_PREK = 8;                // chunks whose R header prefixes k_d1_tab keeps
// per segment in lt.srec (uint2 units, LW_SCAP per segment): table [0, 64), the stitch's (true
// entry | D1_NONE, first output) at [96], (R's entry, its last restart) at [97], R's walk of each
// chunk (exit, outputs, header mask: a uint4) [128, 640), R's entry of each chunk (u32) [640, 768)
constexpr uint32_t D1_RES = 96, D1_RW = 128, D1_RS = D1_RW + 2 * D1_NCH;
static_assert(D1_RS + D1_NCH / 2 <= LW_SCAP, "segment record");
static_assert(D1_NCH == WG, "one thread per chunk");
#ifndef PQG_D1_RB
#define PQG_D1_RB 131072
#endif
constexpr uint32_t D1_RB = PQG_D1_RB;  // bitmap bits per emit round (16 KiB)
constexpr uint32_t D1_RBW = D1_RB / 32;

// Diagnostics (PQG_DIAG builds, PQG_DEBUG 8192): thread 0's s_memtime cycles per phase of each
// workgroup of k_d1_tab (slots 0..2047) and k_d1_emit (2048..4095), 8 words each.
#ifdef PQG_DIAG
#define D1_DIAG_DECL(kid)                                                                            \
  const bool dst_ = (chunks[0].cp.debug & 8192) && chunks[0].cp.dbgbuf && threadIdx.x == 0;       \
  uint64_t dacc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, dt0_ = dst_ ? __builtin_amdgcn_s_memtime() : 0ull; \
  const uint32_t dkid_ = (kid);
#define D1_STAMP(k)                                    \
  if (dst_) {                                          \
    const uint64_t t1_ = __builtin_amdgcn_s_memtime(); \
    dacc_[k] += t1_ - dt0_;                            \
    dt0_ = t1_;                                        \
  }
#define D1_COUNT(k, v) \
  if (dst_) dacc_[k] += (v);
#define D1_DIAG_END()                                                            \
  if (dst_ && blockIdx.x < 2048u) {                                             \
    uint64_t* d_ = chunks[0].cp.dbgbuf + 8ull * (dkid_ * 2048u + blockIdx.x);  \
    for (int i_ = 0; i_ < 8; ++i_) d_[i_] = dacc_[i_];                         \
  }
#else
#define D1_DIAG_DECL(kid)
#define D1_STAMP(k)
#define D1_COUNT(k, v)
#define D1_DIAG_END()
#endif

__device__ inline uint32_t d1_sat(uint64_t v) { return v > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)v; }

// Stage stream bytes [st0, st0 + D1_STB - 16) of stream S (aligned down to 16 bytes; reads past
// the stream are harmless: no header past slen is parsed). Returns the stage byte of st0.
__device__ inline uint32_t d1_stage(const uint8_t* __restrict__ blob, uint64_t blob_len, uint64_t S, uint32_t st0,
                                    uint32_t* st) {
  const uint64_t A = (S + st0) & ~15ull;
  for (uint32_t c = threadIdx.x; c < D1_STB / 16; c += D1_NCH) {
    const uint64_t a = A + (uint64_t)c * 16u;
    reinterpret_cast<uint4*>(st)[c] =
        a + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
  }
  return (uint32_t)(S + st0 - A);
}

// One header at stream position q < slen (w = 1; st0: the stage's origin): next position and
// output count; false for a header the fast parse refuses (lv_parse4's rule).
__device__ __forceinline__ bool d1_hop(const uint32_t* st, uint32_t sb, uint32_t st0, uint32_t slen, uint32_t q,
                                       uint32_t& nx, uint32_t& cnt) {
  const uint32_t rel = q - st0 + sb;
  const uint32_t h = reinterpret_cast<const uint8_t*>(st)[rel];
  if (h < 128u) {
    const uint32_t g = h >> 1;
    const bool bp = (h & 1u) != 0;
    const uint32_t len = bp ? 1u + g : 2u;
    nx = q + len;
    cnt = bp ? g * 8u : g;
    return len <= slen - q;
  }
  uint32_t v;
  bool bpp;
  return lv_parse4(st, rel, q, slen, 1u, 1u, nx, cnt, v, bpp);
}

// The same with the run's kind and RLE value / payload start.
__device__ __forceinline__ bool d1_hop_full(const uint32_t* st, uint32_t sb, uint32_t st0, uint32_t slen, uint32_t q,
                                            uint32_t& nx, uint32_t& cnt, uint32_t& v, bool& bp) {
  const uint32_t rel = q - st0 + sb;
  const uint8_t* b = reinterpret_cast<const uint8_t*>(st);
  const uint32_t h = b[rel];
  if (h < 128u) {
    const uint32_t g = h >> 1;
    bp = (h & 1u) != 0;
    const uint32_t len = bp ? 1u + g : 2u;
    nx = q + len;
    cnt = bp ? g * 8u : g;
    v = bp ? q + 1u : (uint32_t)b[rel + 1u];
    return len <= slen - q;
  }
  return lv_parse4(st, rel, q, slen, 1u, 1u, nx, cnt, v, bp);
}

// The chain from stream position q through the chunk [cb, cb + 64): its header mask, output
// count (saturating) and exit (the first position past the chunk, the stream end, or D1_DEAD).
// q at or past the chunk's end (a hop over it), at the stream end or dead: nothing in the chunk.
struct D1Walk {
  uint64_t hm;
  uint32_t cnt, out;
};

__device__ inline void d1_walk(const uint32_t* st, uint32_t sb, uint32_t st0, uint32_t slen, uint32_t cb,
                               uint32_t q, D1Walk& r) {
  uint32_t hlo = 0, hhi = 0, cnt = 0;
  uint64_t big = 0;
  const uint8_t* b = reinterpret_cast<const uint8_t*>(st);
  const uint32_t lim = min(cb + D1_CH, slen);
#pragma unroll 1
  for (;;) {
    // one-byte headers, branch-free: a single exit condition (left the chunk, a longer header, a
    // run past the stream's end)
#pragma unroll 1
    for (;;) {
      const uint32_t h = b[(q < lim ? q : cb) - st0 + sb];
      const uint32_t g = (h >> 1) & 63u, bp = h & 1u;
      const uint32_t len = bp ? g + 1u : 2u;
      if (!(q < lim && h < 128u && len <= slen - q)) break;
      const uint32_t x = q - cb;
      hlo |= x < 32u ? 1u << (x & 31u) : 0u;
      hhi |= x >= 32u ? 1u << (x & 31u) : 0u;
      cnt += bp ? g << 3 : g;
      q += len;
    }
    if (q >= lim) break;  // (D1_DEAD too)
    uint32_t nx, c, v;
    bool bpp;
    if (!lv_parse4(st, q - st0 + sb, q, slen, 1u, 1u, nx, c, v, bpp)) {
      q = D1_DEAD;
      break;
    }
    const uint32_t x = q - cb;
    hlo |= x < 32u ? 1u << (x & 31u) : 0u;
    hhi |= x >= 32u ? 1u << (x & 31u) : 0u;
    big += c;
    q = nx;
  }
  r.hm = ((uint64_t)hhi << 32) | hlo;
  r.cnt = d1_sat(big + cnt);
  r.out = q;
}

// Guess of the chain's entry into the chunk starting at cb: the exit of a walk from q0 over
// one-byte headers, bytes that are not one skipped (branch-free).
__device__ inline uint32_t d1_guess_entry(const uint32_t* st, uint32_t sb, uint32_t st0, uint32_t slen, uint32_t q0,
                                          uint32_t cb) {
  const uint8_t* b = reinterpret_cast<const uint8_t*>(st);
  uint32_t q = q0;
  const uint32_t lim = min(cb, slen);
#pragma unroll 1
  while (q < lim) {
    const uint32_t h = b[q - st0 + sb];
    const uint32_t len = (h & 1u) ? 1u + ((h >> 1) & 63u) : 2u;
    const bool one = h < 128u;
    q = one && len > slen - q ? D1_DEAD : q + (one ? len : 1u);
  }
  return q;
}

// Settle the segment's chain from `entry` (chunk 0's first header): every thread has walked its
// chunk from guess s (W); chunks whose first header is not the exit of the chunk before walk again
// from it, until no exit changes. Only entries a writer's hop can reach are taken over (inside the
// chunk, or the stream's end): a wrong guess that hops far or dies would otherwise travel down the
// chunks one per round as fast as its correction. A chunk whose entry is a dead exit or a hop
// past it keeps its own walk: a restart (*lastr = the last such chunk, 0 if none; *far = 1 if one
// was a hop, not a death). The chain through the chunks before a restart dies or hops off, so no
// writer's true chain runs through them. Afterwards outs[c] is chunk c's exit; returns the rounds.
__device__ inline uint32_t d1_settle(uint32_t* outs, uint32_t* lastr, uint32_t* far, const uint32_t* st, uint32_t sb,
                                     uint32_t st0, uint32_t slen, uint32_t cb, uint32_t entry, uint32_t& s,
                                     D1Walk& W) {
  const uint32_t c = threadIdx.x;
  outs[c] = W.out;
  if (c == 0) {
    *lastr = 0;
    *far = 0;
  }
  __syncthreads();
  uint32_t rounds = 0;
#pragma unroll 1
  for (;; ++rounds) {
    const uint32_t in = c == 0 ? entry : outs[c - 1];
    bool ch = false;
    if (in != s && (in < cb + D1_CH || (in >= slen && in != D1_DEAD))) {
      const uint32_t old = W.out;
      s = in;
      d1_walk(st, sb, st0, slen, cb, s, W);
      ch = W.out != old;
    }
    __syncthreads();  // every read of outs is done
    if (ch) outs[c] = W.out;
    if (!__syncthreads_or(ch)) break;
  }
  const uint32_t in = c == 0 ? entry : outs[c - 1];
  if (in != s) {  // (an entry no writer's hop reaches: a restart)
    atomicMax(lastr, c);
    if (in != D1_DEAD) atomicOr(far, 1u);
  }
  __syncthreads();
  return rounds;
}

// Exclusive scan of v over the workgroup's 256 threads (total: the sum). wsum: 4 words of LDS.
__device__ inline uint64_t d1_scan_excl(uint64_t v, uint64_t* wsum, uint64_t& total) {
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  uint64_t s = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(s, d, 64);
    if (lane >= (uint32_t)d) s += y;
  }
  if (lane == 63u) wsum[wid] = s;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
#pragma unroll
  for (uint32_t k = 0; k < WG / WAVE; ++k) {
    const uint64_t x = wsum[k];
    pre += k < wid ? x : 0ull;
    tot += x;
  }
  __syncthreads();  // (wsum reusable)
  total = tot;
  return pre + s - v;
}

// A workgroup's contiguous range of the decode's segments (sbase), its page found once and then
// advanced with the segment.
struct D1Range {
  uint32_t g, g1, p, pend;
  __device__ inline bool begin(const LevelTables& lt, int npages) {
    const uint32_t total = lt.sbase[npages];
    const uint32_t per = (total + gridDim.x - 1u) / gridDim.x;
    g = blockIdx.x * per;
    g1 = min(total, g + per);
    if (g >= g1) return false;
    p = lv_page_of(lt.sbase, (uint32_t)npages, g);
    pend = lt.sbase[p + 1];
    return true;
  }
  // page of segment g (g advances monotonically)
  __device__ inline void at(const LevelTables& lt) {
    while (g >= pend) {
      ++p;
      pend = lt.sbase[p + 1];
    }
  }
};

// ------------------------------------------------------------------------------ k_d1_tab
struct D1TabSmem {
  uint32_t st[D1_STW];
  uint32_t outs[D1_NCH];
  uint64_t hm[D1_NCH];
  uint64_t suf[D1_NCH + 1];
  uint32_t pre[D1_PREK][D1_CH];  // R's outputs before each of its headers in chunks 0 .. D1_PREK - 1
  uint64_t wsum[WG / WAVE];
  uint32_t E, lastr, far;
};

__global__ void __launch_bounds__(WG) k_d1_tab(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                               const PageWork* __restrict__ pages, int npages,
                                               const ChunkWork* chunks, int sel, RunTables rt, LevelTables lt) {
  __shared__ D1TabSmem sm;
  const uint32_t c = threadIdx.x;
  D1Range G;
  if (!G.begin(lt, npages)) return;
  D1_DIAG_DECL(0)
  for (; G.g < G.g1; ++G.g) {
    G.at(lt);
    const uint32_t p = G.p;
    Stream s;
    if (rt.pflag[p] != PF_D1 || !lv_stream(blob, pages[p], sel, chunks, s)) continue;
    const uint32_t seg0 = (G.g - lt.sbase[p]) * D1_SEG, slen = s.slen;
    const uint32_t st0 = seg0 ? seg0 - D1_PRE : 0u;  // stage origin (the 64 bytes before the segment)
    __syncthreads();  // the previous segment's LDS reads are done
    D1_STAMP(7)
    const uint32_t sb = d1_stage(blob, blob_len, s.S, st0, sm.st);
    __syncthreads();
    D1_STAMP(0)
    const uint32_t cb = seg0 + c * D1_CH;
    // guesses: every chunk's entry from a walk through the 64 bytes before it (the stream's first
    // header is exact), then the chunk walked exactly from it; R is the chain from chunk 0's guess
    D1Walk W;
    uint32_t q;
    if (cb >= slen) {  // past the stream's end: the chain has ended there
      q = slen;
      W.hm = 0;
      W.cnt = 0;
      W.out = slen;
    } else {
      q = cb == 0 ? 0u : d1_guess_entry(sm.st, sb, st0, slen, cb - D1_CH, cb);
      d1_walk(sm.st, sb, st0, slen, cb, q, W);
    }
    if (c == 0) sm.E = q;
    __syncthreads();
    const uint32_t E = sm.E;
    D1_STAMP(1)
    const uint32_t rounds = d1_settle(sm.outs, &sm.lastr, &sm.far, sm.st, sb, st0, slen, cb, E, q, W);
    D1_STAMP(2)
    D1_COUNT(6, rounds + (sm.lastr ? (1ull << 16) : 0ull) + (1ull << 32))
    (void)rounds;
    // R: header masks, output suffix sums, exit; per chunk its walk (k_d1_emit takes it over)
    uint64_t tot;
    const uint64_t ex = d1_scan_excl(W.cnt, sm.wsum, tot);
    sm.hm[c] = W.hm;
    sm.suf[c] = tot - ex;
    if (c == 0) sm.suf[D1_NCH] = 0;
    uint2* rec = lt.srec + (uint64_t)G.g * LW_SCAP;
    reinterpret_cast<uint4*>(rec + D1_RW)[c] = make_uint4(W.out, W.cnt, (uint32_t)W.hm, (uint32_t)(W.hm >> 32));
    reinterpret_cast<uint32_t*>(rec + D1_RS)[c] = q;
    if (c < D1_PREK) {  // R's outputs before each header of the first chunks
      uint32_t acc = 0;
      for (uint64_t m = W.hm; m; m &= m - 1ull) {
        const uint32_t x = (uint32_t)__builtin_ctzll(m);
        uint32_t nx, cn = 0;
        d1_hop(sm.st, sb, st0, slen, cb + x, nx, cn);  // (a header of R: parses)
        sm.pre[c][x] = acc;
        acc = d1_sat((uint64_t)acc + cn);
      }
    }
    __syncthreads();
    D1_STAMP(3)
    const uint32_t rexit = sm.outs[D1_NCH - 1], lastr = sm.lastr;
    if (c == 0) rec[D1_RES + 1] = make_uint2(E, lastr);
    if (c < D1_ENT) {
      // entry seg0 + c: exact hops until it lands on a header of R (then R's rest: its outputs
      // from there, or a dead chain if R restarts after that chunk), leaves the segment, ends the
      // stream or dies
      uint32_t e = seg0 + c, xo;
      uint64_t acc = 0;
#pragma unroll 1
      for (;;) {
        if (e >= slen) {  // (also D1_DEAD)
          xo = e;
          break;
        }
        const uint32_t k = (e - seg0) / D1_CH, x = (e - seg0) & (D1_CH - 1u);
        if (k >= D1_PREK) {  // not on R within the first chunks: the stitch hands the page back if
          xo = D1_UNKNOWN;   // it is the true entry (an entry meets the true chain within a few
          break;             // headers, and R is the true chain after a few headers)
        }
        if ((sm.hm[k] >> x) & 1ull) {  // on R
          if (k < lastr) {
            xo = D1_DEAD;
            break;
          }
          const uint64_t rest = sm.suf[k] - sm.pre[k][x];
          acc += rest;
          xo = rexit;
          break;
        }
        uint32_t nx, cn;
        if (!d1_hop(sm.st, sb, st0, slen, e, nx, cn)) {
          xo = D1_DEAD;
          break;
        }
        acc += cn;
        e = nx;
      }
      rec[c] = make_uint2(xo, d1_sat(acc));
    }
    D1_STAMP(5)
  }
  D1_DIAG_END()
}

// ------------------------------------------------------------------------------ k_d1_stitch
// One workgroup per page (grid-stride): the segment tables staged through LDS, 64 segments at a
// time, thread 0 follows them from offset 0.
__global__ void __launch_bounds__(WG) k_d1_stitch(const uint8_t* __restrict__ blob, const PageWork* __restrict__ pages,
                                                  int npages, const ChunkWork* chunks, int sel, RunTables rt,
                                                  LevelTables lt) {
  __shared__ uint2 tb[64 * D1_ENT];
  __shared__ uint32_t e_s, jn_s, state_s;
  __shared__ uint64_t acc_s;
  for (int p = (int)blockIdx.x; p < npages; p += (int)gridDim.x) {
    Stream s;
    if (rt.pflag[p] != PF_D1 || !lv_stream(blob, pages[p], sel, chunks, s)) continue;
    const uint32_t g0 = lt.sbase[p], ns = lt.sbase[p + 1] - g0, n = s.n, slen = s.slen;
    __syncthreads();  // (the previous page's shared state)
    if (threadIdx.x == 0) {
      e_s = 0;
      jn_s = 0;
      state_s = 0;  // 0 following the chain, 1 n outputs reached, 2 hand the page back
      acc_s = 0;
    }
    for (uint32_t blk = 0; blk < ns; blk += 64) {
      const uint32_t nb = min(64u, ns - blk);
      for (uint32_t i = threadIdx.x; i < nb * D1_ENT; i += WG)
        tb[i] = lt.srec[(uint64_t)(g0 + blk + i / D1_ENT) * LW_SCAP + (i % D1_ENT)];
      __syncthreads();
      if (threadIdx.x == 0) {
        uint32_t e = e_s, jn = jn_s, state = state_s;
        uint64_t acc = acc_s;
        for (uint32_t k = 0; k < nb; ++k) {
          const uint32_t j = blk + k;
          uint2 res = make_uint2(D1_NONE, 0u);
          if (state == 0 && j == jn) {
            if (e >= D1_ENT) {
              state = 2;  // entered past the table (runs longer than the writer's)
            } else {
              const uint2 t = tb[k * D1_ENT + e];
              res = make_uint2(e, (uint32_t)acc);
              acc += t.y;
              if (acc >= n) {
                state = 1;
              } else if (t.x >= slen) {
                state = 2;  // the chain dies (D1_DEAD), is not known (D1_UNKNOWN) or the stream ends before n outputs
              } else {
                jn = t.x / D1_SEG;
                e = t.x - jn * D1_SEG;
              }
            }
          }
          lt.srec[(uint64_t)(g0 + j) * LW_SCAP + D1_RES] = res;
        }
        e_s = e;
        jn_s = jn;
        state_s = state;
        acc_s = acc;
      }
      __syncthreads();
    }
    if (threadIdx.x == 0 && state_s != 1) LV_BAIL(rt, lt, (uint32_t)p, PF_D1, 8);
  }
}

// ------------------------------------------------------------------------------ k_d1_emit
struct D1EmitSmem {
  uint32_t st[D1_STW];
  uint32_t outs[D1_NCH];
  uint32_t bm[D1_RBW];
  uint64_t wsum[WG / WAVE];
  uint32_t lastr, far;
};

// 32 payload bits from bit j of the run whose payload starts at stream byte v (staged from st0).
__device__ inline uint32_t d1_bits32(const uint32_t* st, uint32_t sb, uint32_t st0, const uint8_t* __restrict__ blob,
                                     uint64_t blob_len, uint64_t S, uint32_t v, uint32_t j) {
  const uint32_t B = (v - st0 + sb) * 8u + j;
  if ((B >> 3) + 8u <= D1_STB) return __builtin_amdgcn_alignbit(st[(B >> 5) + 1u], st[B >> 5], B & 31u);
  return (uint32_t)(gload_u64(blob, blob_len, S + v + (j >> 3)) >> (j & 7u));
}

template <int OUT>
__global__ void __launch_bounds__(WG) k_d1_emit(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                PageWork* pages, int npages, const ChunkWork* chunks, int sel,
                                                RunTables rt, LevelTables lt) {
  __shared__ D1EmitSmem sm;
  const uint32_t c = threadIdx.x;
  D1Range G;
  if (!G.begin(lt, npages)) return;
  D1_DIAG_DECL(1)
  for (; G.g < G.g1; ++G.g) {
    G.at(lt);
    const uint32_t p = G.p;
    Stream s;
    if (rt.pflag[p] != PF_D1 || !lv_stream(blob, pages[p], sel, chunks, s)) continue;
    const uint2* rec = lt.srec + (uint64_t)G.g * LW_SCAP;
    const uint2 res = rec[D1_RES];
    if (res.x == D1_NONE) continue;
    const uint32_t E = rec[D1_RES + 1].x;                                // R's entry
    const uint4 rw = reinterpret_cast<const uint4*>(rec + D1_RW)[c];     // R's walk of this chunk
    const uint32_t rs = reinterpret_cast<const uint32_t*>(rec + D1_RS)[c];  // and its entry
    const uint32_t seg0 = (G.g - lt.sbase[p]) * D1_SEG, slen = s.slen, n = s.n;
    __syncthreads();
    D1_STAMP(7)
    const uint32_t sb = d1_stage(blob, blob_len, s.S, seg0, sm.st);
    __syncthreads();
    D1_STAMP(0)
    const uint32_t cb = seg0 + c * D1_CH, entry = seg0 + res.x;
    // R's walks taken over; chunk 0 walks from the true entry when it is not R's
    D1Walk W;
    uint32_t q;
    if (c == 0 && entry != E) {
      q = entry;
      d1_walk(sm.st, sb, seg0, slen, cb, q, W);
    } else {
      q = c == 0 ? E : rs;
      W.out = rw.x;
      W.cnt = rw.y;
      W.hm = ((uint64_t)rw.w << 32) | rw.z;
    }
    D1_STAMP(1)
    const uint32_t rounds = d1_settle(sm.outs, &sm.lastr, &sm.far, sm.st, sb, seg0, slen, cb, entry, q, W);
    D1_STAMP(2)
    D1_COUNT(6, rounds + (sm.lastr ? (1ull << 16) : 0ull) + (1ull << 32))
    (void)rounds;
    if (sm.far) {  // the true chain hops past a chunk (runs longer than the writer's): not taken here
      if (c == 0) LV_BAIL(rt, lt, p, PF_D1, 10);
      continue;
    }
    uint64_t T;
    const uint64_t ob = (uint64_t)res.y + d1_scan_excl(W.cnt, sm.wsum, T);  // chunk's first output (page)
    const uint64_t go = s.out;  // global index of the page's output 0
    const uint64_t gs = go + res.y, ge = go + min((uint64_t)res.y + T, (uint64_t)n);
    gptr<int16_t> out = (gptr<int16_t>)gp(lv_out(chunks[pages[p].chunk], sel));
    bool bad = false;
    uint32_t ones = 0;
    const uint64_t R0 = gs & ~31ull;
    const int64_t cs0 = (int64_t)(go + ob - R0);  // the chunk's first output, from the bitmap origin
    for (uint64_t r0 = R0; r0 < ge; r0 += D1_RB) {
      // round-relative (32-bit): outputs [lo, hi) of the segment in this round
      const uint32_t lo = (uint32_t)((gs > r0 ? gs : r0) - r0), hi = (uint32_t)((ge < r0 + D1_RB ? ge : r0 + D1_RB) - r0);
      const uint32_t nwd = (hi + 31u) >> 5;
      for (uint32_t i = c; i < nwd; i += WG) sm.bm[i] = 0u;
      __syncthreads();
      const int64_t cs = cs0 - (int64_t)(r0 - R0);
      {
        // the thread's outputs in the round, [a, z), a word at a time: its runs' bits (payload
        // bits, RLE fills) gathered into a register; words no other thread touches stored, the
        // first and last ORed in. Runs before the round are skipped by their counts.
        const int64_t cend = cs + (int64_t)W.cnt;
        const bool mine = cend > (int64_t)lo && cs < (int64_t)hi;
        const uint32_t a = mine ? (uint32_t)(cs > (int64_t)lo ? cs : (int64_t)lo) : 0u;
        const uint32_t z = mine ? (uint32_t)(cend < (int64_t)hi ? cend : (int64_t)hi) : 0u;
        uint64_t m = mine ? W.hm : 0ull;
        int64_t o = cs;  // first output of the next run
        uint32_t pos = a, rl = 0, rv = 0, rj = 0, fill = 0, wacc = 0;
        bool rbp = false;
        const uint32_t wfirst = a >> 5, wlast = z ? (z - 1u) >> 5 : 0u;
#pragma unroll 1
        while (pos < z) {
          if (rl == 0) {  // the next run (a header of the true chain: parses)
            if (!m) break;
            const uint32_t hq = cb + (uint32_t)__builtin_ctzll(m);
            m &= m - 1ull;
            uint32_t nx, cn, v;
            d1_hop_full(sm.st, sb, seg0, slen, hq, nx, cn, v, rbp);
            const int64_t ro = o;
            o += cn;
            if (o <= (int64_t)pos) continue;  // before the round
            if (!rbp && v > 1u) bad = true;  // an RLE value wider than the bit width (rle.rs:498)
            rl = (uint32_t)(o - (int64_t)pos);
            rj = (uint32_t)((int64_t)pos - ro);
            rv = v;
            fill = (!rbp && (v & 1u)) ? 0xFFFFFFFFu : 0u;
          }
          const uint32_t bpos = pos & 31u;
          const uint32_t take = min(min(rl, 32u - bpos), z - pos);
          const uint32_t mk = take >= 32u ? 0xFFFFFFFFu : (1u << take) - 1u;
          const uint32_t bits = rbp ? d1_bits32(sm.st, sb, seg0, blob, blob_len, s.S, rv, rj) : fill;
          wacc |= (bits & mk) << bpos;
          pos += take;
          rl -= take;
          rj += take;
          if ((pos & 31u) == 0 || pos == z) {
            const uint32_t wi = (pos - 1u) >> 5;
            if (wi == wfirst || wi == wlast) atomicOr(&sm.bm[wi], wacc);
            else sm.bm[wi] = wacc;
            wacc = 0;
          }
        }
      }
      __syncthreads();
      D1_STAMP(3)
      // stores: 8 outputs per 16-byte store over the round's outputs [lo, hi)
      gptr<int16_t> orr = out + r0;
      const uint32_t u0 = lo >> 3, u1 = (hi + 7u) >> 3;
#pragma unroll 2
      for (uint32_t u = u0 + c; u < u1; u += WG) {
        const uint32_t rb = u << 3;
        uint32_t bits = (sm.bm[rb >> 5] >> (rb & 31u)) & 0xFFu;
        if (rb >= lo && rb + 8u <= hi) {
          uint32_t d[4];
#pragma unroll
          for (uint32_t t = 0; t < 4; ++t) d[t] = (((bits >> (2u * t)) & 3u) * 0x8001u) & 0x10001u;
          gst16((gptr<uint8_t>)(orr + rb), make_uint4(d[0], d[1], d[2], d[3]));
        } else {
          uint32_t vm = 0;
          for (uint32_t t = 0; t < 8u; ++t) {
            const uint32_t gg = rb + t;
            if (gg >= lo && gg < hi) {
              orr[gg] = (int16_t)((bits >> t) & 1u);
              vm |= 1u << t;
            }
          }
          bits &= vm;
        }
        ones += (uint32_t)__builtin_popcount(bits);
      }
      __syncthreads();  // the bitmap is cleared by the next round
      D1_STAMP(4)
    }
    if (__syncthreads_or(bad)) {
      if (c == 0) LV_BAIL(rt, lt, p, PF_D1, 9);
      continue;
    }
    if (sel == SS_DEF) {
      const uint64_t t = block_sum_u64(ones, sm.wsum);
      if (c == 0 && t) atomicAdd((unsigned long long*)&pages[p].nonnull, (unsigned long long)t);
    }
    D1_STAMP(5)
  }
  D1_DIAG_END()
}

// The one-bit dense pages of stream sel (def / rep levels): tables, stitch, emit.
static void lv_launch_d1(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages, const ChunkWork* chunks,
                         int sel, RunTables rt, LevelTables lt, hipStream_t s) {
#ifndef PQG_D1_GRID
#define PQG_D1_GRID 2048
#endif
#ifndef PQG_D1_TGRID
#define PQG_D1_TGRID 16384  // (k_d1_tab at p_null 0.1: 2048 workgroups 0.33 ms, 4096 0.28, 8192 0.25, 16384 0.24)
#endif
  hipLaunchKernelGGL(k_d1_tab, dim3(PQG_D1_TGRID), dim3(WG), 0, s, blob, blob_len, pages, npages, chunks, sel, rt, lt);
  hipLaunchKernelGGL(k_d1_stitch, dim3(npages < 1024 ? npages : 1024), dim3(WG), 0, s, blob, pages, npages, chunks, sel,
                     rt, lt);
  hipLaunchKernelGGL(k_d1_emit<2>, dim3(PQG_D1_GRID), dim3(WG), 0, s, blob, blob_len, pages, npages, chunks, sel, rt, lt);
}
