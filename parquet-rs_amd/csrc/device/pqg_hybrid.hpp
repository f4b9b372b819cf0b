// pqg_hybrid.hpp — pipelined RLE/bit-packing hybrid decoder (rle.rs:320-509) for one stream
// per 256-thread workgroup.
//
// Run headers sit at data-dependent byte offsets, so discovering them is a serial walk; the
// expansion of discovered runs is embarrassingly parallel. The workgroup therefore runs a
// two-stage pipeline over batches of runs:
//
//   wave 0  (walker)    walks the header chain of batch k+1 inside an LDS-staged region of
//                       the stream: each lane parses a speculative header at its own byte of
//                       a 64-byte window (branchless varint decode from a 16-byte LDS read),
//                       then the wave hops along the real chain with v_readlane, recording
//                       (first output index, RLE value | payload offset) in an LDS run table;
//   waves 1-3 (expanders) expand batch k: 8 consecutive outputs per lane, run found by a
//                       binary search of the batch's run table, bit-packed payload read from
//                       the same LDS region, coalesced stores through the Emit functor.
//
// Regions and run tables are double-buffered; one barrier per batch. A batch covers the
// runs whose header lies in one 8 KiB region (+2 KiB look-ahead holds any bit-packed run the
// reference encoder can write, 1 + 63*32 bytes); longer foreign runs fall back to global
// loads. Every check that makes the reference return Err / panic / spin is reported as a
// status.
#pragma once
#include "pqg_device.hpp"

namespace pqg {

// Diagnostic counters (pqg_debug_set / pqg_debug_read): mode bit 0 skips expansion, bit 1
// skips the walk after the first batch, bit 2 accumulates s_memtime stamps. Mode 0 is the
// production path (one scalar load per workgroup). Each translation unit has its own copy
// (no relocatable device code); the switches act on the kernels of pqg_kernels.hip.
static __device__ uint32_t g_pqg_debug_mode = 0;
static __device__ unsigned long long g_pqg_stats[16];

__device__ inline uint64_t hb_clock() { return __builtin_amdgcn_s_memtime(); }

constexpr int HB_BLK = 8192;
constexpr int HB_PAD = 2112;
constexpr int HB_REGION = HB_BLK + HB_PAD;  // bytes staged per region (multiple of 16)
constexpr int HB_RWORDS = HB_REGION / 4 + 8;
constexpr int HB_RUNCAP = 1024;
constexpr int HB_TILE = 512;                // outputs per expander wave step (64 lanes x 8)

constexpr uint32_t HF_BP = 1u, HF_EOF = 2u, HF_PANIC = 4u;
constexpr uint32_t HB_RLE = 0x80000000u;

struct HbBatch {
  uint64_t A0;
  uint32_t nruns, seg_start, seg_end, buf, done, err;
};

struct HybridSmem {
  uint32_t region[2][HB_RWORDS];
  uint32_t start[2][HB_RUNCAP + 1];
  uint32_t info[2][HB_RUNCAP];
  HbBatch batch[2];
  uint32_t eflag;
  uint64_t red[4];
};

// wave-cooperative copy of [A0, A0 + HB_REGION) into region (called by one wave)
__device__ inline void hb_load_region(const uint8_t* blob, uint64_t blob_len, uint64_t A0,
                                      uint32_t* region, uint32_t lane) {
  for (uint32_t c = lane; c < HB_REGION / 16; c += 64) {
    uint64_t a = A0 + (uint64_t)c * 16;
    uint4 v = (a + 16 <= blob_len) ? *reinterpret_cast<const uint4*>(blob + a)
                                   : gload_u128_tail(blob, blob_len, a);
    reinterpret_cast<uint4*>(region)[c] = v;
  }
  if (lane < 8) region[HB_REGION / 4 + lane] = 0;
}

// Slow, general header parse (varints up to 10 bytes, values up to 8 bytes); the reference
// encoder never needs it (1-2 byte headers, <= 4-byte values). Loops are kept rolled.
__device__ inline void hb_parse_slow(const uint32_t* region, uint32_t ridx, uint32_t q,
                                     uint32_t slen, int w, uint32_t& nxt, uint32_t& cnt,
                                     uint32_t& inf, uint32_t& flg) {
  uint64_t ind = 0;
  int vlen = 0;
  bool complete = false;
#pragma unroll 1
  for (int k = 0; k < 10; ++k) {
    if (q + (uint32_t)k >= slen) break;
    uint32_t b = lbyte(region, ridx + k);
    ind |= (uint64_t)(b & 0x7Fu) << (7 * k);
    vlen = k + 1;
    if (!(b & 0x80u)) {
      complete = true;
      break;
    }
  }
  nxt = 0xFFFFFFFFu;
  cnt = 0;
  inf = 0;
  if (!complete) {  // bit_util.rs:564-580: 11th byte -> assert; end of data -> None
    flg = (vlen == 10 && q + 10 < slen) ? HF_PANIC : HF_EOF;
    return;
  }
  uint32_t p = q + (uint32_t)vlen;
  if (ind & 1) {
    cnt = (uint32_t)((uint64_t)((int64_t)ind >> 1) * 8ull);
    inf = p;
    uint64_t nx = (uint64_t)p + (((uint64_t)cnt * (uint64_t)w) >> 3);
    nxt = nx > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)nx;
    flg = HF_BP;
  } else {
    cnt = (uint32_t)((int64_t)ind >> 1);
    uint32_t vb = ((uint32_t)w + 7u) >> 3;
    if (vb > 8 || (uint64_t)p + vb > slen) {
      flg = HF_PANIC;
      return;
    }
    uint64_t v = 0;
#pragma unroll 1
    for (uint32_t k = 0; k < vb; ++k) v |= (uint64_t)lbyte(region, ridx + (uint32_t)vlen + k) << (8 * k);
    inf = v > 0x7FFFFFFFull ? 0x7FFFFFFFu : (uint32_t)v;
    nxt = p + vb;
    flg = 0;
  }
}

// Header at stream position q: 16-byte LDS read + branchless LEB128 decode for varints of
// <= 8 bytes and RLE values that end within the first 9 bytes; everything else takes the
// slow path. (rle.rs:490-508, bit_util.rs:538-580)
__device__ inline void hb_parse(const uint32_t* region, uint32_t ridx, uint32_t q, uint32_t slen,
                                int w, uint32_t& nxt, uint32_t& cnt, uint32_t& inf,
                                uint32_t& flg) {
  const uint32_t a8 = ridx & ~7u;
  const uint64_t* r64 = reinterpret_cast<const uint64_t*>(region);
  uint64_t lo = r64[a8 >> 3], hi = r64[(a8 >> 3) + 1];
  const uint32_t sh = (ridx & 7u) * 8u;
  if (sh) {
    lo = (lo >> sh) | (hi << (64 - sh));
    hi >>= sh;
  }
  const uint32_t avail = q < slen ? slen - q : 0u;  // stream bytes from q
  const uint64_t t = ~lo & 0x8080808080808080ull;
  const uint32_t vb = ((uint32_t)w + 7u) >> 3;
  const uint32_t vlen = t ? ((uint32_t)__builtin_ctzll(t) >> 3) + 1u : 9u;
  uint64_t y = lo & 0x7F7F7F7F7F7F7F7Full;
  if (vlen < 8) y &= (1ull << (8 * vlen)) - 1ull;
  y = (y & 0x007F007F007F007Full) | ((y & 0x7F007F007F007F00ull) >> 1);
  y = (y & 0x00003FFF00003FFFull) | ((y & 0x3FFF00003FFF0000ull) >> 2);
  const uint64_t ind = (y & 0x000000000FFFFFFFull) | ((y & 0x0FFFFFFF00000000ull) >> 4);
  const uint32_t p = q + vlen;
  const bool bp = (ind & 1) != 0;
  // value bytes [vlen, vlen+vb) of the 16-byte window
  const uint32_t vs = vlen * 8u;
  uint64_t v = (vs < 64) ? ((lo >> vs) | (vs ? (hi << (64 - vs)) : 0ull)) : hi;
  if (vb < 8) v &= (1ull << (8 * vb)) - 1ull;
  // fast path: stream long enough, varint <= 8 bytes, RLE value inside the 16-byte window
  const bool fast = t != 0 && vlen + (bp ? 0u : vb) <= avail && (bp || (vb <= 8 && vlen + vb <= 9));
  if (fast) {
    if (bp) {
      cnt = (uint32_t)((ind >> 1) * 8ull);
      inf = p;
      const uint64_t nx = (uint64_t)p + (((uint64_t)cnt * (uint64_t)w) >> 3);
      nxt = nx > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)nx;
      flg = HF_BP;
    } else {
      cnt = (uint32_t)(ind >> 1);
      inf = v > 0x7FFFFFFFull ? 0x7FFFFFFFu : (uint32_t)v;
      nxt = p + vb;
      flg = 0;
    }
  } else {
    hb_parse_slow(region, ridx, q, slen, w, nxt, cnt, inf, flg);
  }
}

// Walk one batch (wave 0 only, all 64 lanes). Uniform state is passed by reference.
struct HbStats {
  uint64_t walk_cyc = 0, exp_cyc = 0, bar_cyc = 0, load_cyc = 0;
  uint64_t hops = 0, windows = 0, loads = 0, batches = 0, tiles = 0;
};

__device__ inline void hb_walk(const uint8_t* blob, uint64_t blob_len, uint64_t S, uint32_t slen,
                               int w, uint32_t n, HybridSmem& sm, int slot, int avoid_buf,
                               uint32_t& cur, uint32_t& produced, uint64_t& A0, int& buf,
                               bool& loaded, uint32_t lane, HbStats& hs, bool stamps) {
  HbBatch b;
  b.seg_start = produced;
  b.err = 0;
  b.done = 0;
  uint32_t nruns = 0;
  if (produced >= n) {
    b.done = 1;
  } else {
    if (!loaded || S + cur - A0 >= (uint64_t)HB_BLK) {
      uint64_t t0 = stamps ? hb_clock() : 0;
      buf = (avoid_buf < 0) ? 0 : (avoid_buf ^ 1);
      A0 = (S + cur) & ~15ull;
      hb_load_region(blob, blob_len, A0, sm.region[buf], lane);
      loaded = true;
      __builtin_amdgcn_s_waitcnt(0);  // region stores visible to this wave's LDS reads
      __builtin_amdgcn_wave_barrier();
      if (stamps) {
        hs.load_cyc += hb_clock() - t0;
        hs.loads++;
      }
    }
    const uint32_t* region = sm.region[buf];
    uint32_t v_nxt = 0, v_cnt = 0, v_inf = 0, v_flg = 0;
    bool have_win = false;
    uint32_t wbase = 0;
    while (true) {
      if (produced >= n) {
        b.done = 1;
        break;
      }
      if (cur >= slen) {
        b.err = ST_EOF;  // reload() finds no more data: the reference stalls (A.4)
        break;
      }
      if (S + cur - A0 >= (uint64_t)HB_BLK) break;  // next batch, next region
      if (nruns >= HB_RUNCAP) break;
      if (!have_win || cur - wbase >= 64u) {
        wbase = cur;
        have_win = true;
        const uint32_t q = wbase + lane;
        const uint32_t ridx = (uint32_t)(S + q - A0);
        hb_parse(region, ridx, q, slen, w, v_nxt, v_cnt, v_inf, v_flg);
        if (stamps) hs.windows++;
      }
      const int l = (int)(cur - wbase);
      const uint32_t nxt = readlane_u(v_nxt, l);
      const uint32_t cnt = readlane_u(v_cnt, l);
      const uint32_t inf = readlane_u(v_inf, l);
      const uint32_t flg = readlane_u(v_flg, l);
      if (flg & (HF_EOF | HF_PANIC)) {
        b.err = (flg & HF_PANIC) ? ST_PANIC : ST_EOF;
        break;
      }
      if (cnt) {
        const uint32_t left = n - produced;
        const uint32_t need = cnt < left ? cnt : left;
        if (flg & HF_BP) {
          if (w > 32) {  // BitReader::get_batch asserts num_bits <= 32
            b.err = ST_PANIC;
            break;
          }
          if ((uint64_t)inf * 8ull + (uint64_t)need * (uint64_t)w > (uint64_t)slen * 8ull) {
            b.err = ST_EOF;  // truncated bit-packed run: the reference spins (A.4)
            break;
          }
        }
        if (lane == 0) {
          sm.start[slot][nruns] = produced;
          sm.info[slot][nruns] = (flg & HF_BP) ? inf : (HB_RLE | inf);
        }
        nruns++;
        produced += need;
      }
      if (stamps) hs.hops++;
      cur = nxt;
    }
  }
  if (lane == 0) {
    sm.start[slot][nruns] = produced;
    b.nruns = nruns;
    b.seg_end = produced;
    b.buf = (uint32_t)buf;
    b.A0 = A0;
    sm.batch[slot] = b;
  }
}

// Expand one batch with the given waves (wave index widx of nw).
template <class Emit>
__device__ inline void hb_expand(const uint8_t* blob, uint64_t blob_len, uint64_t S, int w,
                                 uint64_t out_base, const HybridSmem& sm, int slot, int widx,
                                 int nw, uint32_t lane, Emit& emit, uint64_t& tiles) {
  const HbBatch& b = sm.batch[slot];
  const uint32_t nruns = b.nruns;
  if (nruns == 0) return;
  const uint32_t* st = sm.start[slot];
  const uint32_t* info = sm.info[slot];
  const uint32_t* region = sm.region[b.buf];
  const uint64_t A0 = b.A0;
  const uint64_t gb = out_base + b.seg_start, ge = out_base + b.seg_end;
  const uint64_t wmask = (w >= 32) ? 0xFFFFFFFFull : ((1ull << w) - 1ull);
  const uint64_t T0 = gb / HB_TILE, T1 = (ge + HB_TILE - 1) / HB_TILE;
  // one tile: 8 consecutive outputs per lane starting at g
  auto tile = [&](uint64_t g, uint32_t* vals) -> uint32_t {
    uint32_t mask = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) vals[j] = 0;
    if (!(g + 8 > gb && g < ge)) return 0;
    const uint32_t o0 = (uint32_t)((g < gb ? gb : g) - out_base);
    int lo = 0, hi = (int)nruns - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (st[mid] <= o0) lo = mid;
      else hi = mid - 1;
    }
    int r = lo;
    const uint32_t o = (uint32_t)(g - out_base);
    const uint32_t inf0 = info[r];
    const uint64_t bit0 = (uint64_t)inf0 * 8ull + (uint64_t)(o - st[r]) * (uint64_t)w;
    const uint64_t ri0 = S + (bit0 >> 3) - A0;  // LDS index of the first payload byte
    const bool one_run = g >= gb && g + 8 <= ge && o + 8 <= st[r + 1];
    const bool in_lds = (inf0 & HB_RLE) || (ri0 + (uint64_t)w + 12 <= (uint64_t)HB_REGION);
    if (one_run && in_lds) {
      // fast path: all 8 outputs in run r, payload staged in LDS
      if (inf0 & HB_RLE) {
#pragma unroll
        for (int j = 0; j < 8; ++j) vals[j] = inf0 & 0x7FFFFFFFu;
      } else if (w <= 7) {
        const uint64_t x = lload_u64(region, (uint32_t)ri0);
        const uint32_t s0 = (uint32_t)(bit0 & 7);
#pragma unroll
        for (int j = 0; j < 8; ++j) vals[j] = (uint32_t)((x >> (s0 + j * w)) & wmask);
      } else {
        const uint32_t rb = (uint32_t)(ri0 * 8ull + (bit0 & 7));  // bit index in region
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t b = rb + (uint32_t)(j * w);
          vals[j] = (uint32_t)((lload_u64(region, b >> 3) >> (b & 7)) & wmask);
        }
      }
      return 0xFFu;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t gj = g + (uint64_t)j;
      if (gj < gb || gj >= ge) continue;
      const uint32_t oj = (uint32_t)(gj - out_base);
      while (oj >= st[r + 1]) ++r;
      const uint32_t inf = info[r];
      if (inf & HB_RLE) {
        vals[j] = inf & 0x7FFFFFFFu;
      } else {
        const uint64_t bit = (uint64_t)inf * 8ull + (uint64_t)(oj - st[r]) * (uint64_t)w;
        const uint64_t abs = S + (bit >> 3);
        const uint64_t ri = abs - A0;
        const uint64_t x = (ri + 12 <= (uint64_t)HB_REGION) ? lload_u64(region, (uint32_t)ri)
                                                             : gload_u64(blob, blob_len, abs);
        vals[j] = (uint32_t)((x >> (bit & 7)) & wmask);
      }
      mask |= 1u << j;
    }
    return mask;
  };
  for (uint64_t t = T0 + (uint64_t)widx; t < T1; t += (uint64_t)nw) {
    uint32_t va[8];
    const uint64_t ga = t * HB_TILE + (uint64_t)lane * 8u;
    const uint32_t ma = tile(ga, va);
    if (ma) emit(ga, va, ma);
    tiles++;
  }
}

// Decode n values of stream [S, S+slen) (absolute blob offsets), bit width w. kind is
// LK_RLE (hybrid, rle.rs) or LK_BIT_PACKED (header-less, levels.rs:203-209).
// Returns 0 or a status; uniform across the workgroup.
template <class Emit>
__device__ int32_t hybrid_decode(const uint8_t* __restrict__ blob, uint64_t blob_len, uint64_t S,
                                 uint32_t slen, int w, uint32_t n, int kind, uint64_t out_base,
                                 HybridSmem& sm, Emit& emit) {
  const uint32_t lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  if (n == 0) return 0;
  if (kind == LK_BIT_PACKED) {
    if ((uint64_t)n * (uint64_t)w > (uint64_t)slen * 8ull) return ST_EOF;
    if (w > 32) return ST_PANIC;
    if (threadIdx.x == 0) {
      sm.start[0][0] = 0;
      sm.info[0][0] = 0;
      sm.start[0][1] = n;
      HbBatch b;
      b.A0 = S & ~15ull;
      b.nruns = 1;
      b.seg_start = 0;
      b.seg_end = n;
      b.buf = 0;
      b.done = 1;
      b.err = 0;
      sm.batch[0] = b;
    }
    if (wave == 0) hb_load_region(blob, blob_len, S & ~15ull, sm.region[0], lane);
    __syncthreads();
    uint64_t tiles = 0;
    hb_expand(blob, blob_len, S, w, out_base, sm, 0, wave, WG / 64, lane, emit, tiles);
    return 0;
  }
  // walker state (meaningful in wave 0)
  uint32_t cur = 0, produced = 0;
  uint64_t A0 = 0;
  int buf = 0;
  bool loaded = false;
  const uint32_t dmode = g_pqg_debug_mode;
  const bool stamps = (dmode & 4) != 0;
  HbStats hs;
  if (threadIdx.x == 0) sm.eflag = 0;
  if (wave == 0) hb_walk(blob, blob_len, S, slen, w, n, sm, 0, -1, cur, produced, A0, buf, loaded, lane, hs, stamps);
  __syncthreads();
  int32_t ret = 0;
  for (int k = 0;; ++k) {
    const int slot = k & 1;
    const uint32_t err = sm.batch[slot].err;
    const bool done = sm.batch[slot].done != 0;
    if (err) {
      ret = (int32_t)err;
      break;
    }
    uint64_t t0 = stamps ? hb_clock() : 0;
    if (wave == 0) {
      // The walker is the pipeline's serial critical path: let it win issue arbitration
      // against the expander waves sharing its SIMD (this and the other workgroups').
      if (!(dmode & 8)) __builtin_amdgcn_s_setprio(3);
      if (!done)
        hb_walk(blob, blob_len, S, slen, w, n, sm, slot ^ 1, (int)sm.batch[slot].buf, cur, produced,
                A0, buf, loaded, lane, hs, stamps);
      __builtin_amdgcn_s_setprio(0);
      if (stamps) hs.walk_cyc += hb_clock() - t0;
    } else {
      if (!(dmode & 1))
        hb_expand(blob, blob_len, S, w, out_base, sm, slot, wave - 1, WG / 64 - 1, lane, emit,
                  hs.tiles);
      if (emit.err) sm.eflag = (uint32_t)emit.err;
      if (stamps) hs.exp_cyc += hb_clock() - t0;
    }
    uint64_t t1 = stamps ? hb_clock() : 0;
    __syncthreads();
    if (stamps) {
      hs.bar_cyc += hb_clock() - t1;
      hs.batches++;
    }
    if (sm.eflag) {
      ret = (int32_t)sm.eflag;
      break;
    }
    if (done) break;
  }
  if (stamps && lane == 0) {
    if (wave == 0) {
      atomicAdd(&g_pqg_stats[0], (unsigned long long)hs.walk_cyc);
      atomicAdd(&g_pqg_stats[3], (unsigned long long)hs.bar_cyc);
      atomicAdd(&g_pqg_stats[4], (unsigned long long)hs.batches);
      atomicAdd(&g_pqg_stats[5], (unsigned long long)hs.hops);
      atomicAdd(&g_pqg_stats[6], (unsigned long long)hs.windows);
      atomicAdd(&g_pqg_stats[7], (unsigned long long)hs.loads);
      atomicAdd(&g_pqg_stats[9], (unsigned long long)hs.load_cyc);
      atomicAdd(&g_pqg_stats[10], 1ull);
    } else if (wave == 1) {
      atomicAdd(&g_pqg_stats[1], (unsigned long long)hs.exp_cyc);
      atomicAdd(&g_pqg_stats[2], (unsigned long long)hs.bar_cyc);
      atomicAdd(&g_pqg_stats[8], (unsigned long long)hs.tiles);
    }
  }
  return ret;
}

}  // namespace pqg
