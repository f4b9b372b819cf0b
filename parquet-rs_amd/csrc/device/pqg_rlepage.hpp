// pqg_rlepage.hpp — page pass of the RLE/bit-packing hybrid decoder (rle.rs:398-487): one
// 256-thread workgroup per page stream decodes the stream tile by tile (RUN_TILE outputs), so
// the header chain is walked once, by the workgroup that expands it, with no index pass, tile
// descriptors or run tables in HBM.
//
// Per tile: the staged window (12 KiB from the payload of the tile's first output, loaded into
// registers while the previous tile was expanded) goes to LDS; wave 0 follows the header chain
// from the run in progress (one-byte headers: an LDS byte read and a few scalar ops per hop;
// any other form: run_parse), then its lanes parse up to 64 of those headers at once, prefix-sum
// their output counts, check them as run_index does and write the tile's run list; all four
// waves expand the tile through tx_range (pqg_texpand.hpp) into the stream's emitter. A stream
// the pass cannot finish (an error the reference reports, a header outside the window, more
// than TX_RCAP runs in a tile, streams of 256 MiB and more) is flagged for the tiled path
// (k_run_index + k_tile_desc + k_texpand_*), which reports errors exactly.
#pragma once
#include "pqg_texpand.hpp"

namespace pqg {

constexpr int RP_CH = TX_STAGE / 16 / WG;  // 16-byte loads per thread per tile

// Run in progress between tiles: outputs [first, end) (page-relative), info as in the run
// list, and the header of the run after it.
struct RpCarry {
  uint32_t first, end, info, next;
};

// Wave 0: the runs producing outputs [lo, hi) into sm.start/info[0, nr) (the carried run
// first), from the window of staged bytes at stream offset sb32. False: leave the stream to the
// tiled path. On success c is the last run listed and the header after it.
__device__ inline bool rp_walk(TileSmem& sm, uint32_t sb32, uint32_t slen, uint32_t n, uint32_t w,
                               uint32_t lo, uint32_t hi, RpCarry& c, uint32_t& nr) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lanes_below = (1ull << lane) - 1ull;
  const uint32_t vb = (w + 7u) >> 3;
  nr = 0;
  if (c.end > lo) {  // the run in progress covers the tile's first output
    if (lane == 0) {
      sm.start[0] = c.first;
      sm.info[0] = c.info;
    }
    nr = 1;
  }
  uint32_t produced = c.end, cur = c.next;
  while (produced < hi) {
    // ---- chain: up to 64 header positions (uniform)
    uint32_t posv = 0, k = 0, acc = produced;
    while (k < 64u && acc < hi) {
      if (cur >= slen) return false;  // the reference stalls at the end of the data
      const uint32_t rel = cur - sb32;
      if (rel + 24u > (uint32_t)TX_STAGE) return false;
      const uint32_t b0 = rfl(lbyte(sm.stage, rel));
      uint32_t cnt, nxt;
      if (!(b0 & 0x80u) && vb <= 3u) {
        const uint32_t half = b0 >> 1;
        cnt = (b0 & 1u) ? half << 3 : half;
        nxt = cur + 1u + ((b0 & 1u) ? half * w : vb);
      } else {
        uint32_t inf, flg;
        run_parse(sm.stage, rel, cur, slen, (int)w, nxt, cnt, inf, flg);
        if (rfl(flg) & (RF_EOF | RF_PANIC)) return false;
        nxt = rfl(nxt);
        cnt = rfl(cnt);
      }
      posv = lane == k ? cur : posv;
      ++k;
      acc += cnt < n - acc ? cnt : n - acc;
      cur = nxt;
    }
    // ---- lanes parse the k headers, count, check and list them
    const bool in = lane < k;
    uint32_t nx, cnt = 0, inf = 0, flg = 0;
    if (in) run_parse(sm.stage, posv - sb32, posv, slen, (int)w, nx, cnt, inf, flg);
    uint64_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t y = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += y;
    }
    const uint64_t before = (uint64_t)produced + incl - cnt;
    const uint32_t need = before >= n ? 0u : (uint32_t)((uint64_t)cnt < n - before ? cnt : n - before);
    const bool bp = (flg & RF_BP) != 0;
    bool bad = false;
    if (in && need && bp && (w > 32u || (uint64_t)inf * 8ull + (uint64_t)need * w > (uint64_t)slen * 8ull))
      bad = true;  // the reference panics / spins on such a run
    if (__ballot(bad)) return false;
    const bool valid = in && need > 0;
    const uint64_t V = __ballot(valid);
    const uint32_t idx = nr + (uint32_t)__builtin_popcountll(V & lanes_below);
    const uint32_t nv = (uint32_t)__builtin_popcountll(V);
    if (nr + nv > (uint32_t)TX_RCAP) return false;
    if (valid) {
      sm.start[idx] = (uint32_t)before;
      sm.info[idx] = bp ? inf : (R_RLE | (inf > 0x7FFFFFFFu ? 0x7FFFFFFFu : inf));
    }
    nr += nv;
    if (V) {
      const int L = 63 - __builtin_clzll(V);
      c.first = rfl(__shfl((uint32_t)before, L, 64));
      c.end = c.first + rfl(__shfl(need, L, 64));
      c.info = rfl(__shfl(bp ? inf : (R_RLE | (inf > 0x7FFFFFFFu ? 0x7FFFFFFFu : inf)), L, 64));
      produced = c.end;
    }
    c.next = cur;
  }
  return true;
}

// Decode stream s of one page with the whole workgroup. mk.make(k) builds the emitter of tile
// k, mk.done(k, em) runs after it. Returns false when the stream is left to the tiled path (its
// outputs may be partly written; the tiled path rewrites them).
template <class M>
__device__ inline bool rle_page(const uint8_t* __restrict__ blob, uint64_t blob_len, const Stream& s,
                                TileSmem& sm, M& mk) {
  const uint32_t tid = threadIdx.x;
  const uint32_t n = s.n, w = (uint32_t)s.w, slen = s.slen;
  const uint64_t S = s.S;
  if (s.err || slen >= (1u << 28)) return false;
  if (n == 0) return true;
  RpCarry c{0u, 0u, 0u, 0u};
  if (s.kind == LK_BIT_PACKED) {  // one header-less run (levels.rs:203-209)
    if ((uint64_t)n * w > (uint64_t)slen * 8ull || w > 32u) return false;
    c = RpCarry{0u, n, 0u, slen};
  }
  uint4 pv[RP_CH];
  auto issue = [&](uint64_t base) {
    const bool fast = base + TX_STAGE <= blob_len;
#pragma unroll
    for (int k = 0; k < RP_CH; ++k) {
      const uint64_t a = base + (uint64_t)(tid + k * WG) * 16;
      pv[k] = fast ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
    }
  };
  uint64_t SB = S & ~15ull;
  issue(SB);
  const uint32_t ntl = (n + RUN_TILE - 1) / RUN_TILE;
  for (uint32_t k = 0; k < ntl; ++k) {
    const uint32_t lo = k * RUN_TILE;
    const uint32_t hi = lo + RUN_TILE < n ? lo + RUN_TILE : n;
#pragma unroll
    for (int j = 0; j < RP_CH; ++j) reinterpret_cast<uint4*>(sm.stage)[tid + j * WG] = pv[j];
    if (tid < 16) sm.stage[TX_STAGE / 4 + tid] = 0;
    __syncthreads();
    const uint32_t sb32 = (uint32_t)(SB - S);
    if (tid < 64) {
      uint32_t nr = 0;
      const bool ok = rp_walk(sm, sb32, slen, n, w, lo, hi, c, nr);
      if (tid == 0) {
        sm.ctl[0] = ok ? 1u : 0u;
        sm.ctl[1] = nr;
        sm.start[nr] = hi;
        sm.start[nr + 1] = hi;
        // next window: from the payload of output hi in the carried bit-packed run, else from
        // the next header
        uint64_t nsb = c.next;
        if (c.end > hi && !(c.info & R_RLE)) nsb = (uint64_t)c.info + (((uint64_t)(hi - c.first) * w) >> 3);
        sm.ctl[2] = (uint32_t)nsb;
      }
    }
    __syncthreads();
    if (!sm.ctl[0]) return false;
    const uint32_t nr = sm.ctl[1];
    const uint64_t SBn = (S + sm.ctl[2]) & ~15ull;
    if (k + 1 < ntl) issue(SBn);
    auto em = mk.make(k);
    tx_range(sm, nr, lo, lo, hi, w, sb32, (uint32_t)TX_STAGE, false, blob, blob_len, S, em);
    mk.done(k, em);
    __syncthreads();
    SB = SBn;
  }
  return true;
}

}  // namespace pqg
