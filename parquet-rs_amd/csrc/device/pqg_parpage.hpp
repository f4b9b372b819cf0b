// pqg_parpage.hpp — fused page pass of dense hybrid streams (bit widths <= 8; rle.rs:398-487,
// levels.rs:191-233): one 256-thread workgroup per page stream decodes the stream region by
// region (FP_REG stream bytes), with no index records, tile descriptors or second pass.
//
// Per region: the parallel chain walk (pqg_runs.hpp: exits, chain, block listing) finds the
// true headers; all threads parse them, a block scan gives every run its first output, and the
// run list goes to LDS (start[] reuses the exits array); then the workgroup expands the
// region's outputs tile by tile through tx_range (pqg_texpand.hpp) out of the same staged
// bytes. The next region's bytes are loaded into registers while this one is worked on.
//
// A stream the pass does not take exactly as the reference reads it (any header outside the
// one- and two-byte forms, an error the reference reports, more than FP_CAP headers in a
// region, a stream that ends early) is left to the tiled passes (k_run_index* + k_tile_desc +
// k_texpand_*), which report errors exactly.
#pragma once
#include "pqg_texpand.hpp"

namespace pqg {

constexpr int FP_REG = 8192;
constexpr int FP_OVL = 512;  // staged bytes past the region: the payload of its last runs
constexpr int FP_CAP = 4096; // headers per region
constexpr int FP_STAGED = FP_REG + FP_OVL;
constexpr int FP_CHUNKS = FP_STAGED / 16;
constexpr int FP_PF = (FP_CHUNKS + WG - 1) / WG;

struct ParPageSmem {
  uint32_t stage[(FP_STAGED + 64) / 4];
  union {
    uint16_t E[PC<FP_REG>::ESZ];  // chain walk
    uint32_t start[FP_CAP + 2];   // run list: first output of each run (page-relative)
  };
  uint32_t info[FP_CAP + 1];      // run list: R_RLE | value, or payload stream offset
  uint16_t pos[FP_CAP];           // true headers of the region, in order (region index)
  uint64_t wsum[4];
  uint32_t wcnt[4];
  uint32_t ctl[8];
};

// Exclusive block scan of (sum, count) over the WG threads; totals in tsum / tcnt.
__device__ inline void fp_scan(ParPageSmem& sm, uint64_t& sum, uint32_t& cnt, uint64_t& tsum,
                               uint32_t& tcnt) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint64_t is = sum;
  uint32_t ic = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t ys = __shfl_up(is, d, 64);
    const uint32_t yc = __shfl_up(ic, d, 64);
    if (lane >= (uint32_t)d) {
      is += ys;
      ic += yc;
    }
  }
  if (lane == 63) {
    sm.wsum[wave] = is;
    sm.wcnt[wave] = ic;
  }
  pr_sync();
  uint64_t bs = 0;
  uint32_t bc = 0;
  tsum = 0;
  tcnt = 0;
#pragma unroll
  for (uint32_t v = 0; v < 4; ++v) {
    if (v < wave) {
      bs += sm.wsum[v];
      bc += sm.wcnt[v];
    }
    tsum += sm.wsum[v];
    tcnt += sm.wcnt[v];
  }
  sum = bs + is - sum;
  cnt = bc + ic - cnt;
}

// Decode stream s of one page with the whole workgroup. mk.make(t) builds the emitter of page
// tile t (outputs [t * RUN_TILE, + RUN_TILE)), mk.done(t, em) runs after it; a tile may be
// handed out twice (split between regions), each time for disjoint outputs. Returns false when
// the stream is left to the tiled path (its outputs may be partly written).
template <class M>
__device__ inline bool par_page(const uint8_t* __restrict__ blob, uint64_t blob_len, const Stream& s,
                                ParPageSmem& sm, M& mk) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (s.err || s.slen >= (1u << 28)) return false;
  const uint32_t n = s.n;
  if (n == 0) return true;
  const uint32_t w = (uint32_t)s.w;
  if (s.kind == LK_BIT_PACKED || w == 0 || w > 8) return false;
  const uint64_t S = s.S;
  const uint32_t slen = s.slen;
  const uint64_t G = S & ~15ull;
  const uint32_t off0 = (uint32_t)(S - G);
  const uint32_t vb = (w + 7u) >> 3;
  const uint32_t nregions = (off0 + slen + FP_REG - 1) / FP_REG;
  uint4 pf[FP_PF];
  auto fetch = [&](uint32_t r) {
    const uint64_t A0 = G + (uint64_t)r * FP_REG;
    const bool fast = A0 + FP_STAGED <= blob_len;
#pragma unroll
    for (int k = 0; k < FP_PF; ++k) {
      const uint32_t c = tid + WG * (uint32_t)k;
      if (c < (uint32_t)FP_CHUNKS)
        pf[k] = fast ? *reinterpret_cast<const uint4*>(blob + A0 + (uint64_t)c * 16)
                     : gload_u128_tail(blob, blob_len, A0 + (uint64_t)c * 16);
    }
  };
  uint32_t cur_r = 0xFFFFFFFFu, pf_r = 0xFFFFFFFFu;
  uint32_t cur = 0;       // next header (stream offset)
  uint32_t produced = 0;  // outputs before it
  while (true) {
    if (produced >= n) return true;
    if (cur >= slen) return false;  // the stream ends early: the tiled path reports it
    const uint32_t r = (off0 + cur) / FP_REG;
    const uint32_t rbase = r * FP_REG - off0;  // stream offset of region byte 0 (mod 2^32)
    if (r != cur_r) {
      if (r != pf_r) fetch(r);
#pragma unroll
      for (int k = 0; k < FP_PF; ++k) {
        const uint32_t c = tid + WG * (uint32_t)k;
        if (c < (uint32_t)FP_CHUNKS) reinterpret_cast<uint4*>(sm.stage)[c] = pf[k];
      }
      cur_r = r;
      pf_r = 0xFFFFFFFFu;
      if (r + 1 < nregions) {
        fetch(r + 1);
        pf_r = r + 1;
      }
      pr_sync();
    }
    pc_exits<FP_REG>(sm.stage, sm.E, r, rbase, off0, slen, w, vb);
    // ---- chain and listing (wave 0)
    if (wave == 0) {
      uint32_t kind, at;
      const uint32_t bent = pc_chain<FP_REG>(sm.E, cur - rbase, rbase, slen, kind, at);
      uint32_t c = 0;
      if (kind == 0) pc_walk<FP_REG>(sm.stage, bent, 0xFFFFFFFFu, rbase, slen, w, vb, [&](uint32_t) { ++c; });
      uint32_t incl = c;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= (uint32_t)d) incl += y;
      }
      const uint32_t H = rfl(__shfl(incl, 63, 64));
      const bool ok = kind == 0 && H <= (uint32_t)FP_CAP;
      if (ok) {
        uint32_t base = incl - c;
        pc_walk<FP_REG>(sm.stage, bent, 0xFFFFFFFFu, rbase, slen, w, vb,
                        [&](uint32_t p) { sm.pos[base++] = (uint16_t)p; });
      }
      if (lane == 0) {
        sm.ctl[0] = ok ? 1u : 0u;
        sm.ctl[1] = H;
        sm.ctl[2] = at;
      }
    }
    pr_sync();
    if (!sm.ctl[0]) return false;
    const uint32_t H = sm.ctl[1], nxt = sm.ctl[2];
    // ---- run list (all threads; E is dead, start[] takes its place)
    const uint32_t K = (H + WG - 1) / WG, h0 = tid * K, h1 = h0 + K < H ? h0 + K : H;
    uint64_t sum = 0;
    uint32_t nv = 0, bad = 0;
    for (uint32_t h = h0; h < h1; ++h) {
      const uint32_t q = sm.pos[h];
      uint32_t nx, cnt, inf, flg;
      run_parse(sm.stage, q, rbase + q, slen, (int)w, nx, cnt, inf, flg);
      sum += cnt;
      nv += cnt ? 1u : 0u;
      bad |= flg & (RF_EOF | RF_PANIC);
    }
    uint64_t tsum;
    uint32_t tcnt;
    fp_scan(sm, sum, nv, tsum, tcnt);
    uint64_t before = (uint64_t)produced + sum;
    uint32_t vi = nv, nw = 0;
    for (uint32_t h = h0; h < h1; ++h) {
      const uint32_t q = sm.pos[h];
      uint32_t nx, cnt, inf, flg;
      run_parse(sm.stage, q, rbase + q, slen, (int)w, nx, cnt, inf, flg);
      if (cnt && before < n) {
        const uint32_t need = (uint64_t)cnt < n - before ? cnt : (uint32_t)(n - before);
        const bool bp = (flg & RF_BP) != 0;
        if (bp && (uint64_t)inf * 8ull + (uint64_t)need * w > (uint64_t)slen * 8ull) bad = 1;  // truncated
        sm.start[vi] = (uint32_t)before;
        sm.info[vi] = bp ? inf : (R_RLE | (inf > 0x7FFFFFFFu ? 0x7FFFFFFFu : inf));
        ++nw;
      }
      vi += cnt ? 1u : 0u;
      before += cnt;
    }
    const uint64_t bn = __ballot(bad != 0);
    uint32_t nwt = nw;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) nwt += __shfl_down(nwt, off, 64);
    if (lane == 0) {
      sm.wcnt[wave] = nwt;
      sm.wsum[wave] = bn ? 1ull : 0ull;
    }
    pr_sync();
    const uint32_t nr = sm.wcnt[0] + sm.wcnt[1] + sm.wcnt[2] + sm.wcnt[3];
    if (sm.wsum[0] | sm.wsum[1] | sm.wsum[2] | sm.wsum[3]) return false;
    const uint64_t pe = (uint64_t)produced + tsum;
    const uint32_t pend = pe < n ? (uint32_t)pe : n;
    if (tid == 0) {
      sm.start[nr] = pend;
      sm.start[nr + 1] = pend;
    }
    pr_sync();
    // ---- expand the region's outputs [produced, pend), tile by tile of the page's tile grid
    if (nr) {
      for (uint32_t t = produced / RUN_TILE; t * RUN_TILE < pend; ++t) {
        const uint32_t lo = t * RUN_TILE;
        const uint32_t sl = lo > produced ? lo : produced;
        const uint32_t sh = lo + RUN_TILE < pend ? lo + RUN_TILE : pend;
        auto em = mk.make(t);
        tx_range(sm, nr, lo, sl, sh, w, rbase, (uint32_t)FP_STAGED, false, blob, blob_len, S, em);
        mk.done(t, em);
      }
    }
    pr_sync();  // stage and run list are rewritten for the next region
    produced = pend;
    cur = nxt;
  }
}

}  // namespace pqg
