// pqg_delta.hip — DELTA_BINARY_PACKED values (decoding.rs:392-619) of the INT32 / INT64 chunks of
// a decode (each kernel is instantiated per value size ES and takes the pages of chunks of that
// size), output to each page's chunk buffer.
#include "pqg_delta.hpp"

// =============================================================================== tiled path
//
// DELTA_BINARY_PACKED over the whole chunk at once (BASELINE config 4):
//   k_delta_index  one wave per page walks the block headers (zigzag min_delta + mini-block
//                  widths, decoding.rs:448-468) over 8 KiB regions prefetched one ahead,
//                  checks everything the reference checks, and gives every tile of
//                  DELTA_TILE values the records of the blocks its values need (with their
//                  mini-block widths);
//   k_delta_sums   one 256-thread workgroup per tile: 16 deltas per thread unpacked from an
//                  LDS-staged window, summed (min_delta + delta, wrapping);
//   k_delta_tscan  per page, the running value at each tile start (value_i = first + sum of
//                  min_delta + delta over d < i, wrapping, decoding.rs:560-566);
//   k_delta_expand the same unpack, a workgroup scan from the tile's start value, and stores
//                  through an LDS transpose (1 KiB of contiguous output per store instruction).
// No workgroup waits on another (no look-back), so no dispatch-order assumption is needed.
// Pages with more than DELTA_MBMAX mini-blocks per block, or a tile needing more than
// DELTA_BCAP blocks, fall back to k_delta above.
#include "pqg_runs.hpp"

namespace pqg {

// DeltaPage::tiled values set by k_delta_page (0 / 1 are the tiled path's own)
constexpr uint32_t DP_DONE = 2u, DP_FALLBACK = 3u;

__device__ inline uint32_t rfl32(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// zigzag/ULEB128 from a wave-uniform 16-byte window (lo, hi): returns bytes used, 0 when the
// stream ends first, -1 for > 10 bytes (get_vlq_int assert).
__device__ inline int vlq16(uint64_t lo, uint64_t hi, uint32_t avail, uint64_t& v) {
  v = 0;
#pragma unroll 1
  for (int k = 0; k < 10; ++k) {
    if ((uint32_t)k >= avail) return 0;
    const uint32_t b = (uint32_t)((k < 8 ? (lo >> (8 * k)) : (hi >> (8 * (k - 8)))) & 0xFF);
    v |= (uint64_t)(b & 0x7F) << (7 * k);
    if (!(b & 0x80)) return k + 1;
  }
  return avail > 10 ? -1 : 0;
}

template <int ES>
__global__ void __launch_bounds__(64) k_delta_index(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                    PageWork* pages, ChunkWork* chunks, DeltaTables dt) {
  __shared__ IndexSmem sm;
  const int p = blockIdx.x;
  const PageWork pw = pages[p];
  const uint32_t lane = threadIdx.x & 63;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  if (pw.encoding != E_DELTA_BINARY_PACKED || chunks[pw.chunk].es != ES) return;
  if (dt.page[p].tiled == DP_DONE) return;  // decoded by k_delta_page
  DeltaPage info{0, 0, 0, 0, 0};
  if (pw.status != 0) {
    if (lane == 0) dt.page[p] = info;
    return;
  }
  const uint64_t S = pw.base + pw.val_off;
  const uint32_t slen = pw.val_bytes;
  const uint8_t* sp = blob + S;
  // ---- stream header (decoding.rs:501-533), parsed by every lane
  uint64_t block_size, nmb, total, fz;
  uint32_t q = 0;
  int32_t err = 0;
  int l;
  if ((l = g_vlq(sp, q, slen, block_size)) <= 0) err = l ? ST_PANIC : ST_EOF;
  q += l > 0 ? l : 0;
  if (!err && (l = g_vlq(sp, q, slen, nmb)) <= 0) err = l ? ST_PANIC : ST_EOF;
  q += l > 0 ? l : 0;
  if (!err && (l = g_vlq(sp, q, slen, total)) <= 0) err = l ? ST_PANIC : ST_EOF;
  q += l > 0 ? l : 0;
  if (!err && (l = g_vlq(sp, q, slen, fz)) <= 0) err = l ? ST_PANIC : ST_EOF;
  q += l > 0 ? l : 0;
  uint64_t vpmb = 0;
  if (!err) {
    if ((int64_t)nmb <= 0) err = ST_PANIC;
    else {
      vpmb = (uint64_t)((int64_t)block_size / (int64_t)nmb);
      if (vpmb % 8 != 0) err = ST_PANIC;
    }
  }
  const uint64_t n = pw.nonnull;
  if (!err && total < n) err = ST_EOF;  // the reference returns a short batch here
  if (!err && n > 1 && vpmb == 0) err = ST_HANG;
  if (err) {
    if (lane == 0) {
      dt.page[p] = info;
      report(pages, chunks, p, err);
    }
    return;
  }
  info.first = (uint64_t)unzigzag(fz);
  info.vpmb = (uint32_t)vpmb;
  info.nmb = (uint32_t)nmb;
  if (nmb > DELTA_MBMAX || vpmb > 0xFFFFFFu) {  // per-page kernel
    if (lane == 0) dt.page[p] = info;
    return;
  }
  const uint32_t need = n > 0 ? (uint32_t)(n - 1) : 0u;  // deltas to decode
  const uint32_t vpb = (uint32_t)(vpmb * nmb);
  const uint32_t wmax = ES == 4 ? 32u : 64u;
  const uint32_t nblocks = vpb ? (need + vpb - 1) / vpb : 0u;
  const uint32_t nmb32 = (uint32_t)nmb, vpmb32 = (uint32_t)vpmb;
  DeltaBlock* const tb = dt.blocks + (uint64_t)pw.ltile0 * DELTA_BCAP;
  // ---- block walk: a scalar hop loop follows up to 64 block headers (varint length and the
  // sum of the mini-block widths give the next header), then the 64 lanes decode, check and
  // record those blocks in parallel
  const uint64_t G = S & ~15ull;
  const uint32_t off0 = (uint32_t)(S - G);
  const uint32_t nregions = (off0 + slen + IX_REG - 1) / IX_REG;
  uint4 pf[IX_PF];
  uint32_t cur_r = 0xFFFFFFFFu, pf_r = 0xFFFFFFFFu;
  uint32_t cur = q, b = 0;
  bool overflow = false;
  while (b < nblocks) {
    if (cur >= slen) {  // "Not enough data to decode 'min_delta'"
      err = ST_EOF;
      break;
    }
    const uint32_t r = (off0 + cur) / IX_REG;
    if (r != cur_r) {
      if (r != pf_r) ix_fetch(blob, blob_len, G + (uint64_t)r * IX_REG, lane, pf);
      ix_install(sm.region, lane, pf);
      cur_r = r;
      pf_r = 0xFFFFFFFFu;
      if (r + 1 < nregions) {
        ix_fetch(blob, blob_len, G + (uint64_t)(r + 1) * IX_REG, lane, pf);
        pf_r = r + 1;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
    const uint32_t rbase = r * IX_REG - off0;  // stream offset of region byte 0
    uint32_t posv = 0, k = 0;
    while (k < 64 && b + k < nblocks) {
      if (cur >= slen || cur - rbase >= (uint32_t)IX_REG) break;  // 64-byte overlap holds the header
      const uint32_t rel = cur - rbase;
      const uint64_t w0 = lload_u64(sm.region, rel);
      const uint32_t x0 = rfl32((uint32_t)w0), x1 = rfl32((uint32_t)(w0 >> 32));
      const uint64_t lo = ((uint64_t)x1 << 32) | x0;
      const uint64_t t8 = ~lo & 0x8080808080808080ull;
      posv = lane == k ? cur : posv;
      ++k;
      if (!t8 || nmb32 > 8) break;  // long varint / many widths: the batch finishes this block
      const uint32_t vl = ((uint32_t)__builtin_ctzll(t8) >> 3) + 1u;
      const uint64_t w1 = lload_u64(sm.region, rel + vl);
      const uint64_t wy = ((uint64_t)rfl32((uint32_t)(w1 >> 32)) << 32) | rfl32((uint32_t)w1);
      const uint64_t y = nmb32 >= 8 ? wy : (wy & ((1ull << (8 * nmb32)) - 1ull));
      uint64_t s16 = (y & 0x00FF00FF00FF00FFull) + ((y >> 8) & 0x00FF00FF00FF00FFull);
      const uint32_t sumw = (uint32_t)((s16 * 0x0001000100010001ull) >> 48);
      cur = cur + vl + nmb32 + (vpmb32 >> 3) * sumw;
    }
    // ---- batch: lane j = block b + j
    const bool in = lane < k;
    const uint32_t bb = b + lane;
    int32_t e = 0;
    uint64_t zz = 0;
    uint32_t vl = 0, wpos = 0, payload = 0, nxt = 0;
    if (in) {
      const uint32_t pos = posv;
      if (pos >= slen) e = ST_EOF;  // "Not enough data to decode 'min_delta'"
      else {
        const uint32_t rel = pos - rbase;
        const uint64_t lo = lload_u64(sm.region, rel), hi = lload_u64(sm.region, rel + 8);
        const int l = vlq16(lo, hi, slen - pos, zz);
        if (l <= 0) e = l ? ST_PANIC : ST_EOF;
        else if ((uint64_t)pos + l + nmb32 > slen) e = ST_EOF;  // "... 'width'"
        else {
          vl = (uint32_t)l;
          wpos = pos + vl;
          payload = wpos + nmb32;
          const uint32_t left = need - bb * vpb;
          const uint32_t inblk = left < vpb ? left : vpb;
          const uint32_t mneed = (inblk + vpmb32 - 1) / vpmb32;
          uint64_t boff = 0;
          for (uint32_t m = 0; m < nmb32; ++m) {
            const uint32_t wdt = lbyte(sm.region, rel + vl + m);
            if (m < mneed && !e) {
              if (wdt > wmax) e = ST_PANIC;  // get_batch / get_value assert on num_bits
              else if ((uint64_t)payload + boff + (vpmb * wdt) / 8 > slen)
                e = (ES == 4) ? ST_PANIC : ST_EOF;  // the whole mini-block is loaded
            }
            boff += (vpmb * wdt) / 8;
          }
          const uint64_t nx = (uint64_t)payload + boff;
          nxt = nx > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)nx;
        }
      }
    }
    const uint64_t emask = __ballot(e != 0);
    if (emask) {
      err = __shfl(e, __builtin_ctzll(emask), 64);
      break;
    }
    if (in) {  // records for the tiles of values whose deltas fall in this block
      const uint32_t d0 = bb * vpb;
      const uint32_t left = need - d0;
      const uint32_t d1 = d0 + (left < vpb ? left : vpb);
      DeltaBlock rec{wpos, payload, (uint64_t)unzigzag(zz), {}};
      {
        const uint32_t rel = posv - rbase + vl;
#pragma unroll
        for (uint32_t m = 0; m < DELTA_MBMAX; ++m) rec.w[m] = m < nmb32 ? (uint8_t)lbyte(sm.region, rel + m) : 0;
      }
      for (uint32_t t = (d0 + 1) / DELTA_TILE; t <= d1 / DELTA_TILE; ++t) {
        const uint32_t vlo = t * DELTA_TILE;
        const uint32_t slot = bb - (vlo > 0 ? vlo - 1 : 0) / vpb;
        if (slot >= DELTA_BCAP) overflow = true;
        else tb[(uint64_t)t * DELTA_BCAP + slot] = rec;
      }
    }
    overflow = __ballot(overflow) != 0;
    // the last block of the batch decides where the next batch starts
    cur = __shfl(nxt, (int)k - 1, 64);
    b += k;
  }
  if (err) {
    if (lane == 0) {
      dt.page[p] = info;
      report(pages, chunks, p, err);
    }
    return;
  }
  info.tiled = overflow ? 0u : 1u;
  if (lane == 0) dt.page[p] = info;
}


constexpr int DX_STAGE = 10240;                        // staged payload bytes per tile
constexpr int DX_OUTB = DELTA_TILE / 2 * 8;            // half a tile of 8-byte values (16 KiB)
constexpr int DX_UNION = DX_OUTB > DX_STAGE + 64 ? DX_OUTB : DX_STAGE + 64;

struct DeltaExpandSmem {
  union {
    uint32_t stage[DX_UNION / 4];   // payload window, then the transposed output halves
    uint4 outq[DX_UNION / 16];
  };
  uint64_t mind[DELTA_BCAP];
  uint32_t pos[DELTA_BCAP];         // block payload offsets (stream-relative)
  uint32_t mboff[DELTA_BCAP][DELTA_MBMAX];  // byte offset of mini-block m from pos
  uint8_t mbw[DELTA_BCAP][DELTA_MBMAX];
  uint64_t wsum[WG / 64];
  uint64_t prefix;
};

// Front of the DELTA_BINARY_PACKED tile passes (decoding.rs:535-566): tile t's block records
// (with their mini-block widths, round trip 1) and payload window (round trip 2), then 16
// consecutive deltas per thread into x (mini-block parameters hoisted, one 32-bit funnel shift
// per delta for widths <= 32) and their wrapping sum into s. False: nothing to do for tile t.
template <int ES>
__device__ inline bool delta_tile_front(DeltaExpandSmem& sm, const uint8_t* __restrict__ blob,
                                        uint64_t blob_len, PageWork* pages, const ChunkWork* chunks,
                                        const uint32_t* __restrict__ tile_page, uint32_t ntiles,
                                        const DeltaTables& dt, uint32_t t, int& p, DeltaPage& info,
                                        uint32_t& lo, uint32_t& hi, uint64_t (&x)[DPT], uint64_t& s) {
  const int tid = threadIdx.x;
  if (t >= ntiles) return false;
  p = (int)tile_page[t];
  const PageWork& pw = pages[p];
  if (pw.status != 0 || pw.encoding != E_DELTA_BINARY_PACKED || chunks[pw.chunk].es != ES) return false;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return false;
  info = dt.page[p];
  if (info.tiled != 1u) return false;
  const uint32_t n = (uint32_t)pw.nonnull;
  const uint32_t k = t - pw.ltile0;
  lo = k * DELTA_TILE;
  if (lo >= n) return false;
  hi = lo + DELTA_TILE < n ? lo + DELTA_TILE : n;
  const uint64_t S = pw.base + pw.val_off;
  const uint32_t vpmb = info.vpmb, nmb = info.nmb, vpb = vpmb * nmb;
  // deltas of the tile: d in [lo - 1, hi - 1), d >= 0
  const uint32_t dlo = lo > 0 ? lo - 1 : 0;
  const bool anyd = hi >= 2;
  const uint32_t blo = dlo / vpb;
  const uint32_t bhi = anyd ? (hi - 2) / vpb : blo;
  const uint32_t nb = bhi - blo + 1;
  const DeltaBlock* recs = dt.blocks + (uint64_t)t * DELTA_BCAP;
  // ---- block records: payload offset, min_delta, widths and mini-block offsets
  if ((uint32_t)tid < nb) {
    const uint4* rq = reinterpret_cast<const uint4*>(recs + tid);
    const uint4 r0 = rq[0], r1 = rq[1];
    sm.pos[tid] = r0.y;
    sm.mind[tid] = (uint64_t)r0.z | ((uint64_t)r0.w << 32);
    const uint32_t wv[4] = {r1.x, r1.y, r1.z, r1.w};
    uint32_t off = 0;
#pragma unroll
    for (uint32_t m = 0; m < DELTA_MBMAX; ++m) {
      const uint32_t wdt = (wv[m >> 2] >> (8 * (m & 3))) & 0xFFu;
      sm.mbw[tid][m] = (uint8_t)wdt;
      sm.mboff[tid][m] = off;
      off += m < nmb ? (vpmb * wdt) >> 3 : 0u;
    }
  }
  __syncthreads();
  // ---- payload window from the tile's first delta on
  uint64_t A0;
  {
    const uint32_t r0 = dlo - blo * vpb;
    const uint32_t m0 = r0 / vpmb;
    const uint64_t bit0 = ((uint64_t)sm.pos[0] + sm.mboff[0][m0]) * 8ull +
                          (uint64_t)(r0 - m0 * vpmb) * sm.mbw[0][m0];
    A0 = (S + (bit0 >> 3)) & ~15ull;
  }
  const uint64_t S_end = S + pw.val_bytes + 16;
  const uint64_t A1 = A0 + DX_STAGE < S_end ? A0 + DX_STAGE : S_end;
  const uint32_t nchunks = (uint32_t)((A1 - A0 + 15) / 16);
  {
    constexpr int PER = (DX_STAGE / 16 + WG - 1) / WG;
    uint4 v[PER];
    const bool fast = A0 + (uint64_t)nchunks * 16 <= blob_len;
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const uint32_t ci = (uint32_t)tid + (uint32_t)(c * WG);
      if (ci < nchunks) {
        const uint64_t a = A0 + (uint64_t)ci * 16;
        v[c] = fast ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
      }
    }
#pragma unroll
    for (int c = 0; c < PER; ++c) {
      const uint32_t ci = (uint32_t)tid + (uint32_t)(c * WG);
      if (ci < nchunks) sm.outq[ci] = v[c];
    }
    if (tid < 16) sm.stage[nchunks * 4 + tid] = 0;
  }
  const uint32_t lim = nchunks * 128u;  // staged bits
  const uint64_t sbase = A0 - S;        // stream offset of staged byte 0
  __syncthreads();
  // ---- 16 deltas per thread: values lo + 16*tid + j
  s = 0;
  const uint32_t i0 = lo + (uint32_t)tid * DPT;
  const uint32_t d0 = i0 > 0 ? i0 - 1 : 0;
  uint32_t bi = d0 / vpb - blo;
  const uint32_t rr = d0 - (bi + blo) * vpb;
  uint32_t m = rr / vpmb;
  uint32_t kk = rr - m * vpmb;
  uint32_t wdt = 0;
  int64_t base = 0;  // bit offset of the mini-block's delta 0 relative to the staged window
  uint64_t mn = 0;
  auto mb = [&]() {
    const uint32_t bs = bi < nb ? bi : 0u;
    wdt = sm.mbw[bs][m];
    base = ((int64_t)sm.pos[bs] + (int64_t)sm.mboff[bs][m] - (int64_t)sbase) * 8;
    mn = sm.mind[bs];
  };
  mb();
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    const uint32_t i = i0 + (uint32_t)j;
    x[j] = 0;
    if (i >= 1 && i < hi && bi < nb) {
      const int64_t bit = base + (int64_t)kk * wdt;
      uint64_t raw = 0;
      if (wdt) {
        if (bit >= 0 && bit + wdt <= (int64_t)lim) {
          const uint32_t b32 = (uint32_t)bit, wi = b32 >> 5;
          const uint32_t w0 = sm.stage[wi], w1 = sm.stage[wi + 1];
          if (wdt <= 32) {  // window bits [sh, sh + 32)
            const uint32_t r = __builtin_amdgcn_alignbit(w1, w0, b32 & 31u);
            raw = wdt == 32 ? r : (r & ((1u << wdt) - 1u));
          } else {          // window bits [sh, sh + 64)
            const uint32_t w2 = sm.stage[wi + 2];
            const uint64_t lo64 = ((uint64_t)__builtin_amdgcn_alignbit(w2, w1, b32 & 31u) << 32) |
                                  __builtin_amdgcn_alignbit(w1, w0, b32 & 31u);
            raw = wdt >= 64 ? lo64 : (lo64 & ((1ull << wdt) - 1ull));
          }
        } else {  // outside the staged window: global memory
          const uint64_t gb = (uint64_t)(bit + (int64_t)sbase * 8);
          const uint64_t abs = S + (gb >> 3);
          const uint32_t sh = (uint32_t)(gb & 7);
          uint64_t r = gload_u64(blob, blob_len, abs) >> sh;
          if (wdt + sh > 64) r |= gload_u64(blob, blob_len, abs + 8) << (64 - sh);
          raw = wdt >= 64 ? r : (r & ((1ull << wdt) - 1ull));
        }
      }
      x[j] = mn + raw;  // min_delta + delta (wrapping)
    }
    if (i >= 1) {  // advance to the next delta
      if (++kk == vpmb) {
        kk = 0;
        if (++m == nmb) {
          m = 0;
          ++bi;
        }
        mb();
      }
    }
    s += x[j];
  }
  return true;
}

// Tile sums: wrapping sum of min_delta + delta over each tile's deltas -> dt.agg[t].
template <int ES>
__device__ inline void delta_sums_tile(DeltaExpandSmem& sm, const uint8_t* __restrict__ blob,
                                       uint64_t blob_len, PageWork* pages, const ChunkWork* chunks,
                                       const uint32_t* __restrict__ tile_page, uint32_t ntiles,
                                       const DeltaTables& dt, uint32_t t) {
  int p;
  DeltaPage info;
  uint32_t lo, hi;
  uint64_t x[DPT], s;
  if (!delta_tile_front<ES>(sm, blob, blob_len, pages, chunks, tile_page, ntiles, dt, t, p, info, lo, hi, x, s))
    return;
  const uint64_t T = block_sum_u64(s, sm.wsum);
  if (threadIdx.x == 0) dt.agg[t] = T;
}

// Grid-stride over the tiles (the pages k_delta_page decoded are skipped inside; with none left
// for this path the kernel exits at once).
template <int ES>
__global__ void __launch_bounds__(WG) k_delta_sums(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                   PageWork* pages, const ChunkWork* chunks,
                                                   const uint32_t* __restrict__ tile_page, uint32_t ntiles,
                                                   DeltaTables dt) {
  __shared__ DeltaExpandSmem sm;
  if (*dt.nfall == 0) return;
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    delta_sums_tile<ES>(sm, blob, blob_len, pages, chunks, tile_page, ntiles, dt, t);
    __syncthreads();
  }
}

// Running value at each tile start: dt.inc[t] = first + the page's earlier tile sums (one
// workgroup per page; wrapping, as the reference's i64 adds).
__global__ void __launch_bounds__(WG) k_delta_tscan(const PageWork* pages, DeltaTables dt) {
  __shared__ uint64_t wsum[WG / 64];
  __shared__ uint64_t carry;
  const int p = blockIdx.x;
  const PageWork& pw = pages[p];
  if (pw.status != 0 || pw.encoding != E_DELTA_BINARY_PACKED) return;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  const DeltaPage info = dt.page[p];
  if (info.tiled != 1u) return;
  const uint32_t n = (uint32_t)pw.nonnull;
  const uint32_t nt = (n + DELTA_TILE - 1) / DELTA_TILE;
  if (threadIdx.x == 0) carry = info.first;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nt; b0 += WG) {
    const uint32_t i = b0 + threadIdx.x;
    const uint64_t v = i < nt ? dt.agg[pw.ltile0 + i] : 0ull;
    uint64_t incl = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint64_t y = __shfl_up(incl, off, 64);
      if ((threadIdx.x & 63) >= (unsigned)off) incl += y;
    }
    if ((threadIdx.x & 63) == 63) wsum[threadIdx.x >> 6] = incl;
    __syncthreads();
    uint64_t pre = carry;
    for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) pre += wsum[w];
    if (i < nt) dt.inc[pw.ltile0 + i] = pre + incl - v;
    __syncthreads();
    if (threadIdx.x == WG - 1) carry = pre + incl;
    __syncthreads();
  }
}

// Tile expand: running values from dt.inc[t] plus the in-tile scan, stored through an LDS
// transpose so that every store instruction writes 1 KiB of contiguous output: half h =
// threads [128h, 128h + 128) hold tile values [2048h, 2048h + 2048) and the half leaves as
// 16-byte chunks, chunk c by thread c % 256.
template <int ES>
__device__ inline void delta_expand_tile(DeltaExpandSmem& sm, const uint8_t* __restrict__ blob,
                                         uint64_t blob_len, PageWork* pages, const ChunkWork* chunks,
                                         const uint32_t* __restrict__ tile_page, uint32_t ntiles,
                                         const DeltaTables& dt, uint32_t t) {
  const int tid = threadIdx.x;
  int p;
  DeltaPage info;
  uint32_t lo, hi;
  uint64_t x[DPT], s;
  if (!delta_tile_front<ES>(sm, blob, blob_len, pages, chunks, tile_page, ntiles, dt, t, p, info, lo, hi, x, s))
    return;
  const PageWork& pw = pages[p];
  const gptr<uint8_t> __restrict__ out = gp(chunks[pw.chunk].val_out);
  // ---- workgroup scan of the thread sums
  uint64_t incl = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off, 64);
    if ((tid & 63) >= off) incl += y;
  }
  if ((tid & 63) == 63) sm.wsum[tid >> 6] = incl;
  if (tid == 0) sm.prefix = dt.inc[t];
  __syncthreads();
  uint64_t acc = sm.prefix + incl - s;
  for (int wv = 0; wv < (tid >> 6); ++wv) acc += sm.wsum[wv];
  uint64_t val[DPT];
#pragma unroll
  for (int j = 0; j < DPT; ++j) {
    acc += x[j];
    val[j] = acc;
  }
  const uint32_t cnt = hi - lo;
  const gptr<uint8_t> ob = out + (pw.value_out + lo) * (uint64_t)ES;
  constexpr uint32_t HALF = DELTA_TILE / 2;  // values per half
  constexpr uint32_t CPT = DPT * ES / 16;    // 16-byte chunks per thread
  constexpr uint32_t NCH = HALF * ES / 16;   // chunks per half
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if ((tid >> 7) == h) {
      const uint32_t tl = (uint32_t)tid & 127u;
#pragma unroll
      for (uint32_t c = 0; c < CPT; ++c) {
        uint4 q;
        if (ES == 8)
          q = make_uint4((uint32_t)val[2 * c], (uint32_t)(val[2 * c] >> 32), (uint32_t)val[2 * c + 1],
                         (uint32_t)(val[2 * c + 1] >> 32));
        else
          q = make_uint4((uint32_t)val[4 * c], (uint32_t)val[4 * c + 1], (uint32_t)val[4 * c + 2],
                         (uint32_t)val[4 * c + 3]);
        const uint32_t ci = tl * CPT + c;   // chunk within the half
        sm.outq[ci ^ (tl & 7u)] = q;        // xor swizzle against bank conflicts
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < NCH / WG; ++r) {
      const uint32_t ci = (uint32_t)tid + r * WG;
      const uint4 q = sm.outq[ci ^ ((ci / CPT) & 7u)];
      const uint32_t v0 = h * HALF + ci * (16 / ES);  // first tile value of the chunk
      gptr<uint8_t> dst = ob + (uint64_t)v0 * ES;
      if (v0 + 16 / ES <= cnt) {
        gst16(dst, q);
      } else if (v0 < cnt) {
        const uint32_t qa[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (uint32_t e = 0; e < 16 / ES; ++e) {
          if (v0 + e >= cnt) break;
          if (ES == 8) reinterpret_cast<gptr<uint64_t>>(dst)[e] = (uint64_t)qa[2 * e] | ((uint64_t)qa[2 * e + 1] << 32);
          else reinterpret_cast<gptr<uint32_t>>(dst)[e] = qa[e];
        }
      }
    }
    __syncthreads();
  }
}

template <int ES>
__global__ void __launch_bounds__(WG) k_delta_expand(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                     PageWork* pages, const ChunkWork* chunks,
                                                     const uint32_t* __restrict__ tile_page, uint32_t ntiles,
                                                     DeltaTables dt) {
  __shared__ DeltaExpandSmem sm;
  if (*dt.nfall == 0) return;
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    delta_expand_tile<ES>(sm, blob, blob_len, pages, chunks, tile_page, ntiles, dt, t);
    __syncthreads();
  }
}

// ============================================================================ page pass
//
// k_delta_page: one workgroup per page (DPG_NT threads) decodes the page's whole value stream tile
// by tile, carrying the running value in registers, so no index pass, tile sums, tile scan or
// cross-workgroup wait is needed. Tiles are DPG_NT * 16 deltas (value i = first + sum of deltas
// d < i, decoding.rs:560-566; the tile of deltas [D0, D1) yields values [D0 + 1, D1 + 1)), and
// blocks must divide the tile, so a block never spans two tiles. Per tile: wave 0 finds the
// tile's block headers by a speculative scan (dpg_headers: lane j guesses block j's offset from
// the previous tile's average block length, the wave's exclusive scan of the lengths parsed there
// checks the guesses, an exact prefix grows each round: one or two rounds for the writer's
// blocks, 512-value or 128-value alike, instead of a serial walk of 8 or 32 headers) and parses
// each block's header on its own lane (the checks of k_delta_index); every thread unpacks 16
// deltas of one mini-block (hoisted parameters, 32-bit bit offsets, one funnel shift per delta),
// the workgroup scans, adds the carry and stores through an LDS transpose (a wave's values per
// round). The next tile's bytes are loaded into registers while the current tile is expanded, as
// many as the current tile spanned plus a margin (a tile that needs more reloads the full window).
// Anything else (an error the reference reports, a header outside the staged window, more than 8
// mini-blocks, mini-blocks of a size not a multiple of 16, blocks not dividing the tile) marks the
// page DP_FALLBACK for the tiled path, which reports errors exactly.
#ifndef PQG_DPG_NT
#define PQG_DPG_NT 256
#endif
constexpr int DPG_NT = PQG_DPG_NT;  // threads per page workgroup (tile = DPG_NT * DPT deltas)

template <int NT>
struct DpgShape {
  static constexpr uint32_t T = NT * DPT;               // deltas per tile
  static constexpr int STAGE = (int)T * 3;              // staged stream bytes per tile (w <= 23 fits)
  static constexpr int CH = STAGE / 16 / NT;            // 16-byte loads per thread per tile
  static constexpr int NB = (int)T / 128;               // blocks per tile at most (blocks of >= 128 values)
  static constexpr int NW = NT / 64;                    // waves
  static_assert(NB <= 64, "one lane per block header");
  static_assert(CH * 16 * NT == STAGE, "whole loads");
};

// The stage doubles as the store transpose buffer; with PQG_DPG_OBUF it holds a whole tile of
// 8-byte values (one store round: every wave's values at once; the per-page grid leaves LDS to
// spare), else as many waves' values as the stream stage holds (measured on config 4: one store
// round 2.48 ms per step, the stage-sized rounds 2.38 ms -- off by default).
#ifndef PQG_DPG_OBUF
#define PQG_DPG_OBUF 0
#endif
template <int NT>
struct DeltaPageSmem {
  using S = DpgShape<NT>;
  static constexpr int OB = PQG_DPG_OBUF && (int)S::T * 8 > S::STAGE ? (int)S::T * 8 : S::STAGE;
  union {
    uint32_t stage[(S::STAGE + 64) / 4];
    uint4 stq[(OB + 64) / 16];
  };
  uint64_t mind[S::NB];
  uint32_t pos[S::NB];
  uint32_t mboff[S::NB][8];
  uint32_t mbw[S::NB][8];
  uint64_t wsum[S::NW];
  uint32_t ctl[4];  // 0: fallback, 1: header of the next tile's first block, 2: window too short
};

// Block header at stream offset hp (stage-relative rel) as the chain needs it: its byte length
// up to the payload's end (hop). ok: the 8-byte window holds the varint's end; in: inside the
// stage (rel + 24 <= lim).
__device__ inline uint32_t dpg_hop(const uint32_t* stage, uint32_t rel, uint32_t nmb32, uint32_t vpmb32, bool& ok) {
  const uint64_t lo8 = lload_u64(stage, rel);
  const uint64_t t8 = ~lo8 & 0x8080808080808080ull;
  ok = t8 != 0;
  const uint32_t vl = ok ? ((uint32_t)__builtin_ctzll(t8) >> 3) + 1u : 8u;
  const uint64_t wy = lload_u64(stage, rel + vl);
  const uint64_t y = nmb32 >= 8 ? wy : (wy & ((1ull << (8 * nmb32)) - 1ull));
  const uint64_t s16 = (y & 0x00FF00FF00FF00FFull) + ((y >> 8) & 0x00FF00FF00FF00FFull);
  const uint32_t sumw = (uint32_t)((s16 * 0x0001000100010001ull) >> 48);
  const uint64_t h = (uint64_t)vl + nmb32 + (uint64_t)(vpmb32 >> 3) * sumw;
  return h > 0x0FFFFFFFull ? 0x0FFFFFFFu : (uint32_t)h;
}

// The stream header of a DELTA page as k_delta_page / k_delta_hdr take it (decoding.rs:501-533):
// false for anything they leave to the tiled path (which reports the reference's errors).
struct DpgHead {
  uint32_t q;          // stream offset of the first block header
  uint32_t nmb, vpmb;  // mini-blocks per block, values per mini-block
  uint32_t need;       // deltas (values - 1)
  uint64_t first;      // first value
};

template <uint32_t TT>
__device__ inline bool dpg_head(const uint8_t* sp, uint32_t slen, uint64_t n, DpgHead& h) {
  uint64_t block_size, nmb, total, fz;
  uint32_t q = 0;
  int l;
  if ((l = g_vlq(sp, q, slen, block_size)) <= 0) return false;
  q += l;
  if ((l = g_vlq(sp, q, slen, nmb)) <= 0) return false;
  q += l;
  if ((l = g_vlq(sp, q, slen, total)) <= 0) return false;
  q += l;
  if ((l = g_vlq(sp, q, slen, fz)) <= 0) return false;
  q += l;
  if ((int64_t)nmb <= 0 || nmb > 8) return false;
  const uint64_t vpmb = (uint64_t)((int64_t)block_size / (int64_t)nmb);
  if (vpmb % 16 != 0 || vpmb == 0 || vpmb * nmb < 128 || TT % (vpmb * nmb) != 0) return false;
  if (total < n || n > 0x7FFFFFFFull || slen >= (1u << 28)) return false;
  h.q = q;
  h.nmb = (uint32_t)nmb;
  h.vpmb = (uint32_t)vpmb;
  h.need = n > 0 ? (uint32_t)n - 1u : 0u;
  h.first = (uint64_t)unzigzag(fz);
  return true;
}

// Wave 0 (all 64 lanes): the block headers of the tile whose first header is at stream offset
// hdr, staged from stream offset sb (win bytes of the STG staged), found by a speculative scan:
// lane j guesses block j's header offset (hdr + j * hguess), parses its length there, and the
// exclusive scan of those lengths gives the next guesses; the prefix of lanes whose guess equals
// the scan is exact and grows by at least one lane per round, so at most nb + 1 rounds (blocks of
// one length, the writer's fixed widths, take one or two). Then lane j parses block j's header
// (min delta, widths: the checks of k_delta_index) into sm. fb: a header the tiled path must
// take; shortwin: a header or payload past the win staged bytes (stage the full window); hp: the
// offset past the tile's last block (the next tile's first header).
template <int NT, int ES>
__device__ inline void dpg_headers(DeltaPageSmem<NT>& sm, uint32_t hdr, uint32_t hguess, uint32_t sb, uint32_t win,
                                   uint32_t slen, uint32_t nb, uint32_t b0, uint32_t need, uint32_t nmb32,
                                   uint32_t vpmb32, bool& fb, bool& shortwin, uint32_t& hp) {
  constexpr int STG = DpgShape<NT>::STAGE;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t vpb = vpmb32 * nmb32;
  const uint32_t wmax = ES == 4 ? 32u : 64u;
  uint32_t P = hdr + lane * hguess;
  fb = true;  // (stays set if the scan never settles)
  shortwin = false;
  hp = hdr;
#pragma unroll 1
  for (uint32_t round = 0; round <= nb; ++round) {
    const uint32_t rel = P - sb;
    const bool act = lane < nb;
    const bool inw = P < slen && rel + 24u <= (uint32_t)STG;  // parseable from the stage
    const bool inwin = rel + 24u <= win;                       // staged for this tile
    bool okv = false;
    uint32_t h = 0;
    if (act && inw && inwin) h = dpg_hop(sm.stage, rel, nmb32, vpmb32, okv);
    const bool good = act && inw && inwin && okv;
    const uint32_t incl = wave_scan_incl_u32(good ? h : 0u);
    const uint64_t Q64 = (uint64_t)hdr + (incl - (good ? h : 0u));
    const uint32_t Q = Q64 > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)Q64;
    const uint64_t diff = __ballot(act && Q != P);
    const uint32_t m = diff ? (uint32_t)__builtin_ctzll(diff) : nb;  // lanes [0, m) exact
    const uint64_t badm = __ballot(act && lane < m && !good);  // an exact lane that cannot be taken
    if (badm) {
      const uint32_t f = (uint32_t)__builtin_ctzll(badm);
      const bool f_inw = __shfl((int)(inw ? 1 : 0), (int)f, 64) != 0;
      const bool f_win = __shfl((int)(inwin ? 1 : 0), (int)f, 64) != 0;
      // past the bytes staged for this tile: stage the full window; past the stream or the
      // stage, or a varint without its end in 8 bytes: the tiled path
      shortwin = f_inw && !f_win;
      fb = !shortwin;
      return;
    }
    if (m >= nb) {  // every block's offset exact: the chain ends past the last one
      const uint32_t e = (uint32_t)__shfl((int)incl, (int)(nb - 1u), 64);
      const uint64_t he = (uint64_t)hdr + e;
      hp = he > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)he;
      fb = false;
      break;
    }
    P = Q;
  }
  bool lfb = false;
  if (lane < nb) {
    const uint32_t pos = P, rel = pos - sb, b = b0 + lane;
    const uint64_t lo8 = lload_u64(sm.stage, rel), hi8 = lload_u64(sm.stage, rel + 8);
    const uint64_t t8 = ~lo8 & 0x8080808080808080ull;
    const uint32_t vl = ((uint32_t)__builtin_ctzll(t8) >> 3) + 1u;  // t8 != 0 (the scan)
    uint64_t y = lo8 & 0x7F7F7F7F7F7F7F7Full;
    if (vl < 8) y &= (1ull << (8 * vl)) - 1ull;
    y = (y & 0x007F007F007F007Full) | ((y & 0x7F007F007F007F00ull) >> 1);
    y = (y & 0x00003FFF00003FFFull) | ((y & 0x3FFF00003FFF0000ull) >> 2);
    const uint64_t zz = (y & 0x000000000FFFFFFFull) | ((y & 0x0FFFFFFF00000000ull) >> 4);
    if ((uint64_t)pos + vl + nmb32 > slen) lfb = true;
    const uint32_t payload = pos + vl + nmb32;
    const uint32_t left = need - b * vpb;
    const uint32_t inblk = left < vpb ? left : vpb;
    const uint32_t mneed = (inblk + vpmb32 - 1) / vpmb32;
    const uint32_t sh = vl * 8u;  // widths: bytes [vl, vl + nmb) of the 16-byte window
    const uint64_t wv = sh < 64 ? ((lo8 >> sh) | (sh ? hi8 << (64 - sh) : 0ull)) : hi8;
    uint32_t boff = 0;
#pragma unroll
    for (uint32_t m = 0; m < 8; ++m) {
      const uint32_t wdt = m < nmb32 ? (uint32_t)((wv >> (8 * m)) & 0xFFu) : 0u;
      if (m < nmb32 && m < mneed && (wdt > wmax || (uint64_t)payload + boff + (vpmb32 * wdt) / 8 > slen)) lfb = true;
      sm.mbw[lane][m] = wdt;
      sm.mboff[lane][m] = boff;
      boff += m < nmb32 ? (vpmb32 * wdt) / 8 : 0u;
    }
    sm.pos[lane] = payload;
    sm.mind[lane] = (uint64_t)unzigzag(zz);
  }
  fb = __ballot(lfb) != 0;
  // the tile's payload must be staged too (its last block's end is the next tile's header)
  if (!fb && hp - sb > win) shortwin = true;
}

// Every thread: its DPT deltas of the tile [D0, D1) (min delta + packed value; from the stage when
// inside the win staged bytes, else global loads); returns their sum.
template <int NT>
__device__ inline uint64_t dpg_unpack(const DeltaPageSmem<NT>& sm, const uint8_t* __restrict__ blob, uint64_t blob_len,
                                      uint64_t S, uint32_t sb, uint32_t win, uint32_t D0, uint32_t D1, uint32_t nmb32,
                                      uint32_t vpmb32, uint64_t (&x)[DPT]) {
  const uint32_t vpb = vpmb32 * nmb32;
  const uint32_t lim = win * 8u;  // staged bits
  const uint32_t r0 = (uint32_t)threadIdx.x * DPT;  // tile-relative first delta
  uint64_t s = 0;
  if (D0 + r0 < D1) {
    const uint32_t bi = r0 / vpb, m = (r0 - bi * vpb) / vpmb32, kk = r0 - bi * vpb - m * vpmb32;
    const uint32_t wdt = sm.mbw[bi][m];
    const uint64_t mn = sm.mind[bi];
    const uint32_t base = (sm.pos[bi] + sm.mboff[bi][m] - sb) * 8u + kk * wdt;  // bit offset in the window
    const uint32_t cnt = D1 - D0 - r0 < (uint32_t)DPT ? D1 - D0 - r0 : (uint32_t)DPT;
    const uint32_t wm = wdt >= 32 ? 0xFFFFFFFFu : (1u << wdt) - 1u;
    if (wdt <= 32 && base + DPT * wdt <= lim) {
#pragma unroll
      for (int j = 0; j < DPT; ++j) {
        const uint32_t bit = base + (uint32_t)j * wdt;
        const uint32_t wi = bit >> 5;
        const uint32_t r = __builtin_amdgcn_alignbit(sm.stage[wi + 1], sm.stage[wi], bit & 31u) & wm;
        x[j] = (uint32_t)j < cnt ? mn + r : 0ull;
        s += x[j];
      }
    } else {  // outside the window or wider than 32 bits: global reads
#pragma unroll
      for (int j = 0; j < DPT; ++j) {
        uint64_t v = 0;
        if ((uint32_t)j < cnt) {
          const uint64_t gb = ((uint64_t)sm.pos[bi] + sm.mboff[bi][m]) * 8ull + (uint64_t)(kk + j) * wdt;
          const uint64_t abs = S + (gb >> 3);
          const uint32_t sh = (uint32_t)(gb & 7);
          uint64_t r = gload_u64(blob, blob_len, abs) >> sh;
          if (wdt + sh > 64) r |= gload_u64(blob, blob_len, abs + 8) << (64 - sh);
          v = mn + (wdt >= 64 ? r : (r & ((1ull << wdt) - 1ull)));
        }
        x[j] = v;
        s += v;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < DPT; ++j) x[j] = 0;
  }
  return s;
}

// The tile's values (deltas [D0, D0 + cnt) -> values [D0 + 1, ...)) from registers through the
// stage buffer: WR waves' values per round, 16-byte stores of contiguous output per instruction.
template <int ES, int NT>
__device__ inline void dpg_store(DeltaPageSmem<NT>& sm, const uint64_t (&val)[DPT], gptr<uint8_t> tb, uint32_t cnt) {
  using SH = DpgShape<NT>;
  const int tid = threadIdx.x;
  constexpr uint32_t CPT = DPT * ES / 16;                   // 16-byte chunks per thread
  constexpr uint32_t WB = 64u * DPT * ES;                   // bytes of one wave's values
  constexpr uint32_t WPR0 = (uint32_t)DeltaPageSmem<NT>::OB / WB;  // waves whose values fit the buffer
  constexpr uint32_t WPR = WPR0 >= 8 ? 8 : WPR0 >= 4 ? 4 : WPR0 >= 2 ? 2 : 1;
  constexpr uint32_t NR = (uint32_t)SH::NW / (WPR < (uint32_t)SH::NW ? WPR : (uint32_t)SH::NW);  // rounds
  constexpr uint32_t WR = (uint32_t)SH::NW / NR;            // waves per round
  constexpr uint32_t QV = WR * 64u * DPT;                   // values per round
  constexpr uint32_t NCH = QV * ES / 16;                    // chunks per round
#pragma unroll 1
  for (uint32_t qq = 0; qq < NR; ++qq) {
    if ((uint32_t)(tid >> 6) / WR == qq) {
      const uint32_t tl = (uint32_t)tid - qq * WR * 64u;
#pragma unroll
      for (uint32_t c = 0; c < CPT; ++c) {
        uint4 v4;
        if (ES == 8)
          v4 = make_uint4((uint32_t)val[2 * c], (uint32_t)(val[2 * c] >> 32), (uint32_t)val[2 * c + 1],
                          (uint32_t)(val[2 * c + 1] >> 32));
        else
          v4 = make_uint4((uint32_t)val[4 * c], (uint32_t)val[4 * c + 1], (uint32_t)val[4 * c + 2],
                          (uint32_t)val[4 * c + 3]);
        const uint32_t ci = tl * CPT + c;
        sm.stq[ci ^ (tl & 7u)] = v4;  // xor swizzle against bank conflicts
      }
    }
    __syncthreads();
#pragma unroll 2
    for (uint32_t r = 0; r < (NCH + NT - 1) / NT; ++r) {
      const uint32_t ci = (uint32_t)tid + r * NT;
      if (ci < NCH) {
        const uint4 v4 = sm.stq[ci ^ ((ci / CPT) & 7u)];
        const uint32_t v0 = qq * QV + ci * (16 / ES);
        gptr<uint8_t> dst = tb + (uint64_t)v0 * ES;
        if (v0 + 16 / ES <= cnt) {
          gst16(dst, v4);
        } else if (v0 < cnt) {
          const uint32_t qa[4] = {v4.x, v4.y, v4.z, v4.w};
#pragma unroll
          for (uint32_t e = 0; e < 16 / ES; ++e) {
            if (v0 + e >= cnt) break;
            if (ES == 8) reinterpret_cast<gptr<uint64_t>>(dst)[e] = (uint64_t)qa[2 * e] | ((uint64_t)qa[2 * e + 1] << 32);
            else reinterpret_cast<gptr<uint32_t>>(dst)[e] = qa[e];
          }
        }
      }
    }
    __syncthreads();
  }
}

// Workgroup scan of the threads' delta sums: acc = the value before this thread's first delta
// (carry + the deltas of the threads before it); returns the tile's sum.
template <int NT>
__device__ inline uint64_t dpg_scan(DeltaPageSmem<NT>& sm, uint64_t s, uint64_t carry, uint64_t& acc) {
  const int tid = threadIdx.x;
  uint64_t incl = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y2 = __shfl_up(incl, off, 64);
    if ((tid & 63) >= off) incl += y2;
  }
  if ((tid & 63) == 63) sm.wsum[tid >> 6] = incl;
  __syncthreads();
  acc = carry + incl - s;
  uint64_t tot = 0;
#pragma unroll
  for (int wv = 0; wv < DpgShape<NT>::NW; ++wv) {
    if (wv < (tid >> 6)) acc += sm.wsum[wv];
    tot += sm.wsum[wv];
  }
  return tot;
}

template <int ES, int NT>
__global__ void __attribute__((amdgpu_waves_per_eu(4, 8))) __launch_bounds__(NT) k_delta_page(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                   PageWork* pages, const ChunkWork* chunks, DeltaTables dt) {
  using SH = DpgShape<NT>;
  constexpr uint32_t TT = SH::T;
  constexpr int STG = SH::STAGE;
  __shared__ DeltaPageSmem<NT> sm;
  const int p = blockIdx.x;
  const int tid = threadIdx.x;
  const PageWork& pw = pages[p];
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  if (pw.encoding != E_DELTA_BINARY_PACKED || chunks[pw.chunk].es != ES) return;
  const gptr<uint8_t> __restrict__ out = gp(chunks[pw.chunk].val_out);
  DeltaPage info{0, 0, DP_FALLBACK, 0, 0};
#ifdef PQG_DPG_OFF  // (experiment builds: every page to the tiled path)
  if (tid == 0) {
    dt.page[p] = info;
    atomicAdd(dt.nfall, 1u);
  }
  return;
#endif
  const uint64_t S = pw.base + pw.val_off;
  const uint32_t slen = pw.val_bytes;
  DpgHead hd;
  if (pw.status != 0 || !dpg_head<TT>(blob + S, slen, pw.nonnull, hd)) {
    if (tid == 0) {
      dt.page[p] = info;
      atomicAdd(dt.nfall, 1u);
    }
    return;
  }
  const uint32_t nmb32 = hd.nmb, vpmb32 = hd.vpmb, vpb = vpmb32 * nmb32, need = hd.need;
  const gptr<uint8_t> ob = out + pw.value_out * (uint64_t)ES;
  if (tid == 0 && pw.nonnull > 0) {  // value 0
    if (ES == 8) *reinterpret_cast<gptr<uint64_t>>(ob) = hd.first;
    else *reinterpret_cast<gptr<uint32_t>>(ob) = (uint32_t)hd.first;
  }
  uint4 pv[SH::CH];
  uint64_t SB = (S + hd.q) & ~15ull;  // stage base of the current tile (absolute)
  uint32_t win = STG;                 // bytes staged for the current tile
  auto issue = [&](uint64_t base, uint32_t nbytes) {
    const bool fast = base + STG <= blob_len;
#pragma unroll
    for (int c = 0; c < SH::CH; ++c) {
      const uint32_t off = (uint32_t)(tid + c * NT) * 16u;
      const uint64_t a = base + off;
      pv[c] = off >= nbytes ? make_uint4(0u, 0u, 0u, 0u)
              : fast        ? *reinterpret_cast<const uint4*>(blob + a)
                            : gload_u128_tail(blob, blob_len, a);
    }
  };
  const uint32_t ntl = (need + TT - 1) / TT;
  if (ntl) issue(SB, win);
#ifdef PQG_DIAG
  // diagnostics (PQG_DEBUG bit 32, tools/diag/diag_delta.py): thread 0's s_memtime cycles per
  // phase over the page's tiles -- stage install, header scan, unpack (with the next tile's load
  // issue), scan, stores -- and the tiles
  const bool dst = tid == 0 && dt.dbg;
  uint64_t dd[8] = {0, 0, 0, 0, 0, 0, 0, 0}, d0 = __builtin_amdgcn_s_memtime();
#define DP_STAMP(k)                                   \
  if (dst) {                                          \
    const uint64_t t1 = __builtin_amdgcn_s_memtime(); \
    dd[k] += t1 - d0;                                 \
    d0 = t1;                                          \
  }
#else
#define DP_STAMP(k)
#endif
  uint32_t hdr = hd.q;        // header of the current tile's first block (stream offset)
  uint64_t carry = hd.first;  // value before the tile's first delta
  uint32_t hguess = 0;        // block length guess for the header scan (the last tile's average)
  for (uint32_t k = 0; k < ntl; ++k) {
    const uint32_t D0 = k * TT;
    const uint32_t D1 = D0 + TT < need ? D0 + TT : need;
    const uint32_t nb = (D1 - D0 + vpb - 1) / vpb;  // blocks of the tile
  restage:
#pragma unroll
    for (int c = 0; c < SH::CH; ++c) sm.stq[tid + c * NT] = pv[c];
    if (tid < 16) sm.stage[STG / 4 + tid] = 0;
    __syncthreads();
    DP_STAMP(0)
    const uint32_t sb = (uint32_t)(SB - S);  // stream offset of staged byte 0 (mod 2^32)
    if (tid < 64) {
      bool fb, shortwin;
      uint32_t hp;
      dpg_headers<NT, ES>(sm, hdr, hguess, sb, win, slen, nb, D0 / vpb, need, nmb32, vpmb32, fb, shortwin, hp);
      if (tid == 0) {
        sm.ctl[0] = fb ? 1u : 0u;
        sm.ctl[1] = hp;
        sm.ctl[2] = shortwin ? 1u : 0u;
      }
    }
    __syncthreads();
    DP_STAMP(1)
    if (sm.ctl[2] && !sm.ctl[0] && win < (uint32_t)STG) {  // stage the full window and redo
      win = STG;
      issue(SB, win);
      __syncthreads();  // every read of the stage is done before the reinstall
      goto restage;
    }
    if (sm.ctl[0]) {  // leave the page to the tiled path (a payload past a full window: global reads)
      if (tid == 0) {
        dt.page[p] = info;
        atomicAdd(dt.nfall, 1u);
      }
      return;
    }
    const uint32_t span = sm.ctl[1] - hdr;  // this tile's bytes: the next tile likely needs as many
    hguess = nb ? span / nb : 0u;
    hdr = sm.ctl[1];
    const uint64_t SBn = (S + hdr) & ~15ull;
    const uint32_t winn = min((uint32_t)STG, (span + span / 8u + 256u + 15u) & ~15u);
    if (k + 1 < ntl) issue(SBn, winn);
    uint64_t x[DPT];
    const uint64_t s = dpg_unpack<NT>(sm, blob, blob_len, S, sb, win, D0, D1, nmb32, vpmb32, x);
    DP_STAMP(2)
    uint64_t acc;
    carry += dpg_scan<NT>(sm, s, carry, acc);  // (the barrier also ends every read of the stage)
    DP_STAMP(3)
    uint64_t val[DPT];
#pragma unroll
    for (int j = 0; j < DPT; ++j) {
      acc += x[j];
      val[j] = acc;
    }
    dpg_store<ES, NT>(sm, val, ob + (uint64_t)(D0 + 1) * ES, D1 - D0);
    DP_STAMP(4)
#ifdef PQG_DIAG
    if (dst) dd[7] += 1;
#endif
    SB = SBn;
    win = winn;
  }
#ifdef PQG_DIAG
  if (dst)
    for (int i = 0; i < 8; ++i) dt.dbg[8 * p + i] = dd[i];
#endif
#undef DP_STAMP
  if (tid == 0) {
    info.first = hd.first;
    info.vpmb = vpmb32;
    info.nmb = nmb32;
    info.tiled = DP_DONE;
    dt.page[p] = info;
  }
}

// Per-page fallback for pages the tiled path does not take (k_delta with a page filter).
template <int ES>
__global__ void __launch_bounds__(WG) k_delta_rest(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                   PageWork* pages, ChunkWork* chunks, DeltaTables dt) {
  __shared__ DeltaSmem sm;
  const int p = blockIdx.x;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  if (pw.encoding != E_DELTA_BINARY_PACKED || chunks[pw.chunk].es != ES) return;
  if (dt.page[p].tiled) return;
  DeltaInfo info;
  int32_t st = delta_stream<ES>(sm, blob, blob_len, pw.base + pw.val_off, pw.val_bytes, pw.nonnull,
                                pw.nonnull, chunks[pw.chunk].val_out + pw.value_out * ES, info);
  if (st && threadIdx.x == 0) report(pages, chunks, p, st);
}

// The page pass; pages it leaves (irregular block shapes, errors) to the tiled kernels, which exit
// at once when it left none (dt.nfall), then the per-page stream decoder for what those refuse.
template <int ES>
static void delta_tiled(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages, ChunkWork* chunks,
                        uint32_t ntiles, const uint32_t* tile_page, DeltaTables dt, hipStream_t s, hipEvent_t* kev) {
  if (kev) (void)hipEventRecord(kev[0], s);
  hipLaunchKernelGGL((k_delta_page<ES, DPG_NT>), dim3(npages), dim3(DPG_NT), 0, s, blob, blob_len, pages, chunks, dt);
  if (kev) (void)hipEventRecord(kev[1], s);
  hipLaunchKernelGGL(k_delta_index<ES>, dim3(npages), dim3(64), 0, s, blob, blob_len, pages, chunks, dt);
  if (ntiles) {
    const dim3 tg(ntiles < 4096u ? ntiles : 4096u);  // grid-stride over the tiles
    hipLaunchKernelGGL(k_delta_sums<ES>, tg, dim3(WG), 0, s, blob, blob_len, pages, chunks, tile_page, ntiles, dt);
    hipLaunchKernelGGL(k_delta_tscan, dim3(npages), dim3(WG), 0, s, pages, dt);
    hipLaunchKernelGGL(k_delta_expand<ES>, tg, dim3(WG), 0, s, blob, blob_len, pages, chunks, tile_page, ntiles, dt);
  }
  hipLaunchKernelGGL(k_delta_rest<ES>, dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, chunks, dt);
}

// es_mask: bit mask of the DELTA_BINARY_PACKED chunks' value sizes (4: INT32, 8: INT64).
extern "C" hipError_t pqg_launch_delta_tiled(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages,
                                             ChunkWork* chunks, uint32_t ntiles, const uint32_t* tile_page,
                                             DeltaTables dt, uint32_t es_mask, hipStream_t s, hipEvent_t* kev) {
  if (es_mask & 8u) delta_tiled<8>(blob, blob_len, pages, npages, chunks, ntiles, tile_page, dt, s, kev);
  if (es_mask & 4u) delta_tiled<4>(blob, blob_len, pages, npages, chunks, ntiles, tile_page, dt, s, (es_mask & 8u) ? nullptr : kev);
  return hipGetLastError();
}

}  // namespace pqg
