// pqg_delta.hip — DELTA_BINARY_PACKED values (decoding.rs:392-619): one 256-thread workgroup
// per page running the stream decoder of pqg_delta.hpp over the page's value stream.
#include "pqg_delta.hpp"

namespace pqg {

template <int ES>  // 4 = INT32, 8 = INT64
__global__ void __launch_bounds__(WG) k_delta(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                              PageWork* pages, uint8_t* __restrict__ out,
                                              ChunkResult* res) {
  __shared__ DeltaSmem sm;
  const int p = blockIdx.x;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  if (pw.encoding != E_DELTA_BINARY_PACKED) return;
  DeltaInfo info;
  // the decoder's set_data ignores num_values; read_batch asks for the non-null count
  int32_t st = delta_stream<ES>(sm, blob, blob_len, pw.base + pw.val_off, pw.val_bytes, pw.nonnull,
                                pw.nonnull, out + pw.value_out * ES, info);
  if (st && threadIdx.x == 0) report(pages, res, p, st);
}

extern "C" hipError_t pqg_launch_delta(const uint8_t* blob, uint64_t blob_len, PageWork* pages,
                                       int npages, int es, uint8_t* out, ChunkResult* res,
                                       hipStream_t s) {
  if (es == 4)
    hipLaunchKernelGGL(k_delta<4>, dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, out, res);
  else if (es == 8)
    hipLaunchKernelGGL(k_delta<8>, dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, out, res);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace pqg

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
                                                    PageWork* pages, DeltaTables dt, ChunkResult* res) {
  __shared__ IndexSmem sm;
  const int p = blockIdx.x;
  const PageWork pw = pages[p];
  const uint32_t lane = threadIdx.x & 63;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  if (pw.encoding != E_DELTA_BINARY_PACKED) return;
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
      report(pages, res, p, err);
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
  const uint64_t below = (1ull << lane) - 1ull;
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
      report(pages, res, p, err);
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
                                        uint64_t blob_len, PageWork* pages,
                                        const uint32_t* __restrict__ tile_page, uint32_t ntiles,
                                        const DeltaTables& dt, uint32_t t, int& p, DeltaPage& info,
                                        uint32_t& lo, uint32_t& hi, uint64_t (&x)[DPT], uint64_t& s) {
  const int tid = threadIdx.x;
  if (t >= ntiles) return false;
  p = (int)tile_page[t];
  const PageWork& pw = pages[p];
  if (pw.status != 0 || pw.encoding != E_DELTA_BINARY_PACKED) return false;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return false;
  info = dt.page[p];
  if (!info.tiled) return false;
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
__global__ void __launch_bounds__(WG) k_delta_sums(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                   PageWork* pages, const uint32_t* __restrict__ tile_page,
                                                   uint32_t ntiles, DeltaTables dt) {
  __shared__ DeltaExpandSmem sm;
  const uint32_t t = blockIdx.x;
  int p;
  DeltaPage info;
  uint32_t lo, hi;
  uint64_t x[DPT], s;
  if (!delta_tile_front<ES>(sm, blob, blob_len, pages, tile_page, ntiles, dt, t, p, info, lo, hi, x, s))
    return;
  const uint64_t T = block_sum_u64(s, sm.wsum);
  if (threadIdx.x == 0) dt.agg[t] = T;
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
  if (!info.tiled) return;
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
__global__ void __launch_bounds__(WG) k_delta_expand(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                     PageWork* pages, const uint32_t* __restrict__ tile_page,
                                                     uint32_t ntiles, DeltaTables dt,
                                                     uint8_t* __restrict__ out) {
  __shared__ DeltaExpandSmem sm;
  const int tid = threadIdx.x;
  const uint32_t t = blockIdx.x;
  int p;
  DeltaPage info;
  uint32_t lo, hi;
  uint64_t x[DPT], s;
  if (!delta_tile_front<ES>(sm, blob, blob_len, pages, tile_page, ntiles, dt, t, p, info, lo, hi, x, s))
    return;
  const PageWork& pw = pages[p];
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
  uint8_t* const ob = out + (pw.value_out + lo) * (uint64_t)ES;
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
      uint8_t* dst = ob + (uint64_t)v0 * ES;
      if (v0 + 16 / ES <= cnt) {
        *reinterpret_cast<uint4*>(dst) = q;
      } else if (v0 < cnt) {
        const uint32_t qa[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
        for (uint32_t e = 0; e < 16 / ES; ++e) {
          if (v0 + e >= cnt) break;
          if (ES == 8) reinterpret_cast<uint64_t*>(dst)[e] = (uint64_t)qa[2 * e] | ((uint64_t)qa[2 * e + 1] << 32);
          else reinterpret_cast<uint32_t*>(dst)[e] = qa[e];
        }
      }
    }
    __syncthreads();
  }
}

// Per-page fallback for pages the tiled path does not take (k_delta with a page filter).
template <int ES>
__global__ void __launch_bounds__(WG) k_delta_rest(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                   PageWork* pages, DeltaTables dt,
                                                   uint8_t* __restrict__ out, ChunkResult* res) {
  __shared__ DeltaSmem sm;
  const int p = blockIdx.x;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  if (pw.encoding != E_DELTA_BINARY_PACKED) return;
  if (dt.page[p].tiled) return;
  DeltaInfo info;
  int32_t st = delta_stream<ES>(sm, blob, blob_len, pw.base + pw.val_off, pw.val_bytes, pw.nonnull,
                                pw.nonnull, out + pw.value_out * ES, info);
  if (st && threadIdx.x == 0) report(pages, res, p, st);
}

template <int ES>
static void delta_tiled(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages,
                        uint32_t ntiles, const uint32_t* tile_page, DeltaTables dt, uint8_t* out,
                        ChunkResult* res, hipStream_t s) {
  hipLaunchKernelGGL(k_delta_index<ES>, dim3(npages), dim3(64), 0, s, blob, blob_len, pages, dt, res);
  if (ntiles) {
    hipLaunchKernelGGL(k_delta_sums<ES>, dim3(ntiles), dim3(WG), 0, s, blob, blob_len, pages, tile_page, ntiles, dt);
    hipLaunchKernelGGL(k_delta_tscan, dim3(npages), dim3(WG), 0, s, pages, dt);
    hipLaunchKernelGGL(k_delta_expand<ES>, dim3(ntiles), dim3(WG), 0, s, blob, blob_len, pages, tile_page, ntiles, dt, out);
  }
  hipLaunchKernelGGL(k_delta_rest<ES>, dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, dt, out, res);
}

extern "C" hipError_t pqg_launch_delta_tiled(const uint8_t* blob, uint64_t blob_len, PageWork* pages,
                                             int npages, uint32_t ntiles, const uint32_t* tile_page,
                                             DeltaTables dt, uint32_t epoch, int es, uint8_t* out,
                                             ChunkResult* res, hipStream_t s) {
  (void)epoch;  // tile prefixes come from k_delta_tscan: no cross-workgroup flags
  if (es == 8) delta_tiled<8>(blob, blob_len, pages, npages, ntiles, tile_page, dt, out, res, s);
  else if (es == 4) delta_tiled<4>(blob, blob_len, pages, npages, ntiles, tile_page, dt, out, res, s);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace pqg
