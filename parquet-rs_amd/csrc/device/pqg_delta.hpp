// pqg_delta.hpp — DELTA_BINARY_PACKED stream decode for one workgroup (decoding.rs:392-619).
//
// Used for DELTA_BINARY_PACKED values (k_delta) and for the length / prefix-length streams of
// DELTA_LENGTH_BYTE_ARRAY and DELTA_BYTE_ARRAY (pqg_bytes.hip).
//
// The stream header (block size, mini-blocks per block, value count, zigzag first value;
// decoding.rs:501-533) is parsed by every thread. Block headers (zigzag min_delta + one width
// byte per mini-block, :448-468) sit at data-dependent offsets, so one lane walks them inside
// an LDS-staged 16 KiB region and records a block table; then all 256 threads unpack 16
// consecutive deltas each, run a workgroup-wide 64-bit prefix sum (wrapping, :564-565) and
// store the values. INT32 is the same computation truncated mod 2^32 (:601-609).
#pragma once
#include "pqg_device.hpp"

namespace pqg {

constexpr int DBLK = 16384;
constexpr int DREGION = DBLK + 128;
constexpr int DREGION_WORDS = DREGION / 4 + 4;
constexpr int NBCAP = 48;     // blocks per batch
constexpr int MBCAP = 64;     // mini-blocks per block-table entry
constexpr int DPT = 16;       // deltas per thread per pass

struct DeltaSmem {
  uint32_t region[DREGION_WORDS];
  uint32_t pay[NBCAP];             // stream-relative payload start of block
  uint64_t mind[NBCAP];            // min_delta
  uint32_t first_delta[NBCAP + 1]; // batch-relative delta index of the entry's first delta
  uint32_t nmbe[NBCAP];            // mini-blocks of the entry (a block of more than MBCAP
                                   // mini-blocks takes several entries)
  uint8_t width[NBCAP][MBCAP];
  uint32_t mboff[NBCAP][MBCAP];    // byte offset of mini-block m from pay[b]
  uint64_t wsum[WG / 64];
  uint64_t carry;
  uint32_t ctl[8];
};

// LEB128 from LDS; returns bytes used, 0 if truncated by the stream end, -1 if > 10 bytes
// with more data (get_vlq_int assert).
__device__ inline int lds_vlq(const uint32_t* region, uint32_t ridx, uint32_t q, uint32_t slen,
                              uint64_t& v) {
  v = 0;
  for (int k = 0; k < 10; ++k) {
    if (q + (uint32_t)k >= slen) return 0;
    uint32_t b = lbyte(region, ridx + k);
    v |= (uint64_t)(b & 0x7F) << (7 * k);
    if (!(b & 0x80)) return k + 1;
  }
  return (q + 10 < slen) ? -1 : 0;
}

__device__ inline int g_vlq(const uint8_t* p, uint32_t q, uint32_t slen, uint64_t& v) {
  v = 0;
  for (int k = 0; k < 10; ++k) {
    if (q + (uint32_t)k >= slen) return 0;
    uint32_t b = p[q + k];
    v |= (uint64_t)(b & 0x7F) << (7 * k);
    if (!(b & 0x80)) return k + 1;
  }
  return (q + 10 < slen) ? -1 : 0;
}

__device__ inline int64_t unzigzag(uint64_t u) { return (int64_t)(u >> 1) ^ -(int64_t)(u & 1); }

__device__ inline void delta_load_region(DeltaSmem& sm, const uint8_t* blob, uint64_t blob_len,
                                         uint64_t a0) {
  const int tid = threadIdx.x;
  for (int c = tid; c < DREGION / 16; c += WG) {
    uint64_t a = a0 + (uint64_t)c * 16;
    uint4 v;
    if (a + 16 <= blob_len) v = *reinterpret_cast<const uint4*>(blob + a);
    else v = gload_u128_tail(blob, blob_len, a);
    reinterpret_cast<uint4*>(sm.region)[c] = v;
  }
  if (tid < 4) sm.region[DREGION / 4 + tid] = 0;
}

// Result of one stream decode (uniform across the workgroup).
struct DeltaInfo {
  uint64_t total;    // the header's value count (values_left() after set_data)
  uint32_t end_off;  // get_offset() after decoding `n_decode` values (stream relative)
};

// Decodes the first `n_decode` values of the DELTA stream at blob[S, S+slen) (all of them
// when n_decode == ~0) and stores the first `n_store` of them to `o` (ES-byte elements).
// Errors follow the reference: EOF for "Not enough data to decode ..." (and for a stream with
// fewer than n_decode values, where the reference would return a short batch), PANIC for its
// asserts. Must be called by all threads of the workgroup.
template <int ES>
__device__ int32_t delta_stream(DeltaSmem& sm, const uint8_t* __restrict__ blob, uint64_t blob_len,
                                uint64_t S, uint32_t slen, uint64_t n_decode, uint64_t n_store,
                                uint8_t* __restrict__ o, DeltaInfo& info) {
  const uint8_t* sp = blob + S;
  const int tid = threadIdx.x;
  uint64_t block_size, nmb, total, fz;
  uint32_t q = 0;
  int32_t err = 0;
  int l;
  info.total = 0;
  info.end_off = 0;
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
    if ((int64_t)nmb <= 0) err = ST_PANIC;  // division by zero / widths[0] (decoding.rs:464)
    else {
      vpmb = (uint64_t)((int64_t)block_size / (int64_t)nmb);
      if (vpmb % 8 != 0) err = ST_PANIC;  // assert!(values_per_mini_block % 8 == 0)
    }
  }
  if (err) return err;
  info.total = total;
  info.end_off = q;
  if (n_decode == ~0ull) n_decode = total;
  if (total < n_decode) return ST_EOF;  // the reference returns a short batch here
  if (n_store > n_decode) n_store = n_decode;
  if (n_decode == 0) return 0;
  const int64_t first = unzigzag(fz);
  if (tid == 0 && n_store > 0) {
    if (ES == 4) *gp(reinterpret_cast<int32_t*>(o)) = (int32_t)first;
    else *gp(reinterpret_cast<int64_t*>(o)) = first;
  }
  if (n_decode == 1) return 0;
  if (vpmb == 0) return ST_HANG;  // block_size < num_mini_blocks: every mini-block is empty
  const uint64_t vpb = vpmb * nmb;  // deltas per block
  const uint64_t need = n_decode - 1;
  uint64_t done = 0;
  uint32_t pos = q;
  uint64_t A0 = (S + pos) & ~15ull;
  uint64_t carry = (uint64_t)first;
  uint32_t end_off = q;
  // Block walk state (lane 0 only; kept across batches, since a block of more than MBCAP
  // mini-blocks is recorded as several table entries of at most MBCAP, possibly in several
  // batches): the next header, and inside a block the next mini-block to record, the block's
  // payload start, the byte offset of that mini-block in it, min_delta, width bytes, needed
  // mini-blocks.
  uint32_t wcur = q, bm = 0, bpay = 0, bw = 0, bmneed = 0;
  uint32_t hguess = 0;    // mean block length of the last batch (the header scan's guesses)
  bool hserial = false;   // the last batch's blocks varied in length: walk them one by one
  uint64_t bboff = 0, bmind = 0;

  delta_load_region(sm, blob, blob_len, A0);
  __syncthreads();

  while (done < need) {
    // ---------------- walk block headers
    if (nmb <= 8 && tid < 64) {
      // wave 0: the batch's headers by a speculative scan (lane j guesses block j's offset from the
      // mean block length so far, parses the hop there -- varint length and the sum of the widths --
      // and the wave's scan of the hops checks the guesses; the exact prefix grows every round, one
      // or two rounds for the writer's blocks), then lane j parses block j and makes every check the
      // serial walk below makes; the first failing block (stream order) ends the batch as there.
      // The batch ends before a header past the staged region and after one past the stream or
      // with a varint of 8 bytes or more (its lane reports or parses it; the next batch goes on)
      const uint32_t lane = tid, nmb32 = (uint32_t)nmb, hs = (uint32_t)(vpmb >> 3);
      const uint64_t want = (need - done + vpb - 1) / vpb;
      const uint32_t kmax = want < (uint64_t)NBCAP ? (uint32_t)want : (uint32_t)NBCAP;
      const uint64_t left_b = slen > wcur ? (uint64_t)(slen - wcur) : 0ull;
      const uint32_t avg = hguess ? hguess : (uint32_t)min(left_b / (want ? want : 1ull), (uint64_t)DBLK);
      uint32_t posv = wcur + lane * avg, k = 0;
      if (!hserial) {
        uint32_t rounds = 0;
#pragma unroll 1
        for (uint32_t round = 0; round <= kmax; ++round) {
          rounds = round + 1u;
          const bool act = lane < kmax;
          const uint64_t rel = S + (uint64_t)posv - A0;
          const bool inreg = posv >= wcur && rel < DBLK;  // (a guess below the batch start: not exact)
          bool good = false, term = false;
          uint32_t h = 0;
          if (act && inreg) {
            if (posv >= slen) {
              term = true;  // (its lane reports the stream end)
            } else {
              const uint64_t w0 = lload_u64(sm.region, (uint32_t)rel);
              const uint64_t t8 = ~w0 & 0x8080808080808080ull;
              if (!t8) {
                term = true;  // a varint of 8 bytes or more: its lane parses it, the batch ends there
              } else {
                const uint32_t vl = ((uint32_t)__builtin_ctzll(t8) >> 3) + 1u;
                const uint64_t wy = lload_u64(sm.region, (uint32_t)rel + vl);
                const uint64_t y = nmb32 >= 8 ? wy : (wy & ((1ull << (8 * nmb32)) - 1ull));
                const uint64_t s16 = (y & 0x00FF00FF00FF00FFull) + ((y >> 8) & 0x00FF00FF00FF00FFull);
                const uint32_t sumw = (uint32_t)((s16 * 0x0001000100010001ull) >> 48);
                const uint64_t hh = (uint64_t)vl + nmb32 + (uint64_t)hs * sumw;
                h = hh > 0x03FFFFFFull ? 0x03FFFFFFu : (uint32_t)hh;  // (64 hops stay below 2^32)
                good = true;
              }
            }
          }
          const uint32_t incl = wave_scan_incl_u32(good ? h : 0u);
          const uint64_t Q64 = (uint64_t)wcur + (incl - (good ? h : 0u));
          const uint32_t Q = Q64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)Q64;
          const uint64_t diff = __ballot(act && Q != posv);
          const uint32_t m = diff ? (uint32_t)__builtin_ctzll(diff) : kmax;  // lanes [0, m) exact
          const uint64_t stop = __ballot(act && lane < m && !good);          // an exact lane that ends it
          if (stop) {
            const uint32_t f = (uint32_t)__builtin_ctzll(stop);
            const bool fterm = __shfl((int)(term ? 1 : 0), (int)f, 64) != 0;
            k = fterm ? f + 1u : f;  // (outside the region: the next batch moves it there)
            break;
          }
          if (m >= kmax) {
            k = kmax;
            break;
          }
          posv = Q;
        }
        // (each round fixes at least one lane; many rounds: block lengths vary, walk them in turn)
        hserial = rounds > 4u;
      } else {
        // blocks of varying length: one walk (every lane alike), one LDS round trip per header
        uint32_t cur = wcur, hmin = 0xFFFFFFFFu, hmax = 0;
#pragma unroll 1
        while (k < kmax) {
          const uint64_t rel = S + (uint64_t)cur - A0;
          if (rel >= DBLK) break;
          posv = lane == k ? cur : posv;
          ++k;
          if (cur >= slen) break;
          const uint32_t wi = (uint32_t)rel >> 2, sh = ((uint32_t)rel & 3u) * 8u;
          const uint32_t x0 = sm.region[wi], x1 = sm.region[wi + 1], x2 = sm.region[wi + 2], x3 = sm.region[wi + 3],
                         x4 = sm.region[wi + 4];
          const uint64_t lo8 = ((uint64_t)__builtin_amdgcn_alignbit(x2, x1, sh) << 32) | __builtin_amdgcn_alignbit(x1, x0, sh);
          const uint64_t hi8 = ((uint64_t)__builtin_amdgcn_alignbit(x4, x3, sh) << 32) | __builtin_amdgcn_alignbit(x3, x2, sh);
          const uint64_t t8 = ~lo8 & 0x8080808080808080ull;
          if (!t8) break;
          const uint32_t vl = ((uint32_t)__builtin_ctzll(t8) >> 3) + 1u, vs = vl * 8u;
          const uint64_t wv = vs < 64 ? ((lo8 >> vs) | (hi8 << (64 - vs))) : hi8;
          const uint64_t y = nmb32 >= 8 ? wv : (wv & ((1ull << (8 * nmb32)) - 1ull));
          const uint64_t s16 = (y & 0x00FF00FF00FF00FFull) + ((y >> 8) & 0x00FF00FF00FF00FFull);
          const uint32_t sumw = (uint32_t)((s16 * 0x0001000100010001ull) >> 48);
          const uint64_t hh = (uint64_t)vl + nmb32 + (uint64_t)hs * sumw;
          const uint32_t h = hh > 0x03FFFFFFull ? 0x03FFFFFFu : (uint32_t)hh;
          hmin = min(hmin, h);
          hmax = max(hmax, h);
          const uint64_t nx = (uint64_t)cur + h;
          cur = nx > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)nx;
        }
        hserial = hmax != hmin;  // blocks of one length: the guesses are exact again
      }
      int32_t e = 0;
      uint32_t nxt = 0, endp = 0;
      if (lane < k) {
        const uint32_t pos = posv, ridx = (uint32_t)(S + pos - A0);
        uint64_t zz;
        const int vl = lds_vlq(sm.region, ridx, pos, slen, zz);
        if (vl <= 0) {
          e = vl ? ST_PANIC : ST_EOF;  // "Not enough data to decode 'min_delta'"
        } else if ((uint64_t)pos + vl + nmb32 > slen) {
          e = ST_EOF;  // "Not enough data to decode 'width'" (every width is read)
        } else {
          const uint64_t left = need - done - (uint64_t)lane * vpb;
          const uint64_t inblk = left < vpb ? left : vpb;
          const uint32_t mneed = (uint32_t)((inblk + vpmb - 1) / vpmb);
          const uint32_t pay = pos + (uint32_t)vl + nmb32;
          uint64_t boff = 0;
          for (uint32_t m = 0; m < nmb32; ++m) {
            const uint32_t wdt = lbyte(sm.region, ridx + (uint32_t)vl + m);
            sm.width[lane][m] = (uint8_t)wdt;
            sm.mboff[lane][m] = (uint32_t)boff;
            if (m < mneed && !e) {
              if (wdt > (ES == 4 ? 32u : 64u)) e = ST_PANIC;  // get_batch / get_value assert on num_bits
              else if ((uint64_t)pay + boff + (vpmb * wdt) / 8 > slen) e = (ES == 4) ? ST_PANIC : ST_EOF;
              else endp = (uint32_t)((uint64_t)pay + boff + (vpmb * wdt) / 8);
            }
            boff += (vpmb * wdt) / 8;
          }
          sm.pay[lane] = pay;
          sm.mind[lane] = (uint64_t)unzigzag(zz);
          sm.nmbe[lane] = nmb32;
          sm.first_delta[lane] = lane * (uint32_t)vpb;
          const uint64_t nx = (uint64_t)pay + boff;
          nxt = nx > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)nx;
        }
      }
      const uint64_t em = __ballot(e != 0);
      const uint32_t nb = em ? (uint32_t)__builtin_ctzll(em) : k;  // blocks before the first failing one
      const int32_t e0 = em ? __shfl(e, (int)nb, 64) : 0;
      if (lane == 0) {
        const uint64_t left = need - done, cap = (uint64_t)nb * vpb;
        const uint32_t dcount = (uint32_t)(left < cap ? left : cap);
        sm.first_delta[nb] = dcount;
        sm.ctl[0] = nb;
        sm.ctl[1] = dcount;
        sm.ctl[2] = (uint32_t)e0;
      }
      const uint32_t last = nb ? nb - 1u : 0u;
      const uint32_t ncur = nb ? (uint32_t)__shfl((int)nxt, (int)last, 64) : wcur;
      if (nb && ncur > wcur) hguess = (ncur - wcur) / nb;
      const uint32_t ep = (uint32_t)__shfl((int)endp, (int)last, 64);
      if (lane == 0) {
        sm.ctl[3] = ncur;
        sm.ctl[4] = ep;
        sm.ctl[5] = 1;  // the batch's entries are whole blocks (expand: entry = delta / vpb)
      }
      wcur = ncur;
    } else if (nmb > 8 && tid == 0) {
      uint32_t nb = 0;
      uint64_t dcount = 0;
      int32_t e = 0;
      uint32_t endp = 0;
      // a width byte: staged when inside the region, else global memory (blocks whose width
      // bytes run past the region: a few thousand mini-blocks per block)
      auto wbyte = [&](uint64_t off) -> uint32_t {
        const uint64_t a = S + off;
        return (a >= A0 && a - A0 < (uint64_t)DREGION) ? lbyte(sm.region, (uint32_t)(a - A0)) : (uint32_t)blob[a];
      };
      while (nb < NBCAP && done + dcount < need) {
        if (bm == 0) {  // at a block header (init_block, decoding.rs:448-468)
          uint64_t rel = S + wcur - A0;
          if (rel >= DBLK) break;
          uint32_t ridx = (uint32_t)rel;
          uint64_t zz;
          int vl = lds_vlq(sm.region, ridx, wcur, slen, zz);
          if (vl <= 0) {
            e = vl ? ST_PANIC : ST_EOF;  // "Not enough data to decode 'min_delta'"
            break;
          }
          if ((uint64_t)wcur + vl + nmb > slen) {
            e = ST_EOF;  // "Not enough data to decode 'width'" (every width is read)
            break;
          }
          uint64_t left = need - done - dcount;
          uint64_t inblk = left < vpb ? left : vpb;
          bmneed = (uint32_t)((inblk + vpmb - 1) / vpmb);
          bw = wcur + (uint32_t)vl;
          bpay = bw + (uint32_t)nmb;
          bboff = 0;
          bmind = (uint64_t)unzigzag(zz);
        }
        // one table entry: mini-blocks [bm, m1) of the block
        const uint32_t m1 = (uint64_t)bm + MBCAP < nmb ? bm + MBCAP : (uint32_t)nmb;
        const uint64_t boff0 = bboff;
        for (uint32_t m = bm; m < m1; ++m) {
          uint32_t wdt = wbyte((uint64_t)bw + m);
          sm.width[nb][m - bm] = (uint8_t)wdt;
          sm.mboff[nb][m - bm] = (uint32_t)(bboff - boff0);
          if (m < bmneed) {
            if (wdt > (ES == 4 ? 32u : 64u)) {
              e = ST_PANIC;  // get_batch / get_value assert on num_bits
              break;
            }
            // the reference loads the whole mini-block, padding included (decoding.rs:472-495)
            if ((uint64_t)bpay + bboff + (vpmb * wdt) / 8 > slen) {
              e = (ES == 4) ? ST_PANIC : ST_EOF;
              break;
            }
            endp = (uint32_t)((uint64_t)bpay + bboff + (vpmb * wdt) / 8);
          }
          bboff += (vpmb * wdt) / 8;
        }
        if (e) break;
        const uint64_t left = need - done - dcount;
        const uint64_t span = (uint64_t)(m1 - bm) * vpmb;
        sm.pay[nb] = (uint32_t)(bpay + boff0);
        sm.mind[nb] = bmind;
        sm.nmbe[nb] = m1 - bm;
        sm.first_delta[nb] = (uint32_t)dcount;
        dcount += left < span ? left : span;
        nb++;
        bm = m1;
        if (bm == (uint32_t)nmb) {  // the block is done: the next header follows its payload
          bm = 0;
          uint64_t nx = (uint64_t)bpay + bboff;
          wcur = nx > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)nx;
        }
      }
      sm.first_delta[nb] = (uint32_t)dcount;
      sm.ctl[0] = nb;
      sm.ctl[1] = (uint32_t)dcount;
      sm.ctl[2] = (uint32_t)e;
      // where the stream continues (the region follows it): the next header, or inside a block
      // the next mini-block's payload
      uint64_t at = bm ? (uint64_t)bpay + bboff : (uint64_t)wcur;
      sm.ctl[3] = at > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)at;
      sm.ctl[4] = endp;
      sm.ctl[5] = 0;
    }
    __syncthreads();
    const uint32_t nb = sm.ctl[0];
    const uint32_t dcount = sm.ctl[1];
    const int32_t e = (int32_t)sm.ctl[2];
    const uint32_t ncur = sm.ctl[3];
    const bool whole = sm.ctl[5] != 0 && vpmb % 16 == 0;  // a thread's 16 deltas: one mini-block
    if (nb) end_off = sm.ctl[4];
    __syncthreads();
    if (e) return e;
    if (nb == 0) {  // next header lies beyond this region: move the region
      A0 = (S + ncur) & ~15ull;
      pos = ncur;
      delta_load_region(sm, blob, blob_len, A0);
      __syncthreads();
      continue;
    }

    // ---------------- expand: 16 deltas per thread per pass
    for (uint32_t pass = 0; pass < dcount; pass += DPT * WG) {
      const uint32_t d0 = pass + (uint32_t)tid * DPT;
      uint64_t v[DPT];
      uint64_t s = 0;
      if (d0 < dcount) {
        int b = 0;
        if (whole) {
          b = (int)(d0 / vpb);
        } else {
          while (b + 1 < (int)nb && sm.first_delta[b + 1] <= d0) ++b;
        }
        uint64_t inb = d0 - sm.first_delta[b];
        uint32_t m = (uint32_t)(inb / vpmb);
        uint32_t k = (uint32_t)(inb - (uint64_t)m * vpmb);
        const uint32_t wd0 = sm.width[b][m];
        const uint64_t sbit = (S + sm.pay[b] + sm.mboff[b][m]) * 8ull + (uint64_t)k * wd0;  // absolute
        const bool fast = whole && wd0 <= 32 && sbit >= A0 * 8ull &&
                          sbit - A0 * 8ull + (uint64_t)DPT * wd0 + 32ull <= (uint64_t)DREGION * 8ull;
        if (fast) {  // staged, one mini-block, at most 32 bits: one funnel shift per delta
          const uint32_t rb = (uint32_t)(sbit - A0 * 8ull);
          const uint32_t wm = wd0 >= 32 ? 0xFFFFFFFFu : (1u << wd0) - 1u;
          const uint64_t mn = sm.mind[b];
#pragma unroll
          for (int j = 0; j < DPT; ++j) {
            const uint32_t bit = rb + (uint32_t)j * wd0, wi = bit >> 5;
            const uint32_t r = __builtin_amdgcn_alignbit(sm.region[wi + 1], sm.region[wi], bit & 31u) & wm;
            v[j] = d0 + j < dcount ? mn + r : 0ull;
            s += v[j];
          }
        } else {
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
          v[j] = 0;
          if (d0 + j < dcount) {
            const uint32_t wdt = sm.width[b][m];
            const uint64_t bit = ((uint64_t)sm.pay[b] + sm.mboff[b][m]) * 8ull + (uint64_t)k * wdt;
            const uint64_t abs = S + (bit >> 3);
            const uint32_t sh = (uint32_t)(bit & 7);
            uint64_t x;
            const uint64_t ri = abs - A0;
            if (abs >= A0 && ri + 12 <= (uint64_t)DREGION) x = lload_u64(sm.region, (uint32_t)ri);
            else x = gload_u64(blob, blob_len, abs);
            uint64_t raw;
            if (wdt == 0) raw = 0;
            else if (wdt + sh <= 64) {
              raw = x >> sh;
              if (wdt < 64) raw &= (1ull << wdt) - 1ull;
            } else {  // 58..64-bit deltas straddle a 64-bit window
              uint64_t hi = (abs >= A0 && ri + 20 <= (uint64_t)DREGION)
                                ? lload_u64(sm.region, (uint32_t)ri + 8)
                                : gload_u64(blob, blob_len, abs + 8);
              raw = (x >> sh) | (hi << (64 - sh));
              if (wdt < 64) raw &= (1ull << wdt) - 1ull;
            }
            v[j] = sm.mind[b] + raw;  // min_delta + delta (wrapping)
            s += v[j];
            if (++k == vpmb) {
              k = 0;
              if (++m == sm.nmbe[b]) {
                m = 0;
                ++b;
              }
            }
          }
        }
        }
      } else {
#pragma unroll
        for (int j = 0; j < DPT; ++j) v[j] = 0;
      }
      // workgroup exclusive scan of s
      uint64_t incl = s;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        uint64_t y = __shfl_up(incl, off, 64);
        if ((tid & 63) >= off) incl += y;
      }
      if ((tid & 63) == 63) sm.wsum[tid >> 6] = incl;
      __syncthreads();
      uint64_t pre = carry;
      for (int w = 0; w < (tid >> 6); ++w) pre += sm.wsum[w];
      pre += incl - s;
      uint64_t tot = carry + sm.wsum[0] + sm.wsum[1] + sm.wsum[2] + sm.wsum[3];
      if (d0 < dcount) {
        const uint64_t oi = done + d0 + 1;  // output index of delta d
        uint64_t acc = pre;
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
          if (d0 + j < dcount) {
            acc += v[j];
            if (oi + j < n_store) {
              if (ES == 8) gp(reinterpret_cast<int64_t*>(o))[oi + j] = (int64_t)acc;  // (global stores:
              else gp(reinterpret_cast<int32_t*>(o))[oi + j] = (int32_t)(uint32_t)acc;  // no lgkmcnt)
            }
          }
        }
      }
      __syncthreads();
      carry = tot;
    }
    done += dcount;
    pos = ncur;
    __syncthreads();
    if (done < need && S + pos - A0 >= DBLK) {
      A0 = (S + pos) & ~15ull;
      delta_load_region(sm, blob, blob_len, A0);
      __syncthreads();
    }
  }
  info.end_off = end_off;
  return 0;
}

}  // namespace pqg
