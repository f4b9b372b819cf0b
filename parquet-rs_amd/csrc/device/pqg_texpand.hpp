// pqg_texpand.hpp — tile expand pass of the RLE/bit-packing hybrid decoder (rle.rs:398-487):
// one 256-thread workgroup per expand tile of RUN_TILE outputs, every page of the chunk in one
// grid.
//
// Per tile, in one memory round trip: the tile descriptor (k_tile_desc) names the run records
// the index pass kept for the tile and the stream bytes holding the tile's bit-packed payload;
// the workgroup loads both into LDS with all loads in flight together. Each thread then owns
// RUN_TILE / 256 = 16 outputs in groups of V consecutive outputs (V = 16 bytes / output size),
// computes all 16 values into registers (run lookup by binary search over the LDS run list,
// then per output an RLE value or a 32-bit funnel shift out of the LDS payload), and hands them
// to an emitter that issues every gather before any store and writes each group with one
// 16-byte store: a wave's store instruction covers 1 KiB of contiguous output.
//
// Tiles with more runs than the index pass keeps (RUN_CAPT) are re-walked from the tile's
// checkpoint by wave 0 in batches, their payload read straight from global memory: only
// hand-made streams (runs averaging under 8 outputs) take that path.
#pragma once
#include <type_traits>

#include "pqg_runs.hpp"

namespace pqg {

constexpr int TX_STAGE = 12288;                // staged payload bytes per tile
constexpr int TX_RCAP = RUN_CAPT;              // run records per batch
constexpr uint32_t TX_PER = RUN_TILE / WG;     // outputs per thread (16)
constexpr int TX_CHUNKS = TX_STAGE / 16 / WG;  // 16-byte payload loads per thread

struct TileSmem {
  uint32_t stage[(TX_STAGE + 64) / 4];
  uint32_t start[TX_RCAP + 2];
  uint32_t info[TX_RCAP + 1];
  uint32_t ctl[4];
};

// Values of outputs [g, g + V) (page-relative) clipped to [seg_lo, seg_hi), from the runs
// sm.start/info[0, nr) (sm.start[nr] = segment end). The bit-packed payload is read from the
// LDS window of `staged` bytes at stream offset sb32, or from global memory outside it.
// Returns the mask of outputs inside the segment.
template <int V>
__device__ inline uint32_t tx_values(const TileSmem& sm, uint32_t nr, uint32_t lgn, uint32_t g,
                                     uint32_t seg_lo, uint32_t seg_hi, uint32_t w, uint32_t wm,
                                     uint32_t sb32, uint32_t staged, bool wide,
                                     const uint8_t* __restrict__ blob, uint64_t blob_len,
                                     uint64_t S, uint32_t (&v)[V]) {
  if (g >= seg_hi || g + V <= seg_lo) {
#pragma unroll
    for (int j = 0; j < V; ++j) v[j] = 0;
    return 0;
  }
  const uint32_t o0 = g < seg_lo ? seg_lo : g;
  uint32_t a = 0;
  for (uint32_t step = lgn; step; step >>= 1)
    if (a + step < nr && sm.start[a + step] <= o0) a += step;
  uint32_t stA = sm.start[a], infA = sm.info[a], stB = sm.start[a + 1];
  const uint32_t lim = staged * 8u;
  uint32_t mask = 0;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const uint32_t o = g + (uint32_t)j;
    if (o >= stB && a + 1 < nr) {  // every run holds >= 1 output: at most one step per output
      ++a;
      stA = stB;
      infA = sm.info[a];
      stB = sm.start[a + 1];
    }
    uint32_t val = infA & 0x7FFFFFFFu;
    if (!(infA & R_RLE)) {
      const uint32_t bit = (infA - sb32) * 8u + (o - stA) * w;  // exact unless `wide`
      if (!wide && bit + w <= lim) {
        const uint32_t wi = bit >> 5;
        val = __builtin_amdgcn_alignbit(sm.stage[wi + 1], sm.stage[wi], bit & 31u) & wm;
      } else {
        const uint64_t b64 = (uint64_t)infA * 8ull + (uint64_t)(o - stA) * (uint64_t)w;
        val = (uint32_t)(gload_u64(blob, blob_len, S + (b64 >> 3)) >> (b64 & 7)) & wm;
      }
    }
    const bool in = o >= seg_lo && o < seg_hi;
    v[j] = in ? val : 0u;
    mask |= (in ? 1u : 0u) << j;
  }
  return mask;
}

// Expand outputs [seg_lo, seg_hi) of the tile starting at page-relative output lo.
template <class E>
__device__ inline void tx_range(const TileSmem& sm, uint32_t nr, uint32_t lo, uint32_t seg_lo,
                                uint32_t seg_hi, uint32_t w, uint32_t sb32, uint32_t staged,
                                bool wide, const uint8_t* __restrict__ blob, uint64_t blob_len,
                                uint64_t S, E& em) {
  constexpr int V = E::V;
  constexpr int NG = (int)TX_PER / V;
  const uint32_t wm = w >= 32 ? 0xFFFFFFFFu : ((1u << w) - 1u);
  const uint32_t lgn = nr > 1 ? 1u << (31 - __builtin_clz(nr - 1)) : 0u;
  const uint32_t g0 = lo + threadIdx.x * (uint32_t)V;
  uint32_t v[NG][V];
  uint32_t m[NG];
#pragma unroll
  for (int s = 0; s < NG; ++s)
    m[s] = tx_values<V>(sm, nr, lgn, g0 + (uint32_t)s * (WG * V), seg_lo, seg_hi, w, wm, sb32,
                        staged, wide, blob, blob_len, S, v[s]);
  em.template put<NG>(g0, (uint32_t)(WG * V), v, m);
}

// Expand the tile described by d (k_tile_desc) through emitter em.
template <class E>
__device__ inline void tile_expand(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                   const QDesc& d, const uint2* __restrict__ runs, TileSmem& sm,
                                   E& em) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lo = d.qlo, hi = d.qhi, w = d.w;
  const bool wide = d.slen >= (1u << 28);  // 32-bit bit offsets could wrap
  if (d.rec != RUN_REWALK) {
    // ---- one batch: run records and payload window, every load in flight together
    const bool hl = d.kind == LK_BIT_PACKED;  // one header-less run from output 0
    const uint32_t nr = hl ? 1u : d.nrec;
    uint2 r0 = make_uint2(0u, 0u), r1 = make_uint2(0u, 0u);
    if (!hl) {
      if (tid < nr) r0 = runs[d.rec + tid];
      if (tid + WG < nr) r1 = runs[d.rec + tid + WG];
    }
    uint64_t A0 = d.S;
    uint32_t nchunks = 0;
    uint4 pv[TX_CHUNKS];
    if (d.bhi && !wide) {
      A0 = (d.S + d.blo) & ~15ull;
      uint64_t A1 = d.S + (uint64_t)d.bhi;
      if (A1 > A0 + TX_STAGE) A1 = A0 + TX_STAGE;
      nchunks = (uint32_t)((A1 - A0 + 15) / 16);
      const bool fast = A0 + (uint64_t)nchunks * 16 <= blob_len;
#pragma unroll
      for (int k = 0; k < TX_CHUNKS; ++k) {
        const uint32_t c = tid + (uint32_t)(k * WG);
        if (c < nchunks) {
          const uint64_t a = A0 + (uint64_t)c * 16;
          pv[k] = fast ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
        }
      }
    }
    if (hl) {
      if (tid == 0) {
        sm.start[0] = 0;
        sm.info[0] = 0;
      }
    } else {
      if (tid < nr) {
        sm.start[tid] = r0.x;
        sm.info[tid] = r0.y;
      }
      if (tid + WG < nr) {
        sm.start[tid + WG] = r1.x;
        sm.info[tid + WG] = r1.y;
      }
    }
    if (tid == 0) {
      sm.start[nr] = hi;
      sm.start[nr + 1] = hi;
    }
#pragma unroll
    for (int k = 0; k < TX_CHUNKS; ++k) {
      const uint32_t c = tid + (uint32_t)(k * WG);
      if (c < nchunks) reinterpret_cast<uint4*>(sm.stage)[c] = pv[k];
    }
    if (tid < 16) sm.stage[nchunks * 4 + tid] = 0;
    __syncthreads();
    tx_range(sm, nr, lo, lo, hi, w, (uint32_t)(A0 - d.S), nchunks * 16, wide, blob, blob_len,
             d.S, em);
    return;
  }
  // ---- more runs than the index kept: wave 0 re-walks from the checkpoint in batches
  uint32_t cur = d.ckpos, produced = d.ckfirst, seg_lo = lo;
  while (seg_lo < hi) {
    if (tid < 64) {
      uint32_t nr = 0;
      while (produced < hi && nr < (uint32_t)TX_RCAP && cur < d.slen) {
        uint32_t nxt, cnt, inf, flg;
        run_parse_global(blob, blob_len, d.S, cur, d.slen, (int)w, nxt, cnt, inf, flg);
        if (flg & (RF_EOF | RF_PANIC)) break;  // cannot happen on a stream run_index accepted
        if (cnt) {
          const uint32_t need = cnt < hi - produced ? cnt : hi - produced;
          if (produced + need > seg_lo) {
            if (tid == 0) {
              sm.start[nr] = produced;
              sm.info[nr] = (flg & RF_BP) ? inf : (R_RLE | inf);
            }
            ++nr;
          }
          produced += need;
        }
        cur = nxt;
      }
      if (tid == 0) {
        const uint32_t sh = produced < hi ? produced : hi;
        sm.ctl[0] = nr;
        sm.ctl[1] = sh;
        sm.start[nr] = sh;
        sm.start[nr + 1] = sh;
      }
    }
    __syncthreads();
    const uint32_t nr = sm.ctl[0], seg_hi = sm.ctl[1];
    if (nr == 0 || seg_hi <= seg_lo) break;
    tx_range(sm, nr, lo, seg_lo, seg_hi, w, 0u, 0u, true, blob, blob_len, d.S, em);
    __syncthreads();
    seg_lo = seg_hi;
  }
}

// ------------------------------------------------------------------------------ emitters
//
// put<NG>(g0, stride, v, m): group s covers page-relative outputs [g0 + s*stride, + V), its
// values in v[s], m[s] the mask of outputs to write.

// Def/rep levels as int16 (column/reader.rs:162-163); def levels also count the values
// read_batch will ask for (def == max_def, column/reader.rs:212-226).
struct TxLevels {
  static constexpr int V = 8;
  int16_t* out;  // page output base
  int16_t maxl;
  bool count;
  uint32_t nonnull;
  template <int NG>
  __device__ void put(uint32_t g0, uint32_t stride, const uint32_t (&v)[NG][V], const uint32_t (&m)[NG]) {
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      if (count) {
#pragma unroll
        for (int j = 0; j < V; ++j)
          nonnull += (((m[s] >> j) & 1u) && (int16_t)v[s][j] == maxl) ? 1u : 0u;
      }
      int16_t* o = out + g0 + (uint32_t)s * stride;
      if (m[s] == 0xFFu) {
        uint4 pk;
        pk.x = (v[s][0] & 0xFFFFu) | (v[s][1] << 16);
        pk.y = (v[s][2] & 0xFFFFu) | (v[s][3] << 16);
        pk.z = (v[s][4] & 0xFFFFu) | (v[s][5] << 16);
        pk.w = (v[s][6] & 0xFFFFu) | (v[s][7] << 16);
        *reinterpret_cast<uint4*>(o) = pk;
      } else if (m[s]) {
#pragma unroll
        for (int j = 0; j < V; ++j)
          if ((m[s] >> j) & 1u) o[j] = (int16_t)v[s][j];
      }
    }
  }
};

// RLE booleans (RleValueDecoder<bool>, decoding.rs:323-384), one byte per value.
struct TxBool {
  static constexpr int V = 16;
  uint8_t* out;
  template <int NG>
  __device__ void put(uint32_t g0, uint32_t stride, const uint32_t (&v)[NG][V], const uint32_t (&m)[NG]) {
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      uint8_t* o = out + g0 + (uint32_t)s * stride;
      if (m[s] == 0xFFFFu) {
        uint32_t q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          q[k] = (v[s][4 * k] & 0xFFu) | ((v[s][4 * k + 1] & 0xFFu) << 8) |
                 ((v[s][4 * k + 2] & 0xFFu) << 16) | ((v[s][4 * k + 3] & 0xFFu) << 24);
        *reinterpret_cast<uint4*>(o) = make_uint4(q[0], q[1], q[2], q[3]);
      } else if (m[s]) {
#pragma unroll
        for (int j = 0; j < V; ++j)
          if ((m[s] >> j) & 1u) o[j] = (uint8_t)v[s][j];
      }
    }
  }
};

// Dictionary gather (DictDecoder::get -> RleDecoder::get_batch_with_dict, decoding.rs:303-315,
// rle.rs:437-487) for fixed-width values of ES bytes: every gather of the thread's 16 outputs
// is issued before the first store. An index past the dictionary is the reference's panic.
template <int ES>
struct TxDictTraits {
  static constexpr int V = ES == 8 ? 2 : ES == 4 ? 4 : ES == 12 ? 4 : 16;
};

template <int ES>
struct TxDict {
  static constexpr int V = TxDictTraits<ES>::V;
  const uint8_t* dict;  // PLAIN dictionary page payload
  uint32_t ndict;
  bool aligned;         // dict payload aligned to its value size
  uint8_t* out;         // page output base
  int32_t err;

  template <int NG>
  __device__ void put(uint32_t g0, uint32_t stride, const uint32_t (&v)[NG][V], const uint32_t (&m)[NG]) {
    if constexpr (ES == 8 || ES == 4) {
      using T = typename std::conditional<ES == 8, uint64_t, uint32_t>::type;
      T x[NG][V];
#pragma unroll
      for (int s = 0; s < NG; ++s)
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const bool want = (m[s] >> j) & 1u;
          const uint32_t idx = v[s][j];
          const bool ok = want && idx < ndict;
          err |= (want && !ok) ? ST_PANIC : 0;
          T t = 0;
          if (ok) {
            if (aligned) {
              t = reinterpret_cast<const T*>(dict)[idx];
            } else {
              const uint8_t* p = dict + (uint64_t)idx * ES;
#pragma unroll
              for (int k = 0; k < ES; ++k) t |= (T)p[k] << (8 * k);
            }
          }
          x[s][j] = t;
        }
#pragma unroll
      for (int s = 0; s < NG; ++s) {
        T* o = reinterpret_cast<T*>(out) + g0 + (uint64_t)s * stride;
        if (m[s] == (1u << V) - 1u) {
          if constexpr (ES == 8)
            *reinterpret_cast<uint4*>(o) = make_uint4((uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32),
                                                      (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32));
          else
            *reinterpret_cast<uint4*>(o) = make_uint4(x[s][0], x[s][1], x[s][2], x[s][3]);
        } else if (m[s]) {
#pragma unroll
          for (int j = 0; j < V; ++j)
            if ((m[s] >> j) & 1u) o[j] = x[s][j];
        }
      }
    } else {  // 1-byte (BOOLEAN) and 12-byte (INT96) values: byte copies
#pragma unroll
      for (int s = 0; s < NG; ++s)
#pragma unroll
        for (int j = 0; j < V; ++j) {
          if (!((m[s] >> j) & 1u)) continue;
          const uint32_t idx = v[s][j];
          if (idx >= ndict) {
            err = ST_PANIC;
            continue;
          }
          uint8_t* o = out + ((uint64_t)g0 + (uint64_t)s * stride + (uint32_t)j) * ES;
          const uint8_t* p = dict + (uint64_t)idx * ES;
          if (ES == 12 && aligned) {
            const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
            const uint32_t a = q[0], b = q[1], c = q[2];
            uint32_t* od = reinterpret_cast<uint32_t*>(o);
            od[0] = a;
            od[1] = b;
            od[2] = c;
          } else {
#pragma unroll
            for (int k = 0; k < ES; ++k) o[k] = p[k];
          }
        }
    }
  }
};

}  // namespace pqg
