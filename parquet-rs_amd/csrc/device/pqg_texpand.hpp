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

// Run holding page-relative output o: binary search over sm.start[0, nr). SM: any LDS layout
// with start[], info[] (run list) and stage[] (payload window) members.
template <class SM>
__device__ inline uint32_t tx_find(const SM& sm, uint32_t nr, uint32_t lgn, uint32_t o) {
  uint32_t a = 0;
  for (uint32_t step = lgn; step; step >>= 1)
    if (a + step < nr && sm.start[a + step] <= o) a += step;
  return a;
}

// Fast path for the V outputs [g, g + V): all inside the segment (caller checks), in at most
// two runs, bit-packed payload inside the LDS window (lim = staged bits). Values go to v;
// returns false when any of that does not hold (the slow path then produces the group).
template <int V, class SM>
__device__ inline bool tx_fast(const SM& sm, uint32_t nr, uint32_t lgn, uint32_t g,
                               uint32_t seg_hi, uint32_t w, uint32_t wm, uint32_t sb32,
                               uint32_t lim, uint32_t (&v)[V]) {
  const uint32_t a = tx_find(sm, nr, lgn, g);
  const uint32_t stA = sm.start[a], infA = sm.info[a];
  const uint32_t stB = sm.start[a + 1];
  const uint32_t infB = sm.info[a + 1 < nr ? a + 1 : a];
  const uint32_t stC = sm.start[a + 2 <= nr ? a + 2 : nr];
  bool ok = g + V <= stC && g + V <= seg_hi;
#pragma unroll
  for (int j = 0; j < V; ++j) {
    const uint32_t o = g + (uint32_t)j;
    const bool inB = o >= stB;
    const uint32_t inf = inB ? infB : infA;
    const uint32_t st = inB ? stB : stA;
    const bool rle = (inf & R_RLE) != 0;
    const uint32_t bit = (inf - sb32) * 8u + (o - st) * w;
    const bool in = rle || bit + w <= lim;
    ok = ok && in;
    const uint32_t wi = (in && !rle) ? bit >> 5 : 0u;
    const uint32_t x = __builtin_amdgcn_alignbit(sm.stage[wi + 1], sm.stage[wi], bit & 31u) & wm;
    v[j] = rle ? (inf & 0x7FFFFFFFu) : x;
  }
  return ok;
}

// One output, any case: LDS window or global memory (64-bit offsets).
template <class SM>
__device__ inline uint32_t tx_one(const SM& sm, uint32_t nr, uint32_t lgn, uint32_t o,
                                  uint32_t w, uint32_t wm, uint32_t sb32, uint32_t lim,
                                  const uint8_t* __restrict__ blob, uint64_t blob_len, uint64_t S) {
  const uint32_t a = tx_find(sm, nr, lgn, o);
  const uint32_t st = sm.start[a], inf = sm.info[a];
  if (inf & R_RLE) return inf & 0x7FFFFFFFu;
  const uint32_t bit = (inf - sb32) * 8u + (o - st) * w;
  if (bit + w <= lim) {
    const uint32_t wi = bit >> 5;
    return __builtin_amdgcn_alignbit(sm.stage[wi + 1], sm.stage[wi], bit & 31u) & wm;
  }
  const uint64_t b64 = (uint64_t)inf * 8ull + (uint64_t)(o - st) * (uint64_t)w;
  return (uint32_t)(gload_u64(blob, blob_len, S + (b64 >> 3)) >> (b64 & 7)) & wm;
}

// Expand outputs [seg_lo, seg_hi) of the tile starting at page-relative output lo. Groups
// that take the fast path are handed to the emitter E::PG at a time (put: all-or-nothing
// masks); the others are produced one output at a time (put1) in a rolled loop.
template <class E, class SM>
__device__ inline void tx_range(const SM& sm, uint32_t nr, uint32_t lo, uint32_t seg_lo,
                                uint32_t seg_hi, uint32_t w, uint32_t sb32, uint32_t staged,
                                bool wide, const uint8_t* __restrict__ blob, uint64_t blob_len,
                                uint64_t S, E& em) {
  constexpr int V = E::V;
  constexpr int NG = (int)TX_PER / V;
  constexpr int PG = E::PG < NG ? E::PG : NG;
  constexpr uint32_t stride = WG * V;
  const uint32_t wm = w >= 32 ? 0xFFFFFFFFu : ((1u << w) - 1u);
  const uint32_t lgn = nr > 1 ? 1u << (31 - __builtin_clz(nr - 1)) : 0u;
  const uint32_t lim = wide ? 0u : staged * 8u;
  const uint32_t g0 = lo + threadIdx.x * (uint32_t)V;
  uint32_t slow = 0;  // groups left to the slow path
#pragma unroll
  for (int c = 0; c < NG; c += PG) {
    uint32_t v[PG][V];
    uint32_t m[PG];
#pragma unroll
    for (int s = 0; s < PG; ++s) {
      const uint32_t g = g0 + (uint32_t)(c + s) * stride;
      const bool inside = g >= seg_lo && g < seg_hi;
      const bool f = inside && tx_fast<V>(sm, nr, lgn, g, seg_hi, w, wm, sb32, lim, v[s]);
      m[s] = f ? (V == 32 ? 0xFFFFFFFFu : (1u << V) - 1u) : 0u;
      if (!f && g + V > seg_lo && g < seg_hi) slow |= 1u << (c + s);
    }
    em.template put<PG>(g0 + (uint32_t)c * stride, stride, v, m);
  }
#pragma unroll 1
  while (slow) {
    const int s = __builtin_ctz(slow);
    slow &= slow - 1;
    const uint32_t g = g0 + (uint32_t)s * stride;
#pragma unroll 1
    for (uint32_t j = 0; j < (uint32_t)V; ++j) {
      const uint32_t o = g + j;
      if (o < seg_lo || o >= seg_hi) continue;
      em.put1(o, tx_one(sm, nr, lgn, o, w, wm, sb32, lim, blob, blob_len, S));
    }
  }
}

// Loads of one tile in flight: run records and the payload window (single-batch tiles).
struct TileLoad {
  uint2 r0, r1;
  uint4 pv[TX_CHUNKS];
  uint32_t nchunks;
  uint64_t A0;
};

__device__ inline bool tx_wide(const QDesc& d) { return d.slen >= (1u << 28); }  // bit offsets could wrap

__device__ inline void tx_issue(const uint8_t* __restrict__ blob, uint64_t blob_len, const QDesc& d,
                                const uint2* __restrict__ runs, TileLoad& f) {
  const uint32_t tid = threadIdx.x;
  f.r0 = f.r1 = make_uint2(0u, 0u);
  f.nchunks = 0;
  f.A0 = d.S;
  if (!d.qhi || d.rec == RUN_REWALK) return;
  if (d.kind != LK_BIT_PACKED) {
    if (tid < d.nrec) f.r0 = runs[d.rec + tid];
    if (tid + WG < d.nrec) f.r1 = runs[d.rec + tid + WG];
  }
  if (d.bhi && !tx_wide(d)) {
    const uint64_t A0 = (d.S + d.blo) & ~15ull;
    uint64_t A1 = d.S + (uint64_t)d.bhi;
    if (A1 > A0 + TX_STAGE) A1 = A0 + TX_STAGE;
    const uint32_t nchunks = (uint32_t)((A1 - A0 + 15) / 16);
    const bool fast = A0 + (uint64_t)nchunks * 16 <= blob_len;
#pragma unroll
    for (int k = 0; k < TX_CHUNKS; ++k) {
      const uint32_t c = tid + (uint32_t)(k * WG);
      if (c < nchunks) {
        const uint64_t a = A0 + (uint64_t)c * 16;
        f.pv[k] = fast ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
      }
    }
    f.A0 = A0;
    f.nchunks = nchunks;
  }
}

__device__ inline uint32_t tx_nrec(const QDesc& d) { return d.kind == LK_BIT_PACKED ? 1u : d.nrec; }

__device__ inline void tx_install(const QDesc& d, const TileLoad& f, TileSmem& sm) {
  const uint32_t tid = threadIdx.x;
  const uint32_t nr = tx_nrec(d);
  if (d.kind == LK_BIT_PACKED) {  // one header-less run from output 0
    if (tid == 0) {
      sm.start[0] = 0;
      sm.info[0] = 0;
    }
  } else {
    if (tid < nr) {
      sm.start[tid] = f.r0.x;
      sm.info[tid] = f.r0.y;
    }
    if (tid + WG < nr) {
      sm.start[tid + WG] = f.r1.x;
      sm.info[tid + WG] = f.r1.y;
    }
  }
  if (tid == 0) {
    sm.start[nr] = d.qhi;
    sm.start[nr + 1] = d.qhi;
  }
#pragma unroll
  for (int k = 0; k < TX_CHUNKS; ++k) {
    const uint32_t c = tid + (uint32_t)(k * WG);
    if (c < f.nchunks) reinterpret_cast<uint4*>(sm.stage)[c] = f.pv[k];
  }
  if (tid < 16) sm.stage[f.nchunks * 4 + tid] = 0;
}

// Tile with more runs than the index kept: wave 0 re-walks from the checkpoint in batches,
// payload read from global memory. Barriers inside; LDS free on entry and on exit.
template <class E>
__device__ inline void tx_rewalk(const uint8_t* __restrict__ blob, uint64_t blob_len, const QDesc& d,
                                 TileSmem& sm, E& em) {
  const uint32_t tid = threadIdx.x;
  const uint32_t lo = d.qlo, hi = d.qhi, w = d.w;
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
  __syncthreads();
}

// Tile t with the whole workgroup: no state carried between tiles, so the fewest live
// registers; the hardware overlaps tiles across workgroups instead.
template <class M>
__device__ inline void tile_one(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                const QDesc* __restrict__ desc, uint32_t t,
                                const uint2* __restrict__ runs, TileSmem& sm, M& mk) {
  const QDesc d = desc[t];
  auto em = mk.make(d);
  if (d.qhi && d.rec != RUN_REWALK) {
    TileLoad f;
    tx_issue(blob, blob_len, d, runs, f);
    tx_install(d, f, sm);
    __syncthreads();
    tx_range(sm, tx_nrec(d), d.qlo, d.qlo, d.qhi, d.w, (uint32_t)(f.A0 - d.S), f.nchunks * 16u,
             tx_wide(d), blob, blob_len, d.S, em);
  } else if (d.qhi) {
    tx_rewalk(blob, blob_len, d, sm, em);
  }
  mk.done(d, t, em);
}

// ------------------------------------------------------------------------------ emitters
//
// put<NG>(g0, stride, v, m): group s covers page-relative outputs [g0 + s*stride, + V), its
// values in v[s], m[s] the mask of outputs to write.

// Def/rep levels as int16 (column/reader.rs:162-163); def levels also count the values
// read_batch will ask for (def == max_def, column/reader.rs:212-226).
struct TxLevels {
  static constexpr int V = 8;
  static constexpr int PG = 2;
  gptr<int16_t> out;  // page output base
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
      gptr<int16_t> o = out + g0 + (uint32_t)s * stride;
      if (m[s]) {
        uint4 pk;
        pk.x = (v[s][0] & 0xFFFFu) | (v[s][1] << 16);
        pk.y = (v[s][2] & 0xFFFFu) | (v[s][3] << 16);
        pk.z = (v[s][4] & 0xFFFFu) | (v[s][5] << 16);
        pk.w = (v[s][6] & 0xFFFFu) | (v[s][7] << 16);
        gst16(reinterpret_cast<gptr<uint8_t>>(o), pk);
      }
    }
  }
  __device__ void put1(uint32_t o, uint32_t v) {
    if (count) nonnull += (int16_t)v == maxl ? 1u : 0u;
    out[o] = (int16_t)v;
  }
};

// RLE booleans (RleValueDecoder<bool>, decoding.rs:323-384), one byte per value.
struct TxBool {
  static constexpr int V = 16;
  static constexpr int PG = 1;
  gptr<uint8_t> out;
  template <int NG>
  __device__ void put(uint32_t g0, uint32_t stride, const uint32_t (&v)[NG][V], const uint32_t (&m)[NG]) {
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      gptr<uint8_t> o = out + g0 + (uint32_t)s * stride;
      if (m[s]) {
        uint32_t q[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          q[k] = (v[s][4 * k] & 0xFFu) | ((v[s][4 * k + 1] & 0xFFu) << 8) |
                 ((v[s][4 * k + 2] & 0xFFu) << 16) | ((v[s][4 * k + 3] & 0xFFu) << 24);
        gst16(o, make_uint4(q[0], q[1], q[2], q[3]));
      }
    }
  }
  __device__ void put1(uint32_t o, uint32_t v) { out[o] = (uint8_t)v; }
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
  static constexpr int PG = ES == 8 ? 4 : 2;
  const uint8_t* dict;  // PLAIN dictionary page payload
  uint32_t ndict;
  bool aligned;         // dict payload aligned to its value size
  gptr<uint8_t> out;    // page output base
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
        gptr<T> o = reinterpret_cast<gptr<T>>(out) + g0 + (uint64_t)s * stride;
        if (m[s]) {
          if constexpr (ES == 8)
            gst16(reinterpret_cast<gptr<uint8_t>>(o), make_uint4((uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32),
                                                                 (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32)));
          else
            gst16(reinterpret_cast<gptr<uint8_t>>(o), make_uint4(x[s][0], x[s][1], x[s][2], x[s][3]));
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
          gptr<uint8_t> o = out + ((uint64_t)g0 + (uint64_t)s * stride + (uint32_t)j) * ES;
          const uint8_t* p = dict + (uint64_t)idx * ES;
          if (ES == 12 && aligned) {
            const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
            const uint32_t a = q[0], b = q[1], c = q[2];
            gptr<uint32_t> od = reinterpret_cast<gptr<uint32_t>>(o);
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
  __device__ void put1(uint32_t o, uint32_t idx) {
    if (idx >= ndict) {
      err = ST_PANIC;
      return;
    }
    gptr<uint8_t> d = out + (uint64_t)o * ES;
    const uint8_t* p = dict + (uint64_t)idx * ES;
    if ((ES == 4 || ES == 8) && aligned) {
      if constexpr (ES == 8) *reinterpret_cast<gptr<uint64_t>>(d) = *reinterpret_cast<const uint64_t*>(p);
      else *reinterpret_cast<gptr<uint32_t>>(d) = *reinterpret_cast<const uint32_t*>(p);
    } else {
#pragma unroll 1
      for (int k = 0; k < ES; ++k) d[k] = p[k];
    }
  }
};

// The same indices kept, not gathered: 16-bit entries into the tile's slot of an index buffer
// (outputs [lo, lo + RUN_TILE) of the tile; dictionaries of at most 65536 entries), for
// k_dict_win's gather through LDS windows. The range check (the reference's panic) stays here.
struct TxDictIdx {
  static constexpr int V = 8;  // one 16-byte store of indices per group
  static constexpr int PG = 2;
  gptr<uint16_t> slot;
  uint32_t lo;
  uint32_t ndict;
  int32_t err;

  template <int NG>
  __device__ void put(uint32_t g0, uint32_t stride, const uint32_t (&v)[NG][V], const uint32_t (&m)[NG]) {
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      uint32_t pk[4] = {0u, 0u, 0u, 0u};
#pragma unroll
      for (int j = 0; j < V; ++j) {
        const bool want = (m[s] >> j) & 1u;
        err |= (want && v[s][j] >= ndict) ? ST_PANIC : 0;
        pk[j >> 1] |= (v[s][j] & 0xFFFFu) << (16 * (j & 1));
      }
      const uint32_t g = g0 + (uint32_t)s * stride - lo;
      if (m[s] == 0xFFu) {
        gst16(reinterpret_cast<gptr<uint8_t>>(slot + g), make_uint4(pk[0], pk[1], pk[2], pk[3]));
      } else if (m[s]) {
#pragma unroll
        for (int j = 0; j < V; ++j)
          if ((m[s] >> j) & 1u) slot[g + j] = (uint16_t)v[s][j];
      }
    }
  }
  __device__ void put1(uint32_t o, uint32_t idx) {
    if (idx >= ndict) err = ST_PANIC;
    slot[o - lo] = (uint16_t)idx;
  }
};

}  // namespace pqg
