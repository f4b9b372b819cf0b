// pqg_runs.hpp — the general RLE/bit-packing hybrid decoder (rle.rs:320-509): index pass +
// tiled expand (pqg_texpand.hpp). It takes every stream: dictionary indices of any width, and
// the level / boolean streams the fast level path (pqg_levels.hip) hands back (malformed
// input, unusual header forms), reproducing every reference error on them.
//
//   index  (run_index, one wave per stream): walks the header chain of a page's stream inside
//          LDS-staged regions, checks everything the reference checks while reading
//          (Err / panic / endless loop), and writes per expand tile a
//          checkpoint (the header of the run holding the tile's first output) and the tile's
//          run records.
//   expand (pqg_texpand.hpp tile_one, one 256-thread workgroup per tile of RUN_TILE outputs,
//          all pages of the chunk in one grid; wave_expand below for byte-array dictionaries).
#pragma once
#include "pqg_device.hpp"

#ifndef PQG_IX_REG
#define PQG_IX_REG 32768
#endif

namespace pqg {

constexpr int IX_REG = PQG_IX_REG;            // index walker region (bytes)
constexpr int IX_WORDS = (IX_REG + 64) / 4;
constexpr uint32_t RF_BP = 1u, RF_EOF = 2u, RF_PANIC = 4u;
constexpr uint32_t R_RLE = 0x80000000u;

enum StreamSel : int { SS_DEF = 0, SS_REP = 1, SS_DICT = 2, SS_BOOL = 3 };

// One hybrid stream of one page.
struct Stream {
  uint64_t S;      // absolute blob offset of the stream
  uint32_t slen;   // stream bytes
  uint32_t n;      // outputs the reader asks for
  int w;           // bit width
  int kind;        // LK_RLE (hybrid) / LK_BIT_PACKED (header-less, levels.rs:203-209)
  uint64_t out;    // global index of the page's first output
  int32_t err;     // error found before any run is read
};

__device__ inline uint32_t rd_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Stream `sel` of page pw; false if the page has none.
//  SS_DEF / SS_REP: level streams located by k_prepare (levels.rs:191-233);
//  SS_DICT: RLE_DICTIONARY indices, [bit width byte][hybrid] (decoding.rs:292-300);
//  SS_BOOL: RleValueDecoder<Bool>, [i32 length][hybrid, w = 1] (decoding.rs:339-349).
__device__ inline bool get_stream(const uint8_t* blob, const PageWork& pw, int sel,
                                  const ColumnParams& cp, Stream& s) {
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return false;
  s.err = 0;
  s.kind = LK_RLE;
  if (sel == SS_DEF || sel == SS_REP) {
    const int kind = sel == SS_DEF ? pw.def_kind : pw.rep_kind;
    if (kind == LK_NONE || !(sel == SS_DEF ? cp.want_def : cp.want_rep)) return false;
    s.kind = kind;
    s.S = pw.base + (sel == SS_DEF ? pw.def_off : pw.rep_off);
    s.slen = sel == SS_DEF ? pw.def_bytes : pw.rep_bytes;
    s.w = sel == SS_DEF ? cp.def_bit_width : cp.rep_bit_width;
    s.n = pw.num_values;
    s.out = pw.level_out;
    return true;
  }
  s.n = (uint32_t)pw.nonnull;
  s.out = pw.value_out;
  if (sel == SS_DICT) {
    if (pw.encoding != E_RLE_DICTIONARY) return false;
    if (pw.val_bytes < 1) {  // data.as_ref()[0]
      s.err = ST_PANIC;
      s.S = pw.base + pw.val_off;
      s.slen = 0;
      s.w = 0;
      return true;
    }
    s.w = blob[pw.base + pw.val_off];
    s.S = pw.base + pw.val_off + 1;
    s.slen = pw.val_bytes - 1;
    return true;
  }
  // SS_BOOL
  if (pw.encoding != E_RLE) return false;
  s.w = 1;
  s.S = pw.base + pw.val_off + 4;
  s.slen = 0;
  if (pw.val_bytes < 4) {
    s.err = ST_PANIC;
    return true;
  }
  const int32_t sz = (int32_t)rd_le32(blob + pw.base + pw.val_off);
  if (sz < 0 || 4ull + (uint64_t)(uint32_t)sz > pw.val_bytes) {  // data.range(4, size) assert
    s.err = ST_PANIC;
    return true;
  }
  s.slen = (uint32_t)sz;
  return true;
}

// ------------------------------------------------------------------------------ header parse

// Slow, general header parse (varints up to 10 bytes, values up to 8 bytes) from an LDS
// image; the reference encoder never needs it (1-2 byte headers, <= 4-byte values).
__device__ inline void run_parse_slow(const uint32_t* region, uint32_t ridx, uint32_t q,
                                      uint32_t slen, int w, uint32_t& nxt, uint32_t& cnt,
                                      uint32_t& inf, uint32_t& flg) {
  uint64_t ind = 0;
  int vlen = 0;
  bool complete = false;
#pragma unroll 1
  for (int k = 0; k < 10; ++k) {
    if (q + (uint32_t)k >= slen) break;
    const uint32_t b = lbyte(region, ridx + k);
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
    flg = (vlen == 10 && q + 10 < slen) ? RF_PANIC : RF_EOF;
    return;
  }
  const uint32_t p = q + (uint32_t)vlen;
  if (ind & 1) {
    cnt = (uint32_t)((uint64_t)((int64_t)ind >> 1) * 8ull);
    inf = p;
    const uint64_t nx = (uint64_t)p + (((uint64_t)cnt * (uint64_t)w) >> 3);
    nxt = nx > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)nx;
    flg = RF_BP;
  } else {
    cnt = (uint32_t)((int64_t)ind >> 1);
    const uint32_t vb = ((uint32_t)w + 7u) >> 3;
    if (vb > 8 || (uint64_t)p + vb > slen) {
      flg = RF_PANIC;
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

// Header at stream position q (LDS index ridx): one-byte headers (every header the reference
// writes for runs < 64 values or <= 63 groups) take a short path; longer varints a branchless
// LEB128 decode of a 16-byte window; anything unusual the slow path. (rle.rs:490-508,
// bit_util.rs:538-580)
__device__ inline void run_parse(const uint32_t* region, uint32_t ridx, uint32_t q, uint32_t slen,
                                 int w, uint32_t& nxt, uint32_t& cnt, uint32_t& inf,
                                 uint32_t& flg) {
  const uint32_t avail = q < slen ? slen - q : 0u;
  const uint32_t vb = ((uint32_t)w + 7u) >> 3;
  const uint64_t lo8 = lload_u64(region, ridx);
  const uint32_t b0 = (uint32_t)lo8 & 0xFFu;
  if (!(b0 & 0x80u) && avail >= 1u + ((b0 & 1u) ? 0u : vb) && vb <= 4u) {
    const uint32_t p = q + 1u;
    if (b0 & 1u) {
      cnt = (b0 >> 1) * 8u;
      inf = p;
      nxt = p + ((cnt * (uint32_t)w) >> 3);
      flg = RF_BP;
    } else {
      cnt = b0 >> 1;
      uint32_t v = (uint32_t)(lo8 >> 8);
      if (vb < 4) v &= (1u << (8 * vb)) - 1u;
      inf = v > 0x7FFFFFFFu ? 0x7FFFFFFFu : v;
      nxt = p + vb;
      flg = 0;
    }
    return;
  }
  const uint64_t hi8 = lload_u64(region, ridx + 8);
  const uint64_t lo = lo8;
  const uint64_t t = ~lo & 0x8080808080808080ull;
  const uint32_t vlen = t ? ((uint32_t)__builtin_ctzll(t) >> 3) + 1u : 9u;
  uint64_t y = lo & 0x7F7F7F7F7F7F7F7Full;
  if (vlen < 8) y &= (1ull << (8 * vlen)) - 1ull;
  y = (y & 0x007F007F007F007Full) | ((y & 0x7F007F007F007F00ull) >> 1);
  y = (y & 0x00003FFF00003FFFull) | ((y & 0x3FFF00003FFF0000ull) >> 2);
  const uint64_t ind = (y & 0x000000000FFFFFFFull) | ((y & 0x0FFFFFFF00000000ull) >> 4);
  const uint32_t p = q + vlen;
  const bool bp = (ind & 1) != 0;
  const uint32_t vs = vlen * 8u;
  uint64_t v = (vs < 64) ? ((lo >> vs) | (vs ? (hi8 << (64 - vs)) : 0ull)) : hi8;
  if (vb < 8) v &= (1ull << (8 * vb)) - 1ull;
  const bool fast = t != 0 && vlen + (bp ? 0u : vb) <= avail && (bp || (vb <= 8 && vlen + vb <= 9));
  if (fast) {
    if (bp) {
      cnt = (uint32_t)((ind >> 1) * 8ull);
      inf = p;
      const uint64_t nx = (uint64_t)p + (((uint64_t)cnt * (uint64_t)w) >> 3);
      nxt = nx > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)nx;
      flg = RF_BP;
    } else {
      cnt = (uint32_t)(ind >> 1);
      inf = v > 0x7FFFFFFFull ? 0x7FFFFFFFu : (uint32_t)v;
      nxt = p + vb;
      flg = 0;
    }
  } else {
    run_parse_slow(region, ridx, q, slen, w, nxt, cnt, inf, flg);
  }
}

// Header parse straight from global memory (walks that leave their staged window).
__device__ inline void run_parse_global(const uint8_t* blob, uint64_t blob_len, uint64_t S,
                                        uint32_t q, uint32_t slen, int w, uint32_t& nxt,
                                        uint32_t& cnt, uint32_t& inf, uint32_t& flg) {
  uint32_t tmp[8];
  const uint64_t a = S + q;
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const uint64_t x = a + 4u * k;
    tmp[k] = gbyte(blob, blob_len, x) | (gbyte(blob, blob_len, x + 1) << 8) |
             (gbyte(blob, blob_len, x + 2) << 16) | (gbyte(blob, blob_len, x + 3) << 24);
  }
  tmp[6] = tmp[7] = 0;
  run_parse(tmp, 0, q, slen, w, nxt, cnt, inf, flg);
}

// ------------------------------------------------------------------------------ density probe
// Whole wave: the chain of a level stream from offset 0 over its first KiB, held in VGPRs (16
// bytes per lane; header bytes read by v_readlane, so a hop costs a few scalar cycles). True when
// its first 64 headers lie within 1 KiB (short RLE runs: the level path's segment walk would stop
// there as dense), i.e. the stream belongs to the level path's window kernels (pqg_levels.hip).
// S, slen, w must be wave-uniform; the caller checks slen >= 1088.
__device__ inline uint32_t probe_dw(const uint32_t (&d)[4], uint32_t i) {  // dword i of the KiB (uniform)
  const int l = (int)(i >> 2);
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)d[0], l), b = (uint32_t)__builtin_amdgcn_readlane((int)d[1], l),
                 c = (uint32_t)__builtin_amdgcn_readlane((int)d[2], l), e = (uint32_t)__builtin_amdgcn_readlane((int)d[3], l);
  const uint32_t k = i & 3u;
  return k == 0 ? a : k == 1 ? b : k == 2 ? c : e;
}

constexpr uint32_t PROBE_SPAN = 1024;  // 64 headers within fewer bytes: dense

__device__ inline bool lv_probe_dense(const uint8_t* __restrict__ blob, uint64_t blob_len, uint64_t S, uint32_t w) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t A = S & ~15ull;
  const uint32_t sb = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(S - A));
  const uint64_t a = A + (uint64_t)lane * 16u;
  const uint4 v = a + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
  const uint32_t d[4] = {v.x, v.y, v.z, v.w};
  const uint32_t vb = (w + 7u) >> 3;
  uint32_t q = 0, k = 0;
  while (k < 64u && q + 20u < PROBE_SPAN) {  // header bytes q .. q + 3 (+ alignment) stay in the staged KiB
    const uint32_t r = q + sb;
    const uint32_t x = __builtin_amdgcn_alignbit(probe_dw(d, (r >> 2) + 1u), probe_dw(d, r >> 2), (r & 3u) * 8u);
    const uint32_t c0 = (x >> 7) & 1u, c1 = (x >> 15) & 1u, c2 = (x >> 23) & 1u, c3 = x >> 31;
    const uint32_t c01 = c0 & c1, c012 = c01 & c2;
    if (c012 & c3) break;  // a varint the fast parse does not take
    const uint32_t hl = 1u + c0 + c01 + c012;
    const uint32_t h = (x & 0x7Fu) | (c0 ? ((x >> 1) & 0x3F80u) : 0u) | (c01 ? ((x >> 2) & 0x1FC000u) : 0u) |
                       (c012 ? ((x >> 3) & 0xFE00000u) : 0u);
    q += (h & 1u) ? hl + (h >> 1) * w : hl + vb;
    ++k;
  }
  return k == 64u && q < PROBE_SPAN;
}

// ------------------------------------------------------------------------------ index pass

struct IndexSmem {
  uint32_t region[IX_WORDS];
};

constexpr int IX_CHUNKS = (IX_REG + 64) / 16;  // 16-byte chunks per region (64-byte overlap)
constexpr int IX_PF = (IX_CHUNKS + 63) / 64;     // 16-byte loads per lane per region

// Region r of the walker's grid: bytes [G + r*IX_REG, G + (r+1)*IX_REG + 64), loaded by the
// whole wave into registers (one wave-instruction per KiB, all in flight together).
__device__ inline void ix_fetch(const uint8_t* __restrict__ blob, uint64_t blob_len, uint64_t A0,
                                uint32_t lane, uint4 (&v)[IX_PF]) {
  if (A0 + IX_REG + 64 <= blob_len) {
#pragma unroll
    for (int k = 0; k < IX_PF; ++k) {
      const uint32_t c = lane + 64u * (uint32_t)k;
      if (k < IX_PF - 1 || c < (uint32_t)IX_CHUNKS) v[k] = *reinterpret_cast<const uint4*>(blob + A0 + (uint64_t)c * 16);
    }
  } else {  // blob tail: guarded byte loads (unrolled: v must stay in registers)
#pragma unroll
    for (int k = 0; k < IX_PF; ++k) {
      const uint32_t c = lane + 64u * (uint32_t)k;
      if (k < IX_PF - 1 || c < (uint32_t)IX_CHUNKS) v[k] = gload_u128_tail(blob, blob_len, A0 + (uint64_t)c * 16);
    }
  }
}

__device__ inline void ix_install(uint32_t* region, uint32_t lane, const uint4 (&v)[IX_PF]) {
#pragma unroll
  for (int k = 0; k < IX_PF; ++k) {
    const uint32_t c = lane + 64u * (uint32_t)k;
    if (k < IX_PF - 1 || c < (uint32_t)IX_CHUNKS) reinterpret_cast<uint4*>(region)[c] = v[k];
  }
}

__device__ inline uint32_t rfl(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }

// True in exactly one workgroup of the grid, the last to arrive here, after every workgroup's
// earlier global writes are visible to it: lets a one-workgroup pass that depends on the whole
// grid (a scan over pages) run in the grid's last workgroup instead of its own launch. Every
// workgroup of the grid must call it (no early exit before it); the ticket counter (zeroed once
// at allocation) is reset by the last workgroup for the next launch using it.
__device__ inline bool last_workgroup(uint32_t* ctr) {
  __shared__ uint32_t last_s;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();  // this workgroup's writes before its ticket
    const uint32_t t = atomicAdd(ctr, 1u);
    last_s = t == gridDim.x * gridDim.y * gridDim.z - 1u;
    if (last_s) atomicExch(ctr, 0u);
  }
  __syncthreads();
  if (last_s) __threadfence();  // acquire: the other workgroups' writes (no stale cache lines)
  return last_s != 0;
}

// One batch of k <= 64 consecutive headers of the chain (lane l: header at stream offset posv,
// staged at region index posv - rbase): parse, prefix-sum output counts, make every check the
// reference makes while reading them and write the run records, tile checkpoints and per-tile
// run counts. Headers whose first output is at or past n are not read by the reference and are
// ignored. Returns a status (0: fine); cy carries the position in the output across batches.
struct IxCarry {
  uint32_t produced;    // outputs before the next batch's first header
  uint32_t carry_tile;  // tile of output `produced`
  uint32_t carry_j;     // records already written for carry_tile
};

// full != 0: every header of the batch is the writer's full bit-packed run (one byte 0x7F: 63
// groups, 504 outputs, payload right after it), read by the walker's fast-forward, not staged.
__device__ inline int32_t ix_batch(const uint32_t* region, uint32_t rbase, uint32_t posv, uint32_t k,
                                   uint32_t slen, uint32_t n, uint32_t w, RunCkpt* __restrict__ ck,
                                   uint2* __restrict__ runs, uint32_t* __restrict__ nruns, IxCarry& cy,
                                   bool full = false) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t lanes_below = (1ull << lane) - 1ull;
  const uint32_t produced = cy.produced, carry_tile = cy.carry_tile, carry_j = cy.carry_j;
  const bool in0 = lane < k;
  uint32_t nx, cnt = 0, inf = 0, flg = 0;
  if (in0) {
    if (full) {
      cnt = 504u;
      inf = posv + 1u;
      flg = RF_BP;
    } else {
      run_parse(region, posv - rbase, posv, slen, (int)w, nx, cnt, inf, flg);
    }
  }
  // exclusive scan of counts
  uint64_t incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += y;
  }
  const uint64_t before = (uint64_t)produced + incl - cnt;
  const bool in = in0 && before < n;
  const uint32_t need = before >= n ? 0u : (uint32_t)((uint64_t)cnt < n - before ? cnt : n - before);
  const bool bp = (flg & RF_BP) != 0;
  int32_t e = 0;
  if (in) {
    if (flg & (RF_EOF | RF_PANIC)) e = (flg & RF_PANIC) ? ST_PANIC : ST_EOF;
    else if (need && bp && w > 32) e = ST_PANIC;  // BitReader::get_batch asserts num_bits <= 32
    else if (need && bp && (uint64_t)inf * 8ull + (uint64_t)need * w > (uint64_t)slen * 8ull)
      e = ST_EOF;  // truncated bit-packed run: the reference spins (A.4)
  }
  const uint64_t emask = __ballot(e != 0);
  if (emask) return __shfl(e, __builtin_ctzll(emask), 64);
  // records: lanes whose run yields outputs
  const bool valid = in && need > 0;
  const uint64_t V = __ballot(valid);
  const uint32_t tile = (uint32_t)(before / RUN_TILE);
  const uint32_t end_level = (uint32_t)before + need;          // one past the run's last output
  const uint32_t end_tile = (end_level - 1u) / RUN_TILE;        // tile of its last output
  // previous valid lane (its tile decides whether this lane starts a tile group)
  const uint64_t vb_below = V & lanes_below;
  const int prev = vb_below ? 63 - __builtin_clzll(vb_below) : -1;
  const uint32_t prev_tile = __shfl(tile, prev < 0 ? 0 : prev, 64);
  const bool head = valid && (prev < 0 || prev_tile != tile);
  const uint64_t H = __ballot(head);
  const uint64_t hb = H & (lanes_below | (1ull << lane));
  const int hl = hb ? 63 - __builtin_clzll(hb) : 0;             // head lane of this lane's group
  const uint32_t rank = (uint32_t)__builtin_popcountll(V & lanes_below & ~((1ull << hl) - 1ull));
  const uint32_t head_before = __shfl((uint32_t)before, hl, 64);
  const uint32_t base = tile == carry_tile ? carry_j : (head_before > tile * RUN_TILE ? 1u : 0u);
  const uint32_t j = base + rank;
  const uint32_t info = bp ? inf : (R_RLE | (inf > 0x7FFFFFFFu ? 0x7FFFFFFFu : inf));
  if (valid) {
    if (j == 0) ck[tile] = RunCkpt{posv, (uint32_t)before};
    if (j < RUN_CAPT) runs[(uint64_t)tile * RUN_CAPT + j] = make_uint2((uint32_t)before, info);
    const bool done_tile = end_tile > tile || end_level == (tile + 1) * RUN_TILE || end_level >= n;
    if (done_tile) nruns[tile] = j + 1;
    for (uint32_t t = tile + 1; t <= end_tile; ++t) {  // the run continues into later tiles
      ck[t] = RunCkpt{posv, (uint32_t)before};
      runs[(uint64_t)t * RUN_CAPT] = make_uint2((uint32_t)before, info);
      if (t < end_tile || end_level == (t + 1) * RUN_TILE || end_level >= n) nruns[t] = 1;
    }
  }
  // carry to the next batch (from the last valid lane)
  if (V) {
    const int L = 63 - __builtin_clzll(V);
    const uint32_t lt = rfl(__shfl(tile, L, 64));
    const uint32_t lj = rfl(__shfl(j, L, 64));
    const uint32_t le = rfl(__shfl(end_level, L, 64));
    const uint32_t let = rfl(__shfl(end_tile, L, 64));
    const uint32_t nt = le / RUN_TILE;
    cy.produced = le;
    cy.carry_tile = nt;
    cy.carry_j = (let == nt) ? (lt == nt ? lj + 1 : 1u) : 0u;
  }
  return 0;
}

// Walks stream s of one page with one wave and writes, per expand tile k of the stream:
// ck[k] = header of the run holding the tile's first output; runs[k*RUN_CAPT + j] = the tile's
// runs (page-relative first output, RLE value | payload offset); nruns[k] = their count
// (> RUN_CAPT: records incomplete, the expand pass re-walks the tile). Every check the
// reference makes while reading the stream is made here. Returns a status.
//
// The serial part is reduced to the header chain itself: a scalar loop follows up to 64
// headers (one LDS read, a few SALU ops and a v_writelane per hop), then the 64 lanes parse
// those headers in parallel, prefix-sum their output counts, check them and write records,
// checkpoints and counts together.
__device__ inline int32_t run_index(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                    const Stream& s, RunCkpt* __restrict__ ck,
                                    uint2* __restrict__ runs, uint32_t* __restrict__ nruns,
                                    IndexSmem& sm, uint64_t* stamps = nullptr) {
  const uint32_t lane = threadIdx.x & 63;
  // diagnostics (PQG_DEBUG bit 5): s_memtime cycles in region fetches, hop loops, batches
  uint64_t t_fetch = 0, t_hop = 0, t_batch = 0, t0 = 0;
  auto stamp = [&](uint64_t& acc) {
    if (stamps) {
      const uint64_t t1 = __builtin_amdgcn_s_memtime();
      acc += t1 - t0;
      t0 = t1;
    }
  };
  auto flush = [&]() {
    if (stamps && lane == 0)
      *reinterpret_cast<uint4*>(stamps) = make_uint4((uint32_t)t_fetch, (uint32_t)t_hop, (uint32_t)t_batch, 0u);
  };
  if (stamps) t0 = __builtin_amdgcn_s_memtime();
  if (s.err) return s.err;
  const uint32_t n = s.n;
  if (n == 0) return 0;
  const uint32_t w = (uint32_t)s.w;
  if (s.kind == LK_BIT_PACKED) {  // one header-less run (levels.rs:203-209)
    if ((uint64_t)n * (uint64_t)w > (uint64_t)s.slen * 8ull) return ST_EOF;
    if (w > 32) return ST_PANIC;
    return 0;
  }
  const uint64_t S = s.S;
  const uint32_t slen = s.slen;
  const uint64_t G = S & ~15ull;            // region grid origin
  const uint32_t off0 = (uint32_t)(S - G);  // stream byte 0 in grid coordinates
  const uint32_t vb = (w + 7u) >> 3;
  const uint32_t nregions = (off0 + slen + IX_REG - 1) / IX_REG;
  uint4 pf[IX_PF];
  uint32_t cur_r = 0xFFFFFFFFu, pf_r = 0xFFFFFFFFu;
  uint32_t cur = 0;            // next header
  IxCarry cy{0u, 0u, 0u};
  const uint32_t& produced = cy.produced;
  const uint32_t P = 1u + 63u * w;  // stream bytes of the writer's full bit-packed run
  while (true) {
    if (cur >= slen) return ST_EOF;  // reload() finds no more data: the reference stalls (A.4)
    if (w > 2u && w <= 32u && slen - cur > P) {
      // fast-forward (wide indices: unique or high-cardinality values leave no RLE runs): lane l
      // reads the header byte l runs on; the prefix of full-run headers (0x7F) is the chain's
      // next headers, recorded in one batch without staging their bytes
      const uint32_t q = cur + lane * P;
      const bool hit = q < slen && blob[S + q] == 0x7Fu;
      const uint64_t m = __ballot(hit);
      const uint32_t run = ~m ? (uint32_t)__builtin_ctzll(~m) : 64u;
      if (run >= 2u) {
        const int32_t e = ix_batch(sm.region, 0u, q, run, slen, n, w, ck, runs, nruns, cy, true);
        if (e) return e;
        if (cy.produced >= n) {
          flush();
          return 0;
        }
        cur = rfl(cur + run * P);
        continue;
      }
    }
    const uint32_t r = (off0 + cur) / IX_REG;
    if (r != cur_r) {
      if (r != pf_r) ix_fetch(blob, blob_len, G + (uint64_t)r * IX_REG, lane, pf);
      ix_install(sm.region, lane, pf);
      cur_r = r;
      pf_r = 0xFFFFFFFFu;
      if (r + 1 < nregions) {  // prefetch the next region while this one is walked
        ix_fetch(blob, blob_len, G + (uint64_t)(r + 1) * IX_REG, lane, pf);
        pf_r = r + 1;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): region writes done (vmcnt untouched)
      __builtin_amdgcn_wave_barrier();
      stamp(t_fetch);
    }
    const uint32_t rbase = r * IX_REG - off0;  // stream offset of region byte 0
    // ---- hop loop: follow up to 64 headers inside this region (uniform, scalar). Sparse headers
    // (bit widths > 2) take one LDS read per hop. Dense ones: the 64 lanes first decode a header
    // at each of the 64 stream positions from the current one (one-byte form: next header and
    // output count); the chain then takes two v_readlane and a few SALU ops per hop until it
    // leaves those 64 bytes. Other header forms take run_parse.
    uint32_t posv = 0, k = 0;
    uint32_t acc = produced;  // < n before each add, so acc + min(cnt, n) < 2^32
    if (w > 2u) {  // sparse headers (runs of >= 64 bytes): one LDS read per hop
      while (k < 64) {
        if (cur >= slen || cur - rbase >= (uint32_t)IX_REG) break;
        const uint32_t rel = cur - rbase;
        const uint32_t wi = rel >> 2;
        const uint32_t x = rfl(__builtin_amdgcn_alignbyte(sm.region[wi + 1], sm.region[wi], rel & 3u));
        const uint32_t b0 = x & 0xFFu;
        uint32_t cnt, nxt;
        bool stop = false;
        if (!(b0 & 0x80u) && vb <= 3u) {
          const uint32_t half = b0 >> 1;
          if (b0 & 1u) {
            cnt = half << 3;
            nxt = cur + 1u + half * w;
          } else {
            cnt = half;
            nxt = cur + 1u + vb;
          }
        } else {
          uint32_t inf, flg;
          run_parse(sm.region, rel, cur, slen, (int)w, nxt, cnt, inf, flg);
          nxt = rfl(nxt);
          cnt = rfl(cnt);
          stop = (rfl(flg) & (RF_EOF | RF_PANIC)) != 0;  // the batch reports it
        }
        posv = lane == k ? cur : posv;  // v_cmp + v_cndmask
        ++k;
        acc += cnt < n ? cnt : n;
        cur = nxt;
        if (stop || acc >= n) break;
      }
    } else {  // dense headers: candidate windows
      bool stop = false;
      while (k < 64 && !stop && acc < n) {
        if (cur >= slen || cur - rbase >= (uint32_t)IX_REG) break;
        // candidate headers at cur + lane (one-byte form); ~0u marks any other form
        const uint32_t wbase = cur;
        uint32_t nxv, cnv;
        {
          const uint32_t q = cur + lane;
          const uint32_t rel = q - rbase;
          const uint32_t b0 = (q < slen && rel < (uint32_t)(IX_REG + 60)) ? lbyte(sm.region, rel) : 0x80u;
          const uint32_t half = b0 >> 1;
          const bool fast = !(b0 & 0x80u) && vb <= 3u;
          nxv = !fast ? 0xFFFFFFFFu : ((b0 & 1u) ? q + 1u + half * w : q + 1u + vb);
          cnv = (b0 & 1u) ? half << 3 : half;
        }
        // tight chain through the candidates: all exits folded into one test; headers stay
        // inside the region (its 64-byte overlap only serves their bytes)
        const uint32_t olim = (rbase + (uint32_t)IX_REG - wbase) < 64u ? rbase + (uint32_t)IX_REG - wbase : 64u;
        uint32_t o = 0;
        while (true) {
          const uint32_t nx = (uint32_t)__builtin_amdgcn_readlane((int)nxv, (int)o);
          if (nx == 0xFFFFFFFFu) break;
          const uint32_t cn = (uint32_t)__builtin_amdgcn_readlane((int)cnv, (int)o);
          posv = lane == k ? cur : posv;
          ++k;
          acc += cn < n ? cn : n;
          cur = nx;
          o = cur - wbase;
          if ((o >= olim) | (k >= 64u) | (acc >= n)) break;
        }
        if (k >= 64u || acc >= n || o >= olim) continue;  // batch full / done / window left
        // header at cur in another form
        if (cur >= slen || cur - rbase >= (uint32_t)IX_REG) break;
        uint32_t nxt, cnt, inf, flg;
        run_parse(sm.region, cur - rbase, cur, slen, (int)w, nxt, cnt, inf, flg);
        nxt = rfl(nxt);
        cnt = rfl(cnt);
        stop = (rfl(flg) & (RF_EOF | RF_PANIC)) != 0;  // the batch reports it
        posv = lane == k ? cur : posv;
        ++k;
        acc += cnt < n ? cnt : n;
        cur = nxt;
      }
    }
    stamp(t_hop);
    if (k == 0) continue;  // region boundary: reload
    // ---- batch: lane l re-parses header l
    {
      const int32_t e = ix_batch(sm.region, rbase, posv, k, slen, n, w, ck, runs, nruns, cy);
      if (e) return e;
    }
    stamp(t_batch);
    if (cy.produced >= n) {
      flush();
      return 0;
    }
  }
}

}  // namespace pqg

// ============================================================================ wave expand
//
// One independent wave per quarter tile (1024 outputs): no workgroup barriers, small LDS,
// so many waves per CU hide the two memory round trips each quarter costs (its tile
// descriptor, then its run records and payload bytes together).
namespace pqg {

constexpr uint32_t WX_OUT = RUN_TILE / 4;  // outputs per wave
constexpr int WX_STAGE = 4096;             // staged payload bytes per batch
constexpr int WX_RCAP = 256;               // runs per batch

struct WaveSmem {
  uint32_t stage[(WX_STAGE + 64) / 4];
  uint32_t start[WX_RCAP + 2];
  uint32_t info[WX_RCAP + 1];
  uint32_t fix[WX_OUT / 8];
  uint32_t ctl[4];
};

__device__ inline void wave_sync() {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes have landed
  __builtin_amdgcn_wave_barrier();
}

__device__ inline uint32_t wave_min_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, off, 64));
  return v;
}
__device__ inline uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
  return v;
}
__device__ inline uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
  return v;
}

// Expand the runs in sm.start/info[0, nr) (sm.start[nr] = end) over outputs
// [seg_lo, seg_hi) of the quarter [qlo, qlo + WX_OUT), payload staged from stream offset
// sbase (sb32 = low 32 bits) for `staged` bytes.
template <class Emit>
__device__ inline void wave_expand_batch(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                         uint64_t S, uint64_t out, uint32_t w, uint32_t qlo,
                                         uint32_t seg_lo, uint32_t seg_hi, uint32_t nr,
                                         uint64_t A0, uint32_t staged, WaveSmem& sm, Emit& emit) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t sb32 = (uint32_t)(A0 - S);
  const uint32_t wm = w >= 32 ? 0xFFFFFFFFu : ((1u << w) - 1u);
  const uint64_t wm64 = w >= 64 ? ~0ull : ((1ull << w) - 1ull);
  if (lane == 0) sm.ctl[1] = 0;
  wave_sync();
#pragma unroll 1
  for (int half = 0; half < 2; ++half) {
    const uint32_t g = qlo + (uint32_t)half * (WX_OUT / 2) + lane * 8u;
    if (g + 8 <= seg_lo || g >= seg_hi) continue;
    const uint32_t o0 = g < seg_lo ? seg_lo : g;
    uint32_t a = 0;
#pragma unroll
    for (uint32_t step = WX_RCAP / 2; step; step >>= 1)
      if (a + step < nr && sm.start[a + step] <= o0) a += step;
    const uint32_t stA = sm.start[a], infA = sm.info[a];
    const uint32_t stB = sm.start[a + 1];
    const uint32_t infB = sm.info[a + 1 < nr ? a + 1 : a];
    const uint32_t stC = sm.start[a + 2 <= nr ? a + 2 : nr];
    const uint32_t end = g + 8 < seg_hi ? g + 8 : seg_hi;
    bool fixup = end > stC;  // three or more runs
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t oj = g + (uint32_t)j;
      const bool inB = oj >= stB;
      const uint32_t inf = inB ? infB : infA;
      const uint32_t d = oj - (inB ? stB : stA);
      const uint32_t rel = inf - sb32;
      const uint32_t bit = rel * 8u + d * w;
      const bool rle = (inf & R_RLE) != 0;
      const bool ok = rle || (d < (1u << 20) && rel < staged && (bit >> 3) + 12u <= staged);
      const uint32_t byte = ok && !rle ? bit >> 3 : 0u;
      uint32_t val;
      if (w <= 24) val = (lload_u32(sm.stage, byte) >> (bit & 7)) & wm;
      else val = (uint32_t)(lload_u64(sm.stage, byte) >> (bit & 7)) & wm;
      val = rle ? (inf & 0x7FFFFFFFu) : val;
      const bool in = oj >= seg_lo && oj < seg_hi;
      fixup |= in && !ok;
      v[j] = in ? val : 0u;
    }
    if (fixup) {
      const uint32_t slot = atomicAdd(&sm.ctl[1], 1u);
      sm.fix[slot] = g;
      continue;
    }
    uint32_t mask = 0xFFu;
    if (g < seg_lo || g + 8 > seg_hi) {
      mask = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (g + j >= seg_lo && g + j < seg_hi) mask |= 1u << j;
    }
    emit(out + g, v, mask);
  }
  wave_sync();
  const uint32_t nfix = sm.ctl[1];
  for (uint32_t f = lane; f < nfix; f += 64) {  // general path, one lane per chunk
    const uint32_t g = sm.fix[f];
    const uint32_t o0 = g < seg_lo ? seg_lo : g;
    uint32_t r = 0;
#pragma unroll
    for (uint32_t step = WX_RCAP / 2; step; step >>= 1)
      if (r + step < nr && sm.start[r + step] <= o0) r += step;
    uint32_t st = sm.start[r], nst = sm.start[r + 1], inf = sm.info[r];
    uint32_t v[8];
    uint32_t mask = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t oj = g + (uint32_t)j;
      v[j] = 0;
      if (oj < seg_lo || oj >= seg_hi) continue;
      while (oj >= nst && r + 1 < nr) {
        ++r;
        st = nst;
        nst = sm.start[r + 1];
        inf = sm.info[r];
      }
      uint32_t val = inf & 0x7FFFFFFFu;
      if (!(inf & R_RLE)) {
        const uint64_t bit = (uint64_t)inf * 8ull + (uint64_t)(oj - st) * (uint64_t)w;
        const uint64_t abs = S + (bit >> 3);
        const uint64_t ri = abs - A0;
        const uint64_t x = (abs >= A0 && ri + 12 <= staged) ? lload_u64(sm.stage, (uint32_t)ri)
                                                            : gload_u64(blob, blob_len, abs);
        val = (uint32_t)((x >> (bit & 7)) & wm64);
      }
      v[j] = val;
      mask |= 1u << j;
    }
    emit(out + g, v, mask);
  }
  wave_sync();
}

// Stage the payload bytes the runs sm.start/info[0, nr) need for outputs [seg_lo, seg_hi).
__device__ inline uint32_t wave_stage(const uint8_t* __restrict__ blob, uint64_t blob_len, uint64_t S,
                                      uint32_t slen, uint32_t w, uint32_t seg_lo, uint32_t seg_hi,
                                      uint32_t nr, WaveSmem& sm, uint64_t& A0) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t lo = 0xFFFFFFFFu, hi = 0;
  for (uint32_t r = lane; r < nr; r += 64) {
    const uint32_t inf = sm.info[r];
    if (inf & R_RLE) continue;
    const uint32_t st = sm.start[r], en = sm.start[r + 1];
    const uint32_t a = seg_lo > st ? seg_lo : st;
    const uint32_t b = seg_hi < en ? seg_hi : en;
    if (a >= b) continue;
    const uint64_t b0 = (uint64_t)inf + (((uint64_t)(a - st) * w) >> 3);
    const uint64_t b1 = (uint64_t)inf + (((uint64_t)(b - st) * w + 7) >> 3) + 8;
    lo = min(lo, (uint32_t)min(b0, (uint64_t)0xFFFFFFFFu));
    hi = max(hi, (uint32_t)min(b1, (uint64_t)0xFFFFFFFFu));
  }
  lo = wave_min_u32(lo);
  hi = wave_max_u32(hi);
  if (lo >= hi) {  // RLE only: nothing to stage
    A0 = S;
    return 0;
  }
  A0 = (S + lo) & ~15ull;
  uint64_t A1 = S + (uint64_t)hi;
  if (A1 > S + slen + 16) A1 = S + slen + 16;
  if (A1 > A0 + WX_STAGE) A1 = A0 + WX_STAGE;
  const uint32_t nchunks = (uint32_t)((A1 - A0 + 15) / 16);
  constexpr int PER = WX_STAGE / 16 / 64;
  uint4 v[PER];
  const bool fast = A0 + (uint64_t)nchunks * 16 <= blob_len;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t c = lane + 64u * (uint32_t)k;
    if (c < nchunks) {
      const uint64_t a = A0 + (uint64_t)c * 16;
      v[k] = fast ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
    }
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t c = lane + 64u * (uint32_t)k;
    if (c < nchunks) reinterpret_cast<uint4*>(sm.stage)[c] = v[k];
  }
  if (lane < 16) sm.stage[nchunks * 4 + lane] = 0;
  wave_sync();
  return nchunks * 16;
}

// Descriptor of outputs [q * span, (q + 1) * span) of tile t for stream `sel` (k_quarter_desc:
// one thread per quarter; k_tile_desc: one thread per tile with span = RUN_TILE).
__device__ inline QDesc quarter_desc(const uint8_t* blob, const PageWork* pages, const ChunkWork* chunks,
                                     const uint32_t* tile_page, const RunTables& rt, int sel, uint32_t t,
                                     uint32_t q, uint32_t span = WX_OUT) {
  QDesc d{};
  const uint32_t p = tile_page[t];
  const PageWork& pw = pages[p];
  d.page = p;
  if (pw.status != 0) return d;
  if (rt.pflag && pf_level_path(rt.pflag[p])) return d;  // decoded by the level path
  const ChunkWork& ck = chunks[pw.chunk];
  if (sel == SS_DICT && !dict_usable(pages, ck)) return d;
  Stream s;
  if (!get_stream(blob, pw, sel, ck.cp, s) || s.err) return d;
  const uint32_t k = t - pw.ltile0;
  const uint32_t lo = k * RUN_TILE + q * span;
  if (lo >= s.n) return d;
  const uint32_t hi = lo + span < s.n ? lo + span : s.n;
  d.S = s.S;
  d.out = s.out;
  d.slen = s.slen;
  d.qlo = lo;
  d.qhi = hi;
  d.w = (uint32_t)s.w;
  d.kind = (uint32_t)s.kind;
  const uint32_t w = d.w;
  if (s.kind == LK_BIT_PACKED) {  // one header-less run from output 0
    d.rec = 0;
    d.nrec = 1;
    d.blo = (uint32_t)(((uint64_t)lo * w) >> 3);
    d.bhi = (uint32_t)min((((uint64_t)hi * w + 7) >> 3) + 8, (uint64_t)s.slen + 8);
    return d;
  }
  const RunCkpt c = rt.ck[t];
  d.ckpos = c.pos;
  d.ckfirst = c.first;
  const uint32_t nrec = rt.nruns[t];
  if (nrec > RUN_CAPT) {
    d.rec = RUN_REWALK;
    return d;
  }
  const uint2* recs = rt.runs + (uint64_t)t * RUN_CAPT;
  // a0: last record starting at or before lo; a1: last record starting before hi
  uint32_t a0 = 0, a1 = 0;
  for (uint32_t step = RUN_CAPT / 2; step; step >>= 1) {
    if (a0 + step < nrec && recs[a0 + step].x <= lo) a0 += step;
    if (a1 + step < nrec && recs[a1 + step].x < hi) a1 += step;
  }
  d.rec = t * RUN_CAPT + a0;
  d.nrec = a1 - a0 + 1;
  // payload bytes of the bit-packed runs among them (stream offsets increase with the index)
  uint32_t blo = 0xFFFFFFFFu, bhi = 0;
  for (uint32_t r = a0; r <= a1; ++r) {
    const uint2 x = recs[r];
    if (x.y & R_RLE) continue;
    const uint32_t st = x.x;
    const uint32_t u = lo > st ? lo : st;
    blo = (uint32_t)min((uint64_t)blo, (uint64_t)x.y + (((uint64_t)(u - st) * w) >> 3));
    break;
  }
  for (uint32_t r = a1 + 1; r-- > a0;) {
    const uint2 x = recs[r];
    if (x.y & R_RLE) continue;
    const uint32_t st = x.x, en = r + 1 < nrec ? recs[r + 1].x : hi;
    const uint32_t v = hi < en ? hi : en;
    bhi = (uint32_t)min((uint64_t)x.y + ((((uint64_t)(v - st)) * w + 7) >> 3) + 8, (uint64_t)0xFFFFFFF0u);
    break;
  }
  if (bhi) {
    d.blo = blo;
    d.bhi = bhi;
  }
  return d;
}

// Loads a quarter descriptor with one wave (16 lanes x 4 bytes), uniform result.
__device__ inline QDesc load_qdesc(const QDesc* dp) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(dp);
  const uint32_t x = lane < 16 ? w[lane] : 0u;
  QDesc d;
  uint32_t* o = reinterpret_cast<uint32_t*>(&d);
#pragma unroll
  for (int k = 0; k < 16; ++k) o[k] = (uint32_t)__builtin_amdgcn_readlane((int)x, k);
  return d;
}

// Expand the quarter described by d: its run records and payload bytes are fetched together
// (one memory round trip), then every lane expands 2 x 8 outputs.
template <class Emit>
__device__ inline void wave_expand(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                   const QDesc& d, const uint2* __restrict__ runs, WaveSmem& sm,
                                   Emit& emit) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t qlo = d.qlo, qhi = d.qhi, w = d.w;
  uint64_t A0 = d.S;
  if (d.rec != RUN_REWALK) {
    for (uint32_t b = 0; b < d.nrec; b += WX_RCAP) {
      const uint32_t nr = d.nrec - b < (uint32_t)WX_RCAP ? d.nrec - b : (uint32_t)WX_RCAP;
      // ---- run records and payload window, all loads in flight together
      uint2 rr[WX_RCAP / 64];
#pragma unroll
      for (int k = 0; k < WX_RCAP / 64; ++k) {
        const uint32_t r = lane + 64u * (uint32_t)k;
        rr[k] = (d.kind == LK_BIT_PACKED) ? make_uint2(0u, 0u)
                                          : (r < nr ? runs[d.rec + b + r] : make_uint2(0u, 0u));
      }
      const uint32_t seg_lo = b == 0 ? qlo : sm.start[WX_RCAP];  // carried from the previous batch
      const uint32_t seg_hi = (d.kind != LK_BIT_PACKED && b + nr < d.nrec) ? runs[d.rec + b + nr].x : qhi;
      uint32_t staged = 0;
      constexpr int PER = WX_STAGE / 16 / 64;
      uint4 v[PER];
      uint32_t nchunks = 0;
      if (d.bhi) {
        A0 = (d.S + d.blo) & ~15ull;
        uint64_t A1 = d.S + (uint64_t)d.bhi;
        if (A1 > A0 + WX_STAGE) A1 = A0 + WX_STAGE;
        nchunks = (uint32_t)((A1 - A0 + 15) / 16);
        const bool fast = A0 + (uint64_t)nchunks * 16 <= blob_len;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
          const uint32_t c = lane + 64u * (uint32_t)k;
          if (c < nchunks) {
            const uint64_t a = A0 + (uint64_t)c * 16;
            v[k] = fast ? *reinterpret_cast<const uint4*>(blob + a) : gload_u128_tail(blob, blob_len, a);
          }
        }
        staged = nchunks * 16;
      }
#pragma unroll
      for (int k = 0; k < WX_RCAP / 64; ++k) {
        const uint32_t r = lane + 64u * (uint32_t)k;
        if (r < nr) {
          sm.start[r] = rr[k].x;
          sm.info[r] = rr[k].y;
        }
      }
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const uint32_t c = lane + 64u * (uint32_t)k;
        if (c < nchunks) reinterpret_cast<uint4*>(sm.stage)[c] = v[k];
      }
      if (lane < 16) sm.stage[nchunks * 4 + lane] = 0;
      if (lane == 0) {
        sm.start[nr] = seg_hi;
        sm.start[nr + 1] = seg_hi;
      }
      wave_sync();
      wave_expand_batch(blob, blob_len, d.S, d.out, w, qlo, seg_lo, seg_hi, nr, A0, staged, sm, emit);
      if (lane == 0) sm.start[WX_RCAP] = seg_hi;
      wave_sync();
    }
    return;
  }
  // more runs than the index kept: re-walk from the checkpoint (uniform, global reads)
  uint32_t cur = d.ckpos, produced = d.ckfirst, seg_lo = qlo;
  while (seg_lo < qhi) {
    uint32_t nr = 0;
    while (produced < qhi && nr < (uint32_t)WX_RCAP && cur < d.slen) {
      uint32_t nxt, cnt, inf, flg;
      run_parse_global(blob, blob_len, d.S, cur, d.slen, (int)w, nxt, cnt, inf, flg);
      if (cnt) {
        const uint32_t need = cnt;
        if (produced + need > seg_lo) {
          if (lane == 0) {
            sm.start[nr] = produced;
            sm.info[nr] = (flg & RF_BP) ? inf : (R_RLE | inf);
          }
          ++nr;
        }
        produced += need;
      }
      cur = nxt;
    }
    if (nr == 0) break;
    const uint32_t seg_hi = produced < qhi ? produced : qhi;
    if (lane == 0) {
      sm.start[nr] = seg_hi;
      sm.start[nr + 1] = seg_hi;
    }
    wave_sync();
    const uint32_t staged = wave_stage(blob, blob_len, d.S, d.slen, w, seg_lo, seg_hi, nr, sm, A0);
    wave_expand_batch(blob, blob_len, d.S, d.out, w, qlo, seg_lo, seg_hi, nr, A0, staged, sm, emit);
    seg_lo = seg_hi;
  }
}

}  // namespace pqg
