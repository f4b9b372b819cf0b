// pqg_balen.hpp — the length streams of large DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY pages
// decoded by the whole chip (included by pqg_bytes.hip, inside namespace pqg).
//
// k_ba_index decodes a page's length streams (DeltaBitPackDecoder<Int32Type>, decoding.rs:392-619,
// called from DeltaLengthByteArrayDecoder::set_data :682-695 and DeltaByteArrayDecoder::set_data
// :768-790) and derives the value slices in one workgroup per page: a page of a million values
// took 4-9 ms. Pages of at least BL_MIN values in the listed page set go through five kernels
// instead, per 4096-value tile of the page (the page table's RUN_TILE tiles) where the work is
// per value:
//   k_bl_walk   one workgroup per page: both stream headers, then every block header of each
//               stream in turn, one thread hopping over LDS-staged 16 KiB regions (the chain is
//               serial in the format: a block's length depends on its widths); each block's
//               offset recorded, every check the reference makes on the way. Anything that
//               is not the common well-formed shape (a stream value count other than the
//               page's, blocks of other than 128..4096 values, more than 8 mini-blocks, a
//               mini-block size not a multiple of 32, a width past 32, a stream past the page,
//               fewer than BL_MIN values) leaves the page to k_ba_index;
//   k_bl_tile<0> per tile: each block's header parsed by its own lane, 16 deltas per thread
//               unpacked from the LDS-staged tile, their wrapping sum per stream;
//   k_bl_scan<0> per page: each tile's first value (the first value + the wrapping sums before);
//   k_bl_tile<1> per tile: the same unpack, a workgroup scan from that value, the lengths
//               (and prefix lengths) stored; per tile their byte sums, negative lengths flagged;
//   k_bl_scan<1> per page: tile byte offsets, the page's output bytes, the data-size check;
//   k_bl_src    per tile: each value's source address (data start + its offset), the prefix
//               length check against the previous value (decoding.rs:804).
// A page any of them finds at fault is handed back (BlPage::fast = 0) before k_ba_index runs,
// which then decodes it whole and reports exactly what the reference reports.

constexpr uint64_t BL_MIN = 65536;  // values: smaller pages stay with k_ba_index
constexpr uint32_t BL_BPT = 32;     // block offsets per tile and stream (blocks of >= 128 values)
constexpr uint32_t BL_REG = 16384;  // k_bl_walk's staged region
constexpr uint32_t BL_TREG = 4096 * 4 + BL_BPT * 18 + 64;  // a tile's blocks staged (widths <= 32)

struct BlPage {
  uint32_t fast;      // 1: the page's length streams and slices come from k_bl_*; 0: k_ba_index
  uint32_t nmb;       // mini-blocks per block
  uint32_t vpmb;      // values per mini-block
  uint32_t bshift;    // log2(block size)
  uint32_t first[2];  // first values of the streams (u32: INT32 wrapping)
  uint32_t e[2];      // stream-relative ends (stream 1 starts at e[0]; the data at e[1] for DBA)
  uint32_t nstream;   // 1: DELTA_LENGTH_BYTE_ARRAY, 2: DELTA_BYTE_ARRAY
  uint32_t pad;
  uint64_t n;         // values
  uint64_t D, dlen;   // data section: absolute start, bytes
};

struct BlTile {
  uint32_t s[2];    // wrapping sums of min_delta + delta over the tile's deltas, per stream
  uint32_t b[2];    // the value at the tile's first value index, per stream (k_bl_scan<0>)
  uint64_t sum[2];  // [0] bytes of the tile's slices (DLBA lengths / DBA suffixes); [1] DBA output bytes
  uint64_t off[2];  // the sums before the tile (k_bl_scan<1>)
};

struct BlArgs {
  const uint32_t* list;  // the candidate pages
  uint32_t nlist;
  uint32_t maxtiles;     // the most tiles of a listed page
  BlPage* pg;            // per page of the decode
  BlTile* tile;          // per tile (page table numbering)
  uint32_t* blk;         // [2][tiles * BL_BPT] block header offsets, stream-relative
  uint64_t blk_stride;   // tiles * BL_BPT
};

// Block-wide exclusive scan of one u64 per thread (256 threads); the total through tot.
__device__ inline uint64_t block_exscan_u64(uint64_t* wsum, uint64_t x, uint64_t& tot) {
  const uint32_t tid = threadIdx.x;
  uint64_t incl = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off, 64);
    if ((tid & 63) >= (uint32_t)off) incl += y;
  }
  __syncthreads();
  if ((tid & 63) == 63) wsum[tid >> 6] = incl;
  __syncthreads();
  uint64_t pre = 0;
  for (uint32_t w = 0; w < (tid >> 6); ++w) pre += wsum[w];
  tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  return pre + incl - x;
}

// One stream header (decoding.rs:501-533) at stream offset q of blob[S, S + slen): false when
// it is not the fast path's shape.
__device__ inline bool bl_stream_header(const uint8_t* sp, uint32_t slen, uint32_t& q, uint64_t want,
                                        uint32_t& nmb, uint32_t& vpmb, uint32_t& bshift, uint32_t& first) {
  uint64_t bs, m, total, fz;
  int l;
  if ((l = g_vlq(sp, q, slen, bs)) <= 0) return false;
  q += l;
  if ((l = g_vlq(sp, q, slen, m)) <= 0) return false;
  q += l;
  if ((l = g_vlq(sp, q, slen, total)) <= 0) return false;
  q += l;
  if ((l = g_vlq(sp, q, slen, fz)) <= 0) return false;
  q += l;
  if (total != want || m < 1 || m > 8 || bs < 128 || bs > 4096 || (bs & (bs - 1)) || bs % m) return false;
  vpmb = (uint32_t)(bs / m);
  if (vpmb % 32) return false;
  nmb = (uint32_t)m;
  bshift = (uint32_t)__builtin_ctzll(bs);
  first = (uint32_t)unzigzag(fz);
  return true;
}

// ------------------------------------------------------------------------------ k_bl_walk
// A block header at stream offset pos (staged at region byte rel) parsed as k_ba_index's walk
// does: hop = varint + nmb width bytes + the mini-blocks' payload. full: a block whose mini-blocks
// all hold values (every width at most 32); else the stream's last block, of `left` deltas
// (only the needed mini-blocks' widths checked, endp = the last needed one's end). False: not
// the fast path's (a varint of 8 bytes or more, a width past 32, a header or payload past sl).
template <bool full>
__device__ inline bool bl_hop(const uint32_t* reg, uint32_t rel, uint64_t pos, uint32_t sl, uint32_t nmb, uint32_t vpmb,
                              uint64_t left, uint64_t& nx, uint64_t& endp) {
  if (pos >= sl) return false;
  const uint64_t w0 = lload_u64(reg, rel);
  const uint64_t t8 = ~w0 & 0x8080808080808080ull;
  if (!t8) return false;
  const uint32_t vl = ((uint32_t)__builtin_ctzll(t8) >> 3) + 1u;
  const uint64_t wy = lload_u64(reg, rel + vl);
  const uint64_t y = nmb >= 8 ? wy : (wy & ((1ull << (8 * nmb)) - 1ull));
  const uint32_t mneed = full ? nmb : (uint32_t)((left + vpmb - 1) / vpmb);
  const uint64_t ym = mneed >= 8 ? y : (y & ((1ull << (8 * mneed)) - 1ull));
  if ((ym | (ym + 0x5F5F5F5F5F5F5F5Full)) & 0x8080808080808080ull & (mneed >= 8 ? ~0ull : ((1ull << (8 * mneed)) - 1ull)))
    return false;  // a needed width past 32 (bytes >= 0xA1 carry, but their own top bit is set)
  const uint64_t s16 = (y & 0x00FF00FF00FF00FFull) + ((y >> 8) & 0x00FF00FF00FF00FFull);
  const uint64_t sm16 = (ym & 0x00FF00FF00FF00FFull) + ((ym >> 8) & 0x00FF00FF00FF00FFull);
  const uint32_t hs = vpmb >> 3;
  const uint64_t pay = pos + vl + nmb;
  endp = pay + (uint64_t)hs * (uint32_t)((sm16 * 0x0001000100010001ull) >> 48);
  nx = pay + (uint64_t)hs * (uint32_t)((s16 * 0x0001000100010001ull) >> 48);
  return pay <= sl && endp <= sl && (!full || nx <= sl);
}

// The walk of one stream, region by region (16 KiB staged in LDS). Per region every position
// is parsed as a full block's header at once (hop16: 0 not a header, BL_HEXIT a hop out of the
// region); random bytes almost never parse (a varint byte and nmb widths <= 32), so the valid
// positions -- the true headers and a few others -- are compacted (position order, at most
// BL_LCAP) and the chain from the region's entry header is found by pointer jumping over them:
// thread j takes the j-th successor (<= 10 table lookups). The stream's last block, a chain that
// leaves the region on its first hop and anything malformed go through one exact hop of thread 0.
constexpr uint32_t BL_PLIM = BL_REG - 24;  // positions parsed from the region (a header's 15 bytes + 3 + slack)
constexpr uint32_t BL_LCAP = 1024;         // compacted headers per region
constexpr uint32_t BLW = 1024;             // k_bl_walk's threads
constexpr uint16_t BL_HEXIT = 0xFFFFu, BL_NONE = 0xFFFFu, BL_TRUNC = 0xFFFEu, BL_DEAD = 0xFFFDu;

struct BlWalkSmem {
  uint32_t reg[BL_REG / 4 + 8];
  uint16_t hop16[BL_PLIM];
  uint16_t imap[BL_PLIM];
  uint16_t lpos[BL_LCAP];
  uint16_t J[10][BL_LCAP];
  uint32_t wcnt[BLW / 64];
  uint32_t ctl[8];  // 0: pos (stream-relative, low), 1: blocks done, 2: state, 3: end, 4: L, 5: stop kind
};

__global__ void __launch_bounds__(BLW) k_bl_walk(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                const PageWork* pages, const ChunkWork* chunks, BlArgs a) {
  __shared__ BlWalkSmem sm;
  const uint32_t p = a.list[blockIdx.x];
  const PageWork& pw = pages[p];
  BlPage& P = a.pg[p];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  if (tid == 0) P.fast = 0;
  const ChunkWork& ck = chunks[pw.chunk];
  if (pw.status != 0 || (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) || ck.es != 0 || !ck.val_out ||
      ck.cp.physical_type == T_FLBA || pw.nonnull < BL_MIN ||
      (pw.encoding != E_DELTA_LENGTH_BYTE_ARRAY && pw.encoding != E_DELTA_BYTE_ARRAY))
    return;
  const uint64_t n = pw.nonnull, S = pw.base + pw.val_off;
  const uint32_t slen = pw.val_bytes;
  const uint32_t ns = pw.encoding == E_DELTA_BYTE_ARRAY ? 2u : 1u;
  uint32_t base = 0;  // the current stream's start (relative to S)
  uint32_t nmb0 = 0, vpmb0 = 0, bsh0 = 0;
  uint32_t e[2] = {0u, 0u}, fst[2] = {0u, 0u};
  for (uint32_t st = 0; st < ns; ++st) {
    uint32_t q = 0, nmb = 0, vpmb = 0, bsh = 0, first = 0;
    const bool ok = bl_stream_header(blob + S + base, slen - base, q, n, nmb, vpmb, bsh, first);
    if (!ok || (st && (nmb != nmb0 || vpmb != vpmb0 || bsh != bsh0))) return;  // (uniform)
    nmb0 = nmb;
    vpmb0 = vpmb;
    bsh0 = bsh;
    fst[st] = first;
    const uint32_t B = 1u << bsh, sl = slen - base;
    const uint64_t need = n - 1;  // deltas
    const uint32_t nblk = (uint32_t)((need + B - 1) >> bsh);
    uint32_t* blk = a.blk + st * a.blk_stride + (uint64_t)pw.ltile0 * BL_BPT;
    const uint64_t Sb = S + base;
    if (tid == 0) {
      sm.ctl[0] = q;
      sm.ctl[1] = 0;
      sm.ctl[2] = 0;
    }
    __syncthreads();
#pragma unroll 1
    while (true) {
      const uint32_t pos = sm.ctl[0], b = sm.ctl[1];
      if (sm.ctl[2]) break;
      const uint64_t R0 = (Sb + pos) & ~15ull;  // region start (absolute)
      const uint32_t xs = (uint32_t)(Sb + pos - R0);  // the entry header's region position
      __syncthreads();
      for (uint32_t c = tid; c < BL_REG / 16; c += BLW) {
        const uint64_t ad = R0 + (uint64_t)c * 16;
        reinterpret_cast<uint4*>(sm.reg)[c] =
            ad + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + ad) : gload_u128_tail(blob, blob_len, ad);
      }
      if (tid < 8) sm.reg[BL_REG / 4 + tid] = 0;
      __syncthreads();
      // the last block, or a single exact hop (thread 0) when the chain cannot be jumped here
      auto serial = [&](bool last) {
        if (tid == 0) {
          uint64_t nx = 0, endp = 0;
          const uint64_t left = need - ((uint64_t)b << bsh);
          const bool good = last ? bl_hop<false>(sm.reg, xs, pos, sl, nmb, vpmb, left, nx, endp)
                                 : bl_hop<true>(sm.reg, xs, pos, sl, nmb, vpmb, left, nx, endp);
          if (!good) {
            sm.ctl[2] = 2;
          } else {
            blk[b] = pos;  // (b < ntiles * BL_BPT: blocks of >= 128 values)
            sm.ctl[1] = b + 1;
            if (last) {
              sm.ctl[3] = (uint32_t)endp;  // get_offset() after the last value (decoding.rs:572-590)
              sm.ctl[2] = 1;
            } else {
              sm.ctl[0] = (uint32_t)nx;
            }
          }
        }
        __syncthreads();
      };
      if (b + 1 == nblk) {
        serial(true);
        continue;
      }
      // hop16 for every region position from the entry on; per wave, valid counts (position order:
      // wave w owns positions [w * 4096, w * 4096 + 4096))
      constexpr uint32_t QW = BL_PLIM / (BLW / 64) + 1;  // positions per wave (rounded up)
      uint32_t cnt = 0;
      for (uint32_t i = 0; i < (QW + 63) / 64; ++i) {
        const uint32_t x = wv * QW + i * 64 + lane;
        bool v = false;
        if (x < BL_PLIM && x < (wv + 1) * QW) {
          uint16_t h = 0;
          if (x >= xs) {
            uint64_t nx = 0, endp = 0;
            const uint64_t sp = pos + (uint64_t)(x - xs);
            if (bl_hop<true>(sm.reg, x, sp, sl, nmb, vpmb, 0, nx, endp)) {
              const uint64_t hp = nx - sp;
              h = (uint64_t)x + hp >= BL_PLIM || hp >= BL_HEXIT ? BL_HEXIT : (uint16_t)hp;
              v = true;
            }
          }
          sm.hop16[x] = h;
        }
        cnt += (uint32_t)__builtin_popcountll(__ballot(v));
      }
      if (lane == 0) sm.wcnt[wv] = cnt;
      __syncthreads();
      uint32_t wb = 0;
      for (uint32_t w = 0; w < wv; ++w) wb += sm.wcnt[w];
      // compaction: list index in position order; imap: position -> index (BL_TRUNC past the cap)
      for (uint32_t i = 0; i < (QW + 63) / 64; ++i) {
        const uint32_t x = wv * QW + i * 64 + lane;
        const bool in = x < BL_PLIM && x < (wv + 1) * QW;
        const bool v = in && x >= xs && sm.hop16[x] != 0;
        const uint64_t m = __ballot(v);
        const uint32_t idx = wb + (uint32_t)__builtin_popcountll(m & ((1ull << lane) - 1ull));
        if (in) sm.imap[x] = !v ? BL_NONE : idx < BL_LCAP ? (uint16_t)idx : BL_TRUNC;
        if (v && idx < BL_LCAP) sm.lpos[idx] = (uint16_t)x;
        wb += (uint32_t)__builtin_popcountll(m);
      }
      __syncthreads();
      uint32_t tot = 0;
      for (uint32_t w = 0; w < BLW / 64; ++w) tot += sm.wcnt[w];
      const uint32_t nl = tot < BL_LCAP ? tot : BL_LCAP;
      // successors: an index, BL_HEXIT (the chain leaves the region or the list: go on from
      // there), BL_DEAD (the next position is not a full block's header)
      for (uint32_t i = tid; i < nl; i += BLW) {
        const uint32_t x = sm.lpos[i], h = sm.hop16[x];
        uint16_t sc = BL_HEXIT;
        if (h != BL_HEXIT) {
          const uint16_t t = sm.imap[x + h];
          sc = t == BL_NONE ? BL_DEAD : t == BL_TRUNC ? BL_HEXIT : t;
        }
        sm.J[0][i] = sc;
      }
      __syncthreads();
#pragma unroll 1
      for (uint32_t k = 1; k < 10; ++k) {
        for (uint32_t i = tid; i < nl; i += BLW) {
          const uint16_t t = sm.J[k - 1][i];
          sm.J[k][i] = t >= BL_DEAD ? t : sm.J[k - 1][t];
        }
        __syncthreads();
      }
      // thread j: the entry's j-th successor (j < 1024: one per thread), recorded
      // while it is not the stream's last block (thread 0 takes that one exactly)
      const uint16_t s0 = sm.imap[xs];
      if (tid == 0) sm.ctl[4] = 0;
      __syncthreads();
      if (s0 < BL_LCAP) {
        for (uint32_t j = tid; j < BL_LCAP; j += BLW) {
          uint32_t e0 = s0;
          bool okj = true;
          for (uint32_t k = 0; k < 10 && okj; ++k)
            if ((j >> k) & 1u) {
              const uint16_t t = sm.J[k][e0];
              okj = t < BL_DEAD;
              e0 = t;
            }
          if (okj) {
            if (b + j + 1 < nblk) blk[b + j] = (uint32_t)(pos + (sm.lpos[e0] - xs));
            atomicMax(&sm.ctl[4], j + 1u);
          }
        }
      }
      __syncthreads();
      if (tid == 0) {
        const uint32_t L = sm.ctl[4];  // chain entries in the region, the entry header included
        auto entry = [&](uint32_t j) -> uint32_t {
          uint32_t e0 = s0;
          for (uint32_t k = 0; k < 10; ++k)
            if ((j >> k) & 1u) e0 = sm.J[k][e0];
          return e0;
        };
        uint32_t mode = 0;  // 1: one exact hop of thread 0 from (pos, b)
        if (L == 0) {
          mode = 1;  // the entry is no full block's header: malformed (thread 0 says so)
        } else if (b + L >= nblk) {
          // the stream's last block is chain entry nblk - 1 - b: thread 0 parses it next
          sm.ctl[0] = pos + (sm.lpos[entry(nblk - 1 - b)] - xs);
          sm.ctl[1] = nblk - 1;
        } else {
          const uint32_t x = sm.lpos[entry(L - 1)], h = sm.hop16[x];
          if (h == BL_HEXIT) {
            // the chain's last entry here hops out of the region: the next region starts at it
            // (it is the entry itself: thread 0 hops it exactly)
            if (L == 1) mode = 1;
            else {
              sm.ctl[0] = pos + (x - xs);
              sm.ctl[1] = b + L - 1;
            }
          } else {
            // its successor is past the compacted list (the next region starts there) or no full
            // block's header (the next round's exact hop reports it)
            sm.ctl[0] = pos + (x - xs) + h;
            sm.ctl[1] = b + L;
          }
        }
        sm.ctl[7] = mode;
      }
      __syncthreads();
      if (sm.ctl[7]) serial(false);
    }
    if (sm.ctl[2] != 1) return;  // (uniform)
    e[st] = sm.ctl[3];
    __syncthreads();
    base += e[st];  // stream-relative ends: e[0] from S, e[1] from S + e[0]
  }
  if (tid == 0) {
    P.nmb = nmb0;
    P.vpmb = vpmb0;
    P.bshift = bsh0;
    P.first[0] = fst[0];
    P.first[1] = fst[1];
    P.e[0] = e[0];
    P.e[1] = e[1];
    P.nstream = ns;
    P.n = n;
    P.D = S + base;
    P.dlen = slen - base;
    P.fast = 1;
  }
}

// ------------------------------------------------------------------------------ k_bl_tile
// Tile k of a listed fast page: deltas [4096 k, 4096 k + 4096) of each stream (delta d gives value
// d + 1). MODE 0: their wrapping sum per stream; MODE 1: the values of the tile's indices
// [4096 k, 4096 k + 4096) stored (v = the tile's first value + the exclusive sum of its deltas
// before), with the tile's byte sums.
struct BlTileSmem {
  uint32_t reg[BL_TREG / 4 + 8];
  uint32_t pay[BL_BPT];
  uint32_t md[BL_BPT];
  uint32_t mboff[BL_BPT][8];
  uint8_t width[BL_BPT][8];
  uint64_t wsum[WG / 64];
  uint32_t bad;
};

template <int MODE>
__global__ void __launch_bounds__(WG) k_bl_tile(const uint8_t* __restrict__ blob, uint64_t blob_len, PageWork* pages,
                                                const ChunkWork* chunks, BlArgs a, uint32_t* vlen0, uint32_t* vpre0) {
  __shared__ BlTileSmem sm;
  const uint32_t p = a.list[blockIdx.y];
  BlPage& P = a.pg[p];
  if (!P.fast) return;
  const PageWork& pw = pages[p];
  const uint64_t n = P.n, i0 = (uint64_t)blockIdx.x * RUN_TILE;
  if (i0 >= n) return;
  const uint32_t t = threadIdx.x, nmb = P.nmb, vpmb = P.vpmb, bsh = P.bshift, B = 1u << bsh;
  const uint64_t need = n - 1;
  const uint32_t nd = i0 < need ? (uint32_t)min((uint64_t)RUN_TILE, need - i0) : 0u;  // the tile's deltas
  const uint32_t nblk = (nd + B - 1) >> bsh, fb = (uint32_t)(i0 >> bsh);
  BlTile& T = a.tile[pw.ltile0 + blockIdx.x];
  const uint64_t S = pw.base + pw.val_off;
  const ChunkWork& ck = chunks[pw.chunk];
  if (MODE == 1 && t == 0) sm.bad = 0;
  uint64_t bsum0 = 0, bsum1 = 0;
  uint32_t prevv[16];  // (MODE 1, DBA: the prefix lengths of the thread's values)
  for (uint32_t st = 0; st < P.nstream; ++st) {
    const uint64_t Sb = S + (st ? P.e[0] : 0u);
    const uint32_t* blk = a.blk + st * a.blk_stride + (uint64_t)pw.ltile0 * BL_BPT;
    uint32_t dd[16];
    uint32_t s = 0;
    if (nblk) {
      // stage the tile's blocks: from the first header to the last block's payload end (the
      // next header, or the stream's end)
      const uint32_t h0 = blk[fb];
      const uint32_t h1 = fb + nblk < ((uint32_t)((need + B - 1) >> bsh)) ? blk[fb + nblk] : P.e[st];
      const uint64_t A0 = (Sb + h0) & ~15ull;
      const uint32_t nch = (uint32_t)((Sb + h1 - A0 + 15) / 16);
      __syncthreads();
      for (uint32_t c = t; c < nch && c < BL_TREG / 16; c += WG) {
        const uint64_t ad = A0 + (uint64_t)c * 16;
        reinterpret_cast<uint4*>(sm.reg)[c] =
            ad + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + ad) : gload_u128_tail(blob, blob_len, ad);
      }
      if (t < 8) sm.reg[BL_TREG / 4 + t] = 0;
      __syncthreads();
      if (t < nblk) {  // block fb + t's header (k_bl_walk checked it)
        const uint32_t rel = (uint32_t)(Sb + blk[fb + t] - A0);
        const uint64_t w0 = lload_u64(sm.reg, rel);
        const uint32_t vl = ((uint32_t)__builtin_ctzll(~w0 & 0x8080808080808080ull) >> 3) + 1u;
        uint64_t zz = 0;
        for (uint32_t k = 0; k < vl; ++k) zz |= ((w0 >> (8 * k)) & 0x7Full) << (7 * k);
        sm.md[t] = (uint32_t)unzigzag(zz);
        const uint64_t y = lload_u64(sm.reg, rel + vl);
        uint32_t off = rel + vl + nmb;
        sm.pay[t] = off;
        for (uint32_t m = 0; m < nmb; ++m) {
          const uint32_t w = (uint32_t)(y >> (8 * m)) & 0xFFu;
          sm.width[t][m] = (uint8_t)w;
          sm.mboff[t][m] = off;
          off += (vpmb >> 3) * w;
        }
      }
      __syncthreads();
      const uint32_t d = 16u * t;
      if (d < nd) {
        const uint32_t b = d >> bsh, inb = d & (B - 1u), m = inb / vpmb, j0 = inb - m * vpmb;
        const uint32_t w = sm.width[b][m], wm = w >= 32 ? 0xFFFFFFFFu : (1u << w) - 1u;
        const uint32_t rb = sm.mboff[b][m] * 8u + j0 * w, mn = sm.md[b];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          const uint32_t bit = rb + (uint32_t)j * w, wi = bit >> 5;
          const uint32_t r = __builtin_amdgcn_alignbit(sm.reg[wi + 1], sm.reg[wi], bit & 31u) & wm;
          dd[j] = d + (uint32_t)j < nd ? mn + r : 0u;  // min_delta + delta (INT32: wrapping)
          s += dd[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 16; ++j) dd[j] = 0;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) dd[j] = 0;
    }
    if (MODE == 0) {
      __syncthreads();
      const uint64_t tot = block_sum_u64(s, sm.wsum);
      if (t == 0) T.s[st] = (uint32_t)tot;
      continue;
    }
    // MODE 1: values 16 t + j of the tile: the tile's first value + the deltas before them
    uint64_t tot;
    __syncthreads();
    uint32_t v = T.b[st] + (uint32_t)block_exscan_u64(sm.wsum, s, tot);
    uint32_t* outp = (P.nstream == 2 && st == 0 ? vpre0 : vlen0) + ck.scr_base + pw.value_out + i0;
    uint64_t ls = 0;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const uint64_t i = i0 + 16u * t + (uint32_t)j;
      if (i < n) {
        gp(outp)[16u * t + (uint32_t)j] = v;
        bad |= (int32_t)v < 0;  // a negative length: data.range asserts (k_ba_index reports it)
        ls += v;
        if (P.nstream == 2 && st == 0) prevv[j] = v;
        else if (P.nstream == 2) bsum1 += (uint64_t)prevv[j] + v;
      }
      v += dd[j];
    }
    if (st == P.nstream - 1) bsum0 = ls;
    if (bad) sm.bad = 1;
  }
  if (MODE == 1) {
    __syncthreads();
    const uint64_t t0 = block_sum_u64(bsum0, sm.wsum);
    const uint64_t t1 = block_sum_u64(bsum1, sm.wsum);
    if (t == 0) {
      T.sum[0] = t0;
      T.sum[1] = P.nstream == 2 ? t1 : t0;
      if (sm.bad) P.fast = 0;
    }
  }
}

// ------------------------------------------------------------------------------ k_bl_scan
// Per listed fast page, over its tiles in order: MODE 0 the tiles' first values (wrapping);
// MODE 1 the byte offsets before each tile, the page's output bytes and the data-size check.
template <int MODE>
__global__ void __launch_bounds__(WG) k_bl_scan(PageWork* pages, BlArgs a) {
  __shared__ uint64_t wsum[WG / 64];
  const uint32_t p = a.list[blockIdx.x];
  BlPage& P = a.pg[p];
  if (!P.fast) return;
  const PageWork& pw = pages[p];
  const uint32_t nt = (uint32_t)((P.n + RUN_TILE - 1) / RUN_TILE);
  BlTile* T = a.tile + pw.ltile0;
  uint64_t c0 = MODE == 0 ? P.first[0] : 0ull, c1 = MODE == 0 ? P.first[1] : 0ull;
  for (uint32_t k0 = 0; k0 < nt; k0 += WG) {
    const uint32_t k = k0 + threadIdx.x;
    const uint64_t x0 = k < nt ? (MODE == 0 ? (uint64_t)T[k].s[0] : T[k].sum[0]) : 0ull;
    const uint64_t x1 = k < nt ? (MODE == 0 ? (uint64_t)T[k].s[1] : T[k].sum[1]) : 0ull;
    uint64_t t0, t1;
    const uint64_t e0 = block_exscan_u64(wsum, x0, t0);
    const uint64_t e1 = block_exscan_u64(wsum, x1, t1);
    if (k < nt) {
      if (MODE == 0) {
        T[k].b[0] = (uint32_t)(c0 + e0);
        T[k].b[1] = (uint32_t)(c1 + e1);
      } else {
        T[k].off[0] = c0 + e0;
        T[k].off[1] = c1 + e1;
      }
    }
    c0 += t0;
    c1 += t1;
  }
  if (MODE == 1 && threadIdx.x == 0) {
    if (c0 > P.dlen) P.fast = 0;  // slices past the data: data.range asserts (k_ba_index reports it)
    else pages[p].nbytes_out = c1;
  }
}

// ------------------------------------------------------------------------------ k_bl_src
// Per tile of a listed fast page: each value's source address (the data start + the slice bytes
// before it), and for DBA each prefix length against the previous value's length (:804; the
// first value's prefix length must be 0).
__global__ void __launch_bounds__(WG) k_bl_src(const PageWork* pages, const ChunkWork* chunks, BlArgs a,
                                               uint64_t* vsrc0, const uint32_t* vlen0, const uint32_t* vpre0) {
  __shared__ uint64_t wsum[WG / 64];
  __shared__ uint32_t bad;
  const uint32_t p = a.list[blockIdx.y];
  BlPage& P = a.pg[p];
  if (!P.fast) return;
  const PageWork& pw = pages[p];
  const uint64_t n = P.n, i0 = (uint64_t)blockIdx.x * RUN_TILE;
  if (i0 >= n) return;
  if (threadIdx.x == 0) bad = 0;
  const ChunkWork& ck = chunks[pw.chunk];
  const uint64_t vb = ck.scr_base + pw.value_out;
  const uint32_t* len = vlen0 + vb;
  const uint32_t* pre = vpre0 + vb;
  const uint64_t ib = i0 + 16u * threadIdx.x;
  uint32_t l[16];
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    l[j] = ib + j < n ? len[ib + j] : 0u;
    s += l[j];
  }
  bool b = false;
  if (P.nstream == 2) {
    uint64_t prevlen = ib == 0 ? 0ull : ib < n ? (uint64_t)pre[ib - 1] + len[ib - 1] : 0ull;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (ib + j < n) {
        const uint32_t pl = pre[ib + j];
        b |= (uint64_t)pl > prevlen;
        prevlen = (uint64_t)pl + l[j];
      }
    }
  }
  uint64_t tot;
  uint64_t off = a.tile[pw.ltile0 + blockIdx.x].off[0] + block_exscan_u64(wsum, s, tot);
  uint64_t* src = vsrc0 + vb;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (ib + j < n) gp(src)[ib + j] = P.D + off;
    off += l[j];
  }
  if (b) bad = 1;
  __syncthreads();
  if (threadIdx.x == 0 && bad) P.fast = 0;
}

static_assert(sizeof(BlPage) <= 64 && sizeof(BlTile) == 48, "the host's state buffer layout (chunk_decoder.cpp)");
