// pqg_bytes.hip — BYTE_ARRAY / FIXED_LEN_BYTE_ARRAY values on CDNA4.
//
// Output layout (pqgpu.h): the dense non-null values' bytes concatenated, plus int64 offsets
// (num_values + 1). The reference hands out ByteArray slices of page memory
// (data_type.rs:70-98) or, for DELTA_BYTE_ARRAY, freshly built vectors; a device layout of
// bytes + offsets carries the same values.
//
// Two passes over each page, with a chunk-wide scan in between:
//   index  k_ba_index / k_ba_dict_idx: per value its source address and length
//          (PLAIN BA :206-226, PLAIN FLBA :228-247, dictionary :256-315 with the dictionary
//          page decoded by k_ba_dict_prep, DELTA_LENGTH_BYTE_ARRAY :682-712, DELTA_BYTE_ARRAY
//          :768-835), and the page's output byte count;
//   scan   k_scan_bytes: page byte offsets, capacity check, final offset;
//   copy   k_ba_copy (gathers slices) and the DELTA_BYTE_ARRAY rebuild (value i = the first
//          prefix_i bytes of value i-1 ++ suffix_i, as slices of earlier suffixes: k_dba_*).
//
// PLAIN BYTE_ARRAY lengths are inline ([u32 len][bytes]...), so value starts form a serial
// chain: one lane walks it over LDS-staged 16 KiB regions of the page.
#include "pqg_delta.hpp"
#include "pqg_runs.hpp"

namespace pqg {

// Walks n PLAIN BYTE_ARRAY values of the stream blob[S, S+slen) (decoding.rs:206-226):
// PANIC when fewer than 4 bytes remain for a length (read_num_bytes! assert), EOF when the
// value bytes run past the stream. Writes absolute source addresses and lengths. One lane
// follows the chain over the LDS-staged region and records each value's (offset, length) in
// LDS; the workgroup then writes them out coalesced (global stores from one lane per value
// would bound the walk).
constexpr uint32_t BW_CAP = 2048;  // values recorded per pass
__device__ int32_t plain_ba_walk(DeltaSmem& sm, const uint8_t* __restrict__ blob, uint64_t blob_len,
                                 uint64_t S, uint32_t slen, uint64_t n, uint64_t* __restrict__ src,
                                 uint32_t* __restrict__ len) {
  __shared__ uint2 rec[BW_CAP];
  __shared__ uint32_t fixed_s;
  // Values of one length L (dates, codes, ids): value i then starts at i * (4 + L) + 4. Checked
  // by the whole workgroup in one pass; the chain is only walked when some length differs.
  if (n > 1 && slen >= 4) {
    const uint32_t L = (uint32_t)blob[S] | ((uint32_t)blob[S + 1] << 8) | ((uint32_t)blob[S + 2] << 16) |
                       ((uint32_t)blob[S + 3] << 24);
    const uint64_t stride = 4ull + L;
    if (threadIdx.x == 0) fixed_s = 1;
    __syncthreads();
    if (n * stride <= (uint64_t)slen) {
      for (uint64_t k = threadIdx.x; k < n; k += WG) {
        const uint64_t a = S + k * stride;
        const uint32_t l = (uint32_t)blob[a] | ((uint32_t)blob[a + 1] << 8) | ((uint32_t)blob[a + 2] << 16) |
                           ((uint32_t)blob[a + 3] << 24);
        if (l != L) fixed_s = 0;
      }
    } else if (threadIdx.x == 0) {
      fixed_s = 0;
    }
    __syncthreads();
    if (fixed_s) {
      for (uint64_t k = threadIdx.x; k < n; k += WG) {
        src[k] = S + k * stride + 4;
        len[k] = L;
      }
      return 0;
    }
  }
  uint64_t i = 0;
  uint32_t pos = 0;
  uint64_t A0 = ~0ull;
  while (i < n) {
    if (A0 == ~0ull || S + pos + 4 - A0 > (uint64_t)DBLK) {  // restage: the next length is past the region
      A0 = (S + pos) & ~15ull;
      __syncthreads();
      delta_load_region(sm, blob, blob_len, A0);
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      int32_t e = 0;
      uint32_t k = 0;
      while (i + k < n && k < BW_CAP) {
        const uint64_t rel = S + pos - A0;
        if (rel + 4 > (uint64_t)DBLK) break;
        if ((uint64_t)pos + 4 > slen) {
          e = ST_PANIC;
          break;
        }
        const uint32_t l = (uint32_t)lload_u64(sm.region, (uint32_t)rel);
        pos += 4;
        if ((uint64_t)pos + l > slen) {
          e = ST_EOF;
          break;
        }
        rec[k++] = make_uint2(pos, l);
        pos += l;
      }
      sm.ctl[0] = (uint32_t)e;
      sm.ctl[1] = pos;
      sm.ctl[2] = k;
    }
    __syncthreads();
    const int32_t e = (int32_t)sm.ctl[0];
    const uint32_t k = sm.ctl[2];
    pos = sm.ctl[1];
    for (uint32_t t = threadIdx.x; t < k; t += WG) {
      const uint2 r = rec[t];
      src[i + t] = S + r.x;
      len[i + t] = r.y;
    }
    i += k;
    __syncthreads();  // rec is refilled by the next pass
    if (e) return e;
  }
  return 0;
}

// Block-wide exclusive scan of one u64 per thread; returns the exclusive prefix and the total
// through `tot`. Uses sm.wsum.
__device__ inline uint64_t block_exscan(DeltaSmem& sm, uint64_t x, uint64_t& tot) {
  const int tid = threadIdx.x;
  uint64_t incl = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint64_t y = __shfl_up(incl, off, 64);
    if ((tid & 63) >= off) incl += y;
  }
  __syncthreads();
  if ((tid & 63) == 63) sm.wsum[tid >> 6] = incl;
  __syncthreads();
  uint64_t pre = 0;
  for (int w = 0; w < (tid >> 6); ++w) pre += sm.wsum[w];
  tot = sm.wsum[0] + sm.wsum[1] + sm.wsum[2] + sm.wsum[3];
  return pre + incl - x;
}

// Source addresses of `n` DELTA_LENGTH-style values whose lengths (int32) are in len[0, n)
// and whose bytes start at D (dlen bytes available). data.range(offset, len) asserts
// (PANIC) on negative lengths or running past the data.
__device__ int32_t slices_from_lengths(DeltaSmem& sm, uint64_t D, uint64_t dlen, uint64_t n,
                                       const uint32_t* len, uint64_t* src, uint64_t& carry) {
  carry = 0;
  int32_t bad = 0;
  constexpr uint32_t PT = 16;  // lengths per thread per pass (one workgroup scan per 4096 values)
  for (uint64_t b = 0; b < n; b += (uint64_t)WG * PT) {
    const uint64_t i0 = b + (uint64_t)threadIdx.x * PT;
    int32_t l[PT];
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k) {
      l[k] = i0 + k < n ? (int32_t)len[i0 + k] : 0;
      s += l[k] > 0 ? (uint64_t)l[k] : 0;
    }
    uint64_t tot;
    uint64_t off = carry + block_exscan(sm, s, tot);
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k) {
      if (i0 + k < n) {
        if (l[k] < 0 || off + (uint64_t)l[k] > dlen) bad = 1;
        else gp(src)[i0 + k] = D + off;
      }
      off += l[k] > 0 ? (uint64_t)l[k] : 0;
    }
    carry += tot;
  }
  __syncthreads();
  if (threadIdx.x == 0) sm.ctl[5] = 0;
  __syncthreads();
  if (bad) sm.ctl[5] = 1;
  __syncthreads();
  return sm.ctl[5] ? ST_PANIC : 0;
}

// DELTA_BYTE_ARRAY after its two length streams (prefix lengths pre[0, n), suffix lengths
// len[0, ns)), in one pass of 16 values per thread per workgroup scan with every load of a pass in
// flight at once: the suffix slices of the first ns values from D (dlen bytes; a negative length
// or one past the data panics, as data.range asserts); values past ns repeat the last suffix
// (decoding.rs:796-801); each prefix length at most the previous value's length
// (previous_value[0..prefix_len], :804; 0 for the first); bytes: the page's output bytes (prefix
// + suffix lengths).
__device__ int32_t dba_slices(DeltaSmem& sm, uint64_t D, uint64_t dlen, uint64_t n, uint64_t ns, const uint32_t* len,
                              const uint32_t* pre, uint64_t* src, uint64_t& bytes) {
  uint64_t carry = 0, by = 0;
  int32_t bad = 0;
  constexpr uint32_t PT = 16;
  const uint32_t lastl = ns ? len[ns - 1] : 0u;
#pragma unroll 1
  for (uint64_t b = 0; b < n; b += (uint64_t)WG * PT) {
    const uint64_t i0 = b + (uint64_t)threadIdx.x * PT;
    int32_t l[PT];
    uint32_t pr[PT];
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k) {
      const uint64_t i = i0 + k;
      l[k] = i < ns ? (int32_t)len[i] : i < n ? (int32_t)lastl : 0;
      pr[k] = i < n ? pre[i] : 0u;
    }
    // the value before the thread's first: its full length
    uint64_t prevlen = 0;
    if (i0 > 0 && i0 < n) {
      const uint64_t j = i0 - 1;
      prevlen = (uint64_t)pre[j] + (uint64_t)(uint32_t)(j < ns ? len[j] : lastl);
    }
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k) {
      const uint64_t i = i0 + k;
      if (i < ns) s += l[k] > 0 ? (uint64_t)l[k] : 0;
      if (i < n) {
        const int32_t pl = (int32_t)pr[k];
        if (pl < 0 || (uint64_t)pl > prevlen) bad = 1;
        prevlen = (uint64_t)pr[k] + (uint64_t)(uint32_t)l[k];
        by += prevlen;
      }
    }
    uint64_t tot;
    uint64_t off = carry + block_exscan(sm, s, tot);
#pragma unroll
    for (uint32_t k = 0; k < PT; ++k) {
      const uint64_t i = i0 + k;
      if (i < ns) {
        if (l[k] < 0 || off + (uint64_t)l[k] > dlen) bad = 1;
        else gp(src)[i] = D + off;
        off += l[k] > 0 ? (uint64_t)l[k] : 0;
      }
    }
    carry += tot;
  }
  __syncthreads();  // (the last scan's reads of sm.wsum)
  const uint64_t tb = block_sum_u64(by, sm.wsum);
  if (threadIdx.x == 0) {
    sm.ctl[5] = 0;
    sm.carry = tb;
  }
  __syncthreads();
  if (bad) sm.ctl[5] = 1;
  __syncthreads();
  bytes = sm.carry;
  return sm.ctl[5] ? ST_PANIC : 0;
}

// Byte arrays of this chunk: FIXED_LEN_BYTE_ARRAY type length, 0 for BYTE_ARRAY.
__device__ inline int ba_type_length(const ChunkWork& ck) {
  return ck.cp.physical_type == T_FLBA ? ck.cp.type_length : 0;
}

// Sum of a page's output value lengths -> pages[p].nbytes_out.
__device__ void page_bytes(DeltaSmem& sm, PageWork* pages, int p, uint64_t n, const uint32_t* len,
                           const uint32_t* pre) {
  uint64_t s = 0;
  for (uint64_t i = threadIdx.x; i < n; i += WG) s += (uint64_t)len[i] + (pre ? (uint64_t)pre[i] : 0);
  uint64_t t = block_sum_u64(s, sm.wsum);
  if (threadIdx.x == 0) pages[p].nbytes_out = t;
}

// Dictionary page of a BYTE_ARRAY / FLBA column: DictDecoder::set_dict decodes every entry
// with PlainDecoder (decoding.rs:282-288). One workgroup per chunk of the decode; the entries go
// to the chunk's slots of the dictionary scratch (dscr_base on).
__global__ void __launch_bounds__(WG) k_ba_dict_prep(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                     PageWork* pages, ChunkWork* chunks, uint64_t* dsrc0,
                                                     uint32_t* dlen0) {
  __shared__ DeltaSmem sm;
  const ChunkWork& ck = chunks[blockIdx.x];
  if (ck.es != 0 || ck.dict_page < 0 || !ck.val_out) return;
  const int dict_page = ck.dict_page;
  const int type_length = ba_type_length(ck);
  uint64_t* dsrc = dsrc0 + ck.dscr_base;
  uint32_t* dlen = dlen0 + ck.dscr_base;
  const PageWork dp = pages[dict_page];
  const uint64_t n = dp.num_values;
  const uint64_t S = dp.base;
  if (dp.status != 0) {  // (failed before: every entry empty, as below -- the scratch is not cleared
                         // between decodes, and the data pages' kernels still read it)
    for (uint64_t i = threadIdx.x; i < n; i += WG) {
      dsrc[i] = S;
      dlen[i] = 0;
    }
    return;
  }
  int32_t st = 0;
  if (type_length > 0) {  // FLBA
    if (n * (uint64_t)type_length > dp.nbytes) st = ST_EOF;
    else
      for (uint64_t i = threadIdx.x; i < n; i += WG) {
        dsrc[i] = S + i * (uint64_t)type_length;
        dlen[i] = (uint32_t)type_length;
      }
  } else {
    st = plain_ba_walk(sm, blob, blob_len, S, dp.nbytes, n, dsrc, dlen);
  }
  // a dictionary that fails to decode: every entry empty, so that the data pages' kernels, which
  // run before the chunk's error is read, never follow an entry the walk did not write (the
  // reference stops at this page, configure_dictionary: column/reader.rs:463-481)
  __shared__ int32_t st_s;
  if (threadIdx.x == 0) st_s = 0;
  __syncthreads();
  if (st) st_s = st;
  __syncthreads();
  if (st_s) {
    for (uint64_t i = threadIdx.x; i < n; i += WG) {
      dsrc[i] = S;
      dlen[i] = 0;
    }
    if (threadIdx.x == 0) report(pages, chunks, dict_page, st_s);
  }
}

struct BaDictEmit {
  const uint64_t* dsrc;
  const uint32_t* dlen;
  uint32_t ndict;
  uint64_t* src;
  uint32_t* len;
  uint64_t bytes;
  int32_t err;
  bool index_only;  // the level path's chunks: the index in the length slot (BaSrc)
  __device__ void operator()(uint64_t g, const uint32_t* v, uint32_t mask) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (!((mask >> j) & 1)) continue;
      const uint32_t idx = v[j];
      if (idx >= ndict) {  // dict[idx] out of bounds: the reference panics
        err = ST_PANIC;
        continue;
      }
      const uint32_t l = dlen[idx];
      if (index_only) {
        len[g + j] = idx;
      } else {
        src[g + j] = dsrc[idx];
        len[g + j] = l;
      }
      bytes += l;
    }
  }
};

// Dictionary indices -> (source, length) of the entry: wave expand pass over the quarters of the
// listed tiles (the index pass: k_run_index with SS_DICT); per quarter-tile byte totals go to
// rt.qcount[4 t + q].
__global__ __attribute__((amdgpu_waves_per_eu(8, 8))) __launch_bounds__(64) void k_wexpand_badict(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                       PageWork* pages, ChunkWork* chunks, RunTables rt,
                                                       const uint32_t* __restrict__ tl, const uint64_t* dsrc,
                                                       const uint32_t* dlen, uint64_t* vsrc, uint32_t* vlen) {
  __shared__ WaveSmem sm;
  const uint32_t qi = 4u * tl[blockIdx.x >> 2] + (blockIdx.x & 3u);
  const QDesc d = load_qdesc(&rt.desc[qi]);
  BaDictEmit em{dsrc, dlen, 0u, vsrc, vlen, 0, 0, false};
  if (d.qhi) {
    const ChunkWork& ck = chunks[pages[d.page].chunk];
    em.dsrc += ck.dscr_base;
    em.dlen += ck.dscr_base;
    em.src += ck.scr_base;
    em.len += ck.scr_base;
    em.ndict = pages[ck.dict_page].num_values;
    wave_expand(blob, blob_len, d, rt.runs, sm, em);
  }
  const uint64_t bad = __ballot(em.err != 0);
  if (bad && (threadIdx.x & 63) == 0) report(pages, chunks, (int)d.page, ST_PANIC);
  uint64_t b = em.bytes;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) b += __shfl_xor(b, off, 64);
  if ((threadIdx.x & 63) == 0) rt.qcount[qi] = (uint32_t)min(b, (uint64_t)0xFFFFFFFFu);
}

// Byte-array dictionary index streams the level path handed back, one workgroup per page (as
// k_dict_fallback for fixed-width values): index walk, then each tile of the page expanded by the
// workgroup's four waves (one quarter each), the page's byte total summed.
__global__ void __launch_bounds__(WG) k_badict_fallback(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                        PageWork* pages, ChunkWork* chunks,
                                                        const uint32_t* __restrict__ tile_page, RunTables rt,
                                                        const uint64_t* dsrc, const uint32_t* dlen, uint64_t* vsrc,
                                                        uint32_t* vlen) {
  __shared__ IndexSmem ism;
  __shared__ WaveSmem wsm[WG / 64];
  __shared__ int32_t st_s;
  __shared__ uint64_t red[WG / 64];
  const int p = blockIdx.x;
  if (rt.pflag[p] != PF_BAIL) return;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  const ChunkWork& ck = chunks[pw.chunk];
  if (ck.es != 0) return;
  Stream s;
  if (!get_stream(blob, pw, SS_DICT, ck.cp, s)) return;
  if (ck.dict_page < 0) {  // "Decoder for dict should have been set"
    if (threadIdx.x == 0) report(pages, chunks, p, ST_PANIC);
    return;
  }
  if (!dict_usable(pages, ck)) return;
  if (threadIdx.x < 64) {
    const int32_t st = run_index(blob, blob_len, s, rt.ck + pw.ltile0, rt.runs + (uint64_t)pw.ltile0 * RUN_CAPT,
                                 rt.nruns + pw.ltile0, ism);
    if (threadIdx.x == 0) {
      st_s = st;
      if (st) report(pages, chunks, p, st);
    }
  }
  __syncthreads();
  if (st_s) return;
  const uint32_t wid = threadIdx.x >> 6;
  BaDictEmit em{dsrc + ck.dscr_base, dlen + ck.dscr_base, pages[ck.dict_page].num_values, vsrc + ck.scr_base,
                vlen + ck.scr_base, 0, 0, ck.lvdict != 0};
  for (uint32_t t = pw.ltile0; t < pw.ltile0 + pw.ntiles; ++t) {
    const QDesc d = quarter_desc(blob, pages, chunks, tile_page, rt, SS_DICT, t, wid);
    if (d.qhi) wave_expand(blob, blob_len, d, rt.runs, wsm[wid], em);
  }
  const uint64_t bad = __ballot(em.err != 0);
  if (bad && (threadIdx.x & 63) == 0) report(pages, chunks, p, ST_PANIC);
  const uint64_t tb = block_sum_u64(em.bytes, red);
  if (threadIdx.x == 0) {
    pages[p].nbytes_out = tb;
    pages[p].tile_bytes = 0;  // (windows the level path emitted before handing the page back)
  }
}

#include "pqg_balen.hpp"

__global__ void __launch_bounds__(WG) k_ba_index(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                                 PageWork* pages, ChunkWork* chunks, uint64_t* vsrc0,
                                                 uint32_t* vlen0, uint32_t* vpre0, const BlPage* blp) {
  __shared__ DeltaSmem sm;
  const int p = blockIdx.x;
  if (blp && blp[p].fast) return;  // (decoded by k_bl_*)
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  const ChunkWork& ck = chunks[pw.chunk];
  if (ck.es != 0 || !ck.val_out) return;
  const int type_length = ba_type_length(ck);
  uint64_t* vsrc = vsrc0 + ck.scr_base;
  uint32_t* vlen = vlen0 + ck.scr_base;
  uint32_t* vpre = vpre0 + ck.scr_base;
  const uint64_t n = pw.nonnull, vo = pw.value_out;
  const uint64_t S = pw.base + pw.val_off;
  const uint32_t slen = pw.val_bytes;
  uint64_t* src = vsrc + vo;
  uint32_t* len = vlen + vo;
  int32_t st = 0;
  bool dba = false, have_bytes = false;
  uint64_t bytes = 0;
  switch (pw.encoding) {
    case E_PLAIN:
      if (type_length > 0) {
        if (n * (uint64_t)type_length > slen) st = ST_EOF;
        else
          for (uint64_t i = threadIdx.x; i < n; i += WG) {
            src[i] = S + i * (uint64_t)type_length;
            len[i] = (uint32_t)type_length;
          }
      } else {
        st = plain_ba_walk(sm, blob, blob_len, S, slen, n, src, len);
      }
      break;
    case E_DELTA_LENGTH_BYTE_ARRAY: {
      // set_data decodes every length, then data.start_from(get_offset()) (:682-695)
      DeltaInfo li;
      st = delta_stream<4>(sm, blob, blob_len, S, slen, ~0ull, n, reinterpret_cast<uint8_t*>(len), li);
      // fewer lengths than values: the decoder's get returns short batches, then none (:697-711):
      // without levels read_batch makes no progress and loops forever (column/reader.rs:159-265);
      // with levels the values run short of the non-null levels (EOF here)
      const int32_t short_st = ck.cp.max_def == 0 && ck.cp.max_rep == 0 ? ST_HANG : ST_EOF;
      if (!st && li.total < n) st = short_st;
      if (!st && li.end_off > slen) st = ST_PANIC;
      if (!st) st = slices_from_lengths(sm, S + li.end_off, slen - li.end_off, n, len, src, bytes);
      have_bytes = true;
      break;
    }
    case E_DELTA_BYTE_ARRAY: {
      dba = true;
      uint32_t* pre = vpre + vo;
      DeltaInfo pi, si;
      st = delta_stream<4>(sm, blob, blob_len, S, slen, ~0ull, n, reinterpret_cast<uint8_t*>(pre), pi);
      if (!st && pi.total < n) st = ck.cp.max_def == 0 && ck.cp.max_rep == 0 ? ST_HANG : ST_EOF;  // (as above)
      if (!st && pi.end_off > slen) st = ST_PANIC;
      const uint32_t e1 = pi.end_off;
      if (!st) {
        __syncthreads();
        st = delta_stream<4>(sm, blob, blob_len, S + e1, slen - e1, ~0ull, n,
                             reinterpret_cast<uint8_t*>(len), si);
      }
      if (!st && (uint64_t)e1 + si.end_off > slen) st = ST_PANIC;
      if (!st) {
        const uint64_t e2 = (uint64_t)e1 + si.end_off;
        const uint64_t ns = si.total < n ? si.total : n;
        if (n > 0 && ns == 0) st = ST_PANIC;  // ByteArray::data() before set_data
        if (!st) st = dba_slices(sm, S + e2, slen - e2, n, ns, len, pre, src, bytes);
        have_bytes = true;
        if (!st && ns < n) {
          // suffix decoder exhausted: `v` keeps the last suffix (decoding.rs:796-801)
          __syncthreads();
          for (uint64_t i = ns + threadIdx.x; i < n; i += WG) {
            src[i] = src[ns - 1];
            len[i] = len[ns - 1];
          }
        }
      }
      break;
    }
    default:
      return;  // dictionary pages of data (k_ba_dict_idx)
  }
  if (st) {
    if (threadIdx.x == 0) report(pages, chunks, p, st);
    return;
  }
  __syncthreads();
  if (have_bytes) {
    if (threadIdx.x == 0) pages[p].nbytes_out = bytes;
  } else {
    page_bytes(sm, pages, p, n, len, nullptr);
  }
}

// Page byte offsets chunk by chunk (exclusive scan of nbytes_out restarted at each chunk's first
// page), the output capacity check and each byte-array chunk's final offset entry. One workgroup.
__global__ void __launch_bounds__(WG) k_scan_bytes(PageWork* pages, ChunkWork* chunks, int npages) {
  seg_scan_pages(
      pages, chunks, npages,
      [&](int p) -> uint64_t {
        const int t = pages[p].page_type;
        return (t == P_DATA || t == P_DATA_V2) ? pages[p].nbytes_out : 0ull;
      },
      [&](int p, uint64_t excl, uint64_t incl) {
        ChunkWork& ck = chunks[pages[p].chunk];
        pages[p].byte_out = excl;
        if (ck.es != 0) return;
        if (incl > excl && incl > ck.val_cap && pages[p].status == 0) report(pages, chunks, p, ST_CAPACITY);
        if ((uint32_t)p == ck.first_page + ck.npages - 1u) {
          ck.res.total_bytes = incl;
          if (ck.off_out) gp(ck.off_out)[ck.res.total_values] = (int64_t)incl;
        }
      });
}

// Gathers value slices into the output and writes their offsets (all encodings but
// DELTA_BYTE_ARRAY), tiled so a page of millions of values (a dictionary column's single data
// page) spreads over the chip: tiles of BA_T values, grid (tile, page).
//   k_ba_tsum   per tile: the tile-relative offset of each value (into `offsets`) and the
//               tile's byte total;
//   k_ba_tscan  per page: the tiles' start offsets (page byte_out + exclusive scan);
//   k_ba_copy   per tile: final offsets and the bytes.
constexpr uint32_t BA_VPT = 16;            // values per thread
constexpr uint32_t BA_T = BA_VPT * WG;     // values per tile: the pages' RUN_TILE tiles (ltile0, ntiles)
static_assert(BA_T == RUN_TILE, "byte-array tiles are the page table's tiles");

// (a dictionary page's data pages: only with a usable dictionary, dict_usable, as their index
// producers take them)
// ba_page_pre: the checks that do not need the chunk's byte total (k_ba_tsum runs before
// k_scan_bytes sets it); ba_page_ok adds the capacity check for the kernels after the scan.
__device__ inline bool ba_page_pre(const PageWork* pages, const PageWork& pw, const ChunkWork& ck) {
  return pw.status == 0 && (pw.page_type == P_DATA || pw.page_type == P_DATA_V2) && ck.es == 0 && ck.val_out &&
         pw.encoding != E_DELTA_BYTE_ARRAY && (pw.encoding != E_RLE_DICTIONARY || dict_usable(pages, ck));
}
__device__ inline bool ba_page_ok(const PageWork* pages, const PageWork& pw, const ChunkWork& ck) {
  return ba_page_pre(pages, pw, ck) && ck.res.total_bytes <= ck.val_cap;
}

// Value k of a byte-array page (k: its index among the chunk's values): source address and length.
// The dictionary pages of the level path's chunks (ChunkWork::lvdict) keep the value's dictionary
// index in the length slot (4 bytes per value instead of 12): the entry comes from the chunk's
// dictionary scratch (k_ba_dict_prep).
struct BaSrc {
  const uint64_t* vsrc;
  const uint32_t* vlen;
  const uint64_t* dsrc;
  const uint32_t* dlen;
  bool via_dict;
  uint32_t nd;  // dictionary entries: the consumers take only pages whose index slots were written
                // (ba_page_ok / dict_usable); an index past the dictionary still reads as empty
  BaSrc() = default;
  __device__ BaSrc(const ChunkWork& ck, const PageWork& pw, const PageWork* pages, const uint64_t* vsrc0,
                   const uint32_t* vlen0, const uint64_t* dsrc0, const uint32_t* dlen0)
      : vsrc(vsrc0 + ck.scr_base), vlen(vlen0 + ck.scr_base), dsrc(dsrc0 + ck.dscr_base),
        dlen(dlen0 + ck.dscr_base), via_dict(pw.encoding == E_RLE_DICTIONARY && ck.lvdict),
        nd(via_dict && ck.dict_page >= 0 ? pages[ck.dict_page].num_values : 0u) {}
  __device__ uint32_t len(uint64_t k) const {
    if (!via_dict) return vlen[k];
    const uint32_t i = vlen[k];
    return i < nd ? dlen[i] : 0u;
  }
  __device__ uint64_t src(uint64_t k) const {
    if (!via_dict) return vsrc[k];
    const uint32_t i = vlen[k];
    return i < nd ? dsrc[i] : 0u;
  }
};

constexpr uint32_t TS_DL = 2048;  // k_ba_tsum: dictionaries of at most this many entries staged in LDS

// Per listed tile (gt, global) of a byte-array page: the tile's byte count into tsum[gt] (the
// offsets themselves are written once, by k_ba_copy, from the scanned tile starts). A workgroup
// takes TS_K consecutive list entries: their tiles and pages are loaded at once, and the page's
// descriptors (and a small dictionary's entry lengths, staged in LDS) only when the page changes
// (config 5: 0.19 ms with one tile per workgroup, 8 tiles 0.17, 16 0.14, 32 0.14; two tiles'
// index loads in flight together took 107 VGPRs and 0.20 ms).
#ifndef PQG_TS_K
#define PQG_TS_K 16
#endif
constexpr uint32_t TS_K = PQG_TS_K;
__global__ void __launch_bounds__(WG) k_ba_tsum(PageWork* pages, const ChunkWork* chunks,
                                                const uint32_t* __restrict__ tile_page, const uint32_t* __restrict__ tl,
                                                uint32_t ntl, const uint64_t* vsrc0, const uint32_t* __restrict__ vlen0,
                                                const uint64_t* dsrc0, const uint32_t* dlen0,
                                                uint64_t* __restrict__ tsum) {
  __shared__ uint64_t red[WG / 64];
  __shared__ uint32_t sdl[TS_DL];  // a small dictionary's entry lengths
  __shared__ uint32_t lgt[TS_K], lpg[TS_K];
  const uint32_t e0 = blockIdx.x * TS_K, ne = min(TS_K, ntl - e0);
  if (threadIdx.x < ne) {
    const uint32_t gt = tl[e0 + threadIdx.x];
    lgt[threadIdx.x] = gt;
    lpg[threadIdx.x] = tile_page[gt];
  }
  __syncthreads();
  uint32_t cur = 0xFFFFFFFFu;  // the page whose descriptors are loaded (uniform)
  bool ok = false, lds = false;
  uint64_t n = 0, vo = 0;
  uint32_t ltile0 = 0, tbytes = 0;
  BaSrc bs;
#pragma unroll 1
  for (uint32_t i = 0; i < ne; ++i) {
    const uint32_t gt = lgt[i], p = lpg[i];
    if (p != cur) {
      cur = p;
      const PageWork pw = pages[p];
      const ChunkWork& ck = chunks[pw.chunk];
      ok = ba_page_pre(pages, pw, ck);  // (before the scan: no byte total yet)
      if (ok) {
        bs = BaSrc(ck, pw, pages, vsrc0, vlen0, dsrc0, dlen0);
        n = pw.nonnull;
        vo = pw.value_out;
        ltile0 = pw.ltile0;
        tbytes = pw.tile_bytes;
#ifdef PQG_TS_OFF
        lds = false;
#else
        lds = bs.via_dict && bs.nd <= TS_DL;  // the level path's dictionary chunks: lengths from LDS
#endif
        if (lds) {
          __syncthreads();  // (the previous page's lengths are read)
          for (uint32_t k = threadIdx.x; k < bs.nd; k += WG) sdl[k] = bs.dlen[k];
          __syncthreads();
        }
      }
    }
    if (!ok) continue;
    const uint32_t t = gt - ltile0;
    if ((uint64_t)t * BA_T >= n) continue;
    uint64_t s = 0;
    if (lds) {
      uint32_t ix[BA_VPT];
#pragma unroll
      for (uint32_t k = 0; k < BA_VPT; ++k) {  // every index load in flight
        const uint64_t j = (uint64_t)t * BA_T + (uint64_t)k * WG + threadIdx.x;
        ix[k] = j < n ? bs.vlen[vo + j] : 0xFFFFFFFFu;
      }
#pragma unroll
      for (uint32_t k = 0; k < BA_VPT; ++k) s += ix[k] < bs.nd ? sdl[ix[k]] : 0u;
    } else {
#pragma unroll
      for (uint32_t k = 0; k < BA_VPT; ++k) {  // lanes on consecutive values: coalesced
        const uint64_t j = (uint64_t)t * BA_T + (uint64_t)k * WG + threadIdx.x;
        s += j < n ? bs.len(vo + j) : 0u;
      }
    }
    const uint64_t tot = block_sum_u64(s, red);
    if (threadIdx.x == 0) {
      tsum[gt] = tot;
      if (tbytes) atomicAdd((unsigned long long*)&pages[p].nbytes_out, (unsigned long long)tot);
    }
  }
}

// Per byte-array page: its tiles' start offsets (page byte_out + exclusive scan of the tile sums).
__global__ void __launch_bounds__(WG) k_ba_tscan(PageWork* pages, const ChunkWork* chunks, uint64_t* __restrict__ tsum) {
  __shared__ DeltaSmem sm;
  const uint32_t p = blockIdx.x;
  const PageWork pw = pages[p];
  if (!ba_page_ok(pages, pw, chunks[pw.chunk])) return;
  const uint32_t nt = (uint32_t)((pw.nonnull + BA_T - 1) / BA_T);
  uint64_t carry = pw.byte_out;
  uint64_t* ts = tsum + pw.ltile0;
  for (uint32_t b = 0; b < nt; b += WG) {
    const uint32_t t = b + threadIdx.x;
    const uint64_t x = t < nt ? ts[t] : 0;
    uint64_t tot;
    const uint64_t pre = block_exscan(sm, x, tot);
    __syncthreads();  // every read of this pass's sums is done before the starts overwrite them
    if (t < nt) ts[t] = carry + pre;
    carry += tot;
  }
}

// Per listed tile of a byte-array page: the values' byte offsets (tile start from k_ba_tscan + an
// in-tile scan of the lengths) and their bytes.
//  - lengths come in coalesced (lanes on consecutive values) into LDS, laid out with one pad word
//    per 16 so that each thread's 16 consecutive values are read without bank conflicts for its
//    scan; their tile-relative offsets replace them in place (32-bit: a tile's bytes come from
//    one page, < 4 GiB); the offsets go out coalesced from LDS;
//  - values of at most BA_SMALL bytes (the common case: short strings) are staged: per round of
//    BA_RN values, each thread loads BA_RV values (lanes on consecutive ones) (16 bytes each, all loads in
//    flight together, no store between them to wait for) and writes their bytes into an LDS image
//    of the round's output, aligned as the output is; the workgroup then stores the image with
//    16-byte stores (byte stores at the round's two ends only);
//  - longer values are copied value by value, 8 bytes at a time.
__device__ inline uint32_t ba_pad(uint32_t j) { return j + (j >> 4); }

// Small dictionaries of the level path's byte-array chunks take k_ba_copy_sd (below).
constexpr uint32_t BSD_N = 1024;
constexpr uint32_t BSD_BYTES = 12288;
constexpr uint32_t BSD_IMG = WG * 8 * 8 + 32;  // round image: BSD_RN (2048) values of up to 8 bytes (longer: byte stores from LDS)

__device__ inline bool ba_small_dict(const PageWork& pw, const ChunkWork& ck, const PageWork* pages) {
  if (!(pw.encoding == E_RLE_DICTIONARY && ck.lvdict && ck.dict_page >= 0)) return false;
  const PageWork& dp = pages[ck.dict_page];
  return dp.num_values <= BSD_N && dp.nbytes <= BSD_BYTES;
}


constexpr uint32_t BA_RV = 4;                     // values per thread per staged round
constexpr uint32_t BA_RN = BA_RV * WG;            // values per round
constexpr uint32_t BA_SMALL = 16;                 // longest value the staged rounds take
constexpr uint32_t BA_IMG = BA_RN * BA_SMALL + 16; // bytes of a round's output image

__device__ inline void ba_load16(const uint8_t* __restrict__ blob, uint64_t blob_len, uint64_t a, uint32_t ln,
                                 uint64_t& x0, uint64_t& x1) {
  x0 = x1 = 0;
  if (ln == 0) return;
  if (a + 16 <= blob_len) {
    __builtin_memcpy(&x0, blob + a, 8);
    __builtin_memcpy(&x1, blob + a + 8, 8);
  } else {
    for (uint32_t q = 0; q < ln && a + q < blob_len; ++q) {
      const uint64_t b = blob[a + q];
      if (q < 8) x0 |= b << (8 * q);
      else x1 |= b << (8 * (q - 8));
    }
  }
}

// (one listed tile; every return is uniform over the workgroup)
__device__ inline void ba_copy_tile(const uint8_t* __restrict__ blob, uint64_t blob_len, PageWork* pages,
                                    const ChunkWork* chunks, uint32_t gt, uint32_t p,
                                    const uint64_t* __restrict__ vsrc0, const uint32_t* __restrict__ vlen0,
                                    const uint64_t* dsrc0, const uint32_t* dlen0, const uint64_t* __restrict__ tsum) {
  __shared__ uint32_t loff[BA_T + BA_T / 16 + 1];  // lengths, then tile-relative offsets (padded)
  __shared__ __attribute__((aligned(16))) uint8_t img[BA_IMG];
  __shared__ uint64_t wsum[WG / 64];
  __shared__ uint32_t wmax[WG / 64];
  const PageWork pw = pages[p];
  const ChunkWork& ck = chunks[pw.chunk];
  if (!ba_page_ok(pages, pw, ck) || ba_small_dict(pw, ck, pages)) return;  // (small dictionaries: k_ba_copy_sd)
  const uint32_t t = gt - pw.ltile0;
  const BaSrc bs(ck, pw, pages, vsrc0, vlen0, dsrc0, dlen0);
  const gptr<int64_t> __restrict__ offsets = gp(ck.off_out);
  const gptr<uint8_t> __restrict__ out = gp(ck.val_out);
  const uint64_t n = pw.nonnull, vo = pw.value_out;
  const uint64_t t0 = (uint64_t)t * BA_T;
  if (t0 >= n) return;
  const uint32_t cnt = (uint32_t)(n - t0 < BA_T ? n - t0 : BA_T);
  const uint64_t base = tsum[gt];
  const uint32_t tid = threadIdx.x;
#pragma unroll
  for (uint32_t k = 0; k < BA_VPT; ++k) {
    const uint32_t j = k * WG + tid;
    loff[ba_pad(j)] = j < cnt ? bs.len(vo + t0 + j) : 0u;
  }
  __syncthreads();
  uint32_t l[BA_VPT];
  uint64_t s = 0;
  uint32_t mx = 0;
#pragma unroll
  for (uint32_t k = 0; k < BA_VPT; ++k) {
    l[k] = loff[tid * 17u + k];  // value tid * 16 + k
    s += l[k];
    mx = l[k] > mx ? l[k] : mx;
  }
  // workgroup exclusive scan of the thread sums, and the longest value
  uint64_t incl = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off, 64);
    if ((tid & 63) >= (uint32_t)off) incl += y;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint32_t y = (uint32_t)__shfl_xor((int)mx, off, 64);
    mx = y > mx ? y : mx;
  }
  if ((tid & 63) == 63) wsum[tid >> 6] = incl;
  if ((tid & 63) == 0) wmax[tid >> 6] = mx;
  __syncthreads();
  uint64_t pre = incl - s, total = 0;
  uint32_t maxlen = 0;
  for (uint32_t w = 0; w < WG / 64; ++w) {
    if (w < (tid >> 6)) pre += wsum[w];
    total += wsum[w];
    maxlen = wmax[w] > maxlen ? wmax[w] : maxlen;
  }
  if (total >> 32) {  // (a tile of > 4 GiB: offsets from registers, values copied one by one)
    uint64_t d = pre;
#pragma unroll 1
    for (uint32_t k = 0; k < BA_VPT; ++k) {
      const uint32_t j = tid * BA_VPT + k;
      if (j >= cnt) break;
      offsets[vo + t0 + j] = (int64_t)(base + d);
      const uint8_t* sp = blob + bs.src(vo + t0 + j);
      for (uint64_t q = 0; q < l[k]; ++q) out[base + d + q] = sp[q];
      d += l[k];
    }
    return;
  }
#pragma unroll
  for (uint32_t k = 0; k < BA_VPT; ++k) {  // lengths -> offsets, in place (each thread its own)
    loff[tid * 17u + k] = (uint32_t)pre;
    pre += l[k];
  }
  if (tid == WG - 1) loff[ba_pad(BA_T)] = (uint32_t)total;
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < BA_VPT; ++k) {  // offsets, coalesced
    const uint32_t j = k * WG + tid;
    if (j < cnt) offsets[vo + t0 + j] = (int64_t)(base + loff[ba_pad(j)]);
  }
  if (maxlen > BA_SMALL) {  // long values: value by value, lanes on consecutive values
#pragma unroll 1
    for (uint32_t k = 0; k < BA_VPT; ++k) {
      const uint32_t j = k * WG + tid;
      if (j >= cnt) break;
      const uint32_t d0 = loff[ba_pad(j)], ln = loff[ba_pad(j + 1)] - d0;
      const uint8_t* sp = blob + bs.src(vo + t0 + j);
      gptr<uint8_t> o = out + base + d0;
      uint32_t q = 0;
      for (; q + 8 <= ln; q += 8) {
        uint64_t x;
        __builtin_memcpy(&x, sp + q, 8);
        __builtin_memcpy(o + q, &x, 8);
      }
      for (; q < ln; ++q) o[q] = sp[q];
    }
    return;
  }
#pragma unroll 1
  for (uint32_t r0 = 0; r0 < cnt; r0 += BA_RN) {
    const uint32_t r1 = r0 + BA_RN < cnt ? r0 + BA_RN : cnt;
    const uint32_t R0 = loff[ba_pad(r0)], R1 = loff[ba_pad(r1)];
    const uint64_t gA = base + R0, gB = base + R1;  // the round's output bytes
    const uint32_t sh = (uint32_t)(gA & 15u);        // image byte i = output byte gA - sh + i
    uint64_t x[BA_RV][2];
    uint32_t dd[BA_RV], ln[BA_RV];
#pragma unroll
    for (uint32_t i = 0; i < BA_RV; ++i) {  // loads of the thread's values, all in flight
      const uint32_t j = r0 + i * WG + tid;  // (lanes on consecutive values: their image bytes
                                             // fall in different LDS banks)
      ln[i] = 0;
      dd[i] = 0;
      if (j < r1) {
        dd[i] = loff[ba_pad(j)];
        ln[i] = loff[ba_pad(j + 1)] - dd[i];
        ba_load16(blob, blob_len, bs.src(vo + t0 + j), ln[i], x[i][0], x[i][1]);
      } else {
        x[i][0] = x[i][1] = 0;
      }
    }
#pragma unroll
    for (uint32_t i = 0; i < BA_RV; ++i) {  // their bytes into the image
      const uint32_t b0 = dd[i] - R0 + sh;
      for (uint32_t q = 0; q < ln[i]; ++q)
        img[b0 + q] = (uint8_t)((q < 8 ? x[i][0] >> (8 * q) : x[i][1] >> (8 * (q - 8))) & 0xFFu);
    }
    __syncthreads();
    const uint64_t c0 = gA & ~15ull;
    for (uint64_t c = c0 + (uint64_t)tid * 16u; c < gB; c += (uint64_t)WG * 16u) {
      const uint32_t ii = (uint32_t)(c - c0);
      if (c >= gA && c + 16 <= gB) {
        gst16(out + c, *reinterpret_cast<const uint4*>(img + ii));
      } else {
        for (uint32_t q = 0; q < 16; ++q)
          if (c + q >= gA && c + q < gB) out[c + q] = img[ii + q];
      }
    }
    __syncthreads();  // (the next round's bytes reuse the image)
  }
}

// BA_CK listed tiles per workgroup: their tiles and pages loaded at once, each page's check made
// once, so that the tiles k_ba_copy_sd takes (and those of pages past their checks) are passed
// over without a chain of dependent loads each
#ifndef PQG_BA_CK
#define PQG_BA_CK 8
#endif
constexpr uint32_t BA_CK = PQG_BA_CK;
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(4))) k_ba_copy(const uint8_t* __restrict__ blob, uint64_t blob_len, PageWork* pages,
                                                const ChunkWork* chunks, const uint32_t* __restrict__ tile_page,
                                                const uint32_t* __restrict__ tl, uint32_t ntl,
                                                const uint64_t* __restrict__ vsrc0, const uint32_t* __restrict__ vlen0,
                                                const uint64_t* dsrc0, const uint32_t* dlen0,
                                                const uint64_t* __restrict__ tsum) {
  __shared__ uint32_t lgt[BA_CK], lpg[BA_CK];
  const uint32_t e0 = blockIdx.x * BA_CK, ne = min(BA_CK, ntl - e0);
  if (threadIdx.x < ne) {
    const uint32_t gt = tl[e0 + threadIdx.x];
    lgt[threadIdx.x] = gt;
    lpg[threadIdx.x] = tile_page[gt];
  }
  __syncthreads();
  uint32_t cur = 0xFFFFFFFFu;
  bool ok = false;
#pragma unroll 1
  for (uint32_t i = 0; i < ne; ++i) {
    const uint32_t p = lpg[i];
    if (p != cur) {
      cur = p;
      const PageWork pw = pages[p];
      const ChunkWork& ck = chunks[pw.chunk];
      ok = ba_page_ok(pages, pw, ck) && !ba_small_dict(pw, ck, pages);
    }
    if (!ok) continue;
    ba_copy_tile(blob, blob_len, pages, chunks, lgt[i], p, vsrc0, vlen0, dsrc0, dlen0, tsum);
    __syncthreads();  // (the next tile reuses the LDS)
  }
}

// k_ba_copy for the dictionary pages of the level path's chunks whose dictionary is small (at most
// BSD_N entries in at most BSD_BYTES bytes: short categorical strings): the dictionary page's bytes
// and its entries' offsets and lengths are staged in LDS, so a value's length and bytes cost LDS
// reads only; the only global loads are the values' indices (coalesced, all 16 in flight at once).
// The tile goes in two rounds of BSD_RN values (lane l: values k * WG + l, k-major): eight wave
// scans of the round's lengths and one exchange of their totals give its offsets (stored
// coalesced); its bytes are assembled in an LDS image of the round's output (8-byte strings of a
// whole round fit) and stored with 16-byte stores. The general kernel exits for these tiles. A
// workgroup takes BSD_K consecutive list entries and stages a dictionary once for those of its
// tiles that share it (one tile per workgroup: 0.56 ms per config-5 step, 4: 0.51, 8: 0.51-0.52,
// 16: 0.54); the list entries and their pages are loaded at once and a page's descriptors once.
#ifndef PQG_BSD_K
#define PQG_BSD_K 4
#endif
constexpr uint32_t BSD_K = PQG_BSD_K;
constexpr uint32_t BSD_RV = 8;                    // values per thread per round
constexpr uint32_t BSD_RN = BSD_RV * WG;          // values per round
static_assert(BSD_RN * 2 == BA_T, "two rounds per tile");

__global__ void __launch_bounds__(WG) k_ba_copy_sd(const uint8_t* __restrict__ blob, uint64_t blob_len, PageWork* pages,
                                                   const ChunkWork* chunks, const uint32_t* __restrict__ tile_page,
                                                   const uint32_t* __restrict__ tl, uint32_t ntl,
                                                   const uint32_t* __restrict__ vlen0, const uint64_t* __restrict__ dsrc0,
                                                   const uint32_t* __restrict__ dlen0, const uint64_t* __restrict__ tsum) {
  __shared__ __attribute__((aligned(16))) uint8_t ldict[BSD_BYTES + 48];
  __shared__ uint32_t doff[BSD_N], dln[BSD_N];
  __shared__ __attribute__((aligned(16))) uint8_t img[BSD_IMG + 32];
  __shared__ uint32_t wsum[BSD_RV][WG / 64];
  __shared__ uint32_t lgt[BSD_K], lpg[BSD_K];
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t e0 = blockIdx.x * BSD_K, ne = min(BSD_K, ntl - e0);
  if (tid < ne) {  // the workgroup's list entries and their pages, loaded at once
    const uint32_t gt = tl[e0 + tid];
    lgt[tid] = gt;
    lpg[tid] = tile_page[gt];
  }
  __syncthreads();
  uint32_t cur = 0xFFFFFFFFu;  // the page whose descriptors are loaded (uniform)
  bool ok = false;
  uint64_t n = 0, vo = 0;
  uint32_t ltile0 = 0, nd = 0;
  gptr<int64_t> offsets = gptr<int64_t>(nullptr);
  gptr<uint8_t> out = gptr<uint8_t>(nullptr);
  const uint32_t* vlen = nullptr;
  int32_t staged = -1;  // the dictionary page ldict / doff / dln hold (uniform)
#pragma unroll 1
  for (uint32_t i = 0; i < ne; ++i) {
    const uint32_t gt = lgt[i], p = lpg[i];
    if (p != cur) {  // the page's descriptors, and its dictionary staged unless it is already
      cur = p;
      const PageWork pw = pages[p];
      const ChunkWork& ck = chunks[pw.chunk];
      ok = ba_page_ok(pages, pw, ck) && ba_small_dict(pw, ck, pages);
      if (ok) {
        n = pw.nonnull;
        vo = pw.value_out;
        ltile0 = pw.ltile0;
        offsets = gp(ck.off_out);
        out = gp(ck.val_out);
        vlen = vlen0 + ck.scr_base;
        // the dictionary page in 16-byte chunks from its aligned start (entry offsets relative to it)
        const PageWork& dp = pages[ck.dict_page];
        nd = dp.num_values;
        if (staged != ck.dict_page) {
          const uint32_t nb = dp.nbytes;
          const uint64_t db = dp.base & ~15ull;
          const uint32_t nch = (uint32_t)((dp.base + nb - db + 15) / 16);
          __syncthreads();  // (the previous dictionary's reads are done)
          for (uint32_t c = tid; c < nch; c += WG) {
            const uint64_t a = db + (uint64_t)c * 16;
            reinterpret_cast<uint4*>(ldict)[c] = a + 16 <= blob_len ? *reinterpret_cast<const uint4*>(blob + a)
                                                                    : gload_u128_tail(blob, blob_len, a);
          }
          for (uint32_t k = tid; k < nd; k += WG) {
            doff[k] = (uint32_t)(dsrc0[ck.dscr_base + k] - db);
            dln[k] = dlen0[ck.dscr_base + k];
          }
          staged = ck.dict_page;
          __syncthreads();
        }
      }
    }
    if (!ok) continue;
    const uint32_t t = gt - ltile0;
    const uint64_t t0 = (uint64_t)t * BA_T;
    if (t0 >= n) continue;
    const uint32_t cnt = (uint32_t)(n - t0 < BA_T ? n - t0 : BA_T);
    // the tile's indices, all loads in flight (lane l: values k * WG + l)
    uint32_t idx[BA_VPT];
#pragma unroll
    for (uint32_t k = 0; k < BA_VPT; ++k) {
      const uint32_t j = k * WG + tid;
      idx[k] = j < cnt ? vlen[vo + t0 + j] : 0u;
    }
    uint64_t run = tsum[gt];  // output byte offset of the round's first value
#pragma unroll 1
    for (uint32_t r = 0; r < 2; ++r) {
      if (r * BSD_RN >= cnt) break;
      uint32_t ln[BSD_RV], so[BSD_RV], pre[BSD_RV];
#pragma unroll
      for (uint32_t k = 0; k < BSD_RV; ++k) {
        const uint32_t kk = r * BSD_RV + k, j = kk * WG + tid;
        // (an index slot past the dictionary: empty, as BaSrc)
        const bool in = j < cnt && idx[kk] < nd;
        ln[k] = in ? dln[idx[kk]] : 0u;
        so[k] = in ? doff[idx[kk]] : 0u;
        const uint32_t inc = wave_scan_incl_u32(ln[k]);
        pre[k] = inc - ln[k];
        if (lane == 63u) wsum[k][wv] = inc;
      }
      __syncthreads();
      uint32_t tot = 0;
#pragma unroll
      for (uint32_t k = 0; k < BSD_RV; ++k) {  // value (k, tid): the rows before, the waves before
        uint32_t rb = 0;
#pragma unroll
        for (uint32_t w = 0; w < WG / 64; ++w) {
          const uint32_t x = wsum[k][w];
          if (w < wv) pre[k] += x;
          rb += x;
        }
        pre[k] += tot;
        tot += rb;
      }
#pragma unroll
      for (uint32_t k = 0; k < BSD_RV; ++k) {
        const uint32_t j = (r * BSD_RV + k) * WG + tid;
        if (j < cnt) offsets[vo + t0 + j] = (int64_t)(run + pre[k]);
      }
      const uint64_t gA = run, gB = run + tot;
      const uint32_t sh = (uint32_t)(gA & 15u);
      if (tot + 32 <= BSD_IMG) {  // staged: the round's bytes in an LDS image aligned as the output is
#pragma unroll
        for (uint32_t k = 0; k < BSD_RV; ++k) {
          const uint32_t b0 = pre[k] + sh;
          for (uint32_t q = 0; q < ln[k]; ++q) img[b0 + q] = ldict[so[k] + q];
        }
        __syncthreads();
        const uint64_t c0 = gA & ~15ull;
        for (uint64_t c = c0 + (uint64_t)tid * 16u; c < gB; c += (uint64_t)WG * 16u) {
          const uint32_t ii = (uint32_t)(c - c0);
          if (c >= gA && c + 16 <= gB) {
            gst16(out + c, *reinterpret_cast<const uint4*>(img + ii));
          } else {
            for (uint32_t q = 0; q < 16; ++q)
              if (c + q >= gA && c + q < gB) out[c + q] = img[ii + q];
          }
        }
      } else {  // long values: straight from the LDS dictionary
#pragma unroll 1
        for (uint32_t k = 0; k < BSD_RV; ++k)
          for (uint32_t q = 0; q < ln[k]; ++q) out[gA + pre[k] + q] = ldict[so[k] + q];
      }
      run += tot;
      __syncthreads();  // (wsum and the image are reused by the next round)
    }
  }
}

// ====================================================================== DELTA_BYTE_ARRAY rebuild
//
// Value i = the first pre_i bytes of value i-1 ++ suffix_i (DeltaByteArrayDecoder::get,
// decoding.rs:794-822): a serial dependency from value to value. Unrolled, byte j of value i is
// byte j of value k = max{k <= i : pre_k <= j}, i.e. a byte of k's suffix. With a = psv(i) =
// max{k < i : pre_k < pre_i} (the previous strictly smaller prefix length), every value in
// (a, i) has pre >= pre_i, so bytes [pre_a, pre_i) of value i are suffix_a's first
// pre_i - pre_a bytes, and bytes [0, pre_a) are value a's, by the same rule from a. A value is
// therefore a few slices of earlier suffixes (its chain i, psv(i), psv(psv(i)), ... down to a
// prefix length of 0), each copied straight from the page into the output; nothing is rebuilt
// value by value and there is no length limit. Four passes over the tiles of BA_T values:
//   k_dba_tiles  per tile: byte total (sum of pre + suffix length), the prefix-length minimum of
//                each 64-value block and of the tile;
//   k_dba_pages  per page: the tiles' byte starts (page byte_out + scan) and each tile's
//                previous tile of smaller minimum (tpsv, a pointer jump over the tiles);
//   k_dba_psv    per tile: value offsets (in-tile scan), psv of every value: its own block, then
//                the tile's blocks (minima in LDS), then earlier tiles through tpsv and their
//                block minima (at most ~64 + 64 steps + the tile jumps + 64 + 64);
//   k_dba_copy   per tile: each lane its values' slices (suffix first, then the chain); slices
//                longer than DBA_LONG are queued in LDS and copied by whole waves.
// Validity (pre_i <= length of value i-1, pre_0 = 0) is checked by k_ba_index, so every chain
// ends at a value of prefix length 0.
constexpr uint32_t DBA_NONE = 0xFFFFFFFFu;
constexpr uint32_t DBA_TSTRIDE = 66;  // per tile: 64 block minima, the tile minimum, tpsv
constexpr uint32_t DBA_LONG = 256;    // slices longer than this: copied by a whole wave
constexpr uint32_t DBA_QCAP = 512;    // queued long slices per tile

__device__ inline bool dba_page_ok(const PageWork& pw, const ChunkWork& ck) {
  return pw.status == 0 && (pw.page_type == P_DATA || pw.page_type == P_DATA_V2) && pw.encoding == E_DELTA_BYTE_ARRAY &&
         ck.es == 0 && ck.val_out && ck.res.total_bytes <= ck.val_cap;
}

__global__ void __launch_bounds__(WG) k_dba_tiles(PageWork* pages, const ChunkWork* chunks,
                                                  const uint32_t* __restrict__ tile_page, const uint32_t* __restrict__ tl,
                                                  const uint32_t* __restrict__ vlen0, const uint32_t* __restrict__ vpre0,
                                                  uint64_t* __restrict__ tsum, uint32_t* __restrict__ dtile) {
  __shared__ uint64_t red[WG / 64];
  __shared__ uint32_t mred[WG / 64];
  const uint32_t gt = tl[blockIdx.x], p = tile_page[gt];
  const PageWork pw = pages[p];
  const ChunkWork& ck = chunks[pw.chunk];
  if (!dba_page_ok(pw, ck)) return;
  const uint64_t n = pw.nonnull, t0 = (uint64_t)(gt - pw.ltile0) * BA_T;
  if (t0 >= n) return;
  const uint32_t cnt = (uint32_t)(n - t0 < BA_T ? n - t0 : BA_T);
  const uint32_t* vlen = vlen0 + ck.scr_base + pw.value_out + t0;
  const uint32_t* vpre = vpre0 + ck.scr_base + pw.value_out + t0;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  uint32_t* dt = dtile + (uint64_t)gt * DBA_TSTRIDE;
  uint64_t s = 0;
  uint32_t tm = DBA_NONE;
#pragma unroll 4
  for (uint32_t k = 0; k < BA_VPT; ++k) {  // block k * 4 + wave: 64 consecutive values
    const uint32_t j = k * WG + tid;
    const uint32_t pre = j < cnt ? vpre[j] : DBA_NONE;
    if (j < cnt) s += (uint64_t)pre + vlen[j];
    const uint32_t bm = wave_min_u32(pre);
    if (lane == 0) dt[k * 4 + wv] = bm;
    tm = bm < tm ? bm : tm;
  }
  if (lane == 0) mred[wv] = tm;
  const uint64_t tot = block_sum_u64(s, red);  // (its barriers order mred too)
  if (tid == 0) {
    tsum[gt] = tot;
    uint32_t m = mred[0];
    for (uint32_t w = 1; w < WG / 64; ++w) m = mred[w] < m ? mred[w] : m;
    dt[64] = m;
  }
}

__global__ void __launch_bounds__(WG) k_dba_pages(PageWork* pages, const ChunkWork* chunks, uint64_t* __restrict__ tsum,
                                                  uint32_t* __restrict__ dtile) {
  __shared__ uint64_t wsum[WG / 64];
  __shared__ uint64_t carry_s;
  const uint32_t p = blockIdx.x;
  const PageWork pw = pages[p];
  if (!dba_page_ok(pw, chunks[pw.chunk])) return;
  const uint32_t nt = (uint32_t)((pw.nonnull + BA_T - 1) / BA_T);
  const uint32_t tid = threadIdx.x;
  uint64_t* ts = tsum + pw.ltile0;
  if (tid == 0) carry_s = pw.byte_out;
  __syncthreads();
  for (uint32_t b = 0; b < nt; b += WG) {  // tile byte starts
    const uint32_t t = b + tid;
    const uint64_t x = t < nt ? ts[t] : 0ull;
    uint64_t incl = x;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint64_t y = __shfl_up(incl, off, 64);
      if ((tid & 63u) >= (uint32_t)off) incl += y;
    }
    if ((tid & 63u) == 63u) wsum[tid >> 6] = incl;
    __syncthreads();
    uint64_t pre = carry_s + incl - x, tot = 0;
    for (uint32_t w = 0; w < WG / 64; ++w) {
      if (w < (tid >> 6)) pre += wsum[w];
      tot += wsum[w];
    }
    if (t < nt) ts[t] = pre;
    __syncthreads();
    if (tid == 0) carry_s += tot;
    __syncthreads();
  }
  if (tid == 0) {  // previous tile of strictly smaller minimum (amortized O(1) per tile)
    uint32_t* dt = dtile + (uint64_t)pw.ltile0 * DBA_TSTRIDE;
    for (uint32_t t = 0; t < nt; ++t) {
      const uint32_t m = dt[(uint64_t)t * DBA_TSTRIDE + 64];
      uint32_t j = t ? t - 1 : DBA_NONE;
      while (j != DBA_NONE && dt[(uint64_t)j * DBA_TSTRIDE + 64] >= m) j = dt[(uint64_t)j * DBA_TSTRIDE + 65];
      dt[(uint64_t)t * DBA_TSTRIDE + 65] = j;
    }
  }
}

__global__ void __launch_bounds__(WG) k_dba_psv(PageWork* pages, const ChunkWork* chunks,
                                                const uint32_t* __restrict__ tile_page, const uint32_t* __restrict__ tl,
                                                const uint32_t* __restrict__ vlen0, const uint32_t* __restrict__ vpre0,
                                                const uint64_t* __restrict__ tsum, const uint32_t* __restrict__ dtile,
                                                uint32_t* __restrict__ vaux0) {
  __shared__ uint32_t pre_s[BA_T + BA_T / 16 + 1];
  __shared__ uint32_t off_s[BA_T + BA_T / 16 + 1];  // value lengths, then tile-relative offsets
  __shared__ uint32_t bmin_s[64];
  __shared__ uint64_t wsum[WG / 64];
  const uint32_t gt = tl[blockIdx.x], p = tile_page[gt];
  const PageWork pw = pages[p];
  const ChunkWork& ck = chunks[pw.chunk];
  if (!dba_page_ok(pw, ck)) return;
  const uint32_t t = gt - pw.ltile0;
  const uint64_t n = pw.nonnull, t0 = (uint64_t)t * BA_T;
  if (t0 >= n) return;
  const uint32_t cnt = (uint32_t)(n - t0 < BA_T ? n - t0 : BA_T);
  const uint64_t vb = ck.scr_base + pw.value_out;  // scratch slot of the page's value 0
  const uint32_t* vpre = vpre0 + vb;
  const uint32_t tid = threadIdx.x;
#pragma unroll 4
  for (uint32_t k = 0; k < BA_VPT; ++k) {
    const uint32_t j = k * WG + tid;
    const uint32_t pr = j < cnt ? vpre[t0 + j] : 0u;
    pre_s[ba_pad(j)] = pr;
    off_s[ba_pad(j)] = j < cnt ? pr + vlen0[vb + t0 + j] : 0u;
  }
  if (tid < 64) bmin_s[tid] = dtile[(uint64_t)gt * DBA_TSTRIDE + tid];
  __syncthreads();
  // ---- value offsets: tile start + in-tile scan (each thread 16 consecutive values)
  uint32_t l[BA_VPT];
  uint64_t s = 0;
#pragma unroll
  for (uint32_t k = 0; k < BA_VPT; ++k) {
    l[k] = off_s[tid * 17u + k];
    s += l[k];
  }
  uint64_t incl = s;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off, 64);
    if ((tid & 63u) >= (uint32_t)off) incl += y;
  }
  if ((tid & 63u) == 63u) wsum[tid >> 6] = incl;
  __syncthreads();
  uint64_t pre = incl - s, total = 0;
  for (uint32_t w = 0; w < WG / 64; ++w) {
    if (w < (tid >> 6)) pre += wsum[w];
    total += wsum[w];
  }
  const gptr<int64_t> __restrict__ offsets = gp(ck.off_out) + pw.value_out + t0;
  const uint64_t base = tsum[gt];
  if (total >> 32) {  // (a tile of > 4 GiB: offsets straight from registers)
#pragma unroll 1
    for (uint32_t k = 0; k < BA_VPT; ++k) {
      const uint32_t j = tid * BA_VPT + k;
      if (j < cnt) offsets[j] = (int64_t)(base + pre);
      pre += l[k];
    }
  } else {
#pragma unroll
    for (uint32_t k = 0; k < BA_VPT; ++k) {
      off_s[tid * 17u + k] = (uint32_t)pre;
      pre += l[k];
    }
    __syncthreads();
#pragma unroll 4
    for (uint32_t k = 0; k < BA_VPT; ++k) {
      const uint32_t j = k * WG + tid;
      if (j < cnt) offsets[j] = (int64_t)(base + off_s[ba_pad(j)]);
    }
  }
  // ---- psv of every value (page-relative index; DBA_NONE for prefix length 0)
  const uint32_t* dtp = dtile + (uint64_t)pw.ltile0 * DBA_TSTRIDE;  // the page's tiles
  uint32_t* vaux = vaux0 + vb;
#pragma unroll 1
  for (uint32_t k = 0; k < BA_VPT; ++k) {
    const uint32_t j = k * WG + tid;
    if (j >= cnt) break;
    const uint32_t x = pre_s[ba_pad(j)];
    uint32_t r = DBA_NONE;
    if (x > 0) {
      // every scan below reads its 64 candidates at once (unrolled, no early exit): a dependent
      // load per step took ~128 global round trips for a value whose psv lies tiles back
      const uint32_t b0 = j & ~63u;
      int lr = -1;
#pragma unroll
      for (int i = 0; i < 64; ++i) {  // own block, before j
        const uint32_t q = b0 + (uint32_t)i;
        lr = (q < j && pre_s[ba_pad(q)] < x) ? i : lr;
      }
      if (lr >= 0) {
        r = (uint32_t)t0 + b0 + (uint32_t)lr;
      } else {
        int lb = -1;  // the tile's earlier blocks
#pragma unroll
        for (int bb = 0; bb < 64; ++bb) lb = ((uint32_t)bb < (j >> 6) && bmin_s[bb] < x) ? bb : lb;
        if (lb >= 0) {
#pragma unroll
          for (int i = 0; i < 64; ++i) lr = pre_s[ba_pad((uint32_t)lb * 64u + (uint32_t)i)] < x ? i : lr;
          r = (uint32_t)t0 + (uint32_t)lb * 64u + (uint32_t)lr;
        } else if (t > 0) {  // earlier tiles: jump to the nearest of minimum < x
          uint32_t u = t - 1;
          while (u != DBA_NONE && dtp[(uint64_t)u * DBA_TSTRIDE + 64] >= x) u = dtp[(uint64_t)u * DBA_TSTRIDE + 65];
          if (u != DBA_NONE) {
            const uint32_t* um = dtp + (uint64_t)u * DBA_TSTRIDE;
#pragma unroll
            for (int bb = 0; bb < 64; ++bb) lb = um[bb] < x ? bb : lb;
            if (lb >= 0) {
              const uint32_t* up = vpre + (uint64_t)u * BA_T + (uint32_t)lb * 64u;
#pragma unroll
              for (int i = 0; i < 64; ++i) lr = up[i] < x ? i : lr;
              if (lr >= 0) r = u * BA_T + (uint32_t)lb * 64u + (uint32_t)lr;
            }
          }
        }
      }
    }
    vaux[t0 + j] = r;
  }
}

// One slice of a value: dst <- src[0, len), 8 bytes at a time.
__device__ inline void dba_slice(gptr<uint8_t> dst, const uint8_t* src, uint32_t len) {
  uint32_t q = 0;
  for (; q + 8 <= len; q += 8) {
    uint64_t x;
    __builtin_memcpy(&x, src + q, 8);
    __builtin_memcpy(dst + q, &x, 8);
  }
  for (; q < len; ++q) dst[q] = src[q];
}

__global__ void __launch_bounds__(WG) k_dba_copy(const uint8_t* __restrict__ blob, PageWork* pages, const ChunkWork* chunks,
                                                 const uint32_t* __restrict__ tile_page, const uint32_t* __restrict__ tl,
                                                 const uint64_t* __restrict__ vsrc0, const uint32_t* __restrict__ vlen0,
                                                 const uint32_t* __restrict__ vpre0, const uint32_t* __restrict__ vaux0) {
  __shared__ uint64_t qdst[DBA_QCAP], qsrc[DBA_QCAP];
  __shared__ uint32_t qlen[DBA_QCAP];
  __shared__ uint32_t qn;
  const uint32_t gt = tl[blockIdx.x], p = tile_page[gt];
  const PageWork pw = pages[p];
  const ChunkWork& ck = chunks[pw.chunk];
  if (!dba_page_ok(pw, ck)) return;
  const uint64_t n = pw.nonnull, t0 = (uint64_t)(gt - pw.ltile0) * BA_T;
  if (t0 >= n) return;
  const uint64_t vb = ck.scr_base + pw.value_out;
  const uint64_t* vsrc = vsrc0 + vb;
  const uint32_t* vlen = vlen0 + vb;
  const uint32_t* vpre = vpre0 + vb;
  const uint32_t* vaux = vaux0 + vb;
  const gptr<int64_t> __restrict__ offsets = gp(ck.off_out) + pw.value_out;
  const gptr<uint8_t> __restrict__ out = gp(ck.val_out);
  const uint32_t tid = threadIdx.x;
  if (tid == 0) qn = 0;
  __syncthreads();
  auto slice = [&](uint64_t d, uint64_t src, uint32_t len) {
    if (len > DBA_LONG) {
      const uint32_t qi = atomicAdd(&qn, 1u);
      if (qi < DBA_QCAP) {
        qdst[qi] = d;
        qsrc[qi] = src;
        qlen[qi] = len;
        return;
      }
    }
    dba_slice(out + d, blob + src, len);
  };
#pragma unroll 1
  for (uint32_t k = 0; k < BA_VPT; ++k) {  // lanes on consecutive values
    const uint64_t i = t0 + k * WG + tid;
    if (i >= n) break;
    const uint64_t o = (uint64_t)offsets[i];
    uint32_t cp = vpre[i];
    slice(o + cp, vsrc[i], vlen[i]);  // its own suffix
    uint64_t cur = i;
    while (cp > 0) {  // then the chain of previous smaller prefix lengths
      const uint32_t a = vaux[cur];
      if (a == DBA_NONE) break;  // (not reached: k_ba_index checked the prefix lengths)
      const uint32_t pa = vpre[a];
      slice(o + pa, vsrc[a], cp - pa);
      cp = pa;
      cur = a;
    }
  }
  __syncthreads();
  const uint32_t nq = qn < DBA_QCAP ? qn : DBA_QCAP;
  const uint32_t lane = tid & 63u;
#pragma unroll 1
  for (uint32_t e = tid >> 6; e < nq; e += WG / 64) {  // long slices: one wave each
    const gptr<uint8_t> d = out + qdst[e];
    const uint8_t* sp = blob + qsrc[e];
    const uint32_t len = qlen[e];
    uint32_t q = lane * 8u;
    for (; q + 8 <= len; q += 512u) {
      uint64_t x;
      __builtin_memcpy(&x, sp + q, 8);
      __builtin_memcpy(d + q, &x, 8);
    }
    if (q < len)  // the lane holding the tail
      for (; q < len; ++q) d[q] = sp[q];
  }
}

extern "C" {

hipError_t pqg_launch_quarter_desc(const uint8_t* blob, PageWork* pages, ChunkWork* chunks, const uint32_t* tile_page,
                                   const uint32_t* tl, uint32_t ntl, RunTables rt, int sel, hipStream_t s);
hipError_t pqg_launch_page_counts(PageWork* pages, int npages, ChunkWork* chunks, RunTables rt, hipStream_t s);

// Dictionary pages of the byte-array chunks (one workgroup per chunk of the decode).
hipError_t pqg_launch_ba_dict_prep(const uint8_t* blob, uint64_t blob_len, PageWork* pages, ChunkWork* chunks,
                                   int nchunks, uint64_t* dsrc, uint32_t* dlen, hipStream_t s) {
  if (nchunks > 0)
    hipLaunchKernelGGL(k_ba_dict_prep, dim3(nchunks), dim3(WG), 0, s, blob, blob_len, pages, chunks, dsrc, dlen);
  return hipGetLastError();
}

// Byte-array dictionary indices off the level path: the pages it handed back (one workgroup per
// page), then the general decoder's expand over the listed tiles of the chunks it does not take
// (larger dictionaries; their index pass ran before), and the page byte totals of those.
hipError_t pqg_launch_badict_general(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages,
                                     ChunkWork* chunks, const uint32_t* tile_page, const uint32_t* tl, uint32_t ntl,
                                     RunTables rt, uint64_t* dsrc, uint32_t* dlen, uint64_t* vsrc, uint32_t* vlen,
                                     int lv, hipStream_t s) {
  if (lv)
    hipLaunchKernelGGL(k_badict_fallback, dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, chunks, tile_page, rt,
                       dsrc, dlen, vsrc, vlen);
  if (ntl) {
    hipError_t e = pqg_launch_quarter_desc(blob, pages, chunks, tile_page, tl, ntl, rt, (int)SS_DICT, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_wexpand_badict, dim3(ntl * 4), dim3(64), 0, s, blob, blob_len, pages, chunks, rt, tl, dsrc,
                       dlen, vsrc, vlen);
    e = pqg_launch_page_counts(pages, npages, chunks, rt, s);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

// Byte-array values of every byte-array chunk: lengths and sources of the PLAIN / DELTA_LENGTH /
// DELTA_BYTE_ARRAY pages, page byte offsets, then the tiled copy over the listed tiles (the tiles
// of the byte-array pages) and the DELTA_BYTE_ARRAY rebuild.
hipError_t pqg_launch_bytes(const uint8_t* blob, uint64_t blob_len, PageWork* pages, int npages, ChunkWork* chunks,
                            const uint32_t* tile_page, const uint32_t* tl, uint32_t ntl, bool has_dba, bool has_lvdict,
                            uint64_t* vsrc, uint32_t* vlen, uint32_t* vpre, const uint64_t* dsrc, const uint32_t* dlen,
                            uint64_t* tsum, uint32_t* vaux, uint32_t* dtile, const uint32_t* bl, uint32_t nbl,
                            uint32_t bl_tiles, uint8_t* blbuf, uint32_t ntiles_all, hipStream_t s) {
  BlPage* blp = nullptr;
  if (nbl) {  // the large DELTA_LENGTH / DELTA_BYTE_ARRAY pages' length streams (pqg_balen.hpp)
    BlArgs a;
    a.list = bl;
    a.nlist = nbl;
    a.maxtiles = bl_tiles;
    a.pg = blp = reinterpret_cast<BlPage*>(blbuf);
    a.tile = reinterpret_cast<BlTile*>(blbuf + (size_t)npages * 64);
    a.blk = reinterpret_cast<uint32_t*>(blbuf + (size_t)npages * 64 + ((size_t)ntiles_all + 1) * sizeof(BlTile));
    a.blk_stride = ((uint64_t)ntiles_all + 1) * BL_BPT;
    (void)hipMemsetAsync(blp, 0, (size_t)npages * sizeof(BlPage), s);
    const dim3 tg(bl_tiles, nbl);
    hipLaunchKernelGGL(k_bl_walk, dim3(nbl), dim3(BLW), 0, s, blob, blob_len, pages, chunks, a);
    hipLaunchKernelGGL(k_bl_tile<0>, tg, dim3(WG), 0, s, blob, blob_len, pages, chunks, a, vlen, vpre);
    hipLaunchKernelGGL(k_bl_scan<0>, dim3(nbl), dim3(WG), 0, s, pages, a);
    hipLaunchKernelGGL(k_bl_tile<1>, tg, dim3(WG), 0, s, blob, blob_len, pages, chunks, a, vlen, vpre);
    hipLaunchKernelGGL(k_bl_scan<1>, dim3(nbl), dim3(WG), 0, s, pages, a);
    hipLaunchKernelGGL(k_bl_src, tg, dim3(WG), 0, s, pages, chunks, a, vsrc, vlen, vpre);
  }
  hipLaunchKernelGGL(k_ba_index, dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, chunks, vsrc, vlen, vpre, blp);
  // tile sums before the page scan: the level path's dictionary pages take their byte totals
  // from them (PageWork::tile_bytes)
  if (ntl)
    hipLaunchKernelGGL(k_ba_tsum, dim3((ntl + TS_K - 1) / TS_K), dim3(WG), 0, s, pages, chunks, tile_page, tl, ntl, vsrc,
                       vlen, dsrc, dlen, tsum);
  hipLaunchKernelGGL(k_scan_bytes, dim3(1), dim3(WG), 0, s, pages, chunks, npages);
  if (ntl) {
    hipLaunchKernelGGL(k_ba_tscan, dim3(npages), dim3(WG), 0, s, pages, chunks, tsum);
    hipLaunchKernelGGL(k_ba_copy, dim3((ntl + BA_CK - 1) / BA_CK), dim3(WG), 0, s, blob, blob_len, pages, chunks,
                       tile_page, tl, ntl, vsrc, vlen,
                       dsrc, dlen, tsum);
    if (has_lvdict)
      hipLaunchKernelGGL(k_ba_copy_sd, dim3((ntl + BSD_K - 1) / BSD_K), dim3(WG), 0, s, blob, blob_len, pages, chunks,
                         tile_page, tl, ntl, vlen,
                         dsrc, dlen, tsum);
  }
  if (has_dba && ntl) {
    hipLaunchKernelGGL(k_dba_tiles, dim3(ntl), dim3(WG), 0, s, pages, chunks, tile_page, tl, vlen, vpre, tsum, dtile);
    hipLaunchKernelGGL(k_dba_pages, dim3(npages), dim3(WG), 0, s, pages, chunks, tsum, dtile);
    hipLaunchKernelGGL(k_dba_psv, dim3(ntl), dim3(WG), 0, s, pages, chunks, tile_page, tl, vlen, vpre, tsum, dtile,
                       vaux);
    hipLaunchKernelGGL(k_dba_copy, dim3(ntl), dim3(WG), 0, s, blob, pages, chunks, tile_page, tl, vsrc, vlen, vpre,
                       vaux);
  }
  return hipGetLastError();
}

}  // extern "C"

}  // namespace pqg
