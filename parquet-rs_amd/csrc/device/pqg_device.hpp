// pqg_device.hpp — device helpers shared by the CDNA4 decode kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../pqg_internal.hpp"

// Global-memory pointers. Output buffers reached through ChunkWork (pointers loaded from memory,
// or held in a struct argument) are generic to the compiler, which then emits flat stores; a flat
// store counts in lgkmcnt as well as vmcnt, so every LDS wait after it waits for the store too.
// Store paths take their output as gptr<T> (gp() at the point the pointer is read).
#define PQG_AS1 __attribute__((address_space(1)))
template <class T>
using gptr = PQG_AS1 T*;
template <class T>
__device__ __forceinline__ gptr<T> gp(T* p) {
  return (gptr<T>)p;
}
// One 16-byte streaming store (never split by the compiler into element stores).
typedef uint32_t pqg_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void gst16(gptr<uint8_t> p, uint4 v) {
  const pqg_u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<gptr<pqg_u32x4>>(p));
}

namespace pqg {

constexpr int WG = 256;       // threads per workgroup (4 waves of 64)
constexpr int WAVE = 64;

// Record the first error of a page and of its chunk. Results must not depend on which
// workgroup reports first: the page status keeps the first code, the chunk keeps the
// lowest bad page index (chunk-relative).
__device__ inline void report(PageWork* pages, ChunkWork* chunks, int page, int32_t code) {
  // the code that sets the page's status is the one the chunk reports for it
  if (atomicCAS(&pages[page].status, 0, code) == 0) {
    ChunkWork& c = chunks[pages[page].chunk];
    atomicMin((unsigned long long*)&c.res.bad,
              ((unsigned long long)((uint32_t)page - c.first_page) << 32) | (uint32_t)code);
  }
}

// A dictionary-encoded page's per-value scratch (kept indices, byte-array index slots and entry
// sources) is written only when its chunk's dictionary page decoded. Every kernel that writes or
// reads such scratch takes a page through this one predicate (with the page's own status), so a
// consumer never reads scratch its producer skipped: the scratch is reused across decodes
// without clearing, and a slot left by an earlier decode may hold any value. The dictionary's
// status is final before any data page's kernel runs (k_prepare / k_ba_dict_prep come first).
__device__ inline bool dict_usable(const PageWork* pages, const ChunkWork& ck) {
  return ck.dict_page >= 0 && pages[ck.dict_page].status == 0;
}

// The column parameters of page pw's chunk.
__device__ inline const ColumnParams& pcp(const ChunkWork* chunks, const PageWork& pw) { return chunks[pw.chunk].cp; }

// One workgroup (WG threads): exclusive scan of per-page counts over pages [0, npages) in order,
// restarted at every chunk's first page. get(p) gives page p's count; put(p, excl, incl) receives
// its chunk-relative exclusive and inclusive prefix.
template <class Get, class Put>
__device__ inline void seg_scan_pages(const PageWork* pages, const ChunkWork* chunks, int npages, Get get, Put put) {
  __shared__ uint64_t sv[WG / 64];
  __shared__ uint32_t sf[WG / 64];
  __shared__ uint64_t carry_s;
  const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
  if (threadIdx.x == 0) carry_s = 0;
  __syncthreads();
  for (int base = 0; base < npages; base += WG) {
    const int p = base + (int)threadIdx.x;
    const bool in = p < npages;
    const uint64_t x = in ? get(p) : 0ull;
    uint32_t f = in && (uint32_t)p == chunks[pages[p].chunk].first_page ? 1u : 0u;
    uint64_t s = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {  // segmented inclusive scan: sums stop at a chunk start
      const uint64_t y = __shfl_up(s, d, 64);
      const uint32_t g = (uint32_t)__shfl_up((int)f, d, 64);
      if (lane >= (uint32_t)d) {
        if (!f) s += y;
        f |= g;
      }
    }
    if (lane == 63) {
      sv[wid] = s;
      sf[wid] = f;
    }
    __syncthreads();
    if (!f) {  // no chunk start between the block's first page and this one: add what came before
      uint64_t c = carry_s;
      for (uint32_t k = 0; k < wid; ++k) c = sf[k] ? sv[k] : c + sv[k];
      s += c;
    }
    if (in) put(p, s - x, s);
    __syncthreads();
    if (threadIdx.x == WG - 1) carry_s = s;
    __syncthreads();
  }
}

// Inclusive scan over the wave's 64 lanes (DPP row shifts and row broadcasts, no LDS).
__device__ inline uint32_t wave_scan_incl_u32(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// Little-endian byte load from global memory, guarded by the blob size.
__device__ inline uint32_t gbyte(const uint8_t* blob, uint64_t blob_len, uint64_t a) {
  return a < blob_len ? blob[a] : 0u;
}

// Guarded byte-wise tail of gload_u64 (only near the end of the blob). A compact loop, not
// a call: calls force scratch spills around every call site on AMDGPU.
__device__ inline uint64_t gload_u64_tail(const uint8_t* blob, uint64_t blob_len, uint64_t a) {
  uint64_t v = 0;
#pragma unroll 1
  for (int k = 0; k < 8; ++k) v |= (uint64_t)gbyte(blob, blob_len, a + k) << (8 * k);
  return v;
}

// 64-bit little-endian window starting at an arbitrary byte address, guarded.
__device__ inline uint64_t gload_u64(const uint8_t* blob, uint64_t blob_len, uint64_t a) {
  uint64_t al = a & ~3ull;
  if (al + 12 > blob_len) return gload_u64_tail(blob, blob_len, a);
  uint32_t sh = (uint32_t)(a - al) * 8u;
  const uint32_t* p = reinterpret_cast<const uint32_t*>(blob + al);
  uint32_t w0 = p[0], w1 = p[1], w2 = p[2];
  uint64_t lo = ((uint64_t)w1 << 32) | w0;
  if (sh == 0) return lo;
  return (lo >> sh) | ((uint64_t)w2 << (64 - sh));
}

// 16 guarded bytes (blob tail) for region staging.
__device__ inline uint4 gload_u128_tail(const uint8_t* blob, uint64_t blob_len, uint64_t a) {
  uint64_t lo = gload_u64_tail(blob, blob_len, a), hi = gload_u64_tail(blob, blob_len, a + 8);
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

// 64-bit little-endian window from an LDS byte image stored as 32-bit words.
__device__ inline uint64_t lload_u64(const uint32_t* words, uint32_t byte_idx) {
  uint32_t wi = byte_idx >> 2;
  uint32_t sh = (byte_idx & 3u) * 8u;
  uint64_t lo = ((uint64_t)words[wi + 1] << 32) | words[wi];
  if (sh == 0) return lo;
  return (lo >> sh) | ((uint64_t)words[wi + 2] << (64 - sh));
}

// 32-bit little-endian window from an LDS byte image (two dword reads + v_alignbyte).
__device__ inline uint32_t lload_u32(const uint32_t* words, uint32_t byte_idx) {
  const uint32_t wi = byte_idx >> 2;
  return __builtin_amdgcn_alignbyte(words[wi + 1], words[wi], byte_idx & 3u);
}

__device__ inline uint32_t lbyte(const uint32_t* words, uint32_t byte_idx) {
  return (words[byte_idx >> 2] >> ((byte_idx & 3u) * 8u)) & 0xFFu;
}

__device__ inline uint32_t lane_id() { return __lane_id(); }

__device__ inline int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ inline uint32_t readlane_u(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

// Block-wide sum of a 64-bit value (256 threads). Uses `scratch` (>= 4 u64) in LDS.
__device__ inline uint64_t block_sum_u64(uint64_t v, uint64_t* scratch) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) scratch[w] = v;
  __syncthreads();
  uint64_t t = 0;
  if (threadIdx.x == 0) t = scratch[0] + scratch[1] + scratch[2] + scratch[3];
  __syncthreads();
  return t;  // valid in thread 0
}

}  // namespace pqg
