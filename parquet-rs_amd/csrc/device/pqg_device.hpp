// pqg_device.hpp — device helpers shared by the CDNA4 decode kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../pqg_internal.hpp"

namespace pqg {

constexpr int WG = 256;       // threads per workgroup (4 waves of 64)
constexpr int WAVE = 64;

// Record the first error of a page and of the chunk. Results must not depend on which
// workgroup reports first: the page status keeps the first code, the chunk keeps the
// lowest bad page index.
__device__ inline void report(PageWork* pages, ChunkResult* res, int page, int32_t code) {
  // the code that sets the page's status is the one the chunk reports for it
  if (atomicCAS(&pages[page].status, 0, code) == 0)
    atomicMin((unsigned long long*)&res->bad, ((unsigned long long)(uint32_t)page << 32) | (uint32_t)code);
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
