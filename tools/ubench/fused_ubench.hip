// Dictionary gather (BASELINE config 3 shape: 1e9 16-bit indices, 65536 x 8-byte dictionary) with
// the work of a CU split between waves: FW filler waves move bytes into LDS by LDS-DMA (the batch's
// index stage, then the dictionary window by window) and never store; the gatherer waves take
// their indices from the stage, gather window by window and store, and never wait on memory (their
// stores drain while the next batch's fills and gathers run). Persistent: one 1024-thread
// workgroup per CU, batches of GW * 64 * 32 values. Against the round-4 windowed kernel (all
// waves fill, 128 KiB windows, stores serialized with the fills).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__device__ inline uint32_t hsh(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__global__ void k_fill_idx(uint16_t* idx, uint64_t n, uint32_t dmask) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) idx[i] = hsh((uint32_t)i) & dmask;
}
__global__ void k_fill_dict(uint64_t* d, uint32_t D) {
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < D; i += gridDim.x * 256) d[i] = ((uint64_t)hsh(i) << 32) | hsh(i + 77777u);
}
__global__ void k_check(const uint64_t* dict, const uint16_t* idx, const uint64_t* out, uint64_t n, unsigned long long* bad) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull)
    if (out[i] != dict[idx[i]]) atomicAdd(bad, 1ull);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define AS1 __attribute__((address_space(1)))
#define AS3 __attribute__((address_space(3)))

__device__ inline void dma16(const void* g, void* l) {
  __builtin_amdgcn_global_load_lds((const AS1 void*)g, (AS3 void*)l, 16, 0, 0);
}
// The same as inline asm: the compiler does not see an LDS write, so it adds no vmcnt wait before
// other waves' LDS reads (a wave with stores in flight would wait for them); the issuing wave waits
// for its own DMAs explicitly. M0 is saved and restored around the instruction.
__device__ inline void dma16a(const void* g, void* l) {
  const uint32_t lds = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uintptr_t)(AS3 void*)l);  // (wave-uniform)
  uint32_t sv;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\ts_nop 0\n\ts_mov_b32 m0, %0"
               : "=&s"(sv) : "s"(lds), "v"(g) : "memory");
}

// round-4 shape: all 16 waves fill 128 KiB windows, values in registers, stores at the end
template <int NT, int NP, int WIN>
__global__ __launch_bounds__(NT) void k_win_r4(const uint64_t* __restrict__ dict, uint32_t D,
                                               const uint16_t* __restrict__ idx, uint64_t* __restrict__ out,
                                               uint64_t n) {
  __shared__ uint4 sd4[WIN / 2];
  const uint64_t* sd = reinterpret_cast<const uint64_t*>(sd4);
  const uint4* dict4 = reinterpret_cast<const uint4*>(dict);
  constexpr int F = WIN / 2 / NT;
  const uint32_t tid = threadIdx.x;
  const uint64_t per = (uint64_t)NT * NP * 2;
  for (uint64_t base = (uint64_t)blockIdx.x * per; base < n; base += (uint64_t)gridDim.x * per) {
    uint32_t ix[NP];
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      const uint64_t o = base + ((uint64_t)s * NT + tid) * 2;
      ix[s] = o + 2 <= n ? *reinterpret_cast<const uint32_t*>(idx + o) : 0u;
    }
    uint64_t x[NP][2];
#pragma unroll
    for (int s = 0; s < NP; ++s) x[s][0] = x[s][1] = 0;
    for (uint32_t w0 = 0; w0 < D; w0 += WIN) {
      __syncthreads();
#pragma unroll
      for (int f = 0; f < F; ++f) {
        const uint32_t i = f * NT + tid;
        dma16(dict4 + w0 / 2 + i, (uint8_t*)sd4 + (f * NT + (tid & ~63u)) * 16);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __syncthreads();
#pragma unroll
      for (int s = 0; s < NP; ++s) {
        const uint32_t r0 = (ix[s] & 0xFFFFu) - w0, r1 = (ix[s] >> 16) - w0;
        if (r0 < (uint32_t)WIN) x[s][0] = sd[r0];
        if (r1 < (uint32_t)WIN) x[s][1] = sd[r1];
      }
    }
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      const uint64_t o = base + ((uint64_t)s * NT + tid) * 2;
      if (o + 2 <= n)
        *reinterpret_cast<uint4*>(out + o) = make_uint4((uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32));
    }
  }
}

// split roles. GW gatherer waves (32 values per lane as 16 pairs), FW filler waves; WIN window
// entries (8 bytes); ROT: each workgroup visits the windows in a rotated order.
template <int GW, int FW, int WIN, bool ROT>
__global__ __launch_bounds__(1024) void k_split(const uint64_t* __restrict__ dict, uint32_t D,
                                                const uint16_t* __restrict__ idx, uint64_t* __restrict__ out,
                                                uint64_t n) {
  static_assert(GW + FW == 16, "16 waves");
  constexpr uint32_t GT = GW * 64;            // gatherer threads
  constexpr uint32_t BV = GT * 32;            // values per batch
  constexpr uint32_t STB = BV * 2;            // stage bytes
  constexpr uint32_t WB = WIN * 8;            // window bytes
  __shared__ uint4 stage[STB / 16];
  __shared__ uint4 win[WB / 16];
  const uint32_t tid = threadIdx.x, wv = tid >> 6, lane = tid & 63u;
  const bool filler = wv >= GW;
  const uint32_t ft = tid - GT;  // filler thread
  const uint64_t nb = (n + BV - 1) / BV;
  const uint32_t nwin = (D + WIN - 1) / WIN;
  const uint64_t* sd = reinterpret_cast<const uint64_t*>(win);
  auto stage_dma = [&](uint64_t b) {  // fillers: the batch's indices into the stage
    const uint8_t* src = reinterpret_cast<const uint8_t*>(idx + b * BV);
    const uint64_t avail = (n - b * BV) * 2;
#pragma unroll 1
    for (uint32_t c = ft; c < STB / 16; c += FW * 64) {
      if ((uint64_t)c * 16 + 16 <= avail) dma16a(src + (uint64_t)c * 16, (uint8_t*)stage + (c & ~63u) * 16);
    }
  };
  auto win_dma = [&](uint32_t w) {
    const uint32_t e0 = w * WIN, ne = D - e0 < WIN ? D - e0 : WIN;
    const uint8_t* src = reinterpret_cast<const uint8_t*>(dict + e0);
#pragma unroll 1
    for (uint32_t c = ft; c < ne / 2; c += FW * 64) dma16a(src + (uint64_t)c * 16, (uint8_t*)win + (c & ~63u) * 16);
  };
  uint64_t b = blockIdx.x;
  if (filler && b < nb) {
    stage_dma(b);
    __builtin_amdgcn_s_waitcnt(0x0F70);
  }
  __syncthreads();
  for (; b < nb; b += gridDim.x) {
    uint32_t ix[16];
    if (!filler) {
#pragma unroll
      for (int s = 0; s < 16; ++s) ix[s] = reinterpret_cast<const uint32_t*>(stage)[s * GT + tid];
    }
    __syncthreads();  // stage free
    const uint64_t bn = b + gridDim.x;
    if (filler && bn < nb) stage_dma(bn);
    uint64_t x[16][2];
#pragma unroll
    for (int s = 0; s < 16; ++s) x[s][0] = x[s][1] = 0;
    for (uint32_t k = 0; k < nwin; ++k) {
      const uint32_t w = ROT ? (uint32_t)((k + blockIdx.x) % nwin) : k;
      if (filler) {
        win_dma(w);
        __builtin_amdgcn_s_waitcnt(0x0F70);
      }
      __syncthreads();
      if (!filler) {
        const uint32_t w0 = w * WIN;
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const uint32_t r0 = (ix[s] & 0xFFFFu) - w0, r1 = (ix[s] >> 16) - w0;
          if (r0 < (uint32_t)WIN) x[s][0] = sd[r0];
          if (r1 < (uint32_t)WIN) x[s][1] = sd[r1];
        }
      }
      __syncthreads();
    }
    if (!filler) {
      const uint64_t base = b * BV;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const uint64_t o = base + ((uint64_t)s * GT + tid) * 2;
        if (o + 2 <= n) {
          const u32x4 v = {(uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32)};
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + o));
        }
      }
    }
  }
}


// Job pipeline: the batch's dictionary windows, then the next batch's index stage, are "jobs",
// each a DMA of exactly NB bytes into buffer (job % 3) of three; the fillers keep two jobs in
// flight ahead of the gatherers (a fixed C instructions per filler lane per job, so a counted
// vmcnt(C) says the older job landed), one barrier per job. Gatherers: stage job -> store the
// finished batch, read the next batch's indices; window job -> gather.
template <int NT, int GW, int FW, int NP, int WENT>
__global__ __launch_bounds__(NT) void k_pipe(const uint64_t* __restrict__ dict, uint32_t D,
                                               const uint16_t* __restrict__ idx, uint64_t* __restrict__ out,
                                               uint64_t n) {
  static_assert((GW + FW) * 64 == NT, "waves");
  constexpr uint32_t GT = GW * 64;
  constexpr uint32_t BV = GT * NP * 2;      // values per batch
  constexpr uint32_t NB = WENT * 8;         // bytes per buffer / job
  static_assert(NB >= BV * 2, "the stage fits a buffer");
  static_assert(NB % (FW * 1024) == 0, "whole DMA rounds");
  constexpr uint32_t C = NB / (FW * 1024);  // DMA instructions per filler lane per job
  static_assert(2 * C <= 63, "two jobs in vmcnt");
  __shared__ uint4 buf[3][NB / 16];
  const uint32_t tid = threadIdx.x, wv = tid >> 6, lane = tid & 63u;
  const bool filler = wv >= GW;
  const uint32_t fw = wv - GW;  // filler wave
  const uint64_t nb = (n + BV - 1) / BV;
  const uint32_t K = (D + WENT - 1) / WENT;  // window jobs per batch
  const uint64_t my_nb = blockIdx.x < nb ? (nb - blockIdx.x + gridDim.x - 1) / gridDim.x : 0;
  // job j of this workgroup: j = 0 stage of batch 0; then per batch t: K windows, then the stage
  // of batch t + 1 (j = 1 + t * (K + 1) + k)
  const uint64_t njobs = my_nb ? 1 + my_nb * (K + 1) : 0;
  auto issue = [&](uint64_t j) {
    const uint8_t* src;
    uint64_t lim;  // source bytes available
    if (j == 0 || (j - 1) % (K + 1) == K) {  // stage of batch t
      const uint64_t t = j == 0 ? 0 : (j - 1) / (K + 1) + 1;
      const uint64_t b = blockIdx.x + t * gridDim.x;
      src = reinterpret_cast<const uint8_t*>(idx + (b < nb ? b : nb - 1) * BV);
      const uint64_t bb = b < nb ? b : nb - 1;
      lim = (n - bb * BV) * 2;
    } else {
      const uint32_t k = (uint32_t)((j - 1) % (K + 1));
      src = reinterpret_cast<const uint8_t*>(dict + (uint64_t)k * WENT);
      lim = (uint64_t)(D - k * WENT) * 8;
    }
    uint8_t* dst = reinterpret_cast<uint8_t*>(buf[j % 3]);
#pragma unroll 1
    for (uint32_t c = 0; c < C; ++c) {
      const uint32_t slot = (c * FW + fw) * 1024u;  // this wave's 1 KiB of the job
      const uint32_t off = slot + lane * 16u;
      const uint32_t so = off + 16 <= lim ? off : 0u;  // (past the source: any valid bytes)
      dma16a(src + so, dst + slot);
    }
  };
  if (filler) {
    if (njobs > 0) issue(0);
    if (njobs > 1) issue(1);
    __builtin_amdgcn_s_waitcnt(0x0F70 & ~0xF | (C & 0xF) | ((C >> 4) << 14));  // vmcnt(C): job 0 landed
  }
  __syncthreads();
  uint32_t ix[NP];
  uint64_t x[NP][2];
#pragma unroll
  for (int s = 0; s < NP; ++s) x[s][0] = x[s][1] = 0;
  for (uint64_t j = 0; j < njobs; ++j) {
    // consume job j (gatherers) while the fillers put job j + 2 in flight
    if (filler) {
      if (j + 2 < njobs) issue(j + 2);
    } else {
      const bool stage = j == 0 || (j - 1) % (K + 1) == K;
      if (stage) {
        if (j > 0) {  // the finished batch
          const uint64_t b = blockIdx.x + ((j - 1) / (K + 1)) * gridDim.x;
          const uint64_t base = b * BV;
#pragma unroll
          for (int s = 0; s < NP; ++s) {
            const uint64_t o = base + ((uint64_t)s * GT + tid) * 2;
            if (o + 2 <= n) {
              const u32x4 v = {(uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32)};
              __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + o));
            }
          }
        }
        const uint32_t* st = reinterpret_cast<const uint32_t*>(buf[j % 3]);
#pragma unroll
        for (int s = 0; s < NP; ++s) ix[s] = st[s * GT + tid];
      } else {
        const uint32_t w0 = (uint32_t)((j - 1) % (K + 1)) * WENT;
        const uint64_t* sd = reinterpret_cast<const uint64_t*>(buf[j % 3]);
#pragma unroll
        for (int s = 0; s < NP; ++s) {
          const uint32_t r0 = (ix[s] & 0xFFFFu) - w0, r1 = (ix[s] >> 16) - w0;
          if (r0 < (uint32_t)WENT) x[s][0] = sd[r0];
          if (r1 < (uint32_t)WENT) x[s][1] = sd[r1];
        }
      }
    }
    if (filler) {
      if (j + 2 < njobs) __builtin_amdgcn_s_waitcnt(0x0F70 & ~0xF | (C & 0xF) | ((C >> 4) << 14));  // job j + 1 landed
      else __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    __syncthreads();
  }
}

// The same job pipeline as nested loops (batch t, job q = 0 stage, 1..K windows), no 64-bit
// job arithmetic, the gather in the round-4 form.
template <int NT, int GW, int FW, int NP, int WENT, int MODE = 0, bool ROT = false>
__global__ __launch_bounds__(NT) void k_pipe2(const uint64_t* __restrict__ dict, uint32_t D,
                                              const uint16_t* __restrict__ idx, uint64_t* __restrict__ out,
                                              uint64_t n) {
  static_assert((GW + FW) * 64 == NT, "waves");
  constexpr uint32_t GT = GW * 64;
  constexpr uint32_t BV = GT * NP * 2;      // values per batch
  constexpr uint32_t NB = WENT * 8;         // bytes per buffer / job
  static_assert(NB >= BV * 2, "the stage fits a buffer");
  static_assert(NB % (FW * 1024) == 0, "whole DMA rounds");
  constexpr uint32_t C = NB / (FW * 1024);  // DMA instructions per filler lane per job
  static_assert(2 * C <= 63, "two jobs in vmcnt");
  __shared__ uint4 buf[3][NB / 16];
  const uint32_t tid = threadIdx.x, wv = tid >> 6, lane = tid & 63u;
  const bool filler = wv >= GW;
  const uint32_t fw = filler ? wv - GW : 0u;
  const uint32_t nb = (uint32_t)((n + BV - 1) / BV);
  const uint32_t K = (D + WENT - 1) / WENT;
  const uint32_t my_nb = blockIdx.x < nb ? (nb - blockIdx.x + gridDim.x - 1) / gridDim.x : 0u;
  // filler: job (t, q) into buffer slot
  auto issue = [&](uint32_t t, uint32_t q, uint32_t slot) {
    if (t >= my_nb) return;
    const uint8_t* src;
    uint32_t lim;
    if (q == 0) {
      const uint32_t b = blockIdx.x + t * gridDim.x;
      src = reinterpret_cast<const uint8_t*>(idx + (uint64_t)b * BV);
      const uint64_t av = (n - (uint64_t)b * BV) * 2;
      lim = av < NB ? (uint32_t)av : NB;
    } else {
      const uint32_t wq = ROT ? (q - 1 + blockIdx.x) % K : q - 1;  // (ROT: each workgroup's own window order)
      src = reinterpret_cast<const uint8_t*>(dict + (uint64_t)wq * WENT);
      lim = (D - wq * WENT) * 8;
    }
    uint8_t* dst = reinterpret_cast<uint8_t*>(buf[slot]);
#pragma unroll 1
    for (uint32_t c = 0; c < C; ++c) {
      const uint32_t sl = (c * FW + fw) * 1024u;
      const uint32_t off = sl + lane * 16u;
      dma16a(src + (off + 16 <= lim ? off : 0u), dst + sl);
    }
  };
  auto wait_c = [&]() { __builtin_amdgcn_s_waitcnt((0x0F70 & ~0xF) | (C & 0xF) | ((C >> 4) << 14)); };
  if (filler) {
    issue(0, 0, 0);
    if (K >= 1) issue(0, 1, 1);
    wait_c();
  }
  __syncthreads();
  uint32_t ix[NP];
  uint64_t x[NP][2];
#pragma unroll
  for (int s = 0; s < NP; ++s) {
    ix[s] = 0;
    x[s][0] = x[s][1] = 0;
  }
  uint32_t slot = 0;
  auto next_slot = [](uint32_t sl) { return sl == 2 ? 0u : sl + 1u; };
  auto prev_slot = [](uint32_t sl) { return sl == 0 ? 2u : sl - 1u; };
  auto ahead = [&](uint32_t t, uint32_t q) {  // fillers: job (t, q) + 2
    uint32_t t2 = t, q2 = q + 2;
    if (q2 > K) {
      q2 -= K + 1;
      ++t2;
    }
    if (MODE == 2 && q2 != 0) return;  // (MODE 2: only the stage jobs move bytes)
    issue(t2, q2, prev_slot(slot));
  };
  for (uint32_t t = 0; t < my_nb; ++t) {
    // job (t, 0): the batch's indices
    if (filler) {
      ahead(t, 0);
    } else {
      if (t > 0) {
        const uint64_t base = (uint64_t)(blockIdx.x + (t - 1) * gridDim.x) * BV;
        u32x4* p = reinterpret_cast<u32x4*>(out + base) + tid;
        const uint64_t lim = n - base;
#pragma unroll
        for (int s = 0; s < NP; ++s) {
          if (((uint64_t)s * GT + tid) * 2 + 2 <= lim) {
            const u32x4 v = {(uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32)};
            __builtin_nontemporal_store(v, p + s * GT);
          }
        }
      }
      const uint32_t* st = reinterpret_cast<const uint32_t*>(buf[slot]);
#pragma unroll
      for (int s = 0; s < NP; ++s) ix[s] = st[s * GT + tid];
    }
    if (filler) {
      if (MODE == 2) __builtin_amdgcn_s_waitcnt(0x0F70);
      else wait_c();
    }
    __syncthreads();
    slot = next_slot(slot);
    // jobs (t, 1..K): the windows
    for (uint32_t k = 0; k < K; ++k) {
      if (filler) {
        ahead(t, k + 1);
      } else if (MODE != 1) {
        const uint32_t w0 = (ROT ? (k + blockIdx.x) % K : k) * WENT;
        const uint64_t* sd = reinterpret_cast<const uint64_t*>(buf[slot]);
#pragma unroll
        for (int s = 0; s < NP; ++s) {
          const uint32_t r0 = (ix[s] & 0xFFFFu) - w0, r1 = (ix[s] >> 16) - w0;
          if (r0 < (uint32_t)WENT) x[s][0] = sd[r0];
          if (r1 < (uint32_t)WENT) x[s][1] = sd[r1];
        }
      }
      if (filler) {
        if (MODE == 2) __builtin_amdgcn_s_waitcnt(0x0F70);
        else wait_c();
      }
      __syncthreads();
      slot = next_slot(slot);
    }
  }
  if (!filler && my_nb) {
    const uint64_t base = (uint64_t)(blockIdx.x + (my_nb - 1) * gridDim.x) * BV;
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      const uint64_t o = base + ((uint64_t)s * GT + tid) * 2;
      if (o + 2 <= n) {
        const u32x4 v = {(uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32)};
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + o));
      }
    }
  }
}

// LDS-DMA fill rate alone: every workgroup streams the dictionary R times into a 128 KiB LDS
// ring, 1 KiB per wave-instruction, each wave keeping DEPTH instructions in flight; PERM: each
// workgroup walks the pieces in its own order.
template <int NW, int DEPTH, bool PERM>
__global__ __launch_bounds__(NW * 64) void k_dmabench(const uint64_t* __restrict__ dict, uint32_t D, uint32_t R,
                                                      uint64_t* __restrict__ sink) {
  __shared__ uint4 ring[128 * 64];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t np = D * 8 / 1024;  // pieces
  const uint8_t* src = reinterpret_cast<const uint8_t*>(dict);
  uint32_t k = 0;
  for (uint32_t r = 0; r < R; ++r) {
    for (uint32_t i = wv; i < np; i += NW) {
      const uint32_t pc = PERM ? (i + blockIdx.x * 37u) % np : i;
      dma16a(src + pc * 1024u + lane * 16u, reinterpret_cast<uint8_t*>(ring) + ((i & 127u) * 1024u));
      if (++k >= DEPTH) __builtin_amdgcn_s_waitcnt((0x0F70 & ~0xF) | ((DEPTH - 1) & 0xF) | (((DEPTH - 1) >> 4) << 14));
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
  if (threadIdx.x == 0) sink[blockIdx.x] = reinterpret_cast<const uint64_t*>(ring)[blockIdx.x & 1023];
}

int main() {
  const uint64_t n = 1000000000ull;
  uint64_t *out, *dict;
  uint16_t* idx;
  unsigned long long* bad;
  hipMalloc(&out, n * 8 + 4096);
  hipMalloc(&idx, n * 2 + 4096);
  hipMalloc(&dict, 65536 * 8);
  hipMalloc(&bad, 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const uint32_t D = 65536;
  k_fill_idx<<<8192, 256>>>(idx, n, D - 1);
  k_fill_dict<<<256, 256>>>(dict, D);
  hipDeviceSynchronize();
  auto run = [&](const char* name, auto fn) {
    hipMemset(out, 0, n * 8);
    fn();
    hipDeviceSynchronize();
    hipMemset(bad, 0, 8);
    k_check<<<8192, 256>>>(dict, idx, out, n, bad);
    unsigned long long nbad = 0;
    hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost);
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) fn();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    printf("%-44s %8.3f ms  %7.0f GB/s in+out  bad %llu\n", name, ms, n * 10 / (ms * 1e-3) / 1e9, nbad);
    fflush(stdout);
  };
  {
    uint64_t* sink;
    hipMalloc(&sink, 4096 * 8);
    auto dm = [&](const char* name, auto fn) {
      fn();
      hipDeviceSynchronize();
      hipEventRecord(a);
      fn();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      printf("%-44s %8.3f ms  %7.2f TB/s LDS-DMA fill (chip)\n", name, ms, 256.0 * 64 * 65536 * 8 / (ms * 1e-3) / 1e12);
      fflush(stdout);
    };
    dm("dma 4 waves depth 12", [&] { k_dmabench<4, 12, false><<<256, 256>>>(dict, D, 64, sink); });
    dm("dma 4 waves depth 24", [&] { k_dmabench<4, 24, false><<<256, 256>>>(dict, D, 64, sink); });
    dm("dma 4 waves depth 24 perm", [&] { k_dmabench<4, 24, true><<<256, 256>>>(dict, D, 64, sink); });
    dm("dma 8 waves depth 16 perm", [&] { k_dmabench<8, 16, true><<<256, 512>>>(dict, D, 64, sink); });
    dm("dma 16 waves depth 8 perm", [&] { k_dmabench<16, 8, true><<<256, 1024>>>(dict, D, 64, sink); });
    dm("dma 16 waves depth 16", [&] { k_dmabench<16, 16, false><<<256, 1024>>>(dict, D, 64, sink); });
    dm("dma 16 waves depth 4", [&] { k_dmabench<16, 4, false><<<256, 1024>>>(dict, D, 64, sink); });
    dm("dma 2 waves depth 32 perm", [&] { k_dmabench<2, 32, true><<<256, 128>>>(dict, D, 64, sink); });
  }
  run("r4: all waves fill, 128 KiB windows", [&] {
    k_win_r4<1024, 16, 16384><<<(uint32_t)(n / 32768 + 1), 1024>>>(dict, D, idx, out, n);
  });
  run("pipe2 1024: GW12 FW4 32/lane 3 x 48 KiB", [&] { k_pipe2<1024, 12, 4, 16, 6144><<<256, 1024>>>(dict, D, idx, out, n); });
  run("pipe2 1024 no gather (DMA pipeline alone)", [&] { k_pipe2<1024, 12, 4, 16, 6144, 1><<<256, 1024>>>(dict, D, idx, out, n); });
  run("pipe2 1024 no gather, ROT", [&] { k_pipe2<1024, 12, 4, 16, 6144, 1, true><<<256, 1024>>>(dict, D, idx, out, n); });
  run("pipe2 1024 ROT", [&] { k_pipe2<1024, 12, 4, 16, 6144, 0, true><<<256, 1024>>>(dict, D, idx, out, n); });
  run("pipe2 1024 no window DMA (gathers, stores)", [&] { k_pipe2<1024, 12, 4, 16, 6144, 2><<<256, 1024>>>(dict, D, idx, out, n); });
  run("split GW12 FW4 WIN 11264 (88 KiB) rot", [&] { k_split<12, 4, 11264, true><<<256, 1024>>>(dict, D, idx, out, n); });
  return 0;
}
