// Dictionary gather with the dictionary streamed through LDS in windows (MI355X): 1e9 outputs of
// 8 bytes from 1e9 16-bit indices read from HBM, dictionary of 65536 entries. Each workgroup takes
// a block of values (indices in registers), then for each window of the dictionary loads the
// window into LDS and gathers the indices that fall inside it; the block is stored at the end.
// Against the L2-served gather (one L2 request per index). Prints ms and GB/s of output.
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

__device__ inline uint32_t idx_of(const uint4& q, int j) {
  const uint32_t w = j < 2 ? q.x : j < 4 ? q.y : j < 6 ? q.z : q.w;
  return (j & 1) ? w >> 16 : w & 0xFFFFu;
}

// baseline: L2-served gather, 8 consecutive values per lane
template <int NS>
__global__ __launch_bounds__(256) void k_gather_idx(const uint64_t* __restrict__ dict, const uint16_t* __restrict__ idx,
                                                    uint64_t* __restrict__ out, uint64_t n) {
  const uint64_t base = (uint64_t)blockIdx.x * 256 * 8 * NS;
  uint4 ix[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const uint64_t o = base + ((uint64_t)s * 256 + threadIdx.x) * 8;
    ix[s] = o + 8 <= n ? *reinterpret_cast<const uint4*>(idx + o) : make_uint4(0, 0, 0, 0);
  }
  uint64_t x[NS][8];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) x[s][j] = dict[idx_of(ix[s], j)];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    const uint64_t o = base + ((uint64_t)s * 256 + threadIdx.x) * 8;
    if (o + 8 <= n)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<uint4*>(out + o + 2 * q) =
            make_uint4((uint32_t)x[s][2 * q], (uint32_t)(x[s][2 * q] >> 32), (uint32_t)x[s][2 * q + 1], (uint32_t)(x[s][2 * q + 1] >> 32));
  }
}

// windowed: NT threads, PT values per thread (8 per 16-byte index load), WIN dictionary entries
// per window
template <int NT, int PT, int WIN>
__global__ __launch_bounds__(NT) void k_gather_win(const uint64_t* __restrict__ dict, uint32_t D,
                                                   const uint16_t* __restrict__ idx, uint64_t* __restrict__ out,
                                                   uint64_t n) {
  __shared__ uint4 sd4[WIN / 2];
  const uint64_t* sd = reinterpret_cast<const uint64_t*>(sd4);
  const uint4* dict4 = reinterpret_cast<const uint4*>(dict);
  constexpr int NS = PT / 8;
  constexpr int F = WIN / 2 / NT;  // 16-byte window loads per thread
  const uint32_t tid = threadIdx.x;
  const uint64_t per = (uint64_t)NT * PT;
  for (uint64_t base = (uint64_t)blockIdx.x * per; base < n; base += (uint64_t)gridDim.x * per) {
    uint4 ix[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint64_t o = base + ((uint64_t)s * NT + tid) * 8;
      ix[s] = o + 8 <= n ? *reinterpret_cast<const uint4*>(idx + o) : make_uint4(0, 0, 0, 0);
    }
    uint64_t x[NS][8];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) x[s][j] = 0;
    for (uint32_t w0 = 0; w0 < D; w0 += WIN) {
      uint4 t[F];
#pragma unroll
      for (int f = 0; f < F; ++f) {
        const uint32_t i = f * NT + tid;
        t[f] = w0 + 2 * i < D ? dict4[w0 / 2 + i] : make_uint4(0, 0, 0, 0);
      }
      __syncthreads();  // (the previous window's gathers are done)
#pragma unroll
      for (int f = 0; f < F; ++f) sd4[f * NT + tid] = t[f];
      __syncthreads();
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t r = idx_of(ix[s], j) - w0;
          if (r < (uint32_t)WIN) x[s][j] = sd[r];
        }
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint64_t o = base + ((uint64_t)s * NT + tid) * 8;
      if (o + 8 <= n)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<uint4*>(out + o + 2 * q) = make_uint4((uint32_t)x[s][2 * q], (uint32_t)(x[s][2 * q] >> 32),
                                                                  (uint32_t)x[s][2 * q + 1], (uint32_t)(x[s][2 * q + 1] >> 32));
    }
  }
}

// layout B: value pairs lane-contiguous (each store instruction one contiguous KiB), indices as
// 32-bit pairs (NP pairs per thread)
template <int NP>
__global__ __launch_bounds__(256) void k_gather_idx2(const uint64_t* __restrict__ dict, const uint16_t* __restrict__ idx,
                                                     uint64_t* __restrict__ out, uint64_t n) {
  const uint64_t base = (uint64_t)blockIdx.x * 256 * 2 * NP;
  uint32_t ix[NP];
#pragma unroll
  for (int s = 0; s < NP; ++s) {
    const uint64_t o = base + ((uint64_t)s * 256 + threadIdx.x) * 2;
    ix[s] = o + 2 <= n ? *reinterpret_cast<const uint32_t*>(idx + o) : 0u;
  }
  uint64_t x[NP][2];
#pragma unroll
  for (int s = 0; s < NP; ++s) {
    x[s][0] = dict[ix[s] & 0xFFFFu];
    x[s][1] = dict[ix[s] >> 16];
  }
#pragma unroll
  for (int s = 0; s < NP; ++s) {
    const uint64_t o = base + ((uint64_t)s * 256 + threadIdx.x) * 2;
    if (o + 2 <= n)
      *reinterpret_cast<uint4*>(out + o) = make_uint4((uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32));
  }
}

template <int NT, int NP, int WIN>
__global__ __launch_bounds__(NT) void k_gather_win2(const uint64_t* __restrict__ dict, uint32_t D,
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
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(dict4 + w0 / 2 + i),
                                         (__attribute__((address_space(3))) void*)((__attribute__((address_space(3))) uint8_t*)sd4 + (f * NT + (tid & ~63u)) * 16), 16, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's fills landed, then the barrier
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

// partial LDS slab (first S entries) + L2 for the rest, indices read from HBM, layout B
template <int NT, int NP>
__global__ __launch_bounds__(NT) void k_gather_slab2(const uint64_t* __restrict__ dict, uint32_t S,
                                                     const uint16_t* __restrict__ idx, uint64_t* __restrict__ out,
                                                     uint64_t n) {
  __shared__ uint64_t sd[19456];
  for (uint32_t i = threadIdx.x; i < S; i += NT) sd[i] = dict[i];
  __syncthreads();
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
    for (int s = 0; s < NP; ++s) {
      const uint32_t a = ix[s] & 0xFFFFu, b = ix[s] >> 16;
      x[s][0] = a < S ? sd[a] : dict[a];
      x[s][1] = b < S ? sd[b] : dict[b];
    }
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      const uint64_t o = base + ((uint64_t)s * NT + tid) * 2;
      if (o + 2 <= n)
        *reinterpret_cast<uint4*>(out + o) = make_uint4((uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32));
    }
  }
}

// u16 index stream write + read alone (the two-kernel split's extra traffic)
__global__ void k_idx_copy(const uint16_t* __restrict__ a, uint16_t* __restrict__ b, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n / 8; i += gridDim.x * 256ull)
    reinterpret_cast<uint4*>(b)[i] = reinterpret_cast<const uint4*>(a)[i];
}

int main() {
  const uint64_t n = 1000000000ull;
  uint64_t *out, *dict;
  uint16_t* idx;
  hipMalloc(&out, n * 8 + 4096);
  hipMalloc(&idx, n * 2 + 4096);
  hipMalloc(&dict, 65536 * 8);
  hipMemset(dict, 1, 65536 * 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto run = [&](const char* name, auto fn) {
    fn();
    hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) fn();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    printf("%-44s %8.3f ms  %7.0f GB/s out  %7.0f GB/s in+out\n", name, ms, n * 8 / (ms * 1e-3) / 1e9,
           n * 10 / (ms * 1e-3) / 1e9);
  };
  for (uint32_t D : {65536u, 16384u}) {
    k_fill_idx<<<8192, 256>>>(idx, n, D - 1);
    hipDeviceSynchronize();
    char nm[80];
    auto g = [&](const char* s) { snprintf(nm, 80, "D=%u %s", D, s); return nm; };
    run(g("L2 gather NS=2"), [&] { k_gather_idx<2><<<(uint32_t)(n / 4096 + 1), 256>>>(dict, idx, out, n); });
    run(g("L2 gather NS=4"), [&] { k_gather_idx<4><<<(uint32_t)(n / 8192 + 1), 256>>>(dict, idx, out, n); });
    run(g("win NT=1024 PT=32 WIN=16384"), [&] {
      k_gather_win<1024, 32, 16384><<<(uint32_t)(n / 32768 + 1), 1024>>>(dict, D, idx, out, n);
    });
    run(g("win NT=1024 PT=16 WIN=16384"), [&] {
      k_gather_win<1024, 16, 16384><<<(uint32_t)(n / 16384 + 1), 1024>>>(dict, D, idx, out, n);
    });
    run(g("win NT=512 PT=32 WIN=8192"), [&] {
      k_gather_win<512, 32, 8192><<<(uint32_t)(n / 16384 + 1), 512>>>(dict, D, idx, out, n);
    });
    run(g("win NT=1024 PT=32 WIN=16384 persistent"), [&] {
      k_gather_win<1024, 32, 16384><<<256, 1024>>>(dict, D, idx, out, n);
    });
    run(g("win NT=512 PT=32 WIN=8192 persistent"), [&] {
      k_gather_win<512, 32, 8192><<<512, 512>>>(dict, D, idx, out, n);
    });
    run(g("B: L2 gather NP=8"), [&] { k_gather_idx2<8><<<(uint32_t)(n / 4096 + 1), 256>>>(dict, idx, out, n); });
    run(g("B: L2 gather NP=16"), [&] { k_gather_idx2<16><<<(uint32_t)(n / 8192 + 1), 256>>>(dict, idx, out, n); });
    run(g("B: win glds NT=1024 NP=16 WIN=16384 pers"), [&] {
      k_gather_win2<1024, 16, 16384><<<256, 1024>>>(dict, D, idx, out, n);
    });
    run(g("B: win glds NT=1024 NP=16 WIN=16384"), [&] {
      k_gather_win2<1024, 16, 16384><<<(uint32_t)(n / 32768 + 1), 1024>>>(dict, D, idx, out, n);
    });
    run(g("B: win glds NT=512 NP=16 WIN=8192 pers"), [&] {
      k_gather_win2<512, 16, 8192><<<512, 512>>>(dict, D, idx, out, n);
    });
    run(g("B: slab S=19456 NT=1024 NP=8 pers"), [&] {
      k_gather_slab2<1024, 8><<<256, 1024>>>(dict, 19456, idx, out, n);
    });
    run(g("B: slab S=19456 NT=1024 NP=16 pers"), [&] {
      k_gather_slab2<1024, 16><<<256, 1024>>>(dict, 19456, idx, out, n);
    });
  }
  run("u16 index copy (2 GB read + 2 GB write)", [&] { k_idx_copy<<<8192, 256>>>(idx, (uint16_t*)out, n); });
  return 0;
}
