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
  }
  return 0;
}
