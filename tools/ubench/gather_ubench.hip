// Random dictionary-gather ceiling on MI355X: 1e9 outputs of 8 bytes, indices from a hash,
// dictionary of D entries (L2/L1 resident). Prints GB/s of output written per variant.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

__device__ inline uint32_t hsh(uint32_t x) { x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x; }

__global__ void k_write(uint64_t* out, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n / 2; i += gridDim.x * 256ull)
    reinterpret_cast<uint4*>(out)[i] = make_uint4(i, 0, i, 1);
}
// thread-per-2-outputs, 16B stores, 8 groups of 2 per thread, gathers all first
template <int NG>
__global__ __launch_bounds__(256) void k_gather(const uint64_t* __restrict__ dict, uint32_t dmask, uint64_t* __restrict__ out, uint64_t n) {
  const uint64_t base = (uint64_t)blockIdx.x * 256 * 2 * NG;
  uint64_t x[NG][2];
#pragma unroll
  for (int s = 0; s < NG; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint64_t o = base + (uint64_t)s * 512 + threadIdx.x * 2 + j;
      x[s][j] = dict[hsh((uint32_t)o) & dmask];
    }
#pragma unroll
  for (int s = 0; s < NG; ++s) {
    uint64_t o = base + (uint64_t)s * 512 + threadIdx.x * 2;
    if (o < n) *reinterpret_cast<uint4*>(out + o) = make_uint4((uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32));
  }
}
// LDS-resident dictionary (first D entries, D <= 8192)
template <int NG>
__global__ __launch_bounds__(256) void k_gather_lds(const uint64_t* __restrict__ dict, uint32_t dmask, uint64_t* __restrict__ out, uint64_t n, int tiles_per_wg) {
  __shared__ uint64_t sd[8192];
  for (uint32_t i = threadIdx.x; i <= dmask; i += 256) sd[i] = dict[i];
  __syncthreads();
  for (int t = 0; t < tiles_per_wg; ++t) {
    const uint64_t base = ((uint64_t)blockIdx.x * tiles_per_wg + t) * 256 * 2 * NG;
    uint64_t x[NG][2];
#pragma unroll
    for (int s = 0; s < NG; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        uint64_t o = base + (uint64_t)s * 512 + threadIdx.x * 2 + j;
        x[s][j] = sd[hsh((uint32_t)o) & dmask];
      }
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      uint64_t o = base + (uint64_t)s * 512 + threadIdx.x * 2;
      if (o < n) *reinterpret_cast<uint4*>(out + o) = make_uint4((uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32));
    }
  }
}

// Partially LDS-resident dictionary: entries [0, S) in LDS (up to 19456 x 8 B = 152 KiB, one
// workgroup of NT threads per CU), the rest gathered from global memory (L2); persistent over
// tiles of NT * 2 * NG outputs.
template <int NG, int NT>
__global__ __launch_bounds__(NT) void k_gather_slab(const uint64_t* __restrict__ dict, uint32_t dmask, uint32_t S,
                                                    uint64_t* __restrict__ out, uint64_t n) {
  __shared__ uint64_t sd[19456];
  for (uint32_t i = threadIdx.x; i < S; i += NT) sd[i] = dict[i];
  __syncthreads();
  const uint64_t per = (uint64_t)NT * 2 * NG;
  for (uint64_t base = (uint64_t)blockIdx.x * per; base < n; base += (uint64_t)gridDim.x * per) {
    uint64_t x[NG][2];
#pragma unroll
    for (int s = 0; s < NG; ++s)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        uint64_t o = base + (uint64_t)s * NT * 2 + threadIdx.x * 2 + j;
        const uint32_t idx = hsh((uint32_t)o) & dmask;
        x[s][j] = idx < S ? sd[idx] : dict[idx];
      }
#pragma unroll
    for (int s = 0; s < NG; ++s) {
      uint64_t o = base + (uint64_t)s * NT * 2 + threadIdx.x * 2;
      if (o < n) *reinterpret_cast<uint4*>(out + o) = make_uint4((uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32));
    }
  }
}

// load flavours for the L2-served gather: 0 plain, 1 nontemporal, 2 agent-scope relaxed atomic (sc1)
template <int NG, int MODE>
__global__ __launch_bounds__(256) void k_gather_m(const uint64_t* __restrict__ dict, uint32_t dmask, uint64_t* __restrict__ out, uint64_t n) {
  const uint64_t base = (uint64_t)blockIdx.x * 256 * 2 * NG;
  uint64_t x[NG][2];
#pragma unroll
  for (int s = 0; s < NG; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint64_t o = base + (uint64_t)s * 512 + threadIdx.x * 2 + j;
      const uint64_t* p = dict + (hsh((uint32_t)o) & dmask);
      if (MODE == 0) x[s][j] = *p;
      else if (MODE == 1) x[s][j] = __builtin_nontemporal_load(p);
      else x[s][j] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
  for (int s = 0; s < NG; ++s) {
    uint64_t o = base + (uint64_t)s * 512 + threadIdx.x * 2;
    if (o < n) *reinterpret_cast<uint4*>(out + o) = make_uint4((uint32_t)x[s][0], (uint32_t)(x[s][0] >> 32), (uint32_t)x[s][1], (uint32_t)(x[s][1] >> 32));
  }
}
// 4-byte dictionary values (same index count, half the bytes)
template <int NG>
__global__ __launch_bounds__(256) void k_gather4(const uint32_t* __restrict__ dict, uint32_t dmask, uint32_t* __restrict__ out, uint64_t n) {
  const uint64_t base = (uint64_t)blockIdx.x * 256 * 4 * NG;
  uint32_t x[NG][4];
#pragma unroll
  for (int s = 0; s < NG; ++s)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint64_t o = base + (uint64_t)s * 1024 + threadIdx.x * 4 + j;
      x[s][j] = dict[hsh((uint32_t)o) & dmask];
    }
#pragma unroll
  for (int s = 0; s < NG; ++s) {
    uint64_t o = base + (uint64_t)s * 1024 + threadIdx.x * 4;
    if (o < n) *reinterpret_cast<uint4*>(out + o) = make_uint4(x[s][0], x[s][1], x[s][2], x[s][3]);
  }
}

int main() {
  const uint64_t n = 1000000000ull;
  uint64_t *out, *dict;
  hipMalloc(&out, n * 8 + 4096);
  hipMalloc(&dict, 65536 * 8 * 4);
  hipMemset(dict, 1, 65536 * 8 * 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](const char* name, auto fn) {
    fn(); hipDeviceSynchronize();
    hipEventRecord(a);
    for (int i = 0; i < 5; ++i) fn();
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
    printf("%-40s %8.3f ms  %7.0f GB/s out\n", name, ms, n * 8 / (ms * 1e-3) / 1e9);
  };
  run("write only 16B", [&] { k_write<<<8192, 256>>>(out, n); });
  const uint32_t tiles8 = (uint32_t)((n + 4095) / 4096);
  for (uint32_t D : {4096u, 16384u, 65536u, 262144u}) {
    char nm[64]; snprintf(nm, 64, "gather D=%u NG=8", D);
    run(nm, [&] { k_gather<8><<<tiles8, 256>>>(dict, D - 1, out, n); });
  }
  run("gather D=65536 NG=4", [&] { k_gather<4><<<tiles8 * 2, 256>>>(dict, 65535, out, n); });
  run("gather D=65536 NG=16", [&] { k_gather<16><<<tiles8 / 2 + 1, 256>>>(dict, 65535, out, n); });
  run("gather D=65536 nt", [&] { k_gather_m<8, 1><<<tiles8, 256>>>(dict, 65535, out, n); });
  int cus = 256;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (uint32_t S : {0u, 8192u, 16384u, 19456u}) {
    char nm[64];
    snprintf(nm, 64, "slab S=%u NT=1024 NG=4", S);
    run(nm, [&] { k_gather_slab<4, 1024><<<cus, 1024>>>(dict, 65535, S, out, n); });
    snprintf(nm, 64, "slab S=%u NT=512 NG=8", S);
    run(nm, [&] { k_gather_slab<8, 512><<<cus, 512>>>(dict, 65535, S, out, n); });
  }
  run("slab S=4096 D=4096 (all LDS)", [&] { k_gather_slab<4, 1024><<<cus, 1024>>>(dict, 4095, 4096, out, n); });
  run("gather D=65536 sc1", [&] { k_gather_m<8, 2><<<tiles8, 256>>>(dict, 65535, out, n); });
  run("gather4 D=65536 (1e9 x 4B)", [&] { k_gather4<4><<<tiles8, 256>>>((const uint32_t*)dict, 65535, (uint32_t*)out, n); });
  run("gather4 D=131072 (1e9 x 4B)", [&] { k_gather4<4><<<tiles8, 256>>>((const uint32_t*)dict, 131071, (uint32_t*)out, n); });
  for (uint32_t D : {4096u, 8192u}) {
    char nm[64]; snprintf(nm, 64, "lds gather D=%u NG=8 x16 tiles", D);
    run(nm, [&] { k_gather_lds<8><<<tiles8 / 16 + 1, 256>>>(dict, D - 1, out, n, 16); });
  }
  return 0;
}
