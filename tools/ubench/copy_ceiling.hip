// copy_ceiling.hip — the achievable HBM copy rate on this device, for bench.py's roofline
// context (measurement tooling; not part of the decode library). A 16-byte-per-lane
// grid-stride copy (the MI355X_MICROARCH.md "float4 copy" shape), plain and non-temporal
// variants at three grid sizes, and a one-pass copy of 2 chunks per lane with one short
// workgroup per 8 KiB (k_plain_copy's shape: many short workgroups copied fastest there); the
// fastest is reported.
#pragma clang diagnostic ignored "-Wunused-result"
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ void __launch_bounds__(256) k_copy16(const v4u* __restrict__ src, v4u* __restrict__ dst,
                                                uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u * 4u;
  for (uint64_t i = (uint64_t)blockIdx.x * 1024u + threadIdx.x; i < n16; i += stride) {
    v4u v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t j = i + (uint64_t)k * 256u;
      if (j < n16) v[k] = NT ? __builtin_nontemporal_load(src + j) : src[j];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t j = i + (uint64_t)k * 256u;
      if (j < n16) {
        if (NT) __builtin_nontemporal_store(v[k], dst + j);
        else dst[j] = v[k];
      }
    }
  }
}

// one pass: workgroup b copies 16-byte chunks [b * 512, b * 512 + 512), two per lane
template <bool NT>
__global__ void __launch_bounds__(256) k_copy16_once(const v4u* __restrict__ src, v4u* __restrict__ dst,
                                                     uint64_t n16) {
  const uint64_t i = (uint64_t)blockIdx.x * 512u + threadIdx.x;
  v4u v[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint64_t j = i + (uint64_t)k * 256u;
    if (j < n16) v[k] = NT ? __builtin_nontemporal_load(src + j) : src[j];
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint64_t j = i + (uint64_t)k * 256u;
    if (j < n16) {
      if (NT) __builtin_nontemporal_store(v[k], dst + j);
      else dst[j] = v[k];
    }
  }
}

extern "C" {

// Best of the plain / non-temporal copy over `iters` launches of a `bytes`-byte buffer, as
// GB/s of bytes read + written. Returns < 0 on a HIP error.
double pqg_copy_ceiling_gbs(uint64_t bytes, int iters) {
  v4u *a = nullptr, *b = nullptr;
  const uint64_t n16 = bytes / 16;
  if (hipMalloc(&a, n16 * 16) != hipSuccess) return -1;
  if (hipMalloc(&b, n16 * 16) != hipSuccess) {
    hipFree(a);
    return -1;
  }
  hipMemset(a, 1, n16 * 16);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  double best = 0;
  // grids of 16, 64 and 256 workgroups per CU (tools/ubench/copy_sweep.hip: the largest grids
  // copy fastest on MI355X, 5.8-6.0 TB/s with non-temporal loads and stores)
  const unsigned grids[3] = {256 * 16, 256 * 64, 256 * 256};
  const unsigned once = (unsigned)((n16 + 511) / 512);
  auto launch = [&](int v) {
    const int nt = v & 1;
    if (v >= 6) {
      if (nt) hipLaunchKernelGGL(k_copy16_once<true>, dim3(once), dim3(256), 0, 0, a, b, n16);
      else hipLaunchKernelGGL(k_copy16_once<false>, dim3(once), dim3(256), 0, 0, a, b, n16);
      return;
    }
    const unsigned grid = grids[v >> 1];
    if (nt) hipLaunchKernelGGL(k_copy16<true>, dim3(grid), dim3(256), 0, 0, a, b, n16);
    else hipLaunchKernelGGL(k_copy16<false>, dim3(grid), dim3(256), 0, 0, a, b, n16);
  };
  for (int v = 0; v < 8 && best >= 0; ++v) {
    for (int w = 0; w < 2; ++w) launch(v);
    hipEventRecord(e0, 0);
    for (int i = 0; i < iters; ++i) launch(v);
    hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) {
      best = -1;
      break;
    }
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double gbs = 2.0 * (double)(n16 * 16) * iters / (ms * 1e-3) / 1e9;
    if (gbs > best) best = gbs;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(a);
  hipFree(b);
  return best;
}

}  // extern "C"
