// pcie_ubench.hip — host <-> device copy rates on this box (measurement tooling, not part of the
// decode library): hipMemcpyAsync H2D / D2H between pinned host memory and HBM, one at a time and
// both directions together (two streams), in 1 / 4 pieces on 1 / 4 streams, and a copy kernel that
// writes into / reads from pinned host memory directly (mapped), the alternative to the DMA engines.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <chrono>
#include <cstring>
#include <thread>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) k_copy(const v4u* __restrict__ src, v4u* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u;
  for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      printf("%s failed: %s\n", #x, hipGetErrorString(e));               \
      return 1;                                                          \
    }                                                                    \
  } while (0)

int main() {
  const size_t B = 512ull << 20;
  void *h_up, *h_dn, *d_a, *d_b;
  CK(hipHostMalloc(&h_up, B, hipHostMallocDefault));
  CK(hipHostMalloc(&h_dn, B, hipHostMallocDefault));
  CK(hipMalloc(&d_a, B));
  CK(hipMalloc(&d_b, B));
  memset(h_up, 1, B);
  memset(h_dn, 2, B);
  hipStream_t s[8];
  for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto gbps = [&](double bytes, std::chrono::steady_clock::time_point t0) {
    return bytes / std::chrono::duration<double>(now() - t0).count() / 1e9;
  };
  for (int rep = 0; rep < 2; ++rep) {
    // H2D alone, pieces over streams
    for (int pieces : {1, 4, 8}) {
      CK(hipDeviceSynchronize());
      auto t0 = now();
      for (int k = 0; k < pieces; ++k)
        CK(hipMemcpyAsync((char*)d_a + k * (B / pieces), (char*)h_up + k * (B / pieces), B / pieces,
                          hipMemcpyHostToDevice, s[k]));
      CK(hipDeviceSynchronize());
      printf("h2d_async pieces=%d GB/s %.1f\n", pieces, gbps(B, t0));
      t0 = now();
      for (int k = 0; k < pieces; ++k)
        CK(hipMemcpyAsync((char*)h_dn + k * (B / pieces), (char*)d_b + k * (B / pieces), B / pieces,
                          hipMemcpyDeviceToHost, s[k]));
      CK(hipDeviceSynchronize());
      printf("d2h_async pieces=%d GB/s %.1f\n", pieces, gbps(B, t0));
    }
    // both directions at once
    {
      CK(hipDeviceSynchronize());
      auto t0 = now();
      CK(hipMemcpyAsync(d_a, h_up, B, hipMemcpyHostToDevice, s[0]));
      CK(hipMemcpyAsync(h_dn, d_b, B, hipMemcpyDeviceToHost, s[1]));
      CK(hipDeviceSynchronize());
      printf("h2d+d2h_async GB/s %.1f (sum)\n", gbps(2.0 * B, t0));
    }
    // kernel over mapped pinned memory
    for (unsigned grid : {256u, 1024u, 4096u}) {
      void *dp_up, *dp_dn;
      CK(hipHostGetDevicePointer(&dp_up, h_up, 0));
      CK(hipHostGetDevicePointer(&dp_dn, h_dn, 0));
      CK(hipDeviceSynchronize());
      auto t0 = now();
      hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, s[0], (const v4u*)dp_up, (v4u*)d_a, B / 16);
      CK(hipDeviceSynchronize());
      printf("kernel_h2d grid=%u GB/s %.1f\n", grid, gbps(B, t0));
      t0 = now();
      hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, s[0], (const v4u*)d_b, (v4u*)dp_dn, B / 16);
      CK(hipDeviceSynchronize());
      printf("kernel_d2h grid=%u GB/s %.1f\n", grid, gbps(B, t0));
    }
    // host memcpy into pinned memory, 1 / 4 / 8 / 16 threads (the staging fill)
    std::vector<char> src(B, 3);
    for (int th : {1, 4, 8, 16}) {
      auto t0 = now();
      std::vector<std::thread> ts;
      for (int k = 0; k < th; ++k)
        ts.emplace_back([&, k] { memcpy((char*)h_up + k * (B / th), src.data() + k * (B / th), B / th); });
      for (auto& t : ts) t.join();
      printf("host_memcpy_to_pinned threads=%d GB/s %.1f\n", th, gbps(B, t0));
    }
    fflush(stdout);
  }
  return 0;
}
