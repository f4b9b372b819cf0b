// copy_sweep.hip — which streaming access shapes reach the HBM ceiling on this MI355X (measurement
// tooling, not part of the decode library). Copies, read-only and write-only passes over 4 GiB
// buffers in several shapes: grid-stride vs. one contiguous span per workgroup, 16-byte lanes
// unrolled 4 / 8, plain vs. non-temporal loads and stores, grid sizes. Prints GB/s of bytes
// moved (read + written) per variant. The shapes that win are the ones the decode kernels'
// stores and the PLAIN copy should take.
#pragma clang diagnostic ignored "-Wunused-result"
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_stride(const v4u* __restrict__ src, v4u* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u * U;
  for (uint64_t i = (uint64_t)blockIdx.x * 256u * U + threadIdx.x; i < n16; i += stride) {
    v4u v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t j = i + (uint64_t)k * 256u;
      if (j < n16) v[k] = NTL ? __builtin_nontemporal_load(src + j) : src[j];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t j = i + (uint64_t)k * 256u;
      if (j < n16) {
        if (NTS) __builtin_nontemporal_store(v[k], dst + j);
        else dst[j] = v[k];
      }
    }
  }
}

// one contiguous span of `per` 16-byte chunks per workgroup
template <int U, bool NTL, bool NTS>
__global__ void __launch_bounds__(256) k_span(const v4u* __restrict__ src, v4u* __restrict__ dst, uint64_t n16,
                                              uint64_t per) {
  const uint64_t lo = (uint64_t)blockIdx.x * per, hi = lo + per < n16 ? lo + per : n16;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += 256u * U) {
    v4u v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t j = i + (uint64_t)k * 256u;
      if (j < hi) v[k] = NTL ? __builtin_nontemporal_load(src + j) : src[j];
    }
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t j = i + (uint64_t)k * 256u;
      if (j < hi) {
        if (NTS) __builtin_nontemporal_store(v[k], dst + j);
        else dst[j] = v[k];
      }
    }
  }
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) k_read(const v4u* __restrict__ src, uint64_t n16, v4u* sink) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u * U;
  v4u acc = {0, 0, 0, 0};
  for (uint64_t i = (uint64_t)blockIdx.x * 256u * U + threadIdx.x; i < n16; i += stride) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t j = i + (uint64_t)k * 256u;
      if (j < n16) acc ^= NT ? __builtin_nontemporal_load(src + j) : src[j];
    }
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[threadIdx.x] = acc;  // keeps the loads
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) k_write(v4u* __restrict__ dst, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256u * U;
  const v4u v = {threadIdx.x, blockIdx.x, 1u, 2u};
  for (uint64_t i = (uint64_t)blockIdx.x * 256u * U + threadIdx.x; i < n16; i += stride) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const uint64_t j = i + (uint64_t)k * 256u;
      if (j < n16) {
        if (NT) __builtin_nontemporal_store(v, dst + j);
        else dst[j] = v;
      }
    }
  }
}

static double timeit(void (*launch)(void*), void* arg, double bytes, int iters = 10) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  launch(arg);
  launch(arg);
  hipEventRecord(e0, 0);
  for (int i = 0; i < iters; ++i) launch(arg);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return bytes * iters / (ms * 1e-3) / 1e9;
}

struct Arg {
  v4u *a, *b;
  uint64_t n16;
  unsigned grid;
};

#define STRIDE(U, L, S)                                                                                  \
  [](void* p) {                                                                                          \
    Arg* x = (Arg*)p;                                                                                    \
    hipLaunchKernelGGL((k_stride<U, L, S>), dim3(x->grid), dim3(256), 0, 0, x->a, x->b, x->n16);         \
  }
#define SPAN(U, L, S)                                                                                    \
  [](void* p) {                                                                                          \
    Arg* x = (Arg*)p;                                                                                    \
    const uint64_t per = (x->n16 + x->grid - 1) / x->grid;                                               \
    hipLaunchKernelGGL((k_span<U, L, S>), dim3(x->grid), dim3(256), 0, 0, x->a, x->b, x->n16, per);      \
  }

int main() {
  const uint64_t bytes = 4ull << 30;
  Arg x{};
  x.n16 = bytes / 16;
  if (hipMalloc(&x.a, bytes) != hipSuccess || hipMalloc(&x.b, bytes) != hipSuccess) return 1;
  hipMemset(x.a, 1, bytes);
  hipMemset(x.b, 2, bytes);
  const unsigned grids[] = {1024, 4096, 16384, 65536};
  printf("variant grid GB/s\n");
  for (unsigned g : grids) {
    x.grid = g;
    printf("copy_stride_u4      %6u %8.1f\n", g, timeit(STRIDE(4, false, false), &x, 2.0 * bytes));
    printf("copy_stride_u4_nt   %6u %8.1f\n", g, timeit(STRIDE(4, true, true), &x, 2.0 * bytes));
    printf("copy_stride_u4_ntl  %6u %8.1f\n", g, timeit(STRIDE(4, true, false), &x, 2.0 * bytes));
    printf("copy_stride_u4_nts  %6u %8.1f\n", g, timeit(STRIDE(4, false, true), &x, 2.0 * bytes));
    printf("copy_stride_u8      %6u %8.1f\n", g, timeit(STRIDE(8, false, false), &x, 2.0 * bytes));
    printf("copy_stride_u8_nt   %6u %8.1f\n", g, timeit(STRIDE(8, true, true), &x, 2.0 * bytes));
    printf("copy_stride_u1      %6u %8.1f\n", g, timeit(STRIDE(1, false, false), &x, 2.0 * bytes));
    printf("copy_span_u4        %6u %8.1f\n", g, timeit(SPAN(4, false, false), &x, 2.0 * bytes));
    printf("copy_span_u4_nt     %6u %8.1f\n", g, timeit(SPAN(4, true, true), &x, 2.0 * bytes));
    printf("copy_span_u8_nt     %6u %8.1f\n", g, timeit(SPAN(8, true, true), &x, 2.0 * bytes));
    printf("read_u4             %6u %8.1f\n", g,
           timeit([](void* p) { Arg* y = (Arg*)p; hipLaunchKernelGGL((k_read<4, false>), dim3(y->grid), dim3(256), 0, 0, y->a, y->n16, y->b); }, &x, (double)bytes));
    printf("read_u8_nt          %6u %8.1f\n", g,
           timeit([](void* p) { Arg* y = (Arg*)p; hipLaunchKernelGGL((k_read<8, true>), dim3(y->grid), dim3(256), 0, 0, y->a, y->n16, y->b); }, &x, (double)bytes));
    printf("write_u4            %6u %8.1f\n", g,
           timeit([](void* p) { Arg* y = (Arg*)p; hipLaunchKernelGGL((k_write<4, false>), dim3(y->grid), dim3(256), 0, 0, y->b, y->n16); }, &x, (double)bytes));
    printf("write_u4_nt         %6u %8.1f\n", g,
           timeit([](void* p) { Arg* y = (Arg*)p; hipLaunchKernelGGL((k_write<4, true>), dim3(y->grid), dim3(256), 0, 0, y->b, y->n16); }, &x, (double)bytes));
    fflush(stdout);
  }
  hipFree(x.a);
  hipFree(x.b);
  return 0;
}
