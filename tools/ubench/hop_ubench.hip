// Micro-benchmark (diagnostic only): cycles per header hop for variants of the walker loop.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

// nxt[i] for 4096 positions in LDS, chain via readlane within 64-lane windows.
template <int V>
__global__ void hop(const uint32_t* nxt_g, int nsteps, unsigned long long* out, uint32_t* sink) {
  __shared__ uint32_t nx[4096 + 64];
  __shared__ uint32_t rec[4096];
  for (int i = threadIdx.x; i < 4096 + 64; i += blockDim.x) nx[i] = i < 4096 ? nxt_g[i] : 0xFFFF;
  __syncthreads();
  if (threadIdx.x >= 64) return;
  const uint32_t lane = threadIdx.x;
  uint32_t cur = 0, wbase = 0, vn = 0, cnt = 0, nrec = 0;
  bool have = false;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  uint32_t hops = 0;
  for (int s = 0; s < nsteps; ++s) {
    cur = 0; have = false;
    while (cur < 4000) {
      if (!have || cur - wbase >= 64u) {
        wbase = cur;
        have = true;
        vn = nx[wbase + lane];
      }
      uint32_t n = (uint32_t)__builtin_amdgcn_readlane((int)vn, (int)(cur - wbase));
      if (V >= 1) {
        if (lane == 0) rec[nrec & 4095] = cur;
        nrec++;
      }
      if (V >= 2) {
        cnt += n & 7;
        if (cnt > 1000000000u) break;
      }
      cur = n;
      hops++;
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[blockIdx.x * 2] = t1 - t0;
    out[blockIdx.x * 2 + 1] = hops;
    sink[blockIdx.x] = cnt + rec[nrec & 4095];
  }
}

int main() {
  std::vector<uint32_t> nxt(4096);
  for (int i = 0; i < 4096; ++i) nxt[i] = i + 1 + ((i * 2654435761u) >> 30);  // hops of 1..4
  uint32_t* d;
  unsigned long long* o;
  uint32_t* sink;
  hipMalloc(&d, 4096 * 4);
  hipMalloc(&o, 2 * 1024 * 8);
  hipMalloc(&sink, 1024 * 4);
  hipMemcpy(d, nxt.data(), 4096 * 4, hipMemcpyHostToDevice);
  for (int blocks : {1, 256, 1024}) {
    for (int v = 0; v < 3; ++v) {
      auto k = v == 0 ? hop<0> : v == 1 ? hop<1> : hop<2>;
      hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d, 20, o, sink);
      hipDeviceSynchronize();
      std::vector<unsigned long long> h(2 * blocks);
      hipMemcpy(h.data(), o, 2 * blocks * 8, hipMemcpyDeviceToHost);
      double cyc = 0, hops = 0;
      for (int b = 0; b < blocks; ++b) { cyc += h[2 * b]; hops += h[2 * b + 1]; }
      printf("blocks %4d variant %d: %.1f cycles/hop\n", blocks, v, cyc / hops);
    }
  }
  return 0;
}
