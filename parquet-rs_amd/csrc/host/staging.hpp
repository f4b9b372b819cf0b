// staging.hpp — buffers of the host readers that only grow: device memory (hipMalloc) or pinned
// host memory (hipHostMalloc), kept across chunks / row groups so steady-state reads allocate nothing.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace pqg {

struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  bool host = false;  // pinned host memory
  hipError_t need(size_t n) {
    if (n <= cap) return hipSuccess;
    release();
    const size_t c = n + n / 8 + 256;
    hipError_t e = host ? hipHostMalloc(&p, c, hipHostMallocDefault) : hipMalloc(&p, c);
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    cap = c;
    return hipSuccess;
  }
  void release() {
    if (p) (void)(host ? hipHostFree(p) : hipFree(p));
    p = nullptr;
    cap = 0;
  }
};

}  // namespace pqg
