// pqg_delta.hip — DELTA_BINARY_PACKED values (decoding.rs:392-619): one 256-thread workgroup
// per page running the stream decoder of pqg_delta.hpp over the page's value stream.
#include "pqg_delta.hpp"

namespace pqg {

template <int ES>  // 4 = INT32, 8 = INT64
__global__ void __launch_bounds__(WG) k_delta(const uint8_t* __restrict__ blob, uint64_t blob_len,
                                              PageWork* pages, uint8_t* __restrict__ out,
                                              ChunkResult* res) {
  __shared__ DeltaSmem sm;
  const int p = blockIdx.x;
  const PageWork pw = pages[p];
  if (pw.status != 0) return;
  if (pw.page_type != P_DATA && pw.page_type != P_DATA_V2) return;
  if (pw.encoding != E_DELTA_BINARY_PACKED) return;
  DeltaInfo info;
  // the decoder's set_data ignores num_values; read_batch asks for the non-null count
  int32_t st = delta_stream<ES>(sm, blob, blob_len, pw.base + pw.val_off, pw.val_bytes, pw.nonnull,
                                pw.nonnull, out + pw.value_out * ES, info);
  if (st && threadIdx.x == 0) report(pages, res, p, st);
}

extern "C" hipError_t pqg_launch_delta(const uint8_t* blob, uint64_t blob_len, PageWork* pages,
                                       int npages, int es, uint8_t* out, ChunkResult* res,
                                       hipStream_t s) {
  if (es == 4)
    hipLaunchKernelGGL(k_delta<4>, dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, out, res);
  else if (es == 8)
    hipLaunchKernelGGL(k_delta<8>, dim3(npages), dim3(WG), 0, s, blob, blob_len, pages, out, res);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

}  // namespace pqg
