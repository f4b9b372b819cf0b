// row_group.cpp — pqg_rg_*: the column chunks of one row group decoded together.
//
// The reference reads a row group column by column, each column chunk through its own
// SerializedPageReader / ColumnReader (file/reader.rs:252-260, 306-330): the chunks share
// nothing. The row-group decoder hands all of them to one batched decode (pqg_decode_chunks): one
// page table for the row group, every kernel launched once for its 11 (or n) chunks on the
// caller's stream, so that a row group costs the launches of one chunk and its chunks' pages fill
// the GPU together. Results per column are delivered by pqg_rg_sync / pqg_rg_sync_call.
#include <hip/hip_runtime.h>

#include <stdio.h>

#include <string>

#include "../../../include/pqgpu.h"

struct pqg_rg_ctx {
  int device = 0;
  pqg_ctx* ctx = nullptr;  // the batched decodes (two in flight: its staging slots)
  std::string msg;
};

extern "C" {

// nstreams is reserved (pqgpu.h): validated, then unused -- the batched decode runs on the caller's stream.
int pqg_rg_ctx_create(int device, int nstreams, pqg_rg_ctx** out) {
  if (!out || nstreams < 1 || nstreams > 16) return PQG_ERR_INVALID;
  *out = nullptr;
  pqg_rg_ctx* g = new pqg_rg_ctx();
  g->device = device;
  const int st = pqg_ctx_create(device, &g->ctx);
  if (st) {
    delete g;
    return st;
  }
  *out = g;
  return PQG_OK;
}

int pqg_rg_ctx_destroy(pqg_rg_ctx* g) {
  if (!g) return PQG_OK;
  pqg_ctx_destroy(g->ctx);  // waits for its decodes
  delete g;
  return PQG_OK;
}

const char* pqg_rg_error_message(pqg_rg_ctx* g) { return g ? g->msg.c_str() : "null ctx"; }

int pqg_rg_decode(pqg_rg_ctx* g, uint32_t ncols, const pqg_column* cols, const uint8_t* blob, uint64_t blob_len,
                  const pqg_page* const* pages, const uint32_t* npages, pqg_output* outs, void* stream) {
  if (!g || (ncols && (!cols || !pages || !npages || !outs))) return PQG_ERR_INVALID;
  for (uint32_t j = 0; j < ncols; ++j)
    if (npages[j] && !pages[j]) {
      g->msg = "column without its page array";
      return PQG_ERR_INVALID;
    }
  g->msg.clear();
  const int st = pqg_decode_chunks(g->ctx, ncols, cols, blob, blob_len, pages, npages, outs, stream);
  if (st) g->msg = pqg_error_message(g->ctx);
  return st;
}

// The failure reported is the one the reference meets first: the earliest row group (decode
// call) with a failing column, and in it the lowest failing column index.
int pqg_rg_sync_call(pqg_rg_ctx* g, int* bad_call, int* bad_column, int* bad_page) {
  if (!g) return PQG_ERR_INVALID;
  int call = -1, col = -1, page = -1;
  const int st = pqg_sync_detail(g->ctx, &call, &col, &page);
  if (bad_call) *bad_call = st ? call : -1;
  if (bad_column) *bad_column = st ? col : -1;
  if (bad_page) *bad_page = st ? page : -1;
  if (st) {
    char buf[400];
    snprintf(buf, sizeof(buf), "row group call %d, column %d: %s", call, col, pqg_error_message(g->ctx));
    g->msg = buf;
  }
  return st;
}

int pqg_rg_sync(pqg_rg_ctx* g, int* bad_column, int* bad_page) {
  return pqg_rg_sync_call(g, nullptr, bad_column, bad_page);
}

}  // extern "C"
