// row_group.cpp — pqg_rg_*: the column chunks of one row group decoded concurrently.
//
// The reference reads a row group column by column, each column chunk through its own
// SerializedPageReader / ColumnReader (file/reader.rs:252-260, 306-330): the chunks share
// nothing. A single chunk of a wide row group (8M rows of a small-dictionary column: one data
// page) leaves most of the GPU idle while its level and index passes run, so the row group
// decoder forks the caller's stream onto `nstreams` HIP streams, gives every column chunk its
// own pqg_ctx (own staging and scratch, reused across row groups), places the chunks on the
// streams by estimated bytes (longest first onto the least-loaded stream) and joins the streams
// back into the caller's stream. Results per column are delivered by pqg_rg_sync.
//
// Enqueueing a chunk decode costs the host ~3 us per kernel launch (~30 launches): for 8M-row
// row groups that is as long as the GPU work itself, so every stream has a host worker thread
// that issues its columns' decodes; the streams' submissions then proceed in parallel.
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../../include/pqgpu.h"

extern "C" {
int pqg_sync_seq(pqg_ctx* ctx, int* first_bad_page, uint64_t* bad_seq);  // chunk_decoder.cpp
uint64_t pqg_decode_seq(pqg_ctx* ctx);
}

// One host thread per stream: runs the enqueue jobs handed to it, one batch per decode call.
struct RgWorker {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::function<void()>> jobs;
  bool busy = false, quit = false;
  int device = 0;

  void start(int dev) {
    device = dev;
    th = std::thread([this] {
      hipSetDevice(device);
      std::unique_lock<std::mutex> lk(mu);
      while (true) {
        cv.wait(lk, [this] { return quit || busy; });
        if (quit) return;
        std::vector<std::function<void()>> todo;
        todo.swap(jobs);
        lk.unlock();
        for (auto& f : todo) f();
        lk.lock();
        busy = false;
        cv.notify_all();
      }
    });
  }
  void run(std::vector<std::function<void()>>&& j) {
    std::lock_guard<std::mutex> lk(mu);
    jobs = std::move(j);
    busy = true;
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [this] { return !busy; });
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(mu);
      quit = true;
      cv.notify_all();
    }
    if (th.joinable()) th.join();
  }
};

struct pqg_rg_ctx {
  int device = 0;
  std::vector<hipStream_t> streams;
  std::vector<hipEvent_t> join;
  hipEvent_t fork = nullptr;
  std::vector<pqg_ctx*> cols;   // one decode context per column index
  std::vector<int> issued;      // decodes pending per column
  // per column, the decodes pending: (the column ctx's issue number, this decoder's call index
  // since the last sync), so that a failure is reported at its (call, column)
  std::vector<std::vector<std::pair<uint64_t, int>>> pend;
  int calls_since_sync = 0;
  std::vector<RgWorker*> workers;
  uint64_t calls = 0;           // decode calls: rotates the stream assignment
  std::string msg;
};

static int rg_fail(pqg_rg_ctx* g, int st, const char* what) {
  g->msg = what;
  return st;
}

extern "C" {

int pqg_rg_ctx_create(int device, int nstreams, pqg_rg_ctx** out) {
  if (!out || nstreams < 1 || nstreams > 16) return PQG_ERR_INVALID;
  *out = nullptr;
  if (hipSetDevice(device) != hipSuccess) return PQG_ERR_HIP;
  pqg_rg_ctx* g = new pqg_rg_ctx();
  g->device = device;
  bool ok = hipEventCreateWithFlags(&g->fork, hipEventDisableTiming) == hipSuccess;
  for (int k = 0; ok && k < nstreams; ++k) {
    hipStream_t s;
    hipEvent_t e;
    ok = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
    if (!ok) break;
    g->streams.push_back(s);
    ok = hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    if (ok) g->join.push_back(e);
  }
  if (!ok) {
    pqg_rg_ctx_destroy(g);
    return PQG_ERR_HIP;
  }
  for (int k = 0; k < nstreams; ++k) {
    g->workers.push_back(new RgWorker());
    g->workers.back()->start(device);
  }
  *out = g;
  return PQG_OK;
}

int pqg_rg_ctx_destroy(pqg_rg_ctx* g) {
  if (!g) return PQG_OK;
  hipSetDevice(g->device);
  for (RgWorker* w : g->workers) {
    w->stop();
    delete w;
  }
  for (pqg_ctx* c : g->cols) pqg_ctx_destroy(c);  // waits for its decodes
  for (hipStream_t s : g->streams) hipStreamDestroy(s);
  for (hipEvent_t e : g->join) hipEventDestroy(e);
  if (g->fork) hipEventDestroy(g->fork);
  delete g;
  return PQG_OK;
}

const char* pqg_rg_error_message(pqg_rg_ctx* g) { return g ? g->msg.c_str() : "null ctx"; }

int pqg_rg_decode(pqg_rg_ctx* g, uint32_t ncols, const pqg_column* cols, const uint8_t* blob, uint64_t blob_len,
                  const pqg_page* const* pages, const uint32_t* npages, pqg_output* outs, void* stream_v) {
  if (!g || (ncols && (!cols || !pages || !npages || !outs))) return PQG_ERR_INVALID;
  for (uint32_t j = 0; j < ncols; ++j)
    if (npages[j] && !pages[j]) return rg_fail(g, PQG_ERR_INVALID, "column without its page array");
  if (hipSetDevice(g->device) != hipSuccess) return rg_fail(g, PQG_ERR_HIP, "hipSetDevice");
  g->msg.clear();
  while (g->cols.size() < ncols) {
    pqg_ctx* c = nullptr;
    const int st = pqg_ctx_create(g->device, &c);
    if (st) return rg_fail(g, st, "pqg_ctx_create");
    g->cols.push_back(c);
    g->issued.push_back(0);
    g->pend.emplace_back();
  }
  const int call = g->calls_since_sync++;
  hipStream_t caller = (hipStream_t)stream_v;
  if (hipEventRecord(g->fork, caller) != hipSuccess) return rg_fail(g, PQG_ERR_HIP, "fork event");
  const size_t K = g->streams.size();
  for (hipStream_t s : g->streams)
    if (hipStreamWaitEvent(s, g->fork, 0) != hipSuccess) return rg_fail(g, PQG_ERR_HIP, "fork wait");
  // bytes each chunk moves (payload in; levels + values out, estimated from the page counts)
  std::vector<std::pair<double, uint32_t>> work(ncols);
  for (uint32_t j = 0; j < ncols; ++j) {
    double b = 0;
    for (uint32_t i = 0; i < npages[j]; ++i) b += pages[j][i].nbytes + 2.0 * pages[j][i].num_values;
    work[j] = {b + (double)outs[j].values_capacity, j};
  }
  std::sort(work.begin(), work.end(), [](const auto& a, const auto& b) { return a.first > b.first; });
  // least-loaded stream first; the streams are rotated per call so that the same column of
  // consecutive row groups lands on different streams (its decodes can then overlap)
  std::vector<double> load(K, 0.0);
  std::vector<std::vector<uint32_t>> per(K);
  const size_t rot = (size_t)((g->calls++ * ncols) % K);
  for (const auto& wj : work) {
    size_t best = 0;
    for (size_t i = 1; i < K; ++i)
      if (load[(rot + i) % K] < load[(rot + best) % K]) best = i;
    const size_t k = (rot + best) % K;
    load[k] += wj.first;
    per[k].push_back(wj.second);
  }
  // every stream's decodes enqueued by its own host thread
  std::vector<int> st(ncols, PQG_OK);
  for (size_t k = 0; k < K; ++k) {
    if (per[k].empty()) continue;
    std::vector<std::function<void()>> jobs;
    for (uint32_t j : per[k])
      jobs.push_back([=, &st] {
        st[j] = pqg_decode_chunk(g->cols[j], &cols[j], blob, blob_len, pages[j], npages[j], &outs[j], g->streams[k]);
      });
    g->workers[k]->run(std::move(jobs));
  }
  for (size_t k = 0; k < K; ++k)
    if (!per[k].empty()) g->workers[k]->wait();
  int first_err = PQG_OK;
  for (uint32_t j = 0; j < ncols; ++j) {
    if (st[j]) {
      if (!first_err) {
        first_err = st[j];
        char buf[320];
        snprintf(buf, sizeof(buf), "column %u: %s", j, pqg_error_message(g->cols[j]));
        g->msg = buf;
      }
      continue;
    }
    g->issued[j]++;
    g->pend[j].emplace_back(pqg_decode_seq(g->cols[j]), call);
  }
  for (size_t k = 0; k < K; ++k) {
    if (hipEventRecord(g->join[k], g->streams[k]) != hipSuccess ||
        hipStreamWaitEvent(caller, g->join[k], 0) != hipSuccess)
      return rg_fail(g, PQG_ERR_HIP, "join");
  }
  return first_err;
}

// The failure reported is the one the reference meets first: the earliest row group (decode
// call) with a failing column, and in it the lowest failing column index.
int pqg_rg_sync_call(pqg_rg_ctx* g, int* bad_call, int* bad_column, int* bad_page) {
  if (!g) return PQG_ERR_INVALID;
  if (bad_call) *bad_call = -1;
  if (bad_column) *bad_column = -1;
  if (bad_page) *bad_page = -1;
  int first = PQG_OK, fcall = 0x7FFFFFFF, fcol = -1;
  for (size_t j = 0; j < g->cols.size(); ++j) {
    if (!g->issued[j]) continue;
    g->issued[j] = 0;
    int page = -1;
    uint64_t seq = 0;
    const int st = pqg_sync_seq(g->cols[j], &page, &seq);
    int call = g->pend[j].empty() ? 0 : g->pend[j].back().second;
    for (const auto& pc : g->pend[j])
      if (pc.first == seq) call = pc.second;
    g->pend[j].clear();
    if (st && (call < fcall || (call == fcall && (int)j < fcol))) {
      first = st;
      fcall = call;
      fcol = (int)j;
      if (bad_page) *bad_page = page;
      char buf[320];
      snprintf(buf, sizeof(buf), "row group call %d, column %zu: %s", call, j, pqg_error_message(g->cols[j]));
      g->msg = buf;
    }
  }
  g->calls_since_sync = 0;
  if (first) {
    if (bad_call) *bad_call = fcall;
    if (bad_column) *bad_column = fcol;
  }
  return first;
}

int pqg_rg_sync(pqg_rg_ctx* g, int* bad_column, int* bad_page) {
  return pqg_rg_sync_call(g, nullptr, bad_column, bad_page);
}

}  // extern "C"
