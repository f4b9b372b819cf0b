// rg_reader.cpp — pqg_rgr_*: row groups from a file to device (and host) memory, pipelined.
//
// The reference reads a column chunk page by page: SerializedPageReader::get_next_page parses a
// page header, reads the payload and decompresses it (file/reader.rs:420-522), and the column
// reader decodes it (column/reader.rs:269-488); row groups are reached through
// SerializedFileReader::get_row_group / get_column_page_reader (file/reader.rs:252-260, 306-330).
// Here a whole row group moves as one unit:
//   host    page headers of every column parsed (plan_chunk_pages), then the payloads copied or
//           decompressed (SNAPPY, GZIP) by a pool of host threads, page by page, straight into
//           pinned staging laid out as the decode's blob;
//   H2D     one async copy of the blob on a copy stream;
//   decode  one batched decode of all the row group's column chunks (pqg_decode_chunks) on the
//           decode stream, after the copy's event;
//   D2H     (PQG_RGR_HOST_OUTPUT) the levels and fixed-width values into pinned host buffers on a
//           second copy stream as soon as the decode ends; byte-array bytes, whose size the
//           decode reports, when the row group is waited for.
// Two row groups may be in flight, so the host work and H2D of row group g + 1 overlap the decode
// of g. Staging, device blobs and outputs belong to three rotating slots and are reused (grown
// only) across row groups; a waited row group's results stay valid until the next wait.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "file_reader.hpp"
#include "staging.hpp"

using namespace pqg;

namespace {

// Host threads that fill a row group's staging: run(n, fn) calls fn(0..n-1) over the workers and
// the calling thread, and returns when all are done.
class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n - 1; ++i) th_.emplace_back([this] { worker(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (std::thread& t : th_) t.join();
  }
  void run(size_t n, const std::function<void(size_t)>& fn) {
    {
      std::lock_guard<std::mutex> lk(m_);
      fn_ = &fn;
      n_ = n;
      next_ = 0;
      active_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [this] { return active_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      const size_t i = next_.fetch_add(1);
      if (i >= n_) break;
      (*fn_)(i);
    }
  }
  void worker() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      work();
      std::lock_guard<std::mutex> lk(m_);
      if (--active_ == 0) done_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t n_ = 0;
  std::atomic<size_t> next_{0};
  int active_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

int value_size(int t, int tl) {
  switch (t) {
    case PQG_BOOLEAN: return 1;
    case PQG_INT32: case PQG_FLOAT: return 4;
    case PQG_INT64: case PQG_DOUBLE: return 8;
    case PQG_INT96: return 12;
    case PQG_FIXED_LEN_BYTE_ARRAY: return tl;
    default: return 0;
  }
}

enum { O_DEF, O_REP, O_VAL, O_OFF, O_N };

struct Col {
  std::vector<PagePlan> plan;
  uint64_t base = 0;      // chunk blob offset in the row group's blob
  uint64_t len = 0;
  uint64_t levels = 0;    // sum of data-page num_values
  uint64_t vcap = 0;      // values capacity (bytes)
  int host_st = 0;        // a header / decompression failure, and the page it is on
  int host_page = -1;
  std::string host_err;
  std::vector<pqg_page> pages;  // offsets into the row group's blob
  Buf dev[O_N];
  Buf hst[O_N];
};

struct Slot {
  int rg = -1;
  pqg_ctx* ctx = nullptr;  // one decode in flight per slot, so each is synced on its own
  hipStream_t s_d2h = nullptr;  // the slot's own D2H copies: waiting for them never waits for the
                                // next row group's decode (its copies are on another slot's stream)
  hipEvent_t ev_h2d = nullptr, ev_dec = nullptr;
  Buf h_blob, d_blob;
  uint64_t blob_len = 0;
  std::vector<Col> cols;
  std::vector<pqg_column> desc;
  std::vector<pqg_output> outs;
  std::vector<const pqg_page*> pp;
  std::vector<uint32_t> np;
  uint32_t ndec = 0;       // columns handed to the decode (those before a host failure)
  int host_col = -1;       // lowest column with a host-side failure
  int status = 0, bad_col = -1, bad_page = -1;
  std::string err;
};

}  // namespace

struct pqg_rgr {
  pqg_file_reader* r = nullptr;
  int device = 0;
  int flags = 0;
  Pool* pool = nullptr;
  hipStream_t s_h2d = nullptr, s_dec = nullptr;
  Slot slot[3];
  int head = 0, count = 0, cur = -1;
  pqg_rgr_stats st{};
  std::string err;
};

static int rgr_fail(pqg_rgr* g, int st, const std::string& m) {
  g->err = m;
  return st;
}

#define RCHK(x, what)                                                                               \
  do {                                                                                              \
    hipError_t e_ = (x);                                                                            \
    if (e_ != hipSuccess) return rgr_fail(g, PQG_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e_)); \
  } while (0)

// Byte-array value bytes a chunk can decode to, from its pages: PLAIN / DELTA_LENGTH_BYTE_ARRAY
// payloads bound their bytes; a dictionary page bounds each index by its longest entry; a
// DELTA_BYTE_ARRAY page's prefixes can grow it (the decode reports the size: wait() retries).
static uint64_t ba_capacity(const Col& c, const uint8_t* blob, int ptype, int tl) {
  if (ptype == PQG_FIXED_LEN_BYTE_ARRAY) return c.levels * (uint64_t)(tl > 0 ? tl : 0) + 64;
  uint64_t maxlen = 0, cap = 64;
  for (const PagePlan& pp : c.plan)
    if (pp.page.page_type == PQG_PAGE_DICTIONARY) {
      const uint8_t* d = blob + c.base + pp.page.offset;
      uint64_t o = 0;
      for (uint32_t i = 0; i < pp.page.num_values && o + 4 <= pp.page.nbytes; ++i) {
        uint32_t l;
        memcpy(&l, d + o, 4);
        if (l > maxlen) maxlen = l;
        o += 4ull + l;
      }
    }
  for (const PagePlan& pp : c.plan) {
    const pqg_page& p = pp.page;
    if (p.page_type == PQG_PAGE_DICTIONARY) continue;
    if (p.encoding == PQG_PLAIN_DICTIONARY || p.encoding == PQG_RLE_DICTIONARY) cap += (uint64_t)p.num_values * maxlen;
    else if (p.encoding == PQG_DELTA_BYTE_ARRAY) cap += 4ull * p.nbytes;
    else cap += p.nbytes;
  }
  return cap;
}

extern "C" {

int pqg_rgr_open(pqg_file_reader* r, int device, int host_threads, int flags, pqg_rgr** out) {
  if (!r || !out || host_threads < 1 || host_threads > 256) return PQG_ERR_INVALID;
  *out = nullptr;
  pqg_rgr* g = new pqg_rgr();
  g->r = r;
  g->device = device;
  g->flags = flags;
  auto bail = [&](int st) {
    pqg_rgr_close(g);
    return st;
  };
  if (hipSetDevice(device) != hipSuccess) return bail(PQG_ERR_HIP);
  if (hipStreamCreateWithFlags(&g->s_h2d, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&g->s_dec, hipStreamNonBlocking) != hipSuccess)
    return bail(PQG_ERR_HIP);
  for (Slot& s : g->slot) {
    if (pqg_ctx_create(device, &s.ctx) != PQG_OK) return bail(PQG_ERR_HIP);
    if (hipStreamCreateWithFlags(&s.s_d2h, hipStreamNonBlocking) != hipSuccess) return bail(PQG_ERR_HIP);
    if (hipEventCreateWithFlags(&s.ev_h2d, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&s.ev_dec, hipEventDisableTiming) != hipSuccess)
      return bail(PQG_ERR_HIP);
    s.h_blob.host = true;
  }
  g->pool = new Pool(host_threads);
  *out = g;
  return PQG_OK;
}

int pqg_rgr_close(pqg_rgr* g) {
  if (!g) return PQG_OK;
  if (g->s_dec) hipStreamSynchronize(g->s_dec);
  if (g->s_h2d) hipStreamSynchronize(g->s_h2d);
  for (Slot& s : g->slot) {
    if (s.s_d2h) {
      hipStreamSynchronize(s.s_d2h);
      hipStreamDestroy(s.s_d2h);
    }
    if (s.ctx) pqg_ctx_destroy(s.ctx);
    if (s.ev_h2d) hipEventDestroy(s.ev_h2d);
    if (s.ev_dec) hipEventDestroy(s.ev_dec);
    s.h_blob.release();
    s.d_blob.release();
    for (Col& c : s.cols)
      for (int k = 0; k < O_N; ++k) {
        c.dev[k].release();
        c.hst[k].release();
      }
  }
  if (g->s_h2d) hipStreamDestroy(g->s_h2d);
  if (g->s_dec) hipStreamDestroy(g->s_dec);
  delete g->pool;
  delete g;
  return PQG_OK;
}

const char* pqg_rgr_error(pqg_rgr* g) { return g ? g->err.c_str() : "null reader"; }

// Enqueue the D2H copies whose sizes the host knows: levels, fixed-width values (up to every level
// slot), byte-array offsets (up to every level slot + 1).
static int enqueue_known_d2h(pqg_rgr* g, Slot& s) {
  if (!(g->flags & PQG_RGR_HOST_OUTPUT)) return PQG_OK;
  RCHK(hipStreamWaitEvent(s.s_d2h, s.ev_dec, 0), "wait decode");
  for (uint32_t j = 0; j < s.ndec; ++j) {
    Col& c = s.cols[j];
    const pqg_column& d = s.desc[j];
    const bool ba = d.physical_type == PQG_BYTE_ARRAY || d.physical_type == PQG_FIXED_LEN_BYTE_ARRAY;
    const uint64_t n = c.levels;
    if (!n) continue;
    if (d.max_def > 0) RCHK(hipMemcpyAsync(c.hst[O_DEF].p, c.dev[O_DEF].p, n * 2, hipMemcpyDeviceToHost, s.s_d2h), "D2H def");
    if (d.max_rep > 0) RCHK(hipMemcpyAsync(c.hst[O_REP].p, c.dev[O_REP].p, n * 2, hipMemcpyDeviceToHost, s.s_d2h), "D2H rep");
    if (ba) {
      RCHK(hipMemcpyAsync(c.hst[O_OFF].p, c.dev[O_OFF].p, (n + 1) * 8, hipMemcpyDeviceToHost, s.s_d2h), "D2H offsets");
    } else {
      RCHK(hipMemcpyAsync(c.hst[O_VAL].p, c.dev[O_VAL].p, c.vcap, hipMemcpyDeviceToHost, s.s_d2h), "D2H values");
    }
  }
  return PQG_OK;
}

// Output buffers of column j sized for the slot's row group (grown, never shrunk).
static int size_outputs(pqg_rgr* g, Slot& s, uint32_t j) {
  Col& c = s.cols[j];
  const pqg_column& d = s.desc[j];
  const bool ba = d.physical_type == PQG_BYTE_ARRAY || d.physical_type == PQG_FIXED_LEN_BYTE_ARRAY;
  const uint64_t n = c.levels;
  const bool host = g->flags & PQG_RGR_HOST_OUTPUT;
  const size_t need[O_N] = {d.max_def > 0 ? n * 2 + 64 : 0, d.max_rep > 0 ? n * 2 + 64 : 0, c.vcap + 64,
                            ba ? (n + 1) * 8 + 64 : 0};
  for (int k = 0; k < O_N; ++k) {
    if (!need[k]) continue;
    RCHK(c.dev[k].need(need[k]), "hipMalloc outputs");
    c.hst[k].host = true;
    if (host) RCHK(c.hst[k].need(need[k]), "hipHostMalloc outputs");
  }
  pqg_output& o = s.outs[j];
  memset(&o, 0, sizeof(o));
  o.def_levels = d.max_def > 0 ? (int16_t*)c.dev[O_DEF].p : nullptr;
  o.rep_levels = d.max_rep > 0 ? (int16_t*)c.dev[O_REP].p : nullptr;
  o.values = c.dev[O_VAL].p;
  o.values_capacity = c.vcap;
  o.offsets = ba ? (int64_t*)c.dev[O_OFF].p : nullptr;
  o.offsets_capacity = ba ? n + 1 : 0;
  return PQG_OK;
}

int pqg_rgr_submit(pqg_rgr* g, int rg) {
  if (!g) return PQG_ERR_INVALID;
  pqg_file_reader* r = g->r;
  if (rg < 0 || rg >= (int)r->meta.row_groups.size()) return rgr_fail(g, PQG_ERR_INVALID, "no such row group");
  if (g->count >= 2) return rgr_fail(g, PQG_ERR_INVALID, "two row groups in flight: wait for one first");
  RCHK(hipSetDevice(g->device), "hipSetDevice");
  const auto t0 = std::chrono::steady_clock::now();
  Slot& s = g->slot[(g->head + g->count) % 3];
  const RowGroupMeta& rgm = r->meta.row_groups[rg];
  const uint32_t nc = (uint32_t)std::min(rgm.columns.size(), r->meta.leaves.size());
  s.rg = rg;
  for (size_t j = nc; j < s.cols.size(); ++j)
    for (int k = 0; k < O_N; ++k) {
      s.cols[j].dev[k].release();
      s.cols[j].hst[k].release();
    }
  s.cols.resize(nc);
  s.desc.resize(nc);
  s.outs.assign(nc, pqg_output{});
  s.pp.assign(nc, nullptr);
  s.np.assign(nc, 0);
  s.host_col = -1;
  s.status = 0;
  s.bad_col = s.bad_page = -1;
  s.err.clear();
  // ---- page headers of every column (in order: a failure stops the row group's decode there)
  uint64_t at = 0, file_bytes = 0;
  for (uint32_t j = 0; j < nc; ++j) {
    Col& c = s.cols[j];
    const LeafColumn& l = r->meta.leaves[j];
    s.desc[j] = pqg_column{l.physical_type, l.type_length, l.max_def, l.max_rep};
    c.plan.clear();
    c.host_st = 0;
    c.host_page = -1;
    c.levels = 0;
    c.len = 0;
    if (s.host_col >= 0) continue;
    c.host_st = plan_chunk_pages(r->data, r->len, rgm.columns[j], c.plan, c.len, c.host_err);
    if (c.host_st) {  // the pages before the failing header are still filled and decoded: a failure
      c.host_page = (int)c.plan.size();  // on one of them is reported first
      s.host_col = (int)j;
    }
    c.base = at;
    at = (at + c.len + 255) & ~255ull;
    file_bytes += (uint64_t)rgm.columns[j].total_compressed_size;
    for (const PagePlan& pp : c.plan)
      if (pp.page.page_type == PQG_PAGE_DATA || pp.page.page_type == PQG_PAGE_DATA_V2) c.levels += pp.page.num_values;
  }
  // columns handed to the decode: up to a failing column, which takes the pages before its failure
  s.ndec = s.host_col < 0 ? nc : (uint32_t)s.host_col + (s.cols[s.host_col].plan.empty() ? 0u : 1u);
  s.blob_len = at;
  const auto tp = std::chrono::steady_clock::now();
  // ---- payloads into pinned staging, page by page over the pool
  RCHK(s.h_blob.need(at + 64), "hipHostMalloc staging");
  RCHK(s.d_blob.need(at + 64), "hipMalloc blob");
  std::vector<std::pair<uint32_t, uint32_t>> work;
  for (uint32_t j = 0; j < s.ndec; ++j)
    for (uint32_t i = 0; i < s.cols[j].plan.size(); ++i) work.emplace_back(j, i);
  std::vector<int> wst(work.size(), 0);
  std::vector<std::string> werr(work.size());
  uint8_t* hb = (uint8_t*)s.h_blob.p;
  g->pool->run(work.size(), [&](size_t k) {
    const Col& c = s.cols[work[k].first];
    const PagePlan& pp = c.plan[work[k].second];
    wst[k] = fill_page(pp, rgm.columns[work[k].first].codec, hb + c.base, werr[k]);
  });
  const auto tf = std::chrono::steady_clock::now();
  for (size_t k = 0; k < work.size(); ++k)  // the lowest failing (column, page): the reference's first
    if (wst[k]) {
      const uint32_t j = work[k].first, i = work[k].second;
      Col& c = s.cols[j];
      c.host_st = wst[k];
      c.host_page = (int)i;
      c.host_err = werr[k];
      s.host_col = (int)j;
      c.plan.resize(i);  // the pages before it are decoded (a decode failure there comes first)
      c.levels = 0;
      for (const PagePlan& pp : c.plan)
        if (pp.page.page_type == PQG_PAGE_DATA || pp.page.page_type == PQG_PAGE_DATA_V2) c.levels += pp.page.num_values;
      s.ndec = j + (i ? 1u : 0u);
      break;
    }
  // ---- tables and outputs
  for (uint32_t j = 0; j < s.ndec; ++j) {
    Col& c = s.cols[j];
    const pqg_column& d = s.desc[j];
    c.pages.resize(c.plan.size());
    for (size_t i = 0; i < c.plan.size(); ++i) {
      c.pages[i] = c.plan[i].page;
      c.pages[i].offset += c.base;
    }
    const bool ba = d.physical_type == PQG_BYTE_ARRAY || d.physical_type == PQG_FIXED_LEN_BYTE_ARRAY;
    c.vcap = ba ? ba_capacity(c, hb, d.physical_type, d.type_length)
                : c.levels * (uint64_t)value_size(d.physical_type, d.type_length);
    const int st = size_outputs(g, s, j);
    if (st) return st;
    s.pp[j] = c.pages.data();
    s.np[j] = (uint32_t)c.pages.size();
  }
  const auto t1 = std::chrono::steady_clock::now();
  // ---- H2D, decode, D2H of what the host can size
  RCHK(hipMemcpyAsync(s.d_blob.p, hb, at, hipMemcpyHostToDevice, g->s_h2d), "H2D pages");
  RCHK(hipEventRecord(s.ev_h2d, g->s_h2d), "event");
  RCHK(hipStreamWaitEvent(g->s_dec, s.ev_h2d, 0), "wait H2D");
  int st = pqg_decode_chunks(s.ctx, s.ndec, s.desc.data(), (const uint8_t*)s.d_blob.p, at, s.pp.data(), s.np.data(),
                             s.outs.data(), g->s_dec);
  if (st) return rgr_fail(g, st, pqg_error_message(s.ctx));
  RCHK(hipEventRecord(s.ev_dec, g->s_dec), "event");
  if ((st = enqueue_known_d2h(g, s))) return st;
  const auto te = std::chrono::steady_clock::now();
  auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  g->st.plan_ms += ms(t0, tp);
  g->st.fill_ms += ms(tp, tf);
  g->st.enqueue_ms += ms(t1, te);
  g->count++;
  g->st.row_groups++;
  g->st.file_bytes += file_bytes;
  g->st.staged_bytes += at;
  g->st.host_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
  return PQG_OK;
}

int pqg_rgr_wait(pqg_rgr* g, int* rg_out, int* bad_column, int* bad_page) {
  if (rg_out) *rg_out = -1;
  if (bad_column) *bad_column = -1;
  if (bad_page) *bad_page = -1;
  if (!g) return PQG_ERR_INVALID;
  if (g->count == 0) return rgr_fail(g, PQG_ERR_INVALID, "no row group in flight");
  RCHK(hipSetDevice(g->device), "hipSetDevice");
  Slot& s = g->slot[g->head];
  g->head = (g->head + 1) % 3;
  g->count--;
  g->cur = (int)(&s - g->slot);
  int call = -1, chunk = -1, page = -1;
  const auto t0 = std::chrono::steady_clock::now();
  int st = pqg_sync_detail(s.ctx, &call, &chunk, &page);
  const auto t1 = std::chrono::steady_clock::now();
  if (st == PQG_ERR_CAPACITY) {  // a byte-array chunk decoded to more than its bound: grow, decode again
    bool grew = false;
    RCHK(hipStreamSynchronize(s.s_d2h), "sync D2H");  // the first pass's copies land before buffers move
    for (uint32_t j = 0; j < s.ndec; ++j)
      if (s.outs[j].num_bytes > s.cols[j].vcap) {
        s.cols[j].vcap = s.outs[j].num_bytes;
        const int e = size_outputs(g, s, j);
        if (e) return e;
        grew = true;
      }
    if (grew) {
      for (uint32_t j = 0; j < s.ndec; ++j) {
        pqg_output& o = s.outs[j];
        Col& c = s.cols[j];
        o.values = c.dev[O_VAL].p;
        o.values_capacity = c.vcap;
      }
      st = pqg_decode_chunks(s.ctx, s.ndec, s.desc.data(), (const uint8_t*)s.d_blob.p, s.blob_len, s.pp.data(),
                             s.np.data(), s.outs.data(), g->s_dec);
      if (st) return rgr_fail(g, st, pqg_error_message(s.ctx));
      RCHK(hipEventRecord(s.ev_dec, g->s_dec), "event");
      if ((st = enqueue_known_d2h(g, s))) return st;
      st = pqg_sync_detail(s.ctx, &call, &chunk, &page);
    }
  }
  s.status = st;
  s.bad_col = st ? chunk : -1;
  s.bad_page = st ? page : -1;
  if (st) s.err = pqg_error_message(s.ctx);
  if (s.host_col >= 0 && (!st || chunk > s.host_col)) {  // the header / decompression failure comes first
    const Col& c = s.cols[s.host_col];
    s.status = st = c.host_st;
    s.bad_col = s.host_col;
    s.bad_page = c.host_page;
    s.err = c.host_err;
  }
  if (g->flags & PQG_RGR_HOST_OUTPUT) {
    for (uint32_t j = 0; j < s.ndec; ++j) {
      const pqg_column& d = s.desc[j];
      Col& c = s.cols[j];
      const bool ba = d.physical_type == PQG_BYTE_ARRAY || d.physical_type == PQG_FIXED_LEN_BYTE_ARRAY;
      const uint64_t nb = s.outs[j].num_bytes < c.vcap ? s.outs[j].num_bytes : c.vcap;
      if (ba && nb) RCHK(hipMemcpyAsync(c.hst[O_VAL].p, c.dev[O_VAL].p, nb, hipMemcpyDeviceToHost, s.s_d2h), "D2H bytes");
    }
    RCHK(hipStreamSynchronize(s.s_d2h), "sync D2H");
  }
  const auto t2 = std::chrono::steady_clock::now();
  g->st.sync_ms += std::chrono::duration<double, std::milli>(t1 - t0).count();
  g->st.d2h_wait_ms += std::chrono::duration<double, std::milli>(t2 - t1).count();
  for (uint32_t j = 0; j < s.ndec; ++j) {
    const pqg_output& o = s.outs[j];
    const bool ba = s.desc[j].physical_type == PQG_BYTE_ARRAY || s.desc[j].physical_type == PQG_FIXED_LEN_BYTE_ARRAY;
    const uint64_t streams = (uint64_t)(s.desc[j].max_def > 0) + (uint64_t)(s.desc[j].max_rep > 0);
    g->st.output_bytes += o.num_levels * 2 * streams +
                          (ba ? o.num_bytes + (o.num_values + 1) * 8
                              : o.num_values * (uint64_t)value_size(s.desc[j].physical_type, s.desc[j].type_length));
  }
  if (rg_out) *rg_out = s.rg;
  if (bad_column) *bad_column = s.bad_col;
  if (bad_page) *bad_page = s.bad_page;
  if (st) g->err = "row group " + std::to_string(s.rg) + ", column " + std::to_string(s.bad_col) + ": " + s.err;
  return st;
}

int pqg_rgr_column(pqg_rgr* g, int col, pqg_rgr_output* out) {
  if (!g || !out || g->cur < 0) return PQG_ERR_INVALID;
  const Slot& s = g->slot[g->cur];
  if (col < 0 || col >= (int)s.cols.size()) return PQG_ERR_INVALID;
  memset(out, 0, sizeof(*out));
  if ((uint32_t)col >= s.ndec) return s.status ? s.status : PQG_ERR_GENERAL;  // not decoded: at / after a host failure
  const Col& c = s.cols[col];
  const pqg_output& o = s.outs[col];
  const bool host = g->flags & PQG_RGR_HOST_OUTPUT;
  out->def_levels = o.def_levels;
  out->rep_levels = o.rep_levels;
  out->values = o.values;
  out->offsets = o.offsets;
  if (host) {
    out->host_def_levels = o.def_levels ? (const int16_t*)c.hst[O_DEF].p : nullptr;
    out->host_rep_levels = o.rep_levels ? (const int16_t*)c.hst[O_REP].p : nullptr;
    out->host_values = (const void*)c.hst[O_VAL].p;
    out->host_offsets = o.offsets ? (const int64_t*)c.hst[O_OFF].p : nullptr;
  }
  out->num_levels = o.num_levels;
  out->num_values = o.num_values;
  out->num_bytes = o.num_bytes;
  return (s.status && col >= s.bad_col) ? s.status : PQG_OK;
}

int pqg_rgr_get_stats(pqg_rgr* g, pqg_rgr_stats* out) {
  if (!g || !out) return PQG_ERR_INVALID;
  *out = g->st;
  return PQG_OK;
}

}  // extern "C"
