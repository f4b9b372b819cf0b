// pqg_gen.cpp — reference-identical page writers and the synthetic workload generators
// (libpqgtools.so: bench and test tooling, not part of the decode library libpqgpu.so).
//
// The writers restate parquet-rs's encoders so the generated pages are byte-for-byte what
// the reference would write:
//   BitWriter            util/bit_util.rs:136-363
//   RleEncoder           encodings/rle.rs:55-317 (runs <= 504 values, rle.rs:49-50)
//   LevelEncoder::v1     encodings/levels.rs:54-143 (RLE, 4-byte length prefix)
//   DictEncoder indices  encodings/encoding.rs:338-355 ([bit width][RLE hybrid])
//   DeltaBitPackEncoder  encodings/encoding.rs:534-714 (block size / mini-block count are
//                        parameters; the reference fixes 128 / 4, encoding.rs:508-509)
// The generators build BASELINE.json configs 2-5 page by page on host threads (pages are
// independent) for bench.py; the pqg_truth_* entry points regenerate one page's raw
// levels / values so the bench can check decoded output against the generator.
#include <stdint.h>
#include <string.h>

#include <stdio.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <unordered_map>
#include <vector>

#include "pqg_gen.h"

namespace {

int64_t ceil_div(int64_t v, int64_t d) { return v / d + (v % d != 0); }

int log2_ceil(uint64_t x) {
  if (x == 1) return 0;
  x -= 1;
  int r = 0;
  while (x) {
    x >>= 1;
    r++;
  }
  return r;
}

size_t num_required_bits(uint64_t x) {
  for (int i = 63; i >= 0; --i)
    if (x & (1ULL << i)) return (size_t)i + 1;
  return 0;
}

struct BitWriter {
  uint8_t* buf;
  size_t max_bytes;
  uint64_t buffered = 0;
  size_t byte_offset;
  size_t bit_offset = 0;
  bool ok = true;
  BitWriter(uint8_t* b, size_t cap, size_t start) : buf(b), max_bytes(cap), byte_offset(start) {}
  void flush() {
    size_t nb = (size_t)ceil_div((int64_t)bit_offset, 8);
    if (byte_offset + nb > max_bytes) {
      ok = false;
      return;
    }
    memcpy(buf + byte_offset, &buffered, nb);
    buffered = 0;
    bit_offset = 0;
    byte_offset += nb;
  }
  long skip(size_t n) {
    flush();
    if (!ok || byte_offset + n > max_bytes) {
      ok = false;
      return -1;
    }
    long r = (long)byte_offset;
    byte_offset += n;
    return r;
  }
  void put_value(uint64_t v, size_t bits) {
    if (byte_offset * 8 + bit_offset + bits > max_bytes * 8) {
      ok = false;
      return;
    }
    buffered |= v << bit_offset;
    bit_offset += bits;
    if (bit_offset >= 64) {
      memcpy(buf + byte_offset, &buffered, 8);
      byte_offset += 8;
      bit_offset -= 64;
      size_t sh = bits - bit_offset;
      buffered = sh < 64 ? (v >> sh) : 0;
    }
  }
  void put_aligned(uint64_t v, size_t nbytes) {
    long off = skip(nbytes);
    if (off >= 0) memcpy(buf + off, &v, nbytes);
  }
  void put_vlq(uint64_t v) {
    while (v & 0xFFFFFFFFFFFFFF80ULL) {
      put_aligned((v & 0x7F) | 0x80, 1);
      v >>= 7;
    }
    put_aligned(v & 0x7F, 1);
  }
  void put_zigzag(int64_t v) { put_vlq(((uint64_t)v << 1) ^ (uint64_t)(v >> 63)); }
};

// RleEncoder, rle.rs:55-317
struct RleEncoder {
  int bit_width;
  BitWriter bw;
  uint64_t buffered_values[8];
  size_t num_buffered = 0;
  uint64_t current_value = 0;
  size_t repeat_count = 0;
  size_t bit_packed_count = 0;
  long indicator_byte_pos = -1;
  RleEncoder(int w, uint8_t* buf, size_t cap, size_t start) : bit_width(w), bw(buf, cap, start) {}

  void flush_rle_run() {
    bw.put_vlq((uint64_t)(repeat_count << 1));
    bw.put_aligned(current_value, (size_t)ceil_div(bit_width, 8));
    num_buffered = 0;
    repeat_count = 0;
  }
  void flush_bit_packed_run(bool update) {
    if (indicator_byte_pos < 0) indicator_byte_pos = bw.skip(1);
    if (indicator_byte_pos < 0) return;
    for (size_t i = 0; i < num_buffered; ++i) bw.put_value(buffered_values[i], (size_t)bit_width);
    num_buffered = 0;
    if (update) {
      bw.buf[indicator_byte_pos] = (uint8_t)(((bit_packed_count / 8) << 1) | 1);
      indicator_byte_pos = -1;
      bit_packed_count = 0;
    }
  }
  void flush_buffered_values() {
    if (repeat_count >= 8) {
      num_buffered = 0;
      if (bit_packed_count > 0) flush_bit_packed_run(true);
      return;
    }
    bit_packed_count += num_buffered;
    size_t groups = bit_packed_count / 8;
    flush_bit_packed_run(groups + 1 >= 64);  // MAX_GROUPS_PER_BIT_PACKED_RUN
    repeat_count = 0;
  }
  inline void put(uint64_t v) {
    if (current_value == v) {
      repeat_count += 1;
      if (repeat_count > 8) return;
    } else {
      if (repeat_count >= 8) flush_rle_run();
      repeat_count = 1;
      current_value = v;
    }
    buffered_values[num_buffered++] = v;
    if (num_buffered == 8) flush_buffered_values();
  }
  void flush() {
    if (bit_packed_count > 0 || repeat_count > 0 || num_buffered > 0) {
      bool all_repeat = bit_packed_count == 0 && (repeat_count == num_buffered || num_buffered == 0);
      if (repeat_count > 0 && all_repeat) {
        flush_rle_run();
      } else {
        if (num_buffered > 0)
          while (num_buffered < 8) buffered_values[num_buffered++] = 0;
        bit_packed_count += num_buffered;
        flush_bit_packed_run(true);
        repeat_count = 0;
      }
    }
  }
  size_t consume() {
    flush();
    bw.flush();
    return bw.ok ? bw.byte_offset : 0;
  }
};

// RleEncoder::max_buffer_size + min_buffer_size (rle.rs:127-150)
uint64_t rle_bound(int w, uint64_t n) {
  uint64_t runs = (uint64_t)ceil_div((int64_t)n, 8);
  uint64_t bp = runs + runs * (uint64_t)w;
  uint64_t rl = runs * (1 + (uint64_t)ceil_div(w, 8));
  uint64_t mx = std::max(bp, rl);
  uint64_t minb = std::max<uint64_t>(1 + (uint64_t)ceil_div(504 * w, 8), 10 + (uint64_t)ceil_div(w, 8));
  return mx + minb + 16;
}

// DeltaBitPackEncoder, encoding.rs:534-714, with block_size / mini_blocks parameters.
template <class T>
uint64_t delta_encode(const T* v, uint64_t n, int block_size, int nmb, uint8_t* out, uint64_t cap) {
  const size_t mini = (size_t)block_size / (size_t)nmb;
  if (mini % 8 != 0 || mini == 0) return 0;
  uint8_t hdr[64];
  BitWriter hw(hdr, sizeof(hdr), 0);
  std::vector<uint8_t> tmp;  // header is written first; body follows it
  // body writer directly into out at an offset reserved for the header (<= 40 bytes)
  const size_t HR = 40;
  if (cap < HR) return 0;
  BitWriter w(out + HR, cap - HR, 0);
  std::vector<int64_t> deltas((size_t)block_size);
  size_t in_block = 0;
  int64_t first = n ? (int64_t)v[0] : 0, cur = first;
  auto sub = [](int64_t l, int64_t r) -> int64_t {
    if (sizeof(T) == 4) return (int64_t)(int32_t)((uint32_t)(int32_t)l - (uint32_t)(int32_t)r);
    return (int64_t)((uint64_t)l - (uint64_t)r);
  };
  auto sub_u64 = [](int64_t l, int64_t r) -> uint64_t {
    if (sizeof(T) == 4) return (uint64_t)(uint32_t)((uint32_t)(int32_t)l - (uint32_t)(int32_t)r);
    return (uint64_t)l - (uint64_t)r;
  };
  auto flush_block = [&]() {
    if (in_block == 0) return;
    int64_t min_delta = INT64_MAX;
    for (size_t i = 0; i < in_block; ++i) min_delta = std::min(min_delta, deltas[i]);
    w.put_zigzag(min_delta);
    long wpos = w.skip((size_t)nmb);
    if (wpos < 0) return;
    for (int i = 0; i < nmb; ++i) {
      size_t m = std::min(mini, in_block);
      if (m == 0) break;
      int64_t max_delta = INT64_MIN;
      for (size_t j = 0; j < m; ++j) max_delta = std::max(max_delta, deltas[i * mini + j]);
      size_t bwid = num_required_bits(sub_u64(max_delta, min_delta));
      w.buf[wpos + i] = (uint8_t)bwid;
      for (size_t j = 0; j < m; ++j) w.put_value(sub_u64(deltas[i * mini + j], min_delta), bwid);
      for (size_t j = m; j < mini; ++j) w.put_value(0, bwid);
      in_block -= m;
    }
  };
  for (uint64_t idx = 1; idx < n; ++idx) {
    int64_t x = (int64_t)v[idx];
    deltas[in_block++] = sub(x, cur);
    cur = x;
    if (in_block == (size_t)block_size) flush_block();
  }
  flush_block();
  hw.put_vlq((uint64_t)block_size);
  hw.put_vlq((uint64_t)nmb);
  hw.put_vlq(n);
  hw.put_zigzag(first);
  hw.flush();
  w.flush();
  if (!w.ok || !hw.ok) return 0;
  size_t hl = hw.byte_offset;
  memmove(out + hl, out + HR, w.byte_offset);
  memcpy(out, hdr, hl);
  return hl + w.byte_offset;
}

// SplitMix64: seeded, counter-based, identical in Python (bench.py) and here.
inline uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

inline uint64_t page_seed(uint64_t seed, uint64_t page) {
  uint64_t s = seed ^ (page * 0xD1B54A32D192ED03ULL);
  return splitmix64(s);
}

template <class F>
void parallel_pages(uint32_t npages, int threads, F&& f) {
  if (threads <= 0) threads = (int)std::max(1u, std::thread::hardware_concurrency());
  threads = std::min<int>(threads, (int)std::max<uint32_t>(npages, 1));
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t)
    ts.emplace_back([&, t]() {
      for (uint32_t p = (uint32_t)t; p < npages; p += (uint32_t)threads) f(p);
    });
  for (auto& th : ts) th.join();
}

inline uint64_t align64(uint64_t x) { return (x + 63) & ~63ull; }

}  // namespace

extern "C" {

uint64_t pqg_encode_rle(const uint64_t* values, uint64_t n, int bit_width, uint8_t* out, uint64_t cap) {
  memset(out, 0, cap);
  RleEncoder e(bit_width, out, cap, 0);
  for (uint64_t i = 0; i < n; ++i) e.put(values[i]);
  return e.consume();
}

uint64_t pqg_encode_levels_v1(const int16_t* levels, uint64_t n, int16_t max_level, uint8_t* out,
                              uint64_t cap) {
  if (cap < 4) return 0;
  memset(out, 0, cap);
  RleEncoder e(log2_ceil((uint64_t)(int64_t)max_level + 1), out, cap, 4);
  for (uint64_t i = 0; i < n; ++i) e.put((uint64_t)(int64_t)levels[i]);
  size_t end = e.consume();
  if (!end) return 0;
  int32_t len = (int32_t)(end - 4);
  memcpy(out, &len, 4);
  return end;
}

uint64_t pqg_encode_delta(int physical_type, const void* values, uint64_t n, int block_size,
                          int mini_blocks, uint8_t* out, uint64_t cap) {
  if (physical_type == PQG_INT32)
    return delta_encode((const int32_t*)values, n, block_size, mini_blocks, out, cap);
  if (physical_type == PQG_INT64)
    return delta_encode((const int64_t*)values, n, block_size, mini_blocks, out, cap);
  return 0;
}

uint64_t pqg_encode_dict_indices(const uint32_t* idx, uint64_t n, int bit_width, uint8_t* out,
                                 uint64_t cap) {
  if (cap < 1) return 0;
  memset(out, 0, cap);
  out[0] = (uint8_t)bit_width;
  RleEncoder e(bit_width, out, cap, 1);
  for (uint64_t i = 0; i < n; ++i) e.put(idx[i]);
  return e.consume();
}

// ------------------------------------------------------------------ config 2
// Raw content of config-2 page p: levels (1 = non-null) and the non-null INT32 values.
static uint64_t levels_page(uint64_t n, double p_null, uint32_t page_levels, uint64_t seed, uint32_t p,
                            std::vector<int16_t>& lv, int32_t* vals) {
  const uint64_t cnt = std::min<uint64_t>(page_levels, n - (uint64_t)p * page_levels);
  // a level is null with probability p_null: compare 53-bit uniforms against the threshold
  const uint64_t thresh = (uint64_t)(p_null * 9007199254740992.0);
  uint64_t s = page_seed(seed, p);
  lv.resize(cnt);
  uint64_t nn = 0;
  for (uint64_t i = 0; i < cnt; ++i) {
    lv[i] = (splitmix64(s) >> 11) >= thresh ? 1 : 0;
    nn += (uint64_t)lv[i];
  }
  for (uint64_t i = 0; i < nn; ++i) {
    int32_t x = (int32_t)(uint32_t)splitmix64(s);
    memcpy((uint8_t*)vals + 4 * i, &x, 4);  // unaligned PLAIN section
  }
  return nn;
}

// Pages [first, first + count) of the config-2 stream (a rank's contiguous share of one stream:
// page p's content depends on the seed and p alone).
int pqg_gen_levels_plain_pages(uint64_t n, double p_null, uint32_t page_levels, uint64_t seed, uint32_t first,
                               uint32_t count, int threads, uint8_t* blob, uint64_t blob_cap, pqg_page* pages,
                               uint32_t pages_cap, pqg_workload_info* info) {
  if (!info || page_levels == 0) return PQG_ERR_INVALID;
  const uint32_t all = (uint32_t)((n + page_levels - 1) / page_levels);
  if (first > all || count > all - first) return PQG_ERR_INVALID;
  const uint32_t np = count;
  const uint64_t slot = align64(4 + rle_bound(1, page_levels) + 4ull * page_levels);
  info->npages = np;
  info->blob_len = slot * np;
  info->total_levels = 0;
  for (uint32_t p = first; p < first + np; ++p) info->total_levels += std::min<uint64_t>(page_levels, n - (uint64_t)p * page_levels);
  info->total_values = 0;
  if (!blob) return PQG_OK;
  if (blob_cap < slot * np || pages_cap < np) return PQG_ERR_CAPACITY;
  std::vector<uint64_t> nonnull(np);
  parallel_pages(np, threads, [&](uint32_t q) {
    const uint32_t p = first + q;
    uint8_t* out = blob + (uint64_t)q * slot;
    std::vector<int16_t> lv;
    std::vector<int32_t> vals(page_levels);
    const uint64_t nn = levels_page(n, p_null, page_levels, seed, p, lv, vals.data());
    const uint64_t cnt = lv.size();
    uint64_t ll = pqg_encode_levels_v1(lv.data(), cnt, 1, out, slot - 4 * cnt);
    memcpy(out + ll, vals.data(), 4 * nn);
    pqg_page& pg = pages[q];
    pg.offset = (uint64_t)q * slot;
    pg.nbytes = (uint32_t)(ll + 4 * nn);
    pg.num_values = (uint32_t)cnt;
    pg.page_type = PQG_PAGE_DATA;
    pg.encoding = PQG_PLAIN;
    pg.def_encoding = PQG_RLE;
    pg.rep_encoding = PQG_BIT_PACKED;
    pg.def_len = pg.rep_len = 0;
    nonnull[q] = nn;
  });
  for (uint64_t x : nonnull) info->total_values += x;
  return PQG_OK;
}

int pqg_gen_levels_plain(uint64_t n, double p_null, uint32_t page_levels, uint64_t seed,
                         int threads, uint8_t* blob, uint64_t blob_cap, pqg_page* pages,
                         uint32_t pages_cap, pqg_workload_info* info) {
  if (page_levels == 0) return PQG_ERR_INVALID;
  return pqg_gen_levels_plain_pages(n, p_null, page_levels, seed, 0, (uint32_t)((n + page_levels - 1) / page_levels),
                                    threads, blob, blob_cap, pages, pages_cap, info);
}

uint64_t pqg_truth_levels_plain(uint64_t n, double p_null, uint32_t page_levels, uint64_t seed,
                                uint32_t page, int16_t* levels, int32_t* values) {
  std::vector<int16_t> lv;
  const uint64_t nn = levels_page(n, p_null, page_levels, seed, page, lv, values);
  memcpy(levels, lv.data(), lv.size() * 2);
  return nn;
}

// ------------------------------------------------------------------ config 3
static void dict_values(uint32_t dict_size, uint64_t seed, uint8_t* out) {
  // distinct values (SplitMix64 of distinct counters is a bijection)
  uint64_t ds = seed ^ 0xD1C7D1C7ull;
  for (uint32_t i = 0; i < dict_size; ++i) {
    uint64_t x = splitmix64(ds);
    memcpy(out + 8ull * i, &x, 8);
  }
}

static void dict_page_indices(uint64_t n, uint32_t dict_size, uint32_t page_values, uint64_t seed,
                              uint32_t p, std::vector<uint32_t>& idx) {
  const uint64_t cnt = std::min<uint64_t>(page_values, n - (uint64_t)p * page_values);
  uint64_t s = page_seed(seed, p);
  idx.resize(cnt);
  for (uint64_t i = 0; i < cnt; ++i) idx[i] = (uint32_t)((splitmix64(s) >> 32) * dict_size >> 32);
}

// The dictionary page and data pages [first, first + count) of the config-3 stream.
int pqg_gen_dict_int64_pages(uint64_t n, uint32_t dict_size, uint32_t page_values, uint64_t seed, uint32_t first,
                             uint32_t count, int threads, uint8_t* blob, uint64_t blob_cap, pqg_page* pages,
                             uint32_t pages_cap, pqg_workload_info* info) {
  if (!info || page_values == 0 || dict_size == 0) return PQG_ERR_INVALID;
  const uint32_t all = (uint32_t)((n + page_values - 1) / page_values);
  if (first > all || count > all - first) return PQG_ERR_INVALID;
  const uint32_t ndata = count;
  const int bw = dict_size == 1 ? 1 : log2_ceil(dict_size);  // encoding.rs:325-334
  const uint64_t dslot = align64(8ull * dict_size);
  const uint64_t slot = align64(1 + rle_bound(bw, page_values));
  info->npages = ndata + 1;
  info->blob_len = dslot + slot * ndata;
  info->total_levels = 0;
  for (uint32_t p = first; p < first + ndata; ++p) info->total_levels += std::min<uint64_t>(page_values, n - (uint64_t)p * page_values);
  info->total_values = info->total_levels;
  if (!blob) return PQG_OK;
  if (blob_cap < info->blob_len || pages_cap < ndata + 1) return PQG_ERR_CAPACITY;
  dict_values(dict_size, seed, blob);
  pages[0] = pqg_page{0, 8u * dict_size, dict_size, PQG_PAGE_DICTIONARY, PQG_PLAIN_DICTIONARY,
                      PQG_RLE, PQG_RLE, 0, 0};
  parallel_pages(ndata, threads, [&](uint32_t q) {
    uint8_t* out = blob + dslot + (uint64_t)q * slot;
    std::vector<uint32_t> idx;
    dict_page_indices(n, dict_size, page_values, seed, first + q, idx);
    uint64_t l = pqg_encode_dict_indices(idx.data(), idx.size(), bw, out, slot);
    pages[q + 1] = pqg_page{dslot + (uint64_t)q * slot, (uint32_t)l, (uint32_t)idx.size(), PQG_PAGE_DATA,
                            PQG_PLAIN_DICTIONARY, PQG_RLE, PQG_BIT_PACKED, 0, 0};
  });
  return PQG_OK;
}

int pqg_gen_dict_int64(uint64_t n, uint32_t dict_size, uint32_t page_values, uint64_t seed,
                       int threads, uint8_t* blob, uint64_t blob_cap, pqg_page* pages,
                       uint32_t pages_cap, pqg_workload_info* info) {
  if (page_values == 0) return PQG_ERR_INVALID;
  return pqg_gen_dict_int64_pages(n, dict_size, page_values, seed, 0, (uint32_t)((n + page_values - 1) / page_values),
                                  threads, blob, blob_cap, pages, pages_cap, info);
}

uint64_t pqg_truth_dict_int64(uint64_t n, uint32_t dict_size, uint32_t page_values, uint64_t seed,
                              uint32_t page, int64_t* values) {
  std::vector<uint8_t> d(8ull * dict_size);
  dict_values(dict_size, seed, d.data());
  std::vector<uint32_t> idx;
  dict_page_indices(n, dict_size, page_values, seed, page, idx);
  for (size_t i = 0; i < idx.size(); ++i) memcpy(values + i, d.data() + 8ull * idx[i], 8);
  return idx.size();
}

// ------------------------------------------------------------------ config 4
static void delta_page_values(uint64_t n, int delta_bits, uint32_t page_values, uint64_t seed,
                              uint32_t p, std::vector<int64_t>& v) {
  const uint64_t cnt = std::min<uint64_t>(page_values, n - (uint64_t)p * page_values);
  uint64_t s = page_seed(seed, p);
  v.resize(cnt);
  uint64_t acc = splitmix64(s);
  const uint64_t span = 1ull << delta_bits;
  const int64_t half = (int64_t)(span >> 1);
  for (uint64_t i = 0; i < cnt; ++i) {
    v[i] = (int64_t)acc;
    int64_t d = (int64_t)((splitmix64(s) >> (64 - delta_bits))) - half;
    acc += (uint64_t)d;  // wrapping prefix sum
  }
}

// Pages [first, first + count) of the config-4 stream.
int pqg_gen_delta_int64_pages(uint64_t n, int delta_bits, uint32_t page_values, int block_size, int mini_blocks,
                              uint64_t seed, uint32_t first, uint32_t count, int threads, uint8_t* blob,
                              uint64_t blob_cap, pqg_page* pages, uint32_t pages_cap, pqg_workload_info* info) {
  if (!info || page_values == 0 || delta_bits < 1 || delta_bits > 63) return PQG_ERR_INVALID;
  const uint32_t all = (uint32_t)((n + page_values - 1) / page_values);
  if (first > all || count > all - first) return PQG_ERR_INVALID;
  const uint32_t np = count;
  const uint64_t blocks = (page_values + block_size - 1) / block_size + 1;
  const uint64_t slot = align64(64 + 8ull * page_values + blocks * (10 + mini_blocks) + 8ull * block_size);
  info->npages = np;
  info->blob_len = slot * np;
  info->total_levels = 0;
  for (uint32_t p = first; p < first + np; ++p) info->total_levels += std::min<uint64_t>(page_values, n - (uint64_t)p * page_values);
  info->total_values = info->total_levels;
  if (!blob) return PQG_OK;
  if (blob_cap < info->blob_len || pages_cap < np) return PQG_ERR_CAPACITY;
  std::atomic<int> rc{PQG_OK};
  parallel_pages(np, threads, [&](uint32_t q) {
    std::vector<int64_t> v;
    delta_page_values(n, delta_bits, page_values, seed, first + q, v);
    uint8_t* out = blob + (uint64_t)q * slot;
    uint64_t l = delta_encode(v.data(), v.size(), block_size, mini_blocks, out, slot);
    if (!l) rc = PQG_ERR_CAPACITY;
    pages[q] = pqg_page{(uint64_t)q * slot, (uint32_t)l, (uint32_t)v.size(), PQG_PAGE_DATA,
                        PQG_DELTA_BINARY_PACKED, PQG_RLE, PQG_BIT_PACKED, 0, 0};
  });
  return rc;
}

int pqg_gen_delta_int64(uint64_t n, int delta_bits, uint32_t page_values, int block_size,
                        int mini_blocks, uint64_t seed, int threads, uint8_t* blob,
                        uint64_t blob_cap, pqg_page* pages, uint32_t pages_cap,
                        pqg_workload_info* info) {
  if (page_values == 0) return PQG_ERR_INVALID;
  return pqg_gen_delta_int64_pages(n, delta_bits, page_values, block_size, mini_blocks, seed, 0,
                                   (uint32_t)((n + page_values - 1) / page_values), threads, blob, blob_cap, pages,
                                   pages_cap, info);
}

uint64_t pqg_truth_delta_int64(uint64_t n, int delta_bits, uint32_t page_values, uint64_t seed,
                               uint32_t page, int64_t* values) {
  std::vector<int64_t> v;
  delta_page_values(n, delta_bits, page_values, seed, page, v);
  memcpy(values, v.data(), v.size() * 8);
  return v.size();
}

}  // extern "C"

// ------------------------------------------------------------------ config 5
// One row group of the alltypes_plain schema (data/alltypes_plain.parquet: 11 OPTIONAL
// columns, max_def 1), written the way ColumnWriterImpl does with the default properties
// (file/properties.rs:56-65: v1 pages, 1 MiB data pages, dictionary on with a 1 MiB limit,
// batches of 1024 levels, no compression):
//   - after each 1024-level mini-batch (column/writer.rs:230-245, 345-364) a data page is cut
//     once the PLAIN encoder's estimate reaches 1 MiB (:406-410); while the dictionary encoder
//     holds the values that estimate stays 0, so a dictionary chunk buffers one data page;
//   - once the dictionary's PLAIN size reaches 1 MiB (:395-402) the dictionary page and the
//     buffered data page are written and the rest of the chunk is PLAIN (:412-420, 543-556);
//   - at the end the dictionary page (if still in use) then the last data page;
//   - BOOLEAN has no dictionary support (:744-756);
//   - data page v1: [i32 length][RLE def levels][values] (:441-480); dictionary data pages
//     PLAIN_DICTIONARY with [bit width][RLE hybrid] indices (encoding.rs:338-355, bit width
//     :324-334), the dictionary page PLAIN_DICTIONARY with the PLAIN uniques.
// Cell contents are counter-based (seed, column, row): the row-group generator and the truth
// function below agree without sharing state.
namespace {

constexpr int AT_NCOL = 11;
const int at_ptype[AT_NCOL] = {PQG_INT32, PQG_BOOLEAN, PQG_INT32, PQG_INT32, PQG_INT32, PQG_INT64,
                               PQG_FLOAT, PQG_DOUBLE, PQG_BYTE_ARRAY, PQG_BYTE_ARRAY, PQG_INT96};
constexpr uint64_t AT_PAGE = 1 << 20;  // data page size limit (properties.rs:56)
constexpr uint64_t AT_DICT = 1 << 20;  // dictionary page size limit (properties.rs:61)
constexpr uint64_t AT_BATCH = 1024;    // write batch size (properties.rs:57)

inline uint64_t at_hash(uint64_t seed, uint32_t col, uint64_t row, uint32_t k) {
  uint64_t s = seed ^ ((uint64_t)col * 0x9E3779B97F4A7C15ULL) ^ (row * 0xD1B54A32D192ED03ULL) ^
               ((uint64_t)k * 0xC2B2AE3D27D4EB4FULL);
  return splitmix64(s);
}

// Cell (col, row): null, or the value's PLAIN bytes (BYTE_ARRAY: the bytes alone).
struct AtCell {
  bool null;
  uint32_t len;
  uint8_t v[16];
};

void at_cell(uint64_t seed, double p_null, uint32_t col, uint64_t row, AtCell& c) {
  const uint64_t thresh = (uint64_t)(p_null * 9007199254740992.0);
  c.null = (at_hash(seed, col, row, 0) >> 11) < thresh;
  const uint64_t h = at_hash(seed, col, row, 1);
  const uint32_t k = (uint32_t)((h >> 32) * 10 >> 32);  // 0..9, as the fixture's small columns
  switch (col) {
    case 0: {  // id: the row number
      const int32_t x = (int32_t)row;
      memcpy(c.v, &x, 4);
      c.len = 4;
      break;
    }
    case 1:  // bool_col: alternating
      c.v[0] = (row & 1) == 0;
      c.len = 1;
      break;
    case 2:
    case 3:
    case 4: {  // tinyint / smallint / int
      const int32_t x = (int32_t)k;
      memcpy(c.v, &x, 4);
      c.len = 4;
      break;
    }
    case 5: {  // bigint
      const int64_t x = (int64_t)k * 10;
      memcpy(c.v, &x, 8);
      c.len = 8;
      break;
    }
    case 6: {  // float
      const float x = (float)k * 1.1f;
      memcpy(c.v, &x, 4);
      c.len = 4;
      break;
    }
    case 7: {  // double
      const double x = (double)k * 10.1;
      memcpy(c.v, &x, 8);
      c.len = 8;
      break;
    }
    case 8: {  // date_string_col "MM/DD/YY" over two years
      const uint32_t d = (uint32_t)(h % 730);
      const uint32_t y = 9 + d / 365, doy = d % 365;
      const uint32_t mo = doy / 31 + 1, dd = doy % 31 + 1;
      char b[16];
      snprintf(b, sizeof(b), "%02u/%02u/%02u", mo, dd, y);
      memcpy(c.v, b, 8);
      c.len = 8;
      break;
    }
    case 9:  // string_col: one digit
      c.v[0] = (uint8_t)('0' + k);
      c.len = 1;
      break;
    default: {  // timestamp_col INT96: nanoseconds of the day, then the Julian day
      const uint64_t ns = h % 86400000000000ULL;
      const uint32_t jd = 2454833u + (uint32_t)(at_hash(seed, col, row, 2) % 730);
      memcpy(c.v, &ns, 8);
      memcpy(c.v + 8, &jd, 4);
      c.len = 12;
      break;
    }
  }
}

// One column chunk of the row group: its pages (offsets relative to the chunk start, each
// payload 64-byte aligned).
struct AtChunk {
  std::vector<uint8_t> buf;
  std::vector<pqg_page> pages;
  uint64_t values = 0, value_bytes = 0;
};

struct AtKey {
  uint8_t v[16];
  uint32_t len;
  bool operator==(const AtKey& o) const { return len == o.len && memcmp(v, o.v, len) == 0; }
};
struct AtKeyHash {
  size_t operator()(const AtKey& k) const {
    uint64_t s = k.len;
    for (uint32_t i = 0; i < k.len; ++i) s = s * 131 + k.v[i];
    return (size_t)splitmix64(s);
  }
};

void at_write_chunk(uint64_t rows, uint64_t row0, double p_null, uint64_t seed, uint32_t col, AtChunk& ch) {
  const int pt = at_ptype[col];
  bool dict = pt != PQG_BOOLEAN;
  std::unordered_map<AtKey, uint32_t, AtKeyHash> map;
  std::vector<uint8_t> uniq;   // PLAIN dictionary page payload
  uint32_t nuniq = 0;
  uint64_t dict_size = 0;      // DictEncoder::dict_encoded_size
  std::vector<uint32_t> idx;   // buffered indices (dictionary data page)
  std::vector<uint8_t> plain;  // PLAIN values of the pending page
  uint64_t nbool = 0;          // PLAIN booleans of the pending page (bit-packed into plain)
  std::vector<int16_t> lv;     // def levels of the pending page
  auto put_page = [&](const uint8_t* p, uint64_t n, uint32_t nv, int type, int enc) {
    const uint64_t off = align64(ch.buf.size());
    ch.buf.resize(off + n);
    memcpy(ch.buf.data() + off, p, n);
    ch.pages.push_back(pqg_page{off, (uint32_t)n, nv, type, enc, PQG_RLE, PQG_RLE, 0, 0});
  };
  auto data_page = [&](bool dict_page) {
    if (lv.empty()) return;
    std::vector<uint8_t> b(8 + rle_bound(1, lv.size()) + plain.size() + rle_bound(32, idx.size()) + 16);
    const uint64_t ll = pqg_encode_levels_v1(lv.data(), lv.size(), 1, b.data(), b.size());
    uint64_t vl;
    if (dict_page) {
      const int bw = nuniq == 0 ? 0 : nuniq == 1 ? 1 : log2_ceil(nuniq);
      vl = pqg_encode_dict_indices(idx.data(), idx.size(), bw, b.data() + ll, b.size() - ll);
    } else {
      memcpy(b.data() + ll, plain.data(), plain.size());
      vl = plain.size();
    }
    put_page(b.data(), ll + vl, (uint32_t)lv.size(), PQG_PAGE_DATA, dict_page ? PQG_PLAIN_DICTIONARY : PQG_PLAIN);
    lv.clear();
    idx.clear();
    plain.clear();
    nbool = 0;
  };
  auto dict_out = [&]() {
    put_page(uniq.data(), uniq.size(), nuniq, PQG_PAGE_DICTIONARY, PQG_PLAIN_DICTIONARY);
    data_page(true);
    dict = false;
  };
  AtCell c;
  for (uint64_t b0 = 0; b0 < rows; b0 += AT_BATCH) {
    const uint64_t b1 = std::min(rows, b0 + AT_BATCH);
    for (uint64_t r = b0; r < b1; ++r) {
      at_cell(seed, p_null, col, row0 + r, c);
      lv.push_back(c.null ? 0 : 1);
      if (c.null) continue;
      ch.values++;
      ch.value_bytes += c.len;
      if (dict) {
        AtKey key;
        memcpy(key.v, c.v, c.len);
        key.len = c.len;
        auto it = map.find(key);
        uint32_t id;
        if (it == map.end()) {
          id = nuniq++;
          map.emplace(key, id);
          if (pt == PQG_BYTE_ARRAY) {
            const uint32_t l = c.len;
            uniq.insert(uniq.end(), (const uint8_t*)&l, (const uint8_t*)&l + 4);
          }
          uniq.insert(uniq.end(), c.v, c.v + c.len);
          dict_size += pt == PQG_BYTE_ARRAY ? 4 + c.len : c.len;
        } else {
          id = it->second;
        }
        idx.push_back(id);
      } else if (pt == PQG_BOOLEAN) {
        if ((nbool & 7) == 0) plain.push_back(0);
        plain.back() |= (uint8_t)(c.v[0] << (nbool & 7));
        ++nbool;
      } else {
        if (pt == PQG_BYTE_ARRAY) {
          const uint32_t l = c.len;
          plain.insert(plain.end(), (const uint8_t*)&l, (const uint8_t*)&l + 4);
        }
        plain.insert(plain.end(), c.v, c.v + c.len);
      }
    }
    // write_mini_batch's tail: page cut on the PLAIN estimate, then the dictionary fallback
    if (!dict && plain.size() >= AT_PAGE) data_page(false);
    if (dict && dict_size >= AT_DICT) dict_out();
  }
  if (dict) dict_out();
  else data_page(false);
}

struct AtGen {
  std::vector<AtChunk> ch;
  pqg_alltypes_info info;
};

}  // namespace

extern "C" {

void* pqg_gen_alltypes(uint64_t rows, uint64_t row0, double p_null, uint64_t seed, int threads,
                       pqg_alltypes_info* info) {
  if (!info) return nullptr;
  AtGen* g = new AtGen();
  g->ch.resize(AT_NCOL);
  parallel_pages(AT_NCOL, threads, [&](uint32_t j) { at_write_chunk(rows, row0, p_null, seed, j, g->ch[j]); });
  pqg_alltypes_info& in = g->info;
  memset(&in, 0, sizeof(in));
  uint64_t off = 0;
  uint32_t np = 0;
  for (int j = 0; j < AT_NCOL; ++j) {
    in.chunk_first[j] = np;
    in.chunk_offset[j] = off;
    np += (uint32_t)g->ch[j].pages.size();
    off = align64(off + g->ch[j].buf.size());
    in.num_values[j] = g->ch[j].values;
    in.value_bytes[j] = g->ch[j].value_bytes;
  }
  in.chunk_first[AT_NCOL] = np;
  in.chunk_offset[AT_NCOL] = off;
  in.npages = np;
  in.blob_len = off;
  in.rows = rows;
  *info = in;
  return g;
}

int pqg_alltypes_copy(void* h, uint8_t* blob, uint64_t cap, pqg_page* pages, uint32_t pages_cap) {
  const AtGen* g = (const AtGen*)h;
  if (!g || cap < g->info.blob_len || pages_cap < g->info.npages) return PQG_ERR_CAPACITY;
  for (int j = 0; j < AT_NCOL; ++j) {
    const AtChunk& c = g->ch[j];
    memcpy(blob + g->info.chunk_offset[j], c.buf.data(), c.buf.size());
    for (size_t i = 0; i < c.pages.size(); ++i) {
      pqg_page p = c.pages[i];
      p.offset += g->info.chunk_offset[j];
      pages[g->info.chunk_first[j] + i] = p;
    }
  }
  return PQG_OK;
}

void pqg_alltypes_free(void* h) { delete (AtGen*)h; }

uint64_t pqg_truth_alltypes(uint64_t row0, uint64_t rows, int col, double p_null, uint64_t seed,
                            int16_t* levels, uint8_t* values, int64_t* offsets) {
  AtCell c;
  uint64_t nv = 0, nb = 0;
  if (offsets) offsets[0] = 0;
  for (uint64_t r = 0; r < rows; ++r) {
    at_cell(seed, p_null, (uint32_t)col, row0 + r, c);
    if (levels) levels[r] = c.null ? 0 : 1;
    if (c.null) continue;
    if (values) memcpy(values + nb, c.v, c.len);
    nb += c.len;
    ++nv;
    if (offsets) offsets[nv] = (int64_t)nb;
  }
  return nv;
}

}  // extern "C"
