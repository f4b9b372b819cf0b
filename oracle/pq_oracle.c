/*
 * pq_oracle.c — CPU restatement of the parquet-rs 0.4.2 decode path (TEST INFRASTRUCTURE;
 * see pq_oracle.h). Each function names the reference lines it restates.
 */
#include "pq_oracle.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ====================================================================== helpers */

/* bit_util.rs:81-88 */
int64_t or_ceil(int64_t value, int64_t divisor) {
  int64_t r = value / divisor;
  if (value % divisor != 0) r += 1;
  return r;
}

/* bit_util.rs:91-104 (ceil(log2(x)); log2(1) = 0) */
int or_log2(uint64_t x) {
  if (x == 1) return 0;
  x -= 1;
  int r = 0;
  while (x > 0) {
    x >>= 1;
    r++;
  }
  return r;
}

/* bit_util.rs:107-116 */
uint64_t or_trailing_bits(uint64_t v, size_t num_bits) {
  if (num_bits == 0) return 0;
  if (num_bits >= 64) return v;
  size_t n = 64 - num_bits;
  return (v << n) >> n;
}

/* bit_util.rs:125-132 */
size_t or_num_required_bits(uint64_t x) {
  for (int i = 63; i >= 0; --i)
    if (x & (1ULL << i)) return (size_t)i + 1;
  return 0;
}

/* read_num_bytes! (bit_util.rs:30-43): little-endian read of `size` bytes into a u64. */
static uint64_t read_le(const uint8_t *p, size_t size) {
  uint64_t v = 0;
  for (size_t i = 0; i < size && i < 8; ++i) v |= (uint64_t)p[i] << (8 * i);
  return v;
}

static void store_elem(void *dst, uint64_t v, int type_size) {
  /* transmute_copy::<u64, T>: the low type_size bytes of v (little-endian host). */
  memcpy(dst, &v, (size_t)type_size);
}

/* ====================================================================== BitReader */

/* BitReader::new / reset, bit_util.rs:395-417 */
void or_br_init(or_bit_reader *r, const uint8_t *buf, size_t len) {
  r->buf = buf;
  r->total_bytes = len;
  size_t nb = len < 8 ? len : 8;
  r->buffered = read_le(buf, nb);
  r->byte_offset = 0;
  r->bit_offset = 0;
  r->status = OR_OK;
}

/* reload_buffer_values, bit_util.rs:599-607 */
static void br_reload(or_bit_reader *r) {
  size_t left = r->total_bytes - r->byte_offset;
  size_t n = left < 8 ? left : 8;
  r->buffered = read_le(r->buf + r->byte_offset, n);
}

/* get_byte_offset, bit_util.rs:421-424 */
size_t or_br_get_byte_offset(const or_bit_reader *r) {
  return r->byte_offset + (size_t)or_ceil((int64_t)r->bit_offset, 8);
}

/* get_value<T>, bit_util.rs:429-453 */
int or_br_get_value(or_bit_reader *r, int num_bits, int type_size, uint64_t *out) {
  if (num_bits > 64 || num_bits > type_size * 8) {
    r->status = OR_PANIC; /* assert!(num_bits <= 64 / size_of::<T>()*8) */
    return 0;
  }
  if (r->byte_offset * 8 + r->bit_offset + (size_t)num_bits > r->total_bytes * 8) return 0;
  uint64_t v = or_trailing_bits(r->buffered, r->bit_offset + (size_t)num_bits) >> r->bit_offset;
  r->bit_offset += (size_t)num_bits;
  if (r->bit_offset >= 64) {
    r->byte_offset += 8;
    r->bit_offset -= 64;
    br_reload(r);
    unsigned sh = (unsigned)(((size_t)num_bits - r->bit_offset) & 63); /* wrapping_shl */
    v |= or_trailing_bits(r->buffered, r->bit_offset) << sh;
  }
  uint64_t res = 0;
  memcpy(&res, &v, (size_t)type_size); /* transmute_copy::<u64, T> */
  *out = res;
  return 1;
}

/* unpack32 (bit_packing.rs:29-72 and the generated unpackN_32 bodies): LSB-first values
 * of num_bits out of num_bits little-endian u32 words. */
void or_unpack32(const uint8_t *in, uint32_t *out, int num_bits) {
  for (int i = 0; i < 32; ++i) {
    if (num_bits == 0) {
      out[i] = 0;
      continue;
    }
    size_t bit = (size_t)i * (size_t)num_bits;
    uint64_t w = read_le(in + bit / 8, (bit % 8 + (size_t)num_bits + 7) / 8);
    w >>= bit % 8;
    out[i] = (uint32_t)(num_bits == 32 ? w : (w & ((1ULL << num_bits) - 1)));
  }
}

/* get_batch<T>, bit_util.rs:456-528 (structure kept so that the 8-byte-T quirk of
 * :498-503 is reproduced: through unpack32 only the low 4 bytes are written). */
size_t or_br_get_batch(or_bit_reader *r, void *batch, size_t n, int type_size, int num_bits) {
  uint8_t *b = (uint8_t *)batch;
  if (num_bits > 32 || num_bits > type_size * 8) {
    r->status = OR_PANIC;
    return 0;
  }
  size_t values_to_read = n;
  size_t needed_bits = (size_t)num_bits * values_to_read;
  size_t remaining_bits = (r->total_bytes - r->byte_offset) * 8 - r->bit_offset;
  if (remaining_bits < needed_bits) values_to_read = remaining_bits / (size_t)num_bits;
  size_t i = 0;
  uint64_t v;
  if (r->bit_offset != 0) {
    while (i < values_to_read && r->bit_offset != 0) {
      if (!or_br_get_value(r, num_bits, type_size, &v)) {
        r->status = OR_PANIC; /* expect("expected to have more data") */
        return i;
      }
      store_elem(b + i * (size_t)type_size, v, type_size);
      i++;
    }
  }
  while (values_to_read - i >= 32) {
    uint32_t tmp[32];
    or_unpack32(r->buf + r->byte_offset, tmp, num_bits);
    r->byte_offset += 4 * (size_t)num_bits;
    for (int k = 0; k < 32; ++k) {
      size_t cp = type_size > 4 ? 4 : (size_t)type_size;
      memcpy(b + (i + (size_t)k) * (size_t)type_size, &tmp[k], cp);
    }
    i += 32;
  }
  br_reload(r);
  while (i < values_to_read) {
    if (!or_br_get_value(r, num_bits, type_size, &v)) {
      r->status = OR_PANIC;
      return i;
    }
    store_elem(b + i * (size_t)type_size, v, type_size);
    i++;
  }
  return values_to_read;
}

/* get_aligned<T>, bit_util.rs:538-557 */
int or_br_get_aligned(or_bit_reader *r, size_t num_bytes, uint64_t *out) {
  size_t bytes_read = (size_t)or_ceil((int64_t)r->bit_offset, 8);
  if (r->byte_offset + bytes_read + num_bytes > r->total_bytes) return 0;
  if (num_bytes > 8) {
    r->status = OR_PANIC; /* copies more bytes than T holds: memory-unsafe in the reference */
    return 0;
  }
  r->byte_offset += bytes_read;
  *out = read_le(r->buf + r->byte_offset, num_bytes);
  r->byte_offset += num_bytes;
  r->bit_offset = 0;
  br_reload(r);
  return 1;
}

/* get_vlq_int, bit_util.rs:564-580 (asserts at most MAX_VLQ_BYTE_LEN = 10 bytes) */
int or_br_get_vlq_int(or_bit_reader *r, int64_t *out) {
  unsigned shift = 0;
  uint64_t v = 0;
  uint64_t byte;
  while (or_br_get_aligned(r, 1, &byte)) {
    if (shift >= 64) {
      r->status = OR_PANIC;
      return 0;
    }
    v |= (byte & 0x7F) << shift;
    shift += 7;
    if (shift > 70) {
      r->status = OR_PANIC;
      return 0;
    }
    if ((byte & 0x80) == 0) {
      *out = (int64_t)v;
      return 1;
    }
  }
  return 0;
}

/* get_zigzag_vlq_int, bit_util.rs:592-597 */
int or_br_get_zigzag_vlq_int(or_bit_reader *r, int64_t *out) {
  int64_t v;
  if (!or_br_get_vlq_int(r, &v)) return 0;
  uint64_t u = (uint64_t)v;
  *out = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
  return 1;
}

/* ====================================================================== RleDecoder */

void or_rle_init(or_rle_decoder *d, int bit_width) {
  memset(d, 0, sizeof(*d));
  d->bit_width = bit_width;
}

/* reload, rle.rs:490-508 */
static int rle_reload(or_rle_decoder *d) {
  int64_t ind;
  if (!or_br_get_vlq_int(&d->br, &ind)) {
    if (d->br.status) d->status = d->br.status;
    return 0;
  }
  if (ind & 1) {
    d->bit_packed_left = (uint32_t)((uint64_t)(ind >> 1) * 8u); /* ((ind >> 1) * 8) as u32 */
  } else {
    d->rle_left = (uint32_t)(ind >> 1);
    size_t value_width = (size_t)or_ceil(d->bit_width, 8);
    uint64_t cv = 0;
    if (!or_br_get_aligned(&d->br, value_width, &cv)) {
      d->status = OR_PANIC; /* assert!(self.current_value.is_some()) */
      d->has_current = 0;
      return 0;
    }
    d->current_value = cv;
    d->has_current = 1;
  }
  return 1;
}

/* set_data, rle.rs:352-361 */
void or_rle_set_data(or_rle_decoder *d, const uint8_t *data, size_t len) {
  or_br_init(&d->br, data, len);
  d->has_reader = 1;
  (void)rle_reload(d);
}

/* get<T>, rle.rs:364-395 */
int or_rle_get(or_rle_decoder *d, int type_size, uint64_t *out, int *has_value) {
  *has_value = 0;
  while (d->rle_left == 0 && d->bit_packed_left == 0) {
    if (!rle_reload(d)) return d->status;
  }
  if (d->rle_left > 0) {
    uint64_t v = 0;
    memcpy(&v, &d->current_value, (size_t)type_size);
    *out = v;
    d->rle_left -= 1;
  } else {
    if (!or_br_get_value(&d->br, d->bit_width, type_size, out)) {
      if (d->br.status) return d->br.status;
      return OR_EOF; /* eof_err!("Not enough data for 'bit_packed_value'") */
    }
    d->bit_packed_left -= 1;
  }
  *has_value = 1;
  return OR_OK;
}

/* get_batch<T>, rle.rs:398-434 */
int or_rle_get_batch(or_rle_decoder *d, void *buf, size_t n, int type_size, size_t *values_read) {
  uint8_t *b = (uint8_t *)buf;
  size_t read = 0;
  *values_read = 0;
  if (!d->has_reader) return OR_PANIC;
  while (read < n) {
    if (d->status) break;
    if (d->rle_left > 0) {
      size_t num = n - read;
      if (num > d->rle_left) num = d->rle_left;
      for (size_t i = 0; i < num; ++i) store_elem(b + (read + i) * (size_t)type_size, d->current_value, type_size);
      d->rle_left -= (uint32_t)num;
      read += num;
    } else if (d->bit_packed_left > 0) {
      size_t num = n - read;
      if (num > d->bit_packed_left) num = d->bit_packed_left;
      num = or_br_get_batch(&d->br, b + read * (size_t)type_size, num, type_size, d->bit_width);
      if (d->br.status) {
        d->status = d->br.status;
        break;
      }
      if (num == 0) {
        d->status = OR_HANG; /* rle.rs:414-425 would spin forever */
        break;
      }
      d->bit_packed_left -= (uint32_t)num;
      read += num;
    } else {
      if (!rle_reload(d)) break;
    }
  }
  *values_read = read;
  return d->status;
}

/* get_batch_with_dict<T>, rle.rs:437-487, including the 1024-index re-loop quirk
 * (:466-477). */
int or_rle_get_batch_with_dict(or_rle_decoder *d, const void *dict, size_t dict_len,
                               size_t elem_size, void *buf, size_t buf_len, size_t max_values,
                               size_t *values_read) {
  const uint8_t *dt = (const uint8_t *)dict;
  uint8_t *b = (uint8_t *)buf;
  size_t read = 0;
  *values_read = 0;
  if (buf_len < max_values) return OR_PANIC; /* assert!(buffer.len() >= max_values) */
  if (!d->has_reader) return OR_PANIC;
  while (read < max_values) {
    if (d->status) break;
    if (d->rle_left > 0) {
      size_t num = max_values - read;
      if (num > d->rle_left) num = d->rle_left;
      uint64_t idx = d->current_value;
      if (num > 0 && idx >= dict_len) {
        d->status = OR_PANIC; /* dict[dict_idx] out of bounds */
        break;
      }
      for (size_t i = 0; i < num; ++i) memcpy(b + (read + i) * elem_size, dt + idx * elem_size, elem_size);
      d->rle_left -= (uint32_t)num;
      read += num;
    } else if (d->bit_packed_left > 0) {
      size_t num = max_values - read;
      if (num > d->bit_packed_left) num = d->bit_packed_left;
      int32_t index_buf[1024];
      if (num > 1024) num = 1024;
      for (;;) {
        num = or_br_get_batch(&d->br, index_buf, num, 4, d->bit_width);
        if (d->br.status) {
          d->status = d->br.status;
          break;
        }
        for (size_t i = 0; i < num; ++i) {
          size_t idx = (size_t)(int64_t)index_buf[i]; /* index_buf[i] as usize */
          if (read + i >= buf_len || idx >= dict_len) {
            d->status = OR_PANIC;
            break;
          }
          memcpy(b + (read + i) * elem_size, dt + idx * elem_size, elem_size);
        }
        if (d->status) break;
        if (num > d->bit_packed_left) {
          d->status = OR_PANIC; /* u32 subtraction overflow */
          break;
        }
        d->bit_packed_left -= (uint32_t)num;
        read += num;
        if (num < 1024) break;
      }
      if (d->status) break;
      if (num == 0) {
        d->status = OR_HANG;
        break;
      }
    } else {
      if (!rle_reload(d)) break;
    }
  }
  *values_read = read;
  return d->status;
}

int or_rle_decode(const uint8_t *data, size_t len, int bit_width, int type_size, void *out,
                  size_t n, size_t *values_read) {
  or_rle_decoder d;
  or_rle_init(&d, bit_width);
  or_rle_set_data(&d, data, len);
  return or_rle_get_batch(&d, out, n, type_size, values_read);
}

int or_rle_decode_dict(const uint8_t *data, size_t len, int bit_width, const void *dict,
                       size_t dict_len, size_t elem_size, void *out, size_t n,
                       size_t *values_read) {
  or_rle_decoder d;
  or_rle_init(&d, bit_width);
  or_rle_set_data(&d, data, len);
  return or_rle_get_batch_with_dict(&d, dict, dict_len, elem_size, out, n, n, values_read);
}

/* ====================================================================== LevelDecoder */

/* LevelDecoder::v1 / v2, levels.rs:162-180 */
void or_level_init_v1(or_level_decoder *d, int encoding, int16_t max_level) {
  memset(d, 0, sizeof(*d));
  d->bit_width = or_log2((uint64_t)(int64_t)max_level + 1);
  if (encoding == OR_ENC_RLE) {
    d->kind = 0;
    or_rle_init(&d->rle, d->bit_width);
  } else if (encoding == OR_ENC_BIT_PACKED) {
    d->kind = 2;
    or_br_init(&d->br, (const uint8_t *)"", 0);
  } else {
    d->status = OR_PANIC; /* panic!("Unsupported encoding type") */
  }
}

void or_level_init_v2(or_level_decoder *d, int16_t max_level) {
  memset(d, 0, sizeof(*d));
  d->kind = 1;
  d->bit_width = or_log2((uint64_t)(int64_t)max_level + 1);
  or_rle_init(&d->rle, d->bit_width);
}

/* set_data, levels.rs:191-211. The slice handed over is page[start .. len). */
size_t or_level_set_data(or_level_decoder *d, size_t num_buffered_values, const uint8_t *page,
                         size_t start, size_t len) {
  if (d->status) return 0;
  size_t slice_len = len - start;
  const uint8_t *data = page + start;
  if (d->kind == 0) {
    d->num_values = num_buffered_values;
    d->has_num_values = 1;
    if (slice_len < 4) {
      d->status = OR_PANIC; /* read_num_bytes! assert */
      return 0;
    }
    int32_t sz = (int32_t)read_le(data, 4);
    size_t data_size = (size_t)(int64_t)sz;
    if (sz < 0 || 4 + data_size > slice_len) {
      d->status = OR_PANIC; /* data.range(i32_size, data_size) assert */
      return 0;
    }
    or_rle_set_data(&d->rle, data + 4, data_size);
    return 4 + data_size;
  } else if (d->kind == 2) {
    d->num_values = num_buffered_values;
    d->has_num_values = 1;
    size_t num_bytes = (size_t)or_ceil((int64_t)(num_buffered_values * (size_t)d->bit_width), 8);
    size_t data_size = num_bytes < slice_len ? num_bytes : slice_len;
    /* data.range(data.start(), data_size): relative to the slice again (quirk A.5) */
    if (start + data_size > slice_len) {
      d->status = OR_PANIC;
      return 0;
    }
    or_br_init(&d->br, data + start, data_size);
    return data_size;
  }
  d->status = OR_PANIC;
  return 0;
}

/* set_data_range, levels.rs:217-233 */
size_t or_level_set_data_range(or_level_decoder *d, size_t num_buffered_values,
                               const uint8_t *buf, size_t buf_len, size_t start, size_t len) {
  if (d->kind != 1) {
    d->status = OR_PANIC;
    return 0;
  }
  if (start + len > buf_len) {
    d->status = OR_PANIC;
    return 0;
  }
  or_rle_set_data(&d->rle, buf + start, len);
  d->num_values = num_buffered_values;
  d->has_num_values = 1;
  return len;
}

/* get, levels.rs:249-271 */
int or_level_get(or_level_decoder *d, int16_t *buf, size_t n, size_t *values_read) {
  *values_read = 0;
  if (d->status) return d->status;
  if (!d->has_num_values) return OR_PANIC; /* "No data set for decoding" */
  size_t len = d->num_values < n ? d->num_values : n;
  size_t read = 0;
  int st;
  if (d->kind == 2) {
    read = or_br_get_batch(&d->br, buf, len, 2, d->bit_width);
    st = d->br.status;
  } else {
    st = or_rle_get_batch(&d->rle, buf, len, 2, &read);
  }
  d->num_values -= read;
  *values_read = read;
  if (st) d->status = st;
  return st;
}

/* ====================================================================== value decoders */

size_t or_type_size(int t) {
  switch (t) {
    case OR_BOOLEAN: return 1;
    case OR_INT32: return 4;
    case OR_INT64: return 8;
    case OR_INT96: return 12;
    case OR_FLOAT: return 4;
    case OR_DOUBLE: return 8;
    default: return sizeof(or_ba);
  }
}

typedef struct or_value_decoder {
  int kind; /* encoding id */
  int physical_type;
  int32_t type_length;
  /* PLAIN (decoding.rs:88-247) */
  const uint8_t *data;
  size_t len;
  size_t start;
  size_t num_values;
  or_bit_reader br;
  /* DICT (decoding.rs:256-315) */
  uint8_t *dictionary;
  size_t dict_len;
  int has_dictionary;
  or_rle_decoder rle;
  int has_rle;
  /* DELTA_BINARY_PACKED (decoding.rs:392-619) */
  int initialized;
  int64_t num_mini_blocks;
  size_t values_per_mini_block;
  size_t values_current_mini_block;
  int64_t first_value;
  int first_value_read;
  int64_t min_delta;
  size_t mini_block_idx;
  uint8_t *delta_bit_widths;
  size_t n_widths;
  uint8_t delta_bit_width;
  int64_t *deltas;
  size_t n_deltas;
  size_t cap_deltas;
  int64_t current_value;
  /* DELTA_LENGTH / DELTA_BYTE_ARRAY (decoding.rs:629-835) */
  int32_t *lengths;
  size_t n_lengths;
  size_t current_idx;
  size_t offset;
  int32_t *prefix_lengths;
  size_t n_prefix;
  struct or_value_decoder *suffix;
  uint8_t *previous;
  size_t previous_len;
  or_ba last_suffix;
  int has_last_suffix;
  /* arena for materialised DELTA_BYTE_ARRAY values */
  uint8_t **arena;
  size_t n_arena;
} or_value_decoder;

static void vd_free(or_value_decoder *d);

static void vd_init(or_value_decoder *d, int kind, int physical_type, int32_t type_length) {
  memset(d, 0, sizeof(*d));
  d->kind = kind;
  d->physical_type = physical_type;
  d->type_length = type_length;
}

/* ---- PLAIN */
static int plain_set_data(or_value_decoder *d, const uint8_t *data, size_t len, size_t nv) {
  d->num_values = nv;
  d->start = 0;
  d->data = data;
  d->len = len;
  if (d->physical_type == OR_BOOLEAN) or_br_init(&d->br, data, len); /* decoding.rs:189-193 */
  return OR_OK;
}

static int plain_get(or_value_decoder *d, void *out, size_t n, size_t *read) {
  *read = 0;
  uint8_t *o = (uint8_t *)out;
  size_t num = n < d->num_values ? n : d->num_values;
  switch (d->physical_type) {
    case OR_BOOLEAN: { /* decoding.rs:195-203: no clamp to num_values */
      size_t r = or_br_get_batch(&d->br, out, n, 1, 1);
      if (d->br.status) return d->br.status;
      if (r > d->num_values) return OR_PANIC; /* usize subtraction overflow */
      d->num_values -= r;
      *read = r;
      return OR_OK;
    }
    case OR_INT96: /* decoding.rs:158-186 */
    case OR_INT32:
    case OR_INT64:
    case OR_FLOAT:
    case OR_DOUBLE: { /* decoding.rs:138-156 */
      size_t sz = or_type_size(d->physical_type);
      size_t bytes = sz * num;
      if (d->len - d->start < bytes) return OR_EOF;
      memcpy(o, d->data + d->start, bytes);
      d->start += bytes;
      d->num_values -= num;
      *read = num;
      return OR_OK;
    }
    case OR_BYTE_ARRAY: { /* decoding.rs:206-226 */
      or_ba *ba = (or_ba *)out;
      for (size_t i = 0; i < num; ++i) {
        if (d->start + 4 > d->len) return OR_PANIC; /* read_num_bytes! assert */
        size_t l = (size_t)(uint32_t)read_le(d->data + d->start, 4);
        d->start += 4;
        if (d->len < d->start + l) return OR_EOF;
        ba[i].ptr = d->data + d->start;
        ba[i].len = l;
        d->start += l;
      }
      d->num_values -= num;
      *read = num;
      return OR_OK;
    }
    case OR_FIXED_LEN_BYTE_ARRAY: { /* decoding.rs:228-247 */
      if (d->type_length <= 0) return OR_PANIC;
      or_ba *ba = (or_ba *)out;
      size_t tl = (size_t)d->type_length;
      for (size_t i = 0; i < num; ++i) {
        if (d->len < d->start + tl) return OR_EOF;
        ba[i].ptr = d->data + d->start;
        ba[i].len = tl;
        d->start += tl;
      }
      d->num_values -= num;
      *read = num;
      return OR_OK;
    }
  }
  return OR_NYI;
}

/* ---- DELTA_BINARY_PACKED */
static int delta_set_data(or_value_decoder *d, const uint8_t *data, size_t len) {
  or_br_init(&d->br, data, len);
  d->initialized = 1;
  int64_t block_size, nmb, nv, fv;
  if (!or_br_get_vlq_int(&d->br, &block_size)) return d->br.status ? d->br.status : OR_EOF;
  if (!or_br_get_vlq_int(&d->br, &nmb)) return d->br.status ? d->br.status : OR_EOF;
  if (!or_br_get_vlq_int(&d->br, &nv)) return d->br.status ? d->br.status : OR_EOF;
  if (!or_br_get_zigzag_vlq_int(&d->br, &fv)) return d->br.status ? d->br.status : OR_EOF;
  d->num_mini_blocks = nmb;
  d->num_values = (size_t)nv;
  d->first_value = fv;
  d->first_value_read = 0;
  d->mini_block_idx = 0;
  d->n_widths = 0;
  d->values_current_mini_block = 0;
  if (nmb == 0) return OR_PANIC; /* division by zero */
  d->values_per_mini_block = (size_t)(block_size / nmb);
  if (d->values_per_mini_block % 8 != 0) return OR_PANIC; /* decoding.rs:529-530 */
  return OR_OK;
}

/* init_block, decoding.rs:448-468 */
static int delta_init_block(or_value_decoder *d) {
  if (!or_br_get_zigzag_vlq_int(&d->br, &d->min_delta)) return d->br.status ? d->br.status : OR_EOF;
  if (d->num_mini_blocks < 0) return OR_PANIC;
  free(d->delta_bit_widths);
  d->delta_bit_widths = (uint8_t *)malloc((size_t)d->num_mini_blocks + 1);
  d->n_widths = 0;
  for (int64_t i = 0; i < d->num_mini_blocks; ++i) {
    uint64_t w;
    if (!or_br_get_aligned(&d->br, 1, &w)) return d->br.status ? d->br.status : OR_EOF;
    d->delta_bit_widths[d->n_widths++] = (uint8_t)w;
  }
  d->mini_block_idx = 0;
  if (d->n_widths == 0) return OR_PANIC; /* delta_bit_widths.data()[0] */
  d->delta_bit_width = d->delta_bit_widths[0];
  d->values_current_mini_block = d->values_per_mini_block;
  return OR_OK;
}

/* load_deltas_in_mini_block, decoding.rs:472-495 */
static int delta_load_mini_block(or_value_decoder *d) {
  size_t n = d->values_current_mini_block;
  if (n > d->cap_deltas) {
    d->deltas = (int64_t *)realloc(d->deltas, n * sizeof(int64_t));
    d->cap_deltas = n;
  }
  d->n_deltas = 0;
  if (d->physical_type == OR_INT32) { /* use_batch: get_batch::<i32> */
    int32_t *tmp = (int32_t *)calloc(n ? n : 1, sizeof(int32_t));
    size_t loaded = or_br_get_batch(&d->br, tmp, n, 4, d->delta_bit_width);
    if (d->br.status) {
      free(tmp);
      return d->br.status;
    }
    if (loaded != n) {
      free(tmp);
      return OR_PANIC; /* assert!(loaded == self.values_current_mini_block) */
    }
    for (size_t i = 0; i < n; ++i) d->deltas[i] = (int64_t)tmp[i]; /* get_delta: as i64 */
    d->n_deltas = n;
    free(tmp);
  } else {
    for (size_t i = 0; i < n; ++i) {
      uint64_t v;
      if (!or_br_get_value(&d->br, d->delta_bit_width, 8, &v)) return d->br.status ? d->br.status : OR_EOF;
      d->deltas[d->n_deltas++] = (int64_t)v;
    }
  }
  return OR_OK;
}

/* get, decoding.rs:535-572 */
static int delta_get(or_value_decoder *d, void *out, size_t n, size_t *read) {
  *read = 0;
  if (!d->initialized) return OR_PANIC;
  size_t num = n < d->num_values ? n : d->num_values;
  for (size_t i = 0; i < num; ++i) {
    int64_t val;
    if (!d->first_value_read) {
      val = d->first_value;
      d->current_value = d->first_value;
      d->first_value_read = 1;
    } else {
      if (d->values_current_mini_block == 0) {
        d->mini_block_idx += 1;
        if (d->mini_block_idx < d->n_widths) {
          d->delta_bit_width = d->delta_bit_widths[d->mini_block_idx];
          d->values_current_mini_block = d->values_per_mini_block;
        } else {
          int st = delta_init_block(d);
          if (st) return st;
        }
        int st = delta_load_mini_block(d);
        if (st) return st;
      }
      int64_t delta = d->deltas[d->n_deltas - d->values_current_mini_block];
      uint64_t cv = (uint64_t)d->current_value + (uint64_t)d->min_delta; /* wrapping_add */
      cv += (uint64_t)delta;
      d->current_value = (int64_t)cv;
      val = d->current_value;
      d->values_current_mini_block -= 1;
    }
    if (d->physical_type == OR_INT32) {
      int32_t v32 = (int32_t)(uint32_t)(uint64_t)val;
      memcpy((uint8_t *)out + i * 4, &v32, 4);
    } else {
      memcpy((uint8_t *)out + i * 8, &val, 8);
    }
  }
  d->num_values -= num;
  *read = num;
  return OR_OK;
}

int or_delta_decode(int physical_type, const uint8_t *data, size_t len, void *out, size_t n,
                    size_t *read, size_t *offset_out, size_t *total_out) {
  or_value_decoder d;
  vd_init(&d, OR_ENC_DELTA_BINARY_PACKED, physical_type, -1);
  *read = 0;
  int st = delta_set_data(&d, data, len);
  if (total_out) *total_out = d.num_values;
  if (!st) st = delta_get(&d, out, n, read);
  if (offset_out) *offset_out = or_br_get_byte_offset(&d.br);
  vd_free(&d);
  return st;
}

/* ---- DELTA_LENGTH_BYTE_ARRAY, decoding.rs:682-712 */
static int dlba_set_data(or_value_decoder *d, const uint8_t *data, size_t len) {
  or_value_decoder ld;
  vd_init(&ld, OR_ENC_DELTA_BINARY_PACKED, OR_INT32, -1);
  int st = delta_set_data(&ld, data, len);
  if (st) {
    vd_free(&ld);
    return st;
  }
  size_t nl = ld.num_values;
  free(d->lengths);
  d->lengths = (int32_t *)calloc(nl ? nl : 1, sizeof(int32_t));
  size_t r;
  st = delta_get(&ld, d->lengths, nl, &r);
  size_t off = or_br_get_byte_offset(&ld.br);
  vd_free(&ld);
  if (st) return st;
  d->n_lengths = nl;
  if (off > len) return OR_PANIC; /* data.start_from(offset) assert */
  d->data = data + off;
  d->len = len - off;
  d->offset = 0;
  d->current_idx = 0;
  d->num_values = nl;
  return OR_OK;
}

static int dlba_get(or_value_decoder *d, or_ba *out, size_t n, size_t *read) {
  *read = 0;
  size_t num = n < d->num_values ? n : d->num_values;
  for (size_t i = 0; i < num; ++i) {
    int32_t l32 = d->lengths[d->current_idx];
    size_t l = (size_t)(int64_t)l32;
    if (l32 < 0 || d->offset + l > d->len) return OR_PANIC; /* data.range assert */
    out[i].ptr = d->data + d->offset;
    out[i].len = l;
    d->offset += l;
    d->current_idx += 1;
  }
  d->num_values -= num;
  *read = num;
  return OR_OK;
}

/* ---- DELTA_BYTE_ARRAY, decoding.rs:768-835 */
static int dba_set_data(or_value_decoder *d, const uint8_t *data, size_t len) {
  or_value_decoder pd;
  vd_init(&pd, OR_ENC_DELTA_BINARY_PACKED, OR_INT32, -1);
  int st = delta_set_data(&pd, data, len);
  if (st) {
    vd_free(&pd);
    return st;
  }
  size_t np = pd.num_values;
  free(d->prefix_lengths);
  d->prefix_lengths = (int32_t *)calloc(np ? np : 1, sizeof(int32_t));
  size_t r;
  st = delta_get(&pd, d->prefix_lengths, np, &r);
  size_t off = or_br_get_byte_offset(&pd.br);
  vd_free(&pd);
  if (st) return st;
  d->n_prefix = np;
  if (off > len) return OR_PANIC;
  if (d->suffix) {
    vd_free(d->suffix);
    free(d->suffix);
  }
  d->suffix = (struct or_value_decoder *)calloc(1, sizeof(or_value_decoder));
  vd_init((or_value_decoder *)d->suffix, OR_ENC_DELTA_LENGTH_BYTE_ARRAY, OR_BYTE_ARRAY, -1);
  st = dlba_set_data((or_value_decoder *)d->suffix, data + off, len - off);
  if (st) return st;
  d->num_values = np;
  d->current_idx = 0;
  d->previous_len = 0;
  d->has_last_suffix = 0;
  return OR_OK;
}

static int dba_get(or_value_decoder *d, or_ba *out, size_t n, size_t *read) {
  *read = 0;
  size_t num = n < d->num_values ? n : d->num_values;
  for (size_t i = 0; i < num; ++i) {
    or_ba v;
    size_t r;
    int st = dlba_get((or_value_decoder *)d->suffix, &v, 1, &r);
    if (st) return st;
    if (r == 1) {
      d->last_suffix = v;
      d->has_last_suffix = 1;
    } else if (!d->has_last_suffix) {
      return OR_PANIC; /* ByteArray::data() on an unset value */
    }
    or_ba suffix = d->last_suffix; /* `v` keeps its old content when get() returned 0 */
    size_t pl = (size_t)(int64_t)d->prefix_lengths[d->current_idx];
    if (d->prefix_lengths[d->current_idx] < 0 || pl > d->previous_len) return OR_PANIC;
    size_t tot = pl + suffix.len;
    uint8_t *res = (uint8_t *)malloc(tot ? tot : 1);
    memcpy(res, d->previous, pl);
    memcpy(res + pl, suffix.ptr, suffix.len);
    d->arena = (uint8_t **)realloc(d->arena, (d->n_arena + 1) * sizeof(uint8_t *));
    d->arena[d->n_arena++] = res;
    out[i].ptr = res;
    out[i].len = tot;
    d->previous = res;
    d->previous_len = tot;
    d->current_idx += 1;
  }
  d->num_values -= num;
  *read = num;
  return OR_OK;
}

/* ---- dictionary, decoding.rs:256-315 */
static int dict_set_data(or_value_decoder *d, const uint8_t *data, size_t len, size_t nv) {
  if (len < 1) return OR_PANIC; /* data.as_ref()[0] */
  int bw = data[0];
  or_rle_init(&d->rle, bw);
  or_rle_set_data(&d->rle, data + 1, len - 1);
  d->has_rle = 1;
  d->num_values = nv;
  return OR_OK;
}

static int dict_get(or_value_decoder *d, void *out, size_t n, size_t *read) {
  *read = 0;
  if (!d->has_rle) return OR_PANIC;
  if (!d->has_dictionary) return OR_PANIC; /* "Must call set_dict() first!" */
  size_t num = n < d->num_values ? n : d->num_values;
  return or_rle_get_batch_with_dict(&d->rle, d->dictionary, d->dict_len,
                                    or_type_size(d->physical_type), out, n, num, read);
}

/* ---- RLE booleans, decoding.rs:323-384 */
static int rlebool_set_data(or_value_decoder *d, const uint8_t *data, size_t len, size_t nv) {
  if (d->physical_type != OR_BOOLEAN) return OR_PANIC; /* "only supports BoolType" */
  if (len < 4) return OR_PANIC;
  int32_t sz = (int32_t)read_le(data, 4);
  if (sz < 0 || 4 + (size_t)sz > len) return OR_PANIC;
  or_rle_init(&d->rle, 1);
  or_rle_set_data(&d->rle, data + 4, (size_t)sz);
  d->has_rle = 1;
  d->num_values = nv;
  return OR_OK;
}

static int rlebool_get(or_value_decoder *d, void *out, size_t n, size_t *read) {
  size_t r;
  int st = or_rle_get_batch(&d->rle, out, n, 1, &r);
  *read = r;
  if (st) return st;
  if (r > d->num_values) return OR_PANIC;
  d->num_values -= r;
  return OR_OK;
}

static void vd_free(or_value_decoder *d) {
  free(d->delta_bit_widths);
  free(d->deltas);
  free(d->lengths);
  free(d->prefix_lengths);
  if (d->suffix) {
    vd_free((or_value_decoder *)d->suffix);
    free(d->suffix);
  }
  for (size_t i = 0; i < d->n_arena; ++i) free(d->arena[i]);
  free(d->arena);
  free(d->dictionary);
  memset(d, 0, sizeof(*d));
}

/* Decoder::set_data dispatch (get_decoder, decoding.rs:60-79) */
static int vd_set_data(or_value_decoder *d, const uint8_t *data, size_t len, size_t nv) {
  switch (d->kind) {
    case OR_ENC_PLAIN: return plain_set_data(d, data, len, nv);
    case OR_ENC_RLE_DICTIONARY: return dict_set_data(d, data, len, nv);
    case OR_ENC_RLE: return rlebool_set_data(d, data, len, nv);
    case OR_ENC_DELTA_BINARY_PACKED:
      if (d->physical_type != OR_INT32 && d->physical_type != OR_INT64) return OR_PANIC;
      return delta_set_data(d, data, len);
    case OR_ENC_DELTA_LENGTH_BYTE_ARRAY:
      if (d->physical_type != OR_BYTE_ARRAY) return OR_GENERAL;
      return dlba_set_data(d, data, len);
    case OR_ENC_DELTA_BYTE_ARRAY:
      if (d->physical_type != OR_BYTE_ARRAY && d->physical_type != OR_FIXED_LEN_BYTE_ARRAY)
        return OR_GENERAL;
      return dba_set_data(d, data, len);
  }
  return OR_NYI;
}

static int vd_get(or_value_decoder *d, void *out, size_t n, size_t *read) {
  switch (d->kind) {
    case OR_ENC_PLAIN: return plain_get(d, out, n, read);
    case OR_ENC_RLE_DICTIONARY: return dict_get(d, out, n, read);
    case OR_ENC_RLE: return rlebool_get(d, out, n, read);
    case OR_ENC_DELTA_BINARY_PACKED: return delta_get(d, out, n, read);
    case OR_ENC_DELTA_LENGTH_BYTE_ARRAY: return dlba_get(d, (or_ba *)out, n, read);
    case OR_ENC_DELTA_BYTE_ARRAY: return dba_get(d, (or_ba *)out, n, read);
  }
  *read = 0;
  return OR_NYI;
}

int or_plain_decode(int physical_type, int32_t type_length, const uint8_t *data, size_t len,
                    size_t num_values, void *out, size_t n, size_t *read) {
  or_value_decoder d;
  vd_init(&d, OR_ENC_PLAIN, physical_type, type_length);
  plain_set_data(&d, data, len, num_values);
  int st = plain_get(&d, out, n, read);
  vd_free(&d);
  return st;
}

/* ====================================================================== column reader */

/* ColumnReaderImpl state, column/reader.rs:106-489 */
#define OR_MAX_ENC 16
typedef struct {
  const or_column *col;
  const or_page *pages;
  size_t npages;
  size_t next_page;
  or_level_decoder def, rep;
  int has_def, has_rep;
  int current_encoding;
  uint32_t num_buffered_values;
  uint32_t num_decoded_values;
  or_value_decoder *decoders[OR_MAX_ENC];
  char *msg;
} or_col_reader;

static int set_msg(or_col_reader *r, int st, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(r->msg, 256, fmt, ap);
  va_end(ap);
  return st;
}

/* configure_dictionary, column/reader.rs:463-488 */
static int configure_dictionary(or_col_reader *r, const or_page *p) {
  int enc = p->encoding;
  if (enc == OR_ENC_PLAIN || enc == OR_ENC_PLAIN_DICTIONARY) enc = OR_ENC_RLE_DICTIONARY;
  if (enc >= 0 && enc < OR_MAX_ENC && r->decoders[enc])
    return set_msg(r, OR_GENERAL, "Column cannot have more than one dictionary");
  if (enc != OR_ENC_RLE_DICTIONARY)
    return set_msg(r, OR_NYI, "Invalid/Unsupported encoding type for dictionary: %d", p->encoding);
  or_value_decoder *dd = (or_value_decoder *)calloc(1, sizeof(or_value_decoder));
  vd_init(dd, OR_ENC_RLE_DICTIONARY, r->col->physical_type, r->col->type_length);
  or_value_decoder pd;
  vd_init(&pd, OR_ENC_PLAIN, r->col->physical_type, r->col->type_length);
  plain_set_data(&pd, p->buf, p->len, p->num_values);
  size_t es = or_type_size(r->col->physical_type);
  dd->dictionary = (uint8_t *)calloc(p->num_values ? p->num_values : 1, es);
  size_t got;
  int st = plain_get(&pd, dd->dictionary, p->num_values, &got); /* set_dict, decoding.rs:282-288 */
  vd_free(&pd);
  dd->dict_len = p->num_values;
  dd->has_dictionary = 1;
  r->decoders[OR_ENC_RLE_DICTIONARY] = dd;
  if (st) return set_msg(r, st, "dictionary decode failed");
  return OR_OK;
}

/* set_current_page_encoding, column/reader.rs:383-413 */
static int set_current_page_encoding(or_col_reader *r, int enc, const uint8_t *buf, size_t len,
                                     size_t nv) {
  if (enc == OR_ENC_PLAIN_DICTIONARY) enc = OR_ENC_RLE_DICTIONARY;
  if (enc < 0 || enc >= OR_MAX_ENC) return set_msg(r, OR_NYI, "Encoding %d is not supported", enc);
  if (enc == OR_ENC_RLE_DICTIONARY) {
    if (!r->decoders[enc]) return set_msg(r, OR_PANIC, "Decoder for dict should have been set");
  } else if (!r->decoders[enc]) {
    if (enc != OR_ENC_PLAIN && enc != OR_ENC_RLE && enc != OR_ENC_DELTA_BINARY_PACKED &&
        enc != OR_ENC_DELTA_LENGTH_BYTE_ARRAY && enc != OR_ENC_DELTA_BYTE_ARRAY)
      return set_msg(r, OR_NYI, "Encoding %d is not supported", enc);
    or_value_decoder *vd = (or_value_decoder *)calloc(1, sizeof(or_value_decoder));
    vd_init(vd, enc, r->col->physical_type, r->col->type_length);
    r->decoders[enc] = vd;
  }
  int st = vd_set_data(r->decoders[enc], buf, len, nv);
  if (st) return set_msg(r, st, "set_data failed for encoding %d", enc);
  r->current_encoding = enc;
  return OR_OK;
}

/* read_new_page, column/reader.rs:269-380. Returns 1 page read, 0 none left, <0 error. */
static int read_new_page(or_col_reader *r, int *st) {
  *st = OR_OK;
  while (r->next_page < r->npages) {
    const or_page *p = &r->pages[r->next_page++];
    if (p->page_type == OR_PAGE_DICTIONARY) {
      *st = configure_dictionary(r, p);
      if (*st) return -1;
      continue;
    }
    if (p->page_type == OR_PAGE_DATA) {
      r->num_buffered_values = p->num_values;
      r->num_decoded_values = 0;
      size_t start = 0; /* buffer_ptr.start() within the page */
      if (r->col->max_rep > 0) {
        or_level_init_v1(&r->rep, p->rep_encoding, r->col->max_rep);
        size_t tb = or_level_set_data(&r->rep, p->num_values, p->buf, start, p->len);
        if (r->rep.status) {
          *st = set_msg(r, r->rep.status, "rep level set_data failed");
          return -1;
        }
        start += tb;
        r->has_rep = 1;
      }
      if (r->col->max_def > 0) {
        or_level_init_v1(&r->def, p->def_encoding, r->col->max_def);
        size_t tb = or_level_set_data(&r->def, p->num_values, p->buf, start, p->len);
        if (r->def.status) {
          *st = set_msg(r, r->def.status, "def level set_data failed");
          return -1;
        }
        start += tb;
        r->has_def = 1;
      }
      *st = set_current_page_encoding(r, p->encoding, p->buf + start, p->len - start, p->num_values);
      if (*st) return -1;
      return 1;
    }
    if (p->page_type == OR_PAGE_DATA_V2) {
      r->num_buffered_values = p->num_values;
      r->num_decoded_values = 0;
      size_t off = 0;
      if (r->col->max_rep > 0) {
        or_level_init_v2(&r->rep, r->col->max_rep);
        off += or_level_set_data_range(&r->rep, p->num_values, p->buf, p->len, off, p->rep_len);
        if (r->rep.status) {
          *st = set_msg(r, r->rep.status, "rep level range failed");
          return -1;
        }
        r->has_rep = 1;
      }
      if (r->col->max_def > 0) {
        or_level_init_v2(&r->def, r->col->max_def);
        off += or_level_set_data_range(&r->def, p->num_values, p->buf, p->len, off, p->def_len);
        if (r->def.status) {
          *st = set_msg(r, r->def.status, "def level range failed");
          return -1;
        }
        r->has_def = 1;
      }
      if (off > p->len) {
        *st = set_msg(r, OR_PANIC, "start_from out of range");
        return -1;
      }
      *st = set_current_page_encoding(r, p->encoding, p->buf + off, p->len - off, p->num_values);
      if (*st) return -1;
      return 1;
    }
    /* other page types are skipped by the page reader (file/reader.rs:512-515) */
  }
  return 0;
}

/* has_next, column/reader.rs:416-430 */
static int has_next(or_col_reader *r, int *st) {
  *st = OR_OK;
  if (r->num_buffered_values == 0 || r->num_buffered_values == r->num_decoded_values) {
    int rv = read_new_page(r, st);
    if (rv < 0) return -1;
    if (rv == 0) return 0;
    return r->num_buffered_values != 0;
  }
  return 1;
}

typedef struct {
  uint8_t *p;
  size_t n, cap;
} vec_u8;

static void vpush(vec_u8 *v, const void *src, size_t n) {
  if (v->n + n > v->cap) {
    size_t c = v->cap ? v->cap : 256;
    while (c < v->n + n) c *= 2;
    v->p = (uint8_t *)realloc(v->p, c);
    v->cap = c;
  }
  if (n) memcpy(v->p + v->n, src, n);
  v->n += n;
}

/* read_batch, column/reader.rs:159-265, for a single call. def/rep/values are the caller's
 * slices of dcap / rcap / vcap elements (def_levels.len(), rep_levels.len(), values.len()). */
static int read_batch(or_col_reader *r, size_t batch_size, int16_t *def, size_t dcap, int16_t *rep,
                      size_t rcap, uint8_t *values, size_t vcap, size_t *values_read_out,
                      size_t *levels_read_out) {
  size_t values_read = 0, levels_read = 0;
  size_t es = or_type_size(r->col->physical_type);
  *values_read_out = *levels_read_out = 0;
  /* the smallest batch the slices allow (:170-177) */
  if (vcap < batch_size) batch_size = vcap;
  if (def && dcap < batch_size) batch_size = dcap;
  if (rep && rcap < batch_size) batch_size = rcap;
  while ((values_read > levels_read ? values_read : levels_read) < batch_size) {
    int st;
    int hn = has_next(r, &st);
    if (hn < 0) return st;
    if (hn == 0) break;
    /* iter_batch_size (:187-205) */
    size_t iter = batch_size;
    size_t left = (size_t)(r->num_buffered_values - r->num_decoded_values);
    if (left < iter) iter = left;
    if (vcap - values_read < iter) iter = vcap - values_read;
    if (def && dcap - levels_read < iter) iter = dcap - levels_read;
    if (rep && rcap - levels_read < iter) iter = rcap - levels_read;

    size_t values_to_read = 0, num_def = 0, num_rep = 0;
    if (r->col->max_def > 0 && def) {
      st = or_level_get(&r->def, def + levels_read, iter, &num_def);
      if (st) return set_msg(r, st, "def level decode failed");
      for (size_t i = levels_read; i < levels_read + num_def; ++i)
        if (def[i] == r->col->max_def) values_to_read++;
    } else {
      values_to_read = iter;
    }
    if (r->col->max_rep > 0 && rep) {
      st = or_level_get(&r->rep, rep + levels_read, iter, &num_rep);
      if (st) return set_msg(r, st, "rep level decode failed");
      if (def && num_def != num_rep) return set_msg(r, OR_PANIC, "Number of decoded rep / def levels did not match");
    }
    size_t cur_values = 0;
    or_value_decoder *vd = r->decoders[r->current_encoding];
    st = vd_get(vd, values + values_read * es, values_to_read, &cur_values);
    if (st) return set_msg(r, st, "value decode failed (encoding %d)", r->current_encoding);
    size_t cur_levels = num_def > num_rep ? num_def : num_rep;
    size_t adv = cur_levels > cur_values ? cur_levels : cur_values;
    if (adv == 0) return set_msg(r, OR_HANG, "no progress in read_batch (reference loops forever)");
    r->num_decoded_values += (uint32_t)adv;
    levels_read += cur_levels;
    values_read += cur_values;
  }
  *values_read_out = values_read;
  *levels_read_out = levels_read;
  return OR_OK;
}

int or_read_column_caps(const or_column *col, const or_page *pages, size_t npages,
                        size_t batch_size, size_t vcap, size_t dcap, size_t rcap, int want_def,
                        int want_rep, uint64_t *counts, size_t counts_cap, or_column_result *res) {
  memset(res, 0, sizeof(*res));
  or_col_reader r;
  memset(&r, 0, sizeof(r));
  r.col = col;
  r.pages = pages;
  r.npages = npages;
  r.msg = res->message;
  size_t es = or_type_size(col->physical_type);
  int isba = col->physical_type == OR_BYTE_ARRAY || col->physical_type == OR_FIXED_LEN_BYTE_ARRAY;
  if (batch_size == 0) batch_size = 1024;
  int16_t *def = want_def ? (int16_t *)malloc((dcap ? dcap : 1) * 2) : NULL;
  int16_t *rep = want_rep ? (int16_t *)malloc((rcap ? rcap : 1) * 2) : NULL;
  uint8_t *vals = (uint8_t *)malloc((vcap ? vcap : 1) * es);
  vec_u8 vdef = {0}, vrep = {0}, vval = {0}, voff = {0}, vbytes = {0};
  int64_t off0 = 0;
  if (isba) vpush(&voff, &off0, 8);
  int st = OR_OK;
  for (;;) {
    size_t vr = 0, lr = 0;
    st = read_batch(&r, batch_size, def, dcap, rep, rcap, vals, vcap, &vr, &lr);
    if (st) break;
    if (vr == 0 && lr == 0) break;
    if (counts && 2 * res->num_batches + 1 < counts_cap) {
      counts[2 * res->num_batches] = vr;
      counts[2 * res->num_batches + 1] = lr;
    }
    res->num_batches++;
    if (def) vpush(&vdef, def, lr * 2);
    if (rep) vpush(&vrep, rep, lr * 2);
    if (isba) {
      or_ba *ba = (or_ba *)vals;
      for (size_t i = 0; i < vr; ++i) {
        vpush(&vbytes, ba[i].ptr, ba[i].len);
        int64_t o = (int64_t)vbytes.n;
        vpush(&voff, &o, 8);
      }
    } else {
      vpush(&vval, vals, vr * es);
    }
    res->num_levels += lr;
    res->num_values += vr;
  }
  res->status = st;
  res->def_levels = (int16_t *)vdef.p;
  res->rep_levels = (int16_t *)vrep.p;
  res->values = vval.p;
  res->offsets = (int64_t *)voff.p;
  res->bytes = vbytes.p;
  res->num_bytes = vbytes.n;
  free(def);
  free(rep);
  free(vals);
  for (int i = 0; i < OR_MAX_ENC; ++i)
    if (r.decoders[i]) {
      vd_free(r.decoders[i]);
      free(r.decoders[i]);
    }
  return st;
}

int or_read_column(const or_column *col, const or_page *pages, size_t npages,
                   size_t batch_size, int want_def, int want_rep, or_column_result *res) {
  if (batch_size == 0) batch_size = 1024;
  return or_read_column_caps(col, pages, npages, batch_size, batch_size, batch_size, batch_size,
                             want_def, want_rep, NULL, 0, res);
}

void or_column_result_free(or_column_result *res) {
  free(res->def_levels);
  free(res->rep_levels);
  free(res->values);
  free(res->offsets);
  free(res->bytes);
  memset(res, 0, sizeof(*res));
}

/* ====================================================================== encoders */

/* BitWriter, bit_util.rs:136-363 */
typedef struct {
  uint8_t *buf;
  size_t max_bytes;
  uint64_t buffered;
  size_t byte_offset;
  size_t bit_offset;
  size_t start;
} or_bit_writer;

static void bw_init(or_bit_writer *w, uint8_t *buf, size_t cap, size_t start) {
  w->buf = buf;
  w->max_bytes = cap;
  w->buffered = 0;
  w->byte_offset = start;
  w->bit_offset = 0;
  w->start = start;
}

static int bw_flush(or_bit_writer *w) {
  size_t nb = (size_t)or_ceil((int64_t)w->bit_offset, 8);
  if (w->byte_offset + nb > w->max_bytes) return 0;
  memcpy(w->buf + w->byte_offset, &w->buffered, nb);
  w->buffered = 0;
  w->bit_offset = 0;
  w->byte_offset += nb;
  return 1;
}

static long bw_skip(or_bit_writer *w, size_t n) {
  if (!bw_flush(w)) return -1;
  if (w->byte_offset + n > w->max_bytes) return -1;
  long r = (long)w->byte_offset;
  w->byte_offset += n;
  return r;
}

static int bw_put_value(or_bit_writer *w, uint64_t v, size_t num_bits) {
  if (w->byte_offset * 8 + w->bit_offset + num_bits > w->max_bytes * 8) return 0;
  w->buffered |= (w->bit_offset < 64) ? (v << w->bit_offset) : 0;
  w->bit_offset += num_bits;
  if (w->bit_offset >= 64) {
    memcpy(w->buf + w->byte_offset, &w->buffered, 8);
    w->byte_offset += 8;
    w->bit_offset -= 64;
    size_t sh = num_bits - w->bit_offset;
    w->buffered = sh < 64 ? (v >> sh) : 0; /* checked_shr(..).unwrap_or(0) */
  }
  return 1;
}

static int bw_put_aligned(or_bit_writer *w, uint64_t v, size_t nbytes) {
  long off = bw_skip(w, nbytes);
  if (off < 0) return 0;
  memcpy(w->buf + off, &v, nbytes);
  return 1;
}

static int bw_put_vlq(or_bit_writer *w, uint64_t v) {
  int ok = 1;
  while (v & 0xFFFFFFFFFFFFFF80ULL) {
    ok &= bw_put_aligned(w, (v & 0x7F) | 0x80, 1);
    v >>= 7;
  }
  ok &= bw_put_aligned(w, v & 0x7F, 1);
  return ok;
}

static int bw_put_zigzag(or_bit_writer *w, int64_t v) {
  uint64_t u = ((uint64_t)v << 1) ^ (uint64_t)(v >> 63);
  return bw_put_vlq(w, u);
}


/* RleEncoder, rle.rs:55-317 */
typedef struct {
  int bit_width;
  or_bit_writer bw;
  int buffer_full;
  uint64_t buffered_values[8];
  size_t num_buffered;
  uint64_t current_value;
  size_t repeat_count;
  size_t bit_packed_count;
  long indicator_byte_pos;
  int err;
} or_rle_encoder;

static void rle_enc_init(or_rle_encoder *e, int bw, uint8_t *buf, size_t cap, size_t start) {
  memset(e, 0, sizeof(*e));
  e->bit_width = bw;
  bw_init(&e->bw, buf, cap, start);
  e->indicator_byte_pos = -1;
}

static void flush_rle_run(or_rle_encoder *e) {
  int ok = bw_put_vlq(&e->bw, (uint64_t)(e->repeat_count << 1));
  ok &= bw_put_aligned(&e->bw, e->current_value, (size_t)or_ceil(e->bit_width, 8));
  if (!ok) e->err = 1;
  e->num_buffered = 0;
  e->repeat_count = 0;
}

static void flush_bit_packed_run(or_rle_encoder *e, int update_indicator) {
  if (e->indicator_byte_pos < 0) {
    e->indicator_byte_pos = bw_skip(&e->bw, 1);
    if (e->indicator_byte_pos < 0) {
      e->err = 1;
      return;
    }
  }
  for (size_t i = 0; i < e->num_buffered; ++i) bw_put_value(&e->bw, e->buffered_values[i], (size_t)e->bit_width);
  e->num_buffered = 0;
  if (update_indicator) {
    size_t num_groups = e->bit_packed_count / 8;
    e->bw.buf[e->indicator_byte_pos] = (uint8_t)((num_groups << 1) | 1);
    e->indicator_byte_pos = -1;
    e->bit_packed_count = 0;
  }
}

static void flush_buffered_values(or_rle_encoder *e) {
  if (e->repeat_count >= 8) {
    e->num_buffered = 0;
    if (e->bit_packed_count > 0) flush_bit_packed_run(e, 1);
    return;
  }
  e->bit_packed_count += e->num_buffered;
  size_t num_groups = e->bit_packed_count / 8;
  if (num_groups + 1 >= 64) /* MAX_GROUPS_PER_BIT_PACKED_RUN */
    flush_bit_packed_run(e, 1);
  else
    flush_bit_packed_run(e, 0);
  e->repeat_count = 0;
}

static void rle_enc_put(or_rle_encoder *e, uint64_t value) {
  if (e->current_value == value) {
    e->repeat_count += 1;
    if (e->repeat_count > 8) return;
  } else {
    if (e->repeat_count >= 8) flush_rle_run(e);
    e->repeat_count = 1;
    e->current_value = value;
  }
  e->buffered_values[e->num_buffered++] = value;
  if (e->num_buffered == 8) flush_buffered_values(e);
}

static void rle_enc_flush(or_rle_encoder *e) {
  if (e->bit_packed_count > 0 || e->repeat_count > 0 || e->num_buffered > 0) {
    int all_repeat = e->bit_packed_count == 0 &&
                     (e->repeat_count == e->num_buffered || e->num_buffered == 0);
    if (e->repeat_count > 0 && all_repeat) {
      flush_rle_run(e);
    } else {
      if (e->num_buffered > 0)
        while (e->num_buffered < 8) e->buffered_values[e->num_buffered++] = 0;
      e->bit_packed_count += e->num_buffered;
      flush_bit_packed_run(e, 1);
      e->repeat_count = 0;
    }
  }
}

static size_t rle_enc_consume(or_rle_encoder *e) {
  rle_enc_flush(e);
  if (!bw_flush(&e->bw)) e->err = 1;
  return e->err ? (size_t)-1 : e->bw.byte_offset;
}

size_t or_rle_encode(const uint64_t *values, size_t n, int bit_width, uint8_t *out, size_t cap) {
  or_rle_encoder e;
  memset(out, 0, cap);
  rle_enc_init(&e, bit_width, out, cap, 0);
  for (size_t i = 0; i < n; ++i) rle_enc_put(&e, values[i]);
  return rle_enc_consume(&e);
}

/* LevelEncoder::v1 / v2 + put + consume, levels.rs:54-143 */
size_t or_level_encode(int encoding, int v2, int16_t max_level, const int16_t *levels,
                       size_t n, uint8_t *out, size_t cap) {
  int bw = or_log2((uint64_t)(int64_t)max_level + 1);
  memset(out, 0, cap);
  if (v2 || encoding == OR_ENC_RLE) {
    or_rle_encoder e;
    size_t start = v2 ? 0 : 4;
    if (cap < start) return (size_t)-1;
    rle_enc_init(&e, bw, out, cap, start);
    for (size_t i = 0; i < n; ++i) rle_enc_put(&e, (uint64_t)(int64_t)levels[i]);
    size_t end = rle_enc_consume(&e);
    if (end == (size_t)-1) return end;
    if (!v2) {
      int32_t len = (int32_t)(end - 4);
      memcpy(out, &len, 4);
    }
    return end;
  }
  if (encoding == OR_ENC_BIT_PACKED) {
    or_bit_writer w;
    bw_init(&w, out, cap, 0);
    for (size_t i = 0; i < n; ++i)
      if (!bw_put_value(&w, (uint64_t)(int64_t)levels[i], (size_t)bw)) return (size_t)-1;
    if (!bw_flush(&w)) return (size_t)-1;
    return w.byte_offset;
  }
  return (size_t)-1;
}

/* PlainEncoder, encoding.rs:94-181 (fixed-width types and BOOLEAN) */
size_t or_plain_encode(int t, const void *values, size_t n, uint8_t *out, size_t cap) {
  if (t == OR_BOOLEAN) {
    or_bit_writer w;
    memset(out, 0, cap);
    bw_init(&w, out, cap, 0);
    const uint8_t *b = (const uint8_t *)values;
    for (size_t i = 0; i < n; ++i)
      if (!bw_put_value(&w, b[i] ? 1 : 0, 1)) return (size_t)-1;
    if (!bw_flush(&w)) return (size_t)-1;
    return w.byte_offset;
  }
  size_t sz = or_type_size(t);
  if (sz * n > cap) return (size_t)-1;
  memcpy(out, values, sz * n);
  return sz * n;
}

size_t or_plain_encode_ba(const uint8_t *bytes, const int64_t *offsets, size_t n, int fixed,
                          uint8_t *out, size_t cap) {
  size_t o = 0;
  for (size_t i = 0; i < n; ++i) {
    uint32_t l = (uint32_t)(offsets[i + 1] - offsets[i]);
    if (!fixed) {
      if (o + 4 > cap) return (size_t)-1;
      memcpy(out + o, &l, 4);
      o += 4;
    }
    if (o + l > cap) return (size_t)-1;
    memcpy(out + o, bytes + offsets[i], l);
    o += l;
  }
  return o;
}

/* DeltaBitPackEncoder, encoding.rs:534-714 */
static int64_t delta_sub(int t, int64_t l, int64_t r) {
  if (t == OR_INT32) return (int64_t)(int32_t)((uint32_t)(int32_t)l - (uint32_t)(int32_t)r);
  return (int64_t)((uint64_t)l - (uint64_t)r);
}
static uint64_t delta_sub_u64(int t, int64_t l, int64_t r) {
  if (t == OR_INT32) return (uint64_t)(uint32_t)((uint32_t)(int32_t)l - (uint32_t)(int32_t)r);
  return (uint64_t)l - (uint64_t)r;
}

/* Block shape: the reference encoder always writes 128 / 4 x 32 (encoding.rs:508-509); the
 * decoder accepts any block with values_per_mini_block % 8 == 0 (decoding.rs:529-530), so the
 * generator also takes other shapes (BASELINE config 4: 512 / 4 x 128). */
size_t or_delta_encode_shape(int t, const void *values, size_t n, size_t block_size,
                             size_t num_mini_blocks, uint8_t *out, size_t cap) {
  if (block_size == 0 || num_mini_blocks == 0 || block_size % num_mini_blocks ||
      (block_size / num_mini_blocks) % 8 || block_size > (1u << 22))
    return (size_t)-1;
  const size_t mini = block_size / num_mini_blocks;
  uint8_t hdr[32];
  or_bit_writer hw;
  memset(hdr, 0, sizeof(hdr));
  bw_init(&hw, hdr, sizeof(hdr), 0);
  size_t body_cap = cap;
  uint8_t *body = (uint8_t *)calloc(body_cap ? body_cap : 1, 1);
  or_bit_writer w;
  bw_init(&w, body, body_cap, 0);
  int64_t *deltas = (int64_t *)malloc(block_size * sizeof(int64_t));
  size_t in_block = 0;
  int64_t first = 0, cur = 0;
  int ok = 1;
#define VAL(i) (t == OR_INT32 ? (int64_t)((const int32_t *)values)[i] : ((const int64_t *)values)[i])
  if (n > 0) {
    first = VAL(0);
    cur = first;
  }
  for (size_t idx = 1; idx <= n; ++idx) {
    int flush = 0;
    if (idx < n) {
      int64_t v = VAL(idx);
      deltas[in_block++] = delta_sub(t, v, cur);
      cur = v;
      if (in_block == block_size) flush = 1;
    } else {
      flush = in_block > 0;
    }
    if (!flush) continue;
    /* flush_block_values, encoding.rs:611-664 */
    int64_t min_delta = INT64_MAX;
    for (size_t i = 0; i < in_block; ++i)
      if (deltas[i] < min_delta) min_delta = deltas[i];
    ok &= bw_put_zigzag(&w, min_delta);
    long wpos = bw_skip(&w, num_mini_blocks);
    if (wpos < 0) {
      ok = 0;
      break;
    }
    for (size_t i = 0; i < num_mini_blocks; ++i) {
      size_t m = in_block < mini ? in_block : mini;
      if (m == 0) break;
      int64_t max_delta = INT64_MIN;
      for (size_t j = 0; j < m; ++j)
        if (deltas[i * mini + j] > max_delta) max_delta = deltas[i * mini + j];
      size_t bwid = or_num_required_bits(delta_sub_u64(t, max_delta, min_delta));
      body[wpos + (long)i] = (uint8_t)bwid;
      for (size_t j = 0; j < m; ++j) ok &= bw_put_value(&w, delta_sub_u64(t, deltas[i * mini + j], min_delta), bwid);
      for (size_t j = m; j < mini; ++j) ok &= bw_put_value(&w, 0, bwid);
      in_block -= m;
    }
  }
#undef VAL
  /* write_page_header, encoding.rs:589-607 */
  ok &= bw_put_vlq(&hw, block_size);
  ok &= bw_put_vlq(&hw, num_mini_blocks);
  ok &= bw_put_vlq(&hw, n);
  ok &= bw_put_zigzag(&hw, first);
  ok &= bw_flush(&hw);
  ok &= bw_flush(&w);
  size_t total = hw.byte_offset + w.byte_offset;
  free(deltas);
  if (!ok || total > cap) {
    free(body);
    return (size_t)-1;
  }
  memcpy(out, hdr, hw.byte_offset);
  memcpy(out + hw.byte_offset, body, w.byte_offset);
  free(body);
  return total;
}

size_t or_delta_encode(int t, const void *values, size_t n, uint8_t *out, size_t cap) {
  return or_delta_encode_shape(t, values, n, 128, 4, out, cap);
}

/* DeltaLengthByteArrayEncoder, encoding.rs:796-859 */
size_t or_delta_length_encode(const uint8_t *bytes, const int64_t *offsets, size_t n,
                              uint8_t *out, size_t cap) {
  int32_t *lens = (int32_t *)malloc((n ? n : 1) * 4);
  for (size_t i = 0; i < n; ++i) lens[i] = (int32_t)(offsets[i + 1] - offsets[i]);
  size_t o = or_delta_encode(OR_INT32, lens, n, out, cap);
  free(lens);
  if (o == (size_t)-1) return o;
  size_t tot = (size_t)(offsets[n] - offsets[0]);
  if (o + tot > cap) return (size_t)-1;
  memcpy(out + o, bytes + offsets[0], tot);
  return o + tot;
}

/* DeltaByteArrayEncoder, encoding.rs:866-952 */
size_t or_delta_byte_array_encode(const uint8_t *bytes, const int64_t *offsets, size_t n,
                                  uint8_t *out, size_t cap) {
  int32_t *pl = (int32_t *)malloc((n ? n : 1) * 4);
  int64_t *soff = (int64_t *)malloc((n + 1) * 8);
  uint8_t *sbytes = (uint8_t *)malloc((size_t)(offsets[n] - offsets[0]) + 1);
  size_t sb = 0;
  soff[0] = 0;
  const uint8_t *prev = NULL;
  size_t prev_len = 0;
  for (size_t i = 0; i < n; ++i) {
    const uint8_t *c = bytes + offsets[i];
    size_t cl = (size_t)(offsets[i + 1] - offsets[i]);
    size_t lim = prev_len < cl ? prev_len : cl;
    size_t m = 0;
    while (m < lim && prev[m] == c[m]) m++;
    pl[i] = (int32_t)m;
    memcpy(sbytes + sb, c + m, cl - m);
    sb += cl - m;
    soff[i + 1] = (int64_t)sb;
    prev = c;
    prev_len = cl;
  }
  size_t o = or_delta_encode(OR_INT32, pl, n, out, cap);
  size_t r = (size_t)-1;
  if (o != (size_t)-1) {
    size_t o2 = or_delta_length_encode(sbytes, soff, n, out + o, cap - o);
    if (o2 != (size_t)-1) r = o + o2;
  }
  free(pl);
  free(soff);
  free(sbytes);
  return r;
}

/* RleValueEncoder<Bool>::flush_buffer, encoding.rs:475-500 */
size_t or_rle_bool_encode(const uint8_t *values, size_t n, uint8_t *out, size_t cap) {
  if (cap < 4) return (size_t)-1;
  uint64_t *v = (uint64_t *)malloc((n ? n : 1) * 8);
  for (size_t i = 0; i < n; ++i) v[i] = values[i] ? 1 : 0;
  size_t l = or_rle_encode(v, n, 1, out + 4, cap - 4);
  free(v);
  if (l == (size_t)-1) return l;
  int32_t li = (int32_t)l;
  memcpy(out, &li, 4);
  return l + 4;
}

/* DictEncoder, encoding.rs:200-387. Uniques are kept in insertion order (the hash only
 * decides probing, encoding.rs:291-315, so it does not change the bytes). */
size_t or_dict_encode(const void *values, size_t n, size_t es, uint8_t *dict_out,
                      size_t dict_cap, size_t *dict_len, uint8_t *idx_out, size_t idx_cap,
                      size_t *idx_len) {
  const uint8_t *v = (const uint8_t *)values;
  size_t hsize = 1024;
  while (hsize < 2 * n + 2) hsize *= 2;
  int64_t *slots = (int64_t *)malloc(hsize * sizeof(int64_t));
  for (size_t i = 0; i < hsize; ++i) slots[i] = -1;
  uint64_t *idx = (uint64_t *)malloc((n ? n : 1) * 8);
  size_t nuniq = 0;
  for (size_t i = 0; i < n; ++i) {
    uint64_t h = 1469598103934665603ULL;
    for (size_t k = 0; k < es; ++k) h = (h ^ v[i * es + k]) * 1099511628211ULL;
    size_t j = (size_t)(h & (hsize - 1));
    while (slots[j] >= 0 && memcmp(dict_out + (size_t)slots[j] * es, v + i * es, es) != 0)
      j = (j + 1) & (hsize - 1);
    if (slots[j] < 0) {
      if ((nuniq + 1) * es > dict_cap) {
        free(slots);
        free(idx);
        return (size_t)-1;
      }
      memcpy(dict_out + nuniq * es, v + i * es, es);
      slots[j] = (int64_t)nuniq++;
    }
    idx[i] = (uint64_t)slots[j];
  }
  free(slots);
  *dict_len = nuniq * es;
  int bw = nuniq == 0 ? 0 : (nuniq == 1 ? 1 : or_log2(nuniq));
  if (idx_cap < 1) {
    free(idx);
    return (size_t)-1;
  }
  idx_out[0] = (uint8_t)bw;
  or_rle_encoder e;
  memset(idx_out + 1, 0, idx_cap - 1);
  rle_enc_init(&e, bw, idx_out, idx_cap, 1);
  for (size_t i = 0; i < n; ++i) rle_enc_put(&e, idx[i]);
  size_t end = rle_enc_consume(&e);
  free(idx);
  if (end == (size_t)-1) return end;
  *idx_len = end;
  return nuniq;
}
