/*
 * pq_oracle.h — CPU restatement of parquet-rs 0.4.2's decode path (TEST INFRASTRUCTURE).
 *
 * THIS IS THE PARITY ORACLE, NOT PRODUCT CODE. Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker / CPU baseline.
 *
 * Every function restates the behaviour of a reference item, cited as path:line into
 * /root/reference (sunchao/parquet-rs v0.4.2). The reference is Rust and cannot be built
 * in this image (no rustc/cargo, nightly-2018-12-06 features, un-vendored crates), so
 * parity is pinned by the reference's own known-answer tests (tests/test_oracle_kat.py)
 * and by the reference data files under tests/golden (values cross-checked with pyarrow,
 * an independent Parquet implementation; see tests/golden/make_golden.py).
 *
 * Status codes mirror ParquetError (src/errors.rs:24-51) plus the two non-error outcomes
 * the reference can reach on malformed input: a Rust panic (assert!/index) and an
 * infinite loop. The oracle reports those instead of crashing.
 */
#ifndef PQ_ORACLE_H
#define PQ_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  OR_OK = 0,
  OR_GENERAL = 1, /* ParquetError::General */
  OR_NYI = 2,     /* ParquetError::NYI */
  OR_EOF = 3,     /* ParquetError::EOF */
  OR_PANIC = 4,   /* the reference would panic (assert!/bounds check) */
  OR_HANG = 5     /* the reference would loop forever (rle.rs:414-425 with 0-value progress) */
};

/* Thrift enum ids (basic.rs:38-47, 169-218 via 508-521). */
enum {
  OR_BOOLEAN = 0, OR_INT32 = 1, OR_INT64 = 2, OR_INT96 = 3, OR_FLOAT = 4, OR_DOUBLE = 5,
  OR_BYTE_ARRAY = 6, OR_FIXED_LEN_BYTE_ARRAY = 7
};
enum {
  OR_ENC_PLAIN = 0, OR_ENC_PLAIN_DICTIONARY = 2, OR_ENC_RLE = 3, OR_ENC_BIT_PACKED = 4,
  OR_ENC_DELTA_BINARY_PACKED = 5, OR_ENC_DELTA_LENGTH_BYTE_ARRAY = 6,
  OR_ENC_DELTA_BYTE_ARRAY = 7, OR_ENC_RLE_DICTIONARY = 8
};
enum { OR_PAGE_DATA = 0, OR_PAGE_INDEX = 1, OR_PAGE_DICTIONARY = 2, OR_PAGE_DATA_V2 = 3 };

/* ---------------------------------------------------------------- bit utilities */
/* bit_util.rs:81-132 */
int64_t or_ceil(int64_t value, int64_t divisor);
int or_log2(uint64_t x);
uint64_t or_trailing_bits(uint64_t v, size_t num_bits);
size_t or_num_required_bits(uint64_t x);

/* BitReader, bit_util.rs:369-608 */
typedef struct {
  const uint8_t *buf;
  size_t total_bytes;
  size_t byte_offset;
  size_t bit_offset;
  uint64_t buffered;
  int status; /* sticky: OR_PANIC once an assert! of the reference would fire */
} or_bit_reader;

void or_br_init(or_bit_reader *r, const uint8_t *buf, size_t len);
/* get_value<T>(num_bits): returns 1 (Some) / 0 (None); *out holds the low type_size bytes. */
int or_br_get_value(or_bit_reader *r, int num_bits, int type_size, uint64_t *out);
/* get_batch<T>: writes type_size-byte elements (quirk: 8-byte T gets only the low 4 bytes
 * through the unpack32 path, bit_util.rs:498-503). Returns values read. */
size_t or_br_get_batch(or_bit_reader *r, void *batch, size_t n, int type_size, int num_bits);
int or_br_get_aligned(or_bit_reader *r, size_t num_bytes, uint64_t *out);
int or_br_get_vlq_int(or_bit_reader *r, int64_t *out);
int or_br_get_zigzag_vlq_int(or_bit_reader *r, int64_t *out);
size_t or_br_get_byte_offset(const or_bit_reader *r);

/* unpack32, bit_packing.rs:29-72: 32 values of num_bits from 4*num_bits bytes. */
void or_unpack32(const uint8_t *in, uint32_t *out, int num_bits);

/* ---------------------------------------------------------------- RLE hybrid */
/* RleDecoder, rle.rs:320-509 */
typedef struct {
  int bit_width;
  or_bit_reader br;
  int has_reader;
  uint32_t rle_left;
  uint32_t bit_packed_left;
  uint64_t current_value;
  int has_current;
  int status;
} or_rle_decoder;

void or_rle_init(or_rle_decoder *d, int bit_width);
void or_rle_set_data(or_rle_decoder *d, const uint8_t *data, size_t len);
int or_rle_get(or_rle_decoder *d, int type_size, uint64_t *out, int *has_value);
int or_rle_get_batch(or_rle_decoder *d, void *buf, size_t n, int type_size, size_t *values_read);
int or_rle_get_batch_with_dict(or_rle_decoder *d, const void *dict, size_t dict_len,
                               size_t elem_size, void *buf, size_t buf_len, size_t max_values,
                               size_t *values_read);

/* Convenience for tests: set_data + get_batch<T>. */
int or_rle_decode(const uint8_t *data, size_t len, int bit_width, int type_size, void *out,
                  size_t n, size_t *values_read);
int or_rle_decode_dict(const uint8_t *data, size_t len, int bit_width, const void *dict,
                       size_t dict_len, size_t elem_size, void *out, size_t n,
                       size_t *values_read);

/* ---------------------------------------------------------------- levels */
/* LevelDecoder, levels.rs:148-272.  For v1 (`v2 == 0`) the data pointer is the
 * (page-relative) slice handed to set_data and `slice_start` is BufferPtr::start() of that
 * slice (needed for the BIT_PACKED double-offset quirk, levels.rs:206). For v2 the range
 * [start, start+len) of `data` is used (set_data_range, levels.rs:217-233). */
typedef struct {
  int kind; /* 0 RLE, 1 RLE_V2, 2 BIT_PACKED */
  int bit_width;
  size_t num_values;
  int has_num_values;
  or_rle_decoder rle;
  or_bit_reader br;
  int status;
} or_level_decoder;

void or_level_init_v1(or_level_decoder *d, int encoding, int16_t max_level);
void or_level_init_v2(or_level_decoder *d, int16_t max_level);
/* set_data: `page` is the whole page buffer, `start` the BufferPtr start of the slice
 * (the slice is page[start:len]). Returns bytes consumed (or 0 with d->status set). */
size_t or_level_set_data(or_level_decoder *d, size_t num_buffered_values, const uint8_t *page,
                         size_t start, size_t len);
size_t or_level_set_data_range(or_level_decoder *d, size_t num_buffered_values,
                               const uint8_t *buf, size_t buf_len, size_t start, size_t len);
int or_level_get(or_level_decoder *d, int16_t *buf, size_t n, size_t *values_read);

/* ---------------------------------------------------------------- values */
/* A byte-array value (ByteArray, data_type.rs:70-98): a slice, possibly of page bytes. */
typedef struct {
  const uint8_t *ptr;
  uint64_t len;
} or_ba;

/* Element layout per physical type on the output side (data_type.rs:308-345):
 * BOOLEAN 1 B, INT32 4, INT64 8, INT96 12, FLOAT 4, DOUBLE 8, BYTE_ARRAY/FLBA or_ba. */
size_t or_type_size(int physical_type);

/* PLAIN decode of up to n values (decoding.rs:88-247). Returns status; *read = count. */
int or_plain_decode(int physical_type, int32_t type_length, const uint8_t *data, size_t len,
                    size_t num_values, void *out, size_t n, size_t *read);

/* DELTA_BINARY_PACKED (decoding.rs:392-619). Decodes min(n, header count) values.
 * *offset_out = get_offset() after decoding (decoding.rs:441-444). *total_out = header
 * value count (values_left() right after set_data). */
int or_delta_decode(int physical_type, const uint8_t *data, size_t len, void *out, size_t n,
                    size_t *read, size_t *offset_out, size_t *total_out);

/* ---------------------------------------------------------------- column chunk */
typedef struct {
  int page_type;        /* OR_PAGE_* */
  const uint8_t *buf;   /* uncompressed payload */
  size_t len;
  uint32_t num_values;
  int encoding;
  int def_encoding;     /* v1 only */
  int rep_encoding;     /* v1 only */
  uint32_t def_len;     /* v2 only */
  uint32_t rep_len;     /* v2 only */
} or_page;

typedef struct {
  int physical_type;
  int32_t type_length;
  int16_t max_def;
  int16_t max_rep;
} or_column;

/* Result of reading a whole chunk through ColumnReaderImpl::read_batch (column/reader.rs
 * :159-265) in batches of `batch_size`. Fixed-width values are packed in `values` (element
 * size or_type_size); BYTE_ARRAY/FLBA values are concatenated in `bytes` with int64
 * `offsets` (n+1 entries). Buffers are malloc'd; free with or_column_result_free. */
typedef struct {
  int status;
  char message[256];
  int16_t *def_levels;
  int16_t *rep_levels;
  uint8_t *values;
  int64_t *offsets;
  uint8_t *bytes;
  size_t num_levels;
  size_t num_values;
  size_t num_bytes;
  size_t num_batches;
} or_column_result;

int or_read_column(const or_column *col, const or_page *pages, size_t npages,
                   size_t batch_size, int want_def, int want_rep, or_column_result *res);
/* The same with the reference's slice lengths: values / def / rep slices of vcap / dcap / rcap
 * elements (column/reader.rs:170-205); counts (if given) receives (values_read, levels_read) of
 * each read_batch call, counts_cap entries. */
int or_read_column_caps(const or_column *col, const or_page *pages, size_t npages,
                        size_t batch_size, size_t vcap, size_t dcap, size_t rcap, int want_def,
                        int want_rep, uint64_t *counts, size_t counts_cap, or_column_result *res);
void or_column_result_free(or_column_result *res);

/* ---------------------------------------------------------------- encoders (generators) */
/* Restated writers used to produce pages byte-identical to the reference's (encoding.rs,
 * rle.rs:55-317, levels.rs:54-143). All return bytes written or (size_t)-1 on overflow. */
size_t or_rle_encode(const uint64_t *values, size_t n, int bit_width, uint8_t *out, size_t cap);
size_t or_level_encode(int encoding, int v2, int16_t max_level, const int16_t *levels,
                       size_t n, uint8_t *out, size_t cap);
size_t or_plain_encode(int physical_type, const void *values, size_t n, uint8_t *out,
                       size_t cap);
size_t or_delta_encode(int physical_type, const void *values, size_t n, uint8_t *out,
                       size_t cap);
/* Same with any block shape (block_size / num_mini_blocks values per mini-block, a multiple of 8). */
size_t or_delta_encode_shape(int physical_type, const void *values, size_t n, size_t block_size,
                             size_t num_mini_blocks, uint8_t *out, size_t cap);
/* DictEncoder (encoding.rs:200-387): returns number of uniques; writes the PLAIN dict page
 * to dict_out (*dict_len) and [bit_width][RLE] indices to idx_out (*idx_len). For
 * fixed-width types only (elem_size bytes per value). */
size_t or_dict_encode(const void *values, size_t n, size_t elem_size, uint8_t *dict_out,
                      size_t dict_cap, size_t *dict_len, uint8_t *idx_out, size_t idx_cap,
                      size_t *idx_len);
/* RleValueEncoder<Bool> (encoding.rs:422-501): [i32 len][RLE w=1]. */
size_t or_rle_bool_encode(const uint8_t *values, size_t n, uint8_t *out, size_t cap);
/* Byte arrays given as concatenated bytes + int64 offsets (n+1). */
size_t or_plain_encode_ba(const uint8_t *bytes, const int64_t *offsets, size_t n, int fixed,
                          uint8_t *out, size_t cap);
size_t or_delta_length_encode(const uint8_t *bytes, const int64_t *offsets, size_t n,
                              uint8_t *out, size_t cap);
size_t or_delta_byte_array_encode(const uint8_t *bytes, const int64_t *offsets, size_t n,
                                  uint8_t *out, size_t cap);

#ifdef __cplusplus
}
#endif
#endif
