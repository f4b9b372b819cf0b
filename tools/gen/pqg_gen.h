/*
 * pqg_gen.h — bench / test tooling (libpqgtools.so), NOT part of the decode library.
 *
 * Reference-identical page writers (RleEncoder rle.rs:55-317, LevelEncoder levels.rs:54-143,
 * PlainEncoder / DictEncoder / DeltaBitPackEncoder encoding.rs:94-714) and the multi-threaded
 * generators of the BASELINE.json workloads, plus pqg_truth_* functions that regenerate one
 * page's raw content so a benchmark can check decoded output against the generator.
 */
#ifndef PQG_GEN_H
#define PQG_GEN_H

#include "../../include/pqgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Writers: each returns bytes written or 0 on overflow. */
uint64_t pqg_encode_rle(const uint64_t *values, uint64_t n, int bit_width, uint8_t *out,
                        uint64_t cap);
uint64_t pqg_encode_levels_v1(const int16_t *levels, uint64_t n, int16_t max_level,
                              uint8_t *out, uint64_t cap);
uint64_t pqg_encode_delta(int physical_type, const void *values, uint64_t n, int block_size,
                          int mini_blocks, uint8_t *out, uint64_t cap);
/* Dictionary indices page body: [bit_width byte][RLE hybrid of the indices]. */
uint64_t pqg_encode_dict_indices(const uint32_t *indices, uint64_t n, int bit_width,
                                 uint8_t *out, uint64_t cap);

/* Multi-threaded synthetic workload generators (one page per task): see DESIGN.md §4. */
typedef struct {
  uint64_t blob_len;
  uint32_t npages;
  uint64_t total_levels;
  uint64_t total_values;
} pqg_workload_info;

/* Config 2: n levels with Bernoulli(p_null) nulls, max_def 1, PLAIN INT32 values; data
 * page v1 with `page_levels` levels per page. Pages written into `blob` (host) at 64-byte
 * aligned offsets; descriptors to `pages`. Call with blob == NULL to size. */
int pqg_gen_levels_plain(uint64_t n, double p_null, uint32_t page_levels, uint64_t seed,
                         int threads, uint8_t *blob, uint64_t blob_cap, pqg_page *pages,
                         uint32_t pages_cap, pqg_workload_info *info);
/* Config 3: required INT64 column, dictionary of `dict_size` distinct values, n indices
 * uniform in [0, dict_size): page 0 is the dictionary page. */
int pqg_gen_dict_int64(uint64_t n, uint32_t dict_size, uint32_t page_values, uint64_t seed,
                       int threads, uint8_t *blob, uint64_t blob_cap, pqg_page *pages,
                       uint32_t pages_cap, pqg_workload_info *info);
/* Config 4: required INT64 column, DELTA_BINARY_PACKED, deltas uniform in
 * [-2^(delta_bits-1), 2^(delta_bits-1)). */
int pqg_gen_delta_int64(uint64_t n, int delta_bits, uint32_t page_values, int block_size,
                        int mini_blocks, uint64_t seed, int threads, uint8_t *blob,
                        uint64_t blob_cap, pqg_page *pages, uint32_t pages_cap,
                        pqg_workload_info *info);

/* The same streams, pages [first, first + count) only (config 3: with the dictionary page first):
 * a rank's contiguous share of one stream, byte-identical to those pages of the whole. */
int pqg_gen_levels_plain_pages(uint64_t n, double p_null, uint32_t page_levels, uint64_t seed,
                               uint32_t first, uint32_t count, int threads, uint8_t *blob,
                               uint64_t blob_cap, pqg_page *pages, uint32_t pages_cap,
                               pqg_workload_info *info);
int pqg_gen_dict_int64_pages(uint64_t n, uint32_t dict_size, uint32_t page_values, uint64_t seed,
                             uint32_t first, uint32_t count, int threads, uint8_t *blob,
                             uint64_t blob_cap, pqg_page *pages, uint32_t pages_cap,
                             pqg_workload_info *info);
int pqg_gen_delta_int64_pages(uint64_t n, int delta_bits, uint32_t page_values, int block_size,
                              int mini_blocks, uint64_t seed, uint32_t first, uint32_t count,
                              int threads, uint8_t *blob, uint64_t blob_cap, pqg_page *pages,
                              uint32_t pages_cap, pqg_workload_info *info);

/* Config 5: one row group (`rows` rows from global row `row0`) of the alltypes_plain schema (11
 * OPTIONAL columns: id INT32, bool_col BOOLEAN, tinyint/smallint/int INT32, bigint INT64, float,
 * double, date_string / string BYTE_ARRAY, timestamp INT96), written with the reference writer's
 * defaults (see pqg_gen.cpp). pqg_gen_alltypes builds it in host memory (one thread per column)
 * and returns a handle; pqg_alltypes_copy lays the 11 column chunks out in `blob` (64-byte
 * aligned pages; chunk j's pages are [chunk_first[j], chunk_first[j + 1])). */
typedef struct {
  uint64_t blob_len;
  uint64_t rows;
  uint32_t npages;
  uint32_t chunk_first[12];
  uint64_t chunk_offset[12];
  uint64_t num_values[11];   /* non-null values per column */
  uint64_t value_bytes[11];  /* decoded value bytes (BYTE_ARRAY: the concatenated bytes) */
} pqg_alltypes_info;
void *pqg_gen_alltypes(uint64_t rows, uint64_t row0, double p_null, uint64_t seed, int threads,
                       pqg_alltypes_info *info);
int pqg_alltypes_copy(void *handle, uint8_t *blob, uint64_t cap, pqg_page *pages, uint32_t pages_cap);
void pqg_alltypes_free(void *handle);
/* Raw content of column `col` over rows [row0, row0 + rows): levels (0/1), the non-null values'
 * bytes (PLAIN form; BYTE_ARRAY: the bytes alone, with int64 offsets[values + 1]). Returns the
 * non-null count. Any output pointer may be NULL. */
/* Row groups [row0 / rows_per_group, ...) of the alltypes workload written as a parquet file
 * (row group g = pqg_gen_alltypes(rows_per_group, row0 + g * rows_per_group, ...)); codec 0 none,
 * 1 SNAPPY, 2 GZIP. Returns PQG_OK or a PQG_ERR_* status. */
int pqg_write_alltypes_file(const char *path, uint64_t rows_per_group, uint32_t row_groups, uint64_t row0,
                            double p_null, uint64_t seed, int codec, int threads);
uint64_t pqg_truth_alltypes(uint64_t row0, uint64_t rows, int col, double p_null, uint64_t seed,
                            int16_t *levels, uint8_t *values, int64_t *offsets);

/* Raw content of one generated page (same seeds as the generators): */
/* config 2: levels (0/1) of page `page` and its non-null INT32 values; returns the count. */
uint64_t pqg_truth_levels_plain(uint64_t n, double p_null, uint32_t page_levels, uint64_t seed,
                                uint32_t page, int16_t *levels, int32_t *values);
/* config 3: the decoded INT64 values of data page `page` (0-based, after the dictionary page). */
uint64_t pqg_truth_dict_int64(uint64_t n, uint32_t dict_size, uint32_t page_values, uint64_t seed,
                              uint32_t page, int64_t *values);
/* config 4: the INT64 values of page `page`. */
uint64_t pqg_truth_delta_int64(uint64_t n, int delta_bits, uint32_t page_values, uint64_t seed,
                               uint32_t page, int64_t *values);

#ifdef __cplusplus
}
#endif
#endif
