/*
 * pqgpu.h — C ABI of the MI355X-native parquet page decoder.
 *
 * This is the drop-in boundary for the decode half of parquet-rs 0.4.2 (sunchao/parquet-rs,
 * /root/reference). It replaces, for a whole column chunk at a time:
 *
 *   Decoder<T>::set_data / get           src/encodings/decoding.rs:37-54 (all decoders,
 *                                        :88-835, via get_decoder :60-79)
 *   DictDecoder<T>::set_dict             src/encodings/decoding.rs:282-288
 *   LevelDecoder::{v1,v2,set_data,set_data_range,get}   src/encodings/levels.rs:148-272
 *   RleDecoder::{get_batch,get_batch_with_dict}         src/encodings/rle.rs:398-487
 *   BitReader::{get_value,get_batch,...}, unpack32      src/util/bit_util.rs:369-608,
 *                                                       src/util/bit_packing.rs:29-72
 *   the decode loop of ColumnReaderImpl::read_batch     src/column/reader.rs:159-265
 *       (def-level count :212-226, dense values :252-253) and read_new_page /
 *       set_current_page_encoding / configure_dictionary :269-488
 *
 * The reference pulls `batch_size` values at a time through those traits; a GPU cannot be
 * fed that way, so the ABI decodes whole chunks (all pages of a column chunk in one call)
 * and a host-side ColumnReader serves read_batch slices from the decoded chunk
 * (pqg_column_reader_* below). Results are identical to the concatenation of the
 * reference's read_batch outputs.
 *
 * Conventions
 *  - Plain pointers and sizes only. Device buffers are HIP device pointers on the ctx's
 *    device; the stream argument is a hipStream_t (may be NULL = default stream).
 *  - The caller owns every buffer; the library never frees caller memory. Page bytes are
 *    read-only (mirrors ByteBufferPtr, src/util/memory.rs:245-356).
 *  - One pqg_ctx per GPU; a ctx is single-owner (like the reference's !Send readers).
 *    Distinct contexts may be used concurrently from different host threads.
 *  - Status codes: 0 OK; 1 General, 2 NYI, 3 EOF (ParquetError, src/errors.rs:24-51);
 *    4 = input on which the reference panics; 5 = input on which the reference loops
 *    forever; 6 = output capacity too small; 7 = invalid argument; 8 = HIP runtime error.
 *    The library never aborts the process.
 *  - Encoding / type / page-type ids are the on-disk thrift ids (src/basic.rs:38-47,
 *    169-218, converted at :387-400, :508-521).
 */
#ifndef PQGPU_H
#define PQGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PQG_OK 0
#define PQG_ERR_GENERAL 1
#define PQG_ERR_NYI 2
#define PQG_ERR_EOF 3
#define PQG_ERR_PANIC 4
#define PQG_ERR_HANG 5
#define PQG_ERR_CAPACITY 6
#define PQG_ERR_INVALID 7
#define PQG_ERR_HIP 8

/* physical types (basic.rs:38-47) */
#define PQG_BOOLEAN 0
#define PQG_INT32 1
#define PQG_INT64 2
#define PQG_INT96 3
#define PQG_FLOAT 4
#define PQG_DOUBLE 5
#define PQG_BYTE_ARRAY 6
#define PQG_FIXED_LEN_BYTE_ARRAY 7

/* encodings (thrift ids) */
#define PQG_PLAIN 0
#define PQG_PLAIN_DICTIONARY 2
#define PQG_RLE 3
#define PQG_BIT_PACKED 4
#define PQG_DELTA_BINARY_PACKED 5
#define PQG_DELTA_LENGTH_BYTE_ARRAY 6
#define PQG_DELTA_BYTE_ARRAY 7
#define PQG_RLE_DICTIONARY 8

/* page types (thrift PageType) */
#define PQG_PAGE_DATA 0
#define PQG_PAGE_DICTIONARY 2
#define PQG_PAGE_DATA_V2 3

/* One uncompressed page of a column chunk (Page, src/column/page.rs:28-57). Pages are
 * given in file order, the dictionary page (if any) first. `offset` locates the payload in
 * the chunk blob; 16-byte aligned offsets give the fastest dictionary gathers. */
typedef struct {
  uint64_t offset;       /* payload offset inside the blob */
  uint32_t nbytes;       /* uncompressed payload length */
  uint32_t num_values;   /* DataPage(V2).num_values / DictionaryPage.num_values */
  int32_t page_type;     /* PQG_PAGE_* */
  int32_t encoding;      /* value encoding */
  int32_t def_encoding;  /* data page v1: definition level encoding (RLE / BIT_PACKED) */
  int32_t rep_encoding;  /* data page v1: repetition level encoding */
  uint32_t def_len;      /* data page v2: definition_levels_byte_length */
  uint32_t rep_len;      /* data page v2: repetition_levels_byte_length */
} pqg_page;

/* Column descriptor subset the decode needs (ColumnDescriptor, schema/types.rs:546-640). */
typedef struct {
  int32_t physical_type;
  int32_t type_length;  /* FIXED_LEN_BYTE_ARRAY only */
  int16_t max_def;
  int16_t max_rep;
} pqg_column;

/* Outputs of one chunk decode, all device memory, 16-byte aligned.
 *  def_levels / rep_levels: int16, capacity >= sum of data-page num_values; NULL skips the
 *    stream exactly as read_batch(.., None, ..) does (column/reader.rs:212-250).
 *  values: dense non-null values (fixed width: 1 B bool, 4 B INT32/FLOAT, 8 B INT64/DOUBLE,
 *    12 B INT96; BYTE_ARRAY/FLBA: concatenated bytes) with `values_capacity` bytes.
 *  offsets: BYTE_ARRAY/FLBA only, int64[num_values + 1] byte offsets into `values`.
 *  The counters are filled by pqg_sync. */
typedef struct {
  int16_t *def_levels;
  int16_t *rep_levels;
  void *values;
  uint64_t values_capacity;
  int64_t *offsets;
  uint64_t offsets_capacity; /* entries */
  uint64_t num_levels;       /* out */
  uint64_t num_values;       /* out */
  uint64_t num_bytes;        /* out (BYTE_ARRAY/FLBA) */
} pqg_output;

typedef struct pqg_ctx pqg_ctx;

/* Per-stage device times (ms) measured with HIP events on the decode stream. */
typedef struct {
  float prepare_ms, levels_ms, scan_ms, values_ms, total_ms;
  uint32_t values_kernel; /* encoding whose kernel dominated values_ms */
  float levels_kernel_ms; /* the def-level path kernels alone, 0 if none */
  float values_kernel_ms; /* the values stage's dominant kernel alone, 0 if none */
} pqg_timings;

int pqg_ctx_create(int device, pqg_ctx **out);
int pqg_ctx_destroy(pqg_ctx *ctx);
int pqg_ctx_set_timing(pqg_ctx *ctx, int enabled);
/* PLAIN fixed-width values of chunks read with def levels, whose data pages are all PLAIN: copied
 * on a side stream while the def levels decode, at the offsets the value sections' sizes give
 * (a page's value section holds exactly its non-null values in every file the reference writes);
 * the value-offset scan checks every such page and the chunks where a count or offset differs are
 * copied again at the true offsets. enabled = 0 copies after the levels only (the default: the
 * copy and the level kernels share HBM; measured on MI355X the side copy pays off only for sparse
 * def streams); 1 forks the side copy right after the page preparation, one workgroup per page
 * (p_null 0.5: 1.72 -> 1.63 ms, but p_null 0: 1.96 -> 2.3-2.6 ms); 2 forks it after the def
 * levels' front end, beside their emit, on a full grid. */
int pqg_ctx_set_overlap(pqg_ctx *ctx, int enabled);

/* Enqueue the decode of one column chunk on `stream` (asynchronous). `blob` is a device
 * buffer of `blob_len` bytes holding every page payload; `pages` is host memory (copied
 * during the call). Returns immediately with PQG_OK or an argument error.
 * `out` is written again later, when the decode's counters are delivered (by pqg_sync, or
 * when the ctx reuses the decode's staging two decodes on): the pqg_output struct itself must
 * stay valid until the pqg_sync that follows this call. */
int pqg_decode_chunk(pqg_ctx *ctx, const pqg_column *col, const uint8_t *blob,
                     uint64_t blob_len, const pqg_page *pages, uint32_t npages,
                     pqg_output *out, void *stream);

/* Enqueue the decode of a batch of column chunks in one pass (asynchronous): chunk j is
 * cols[j], its pages pages[j][0 .. npages[j]) (offsets into the one device blob) and its outputs
 * outs[j], as pqg_decode_chunk takes them. The chunks share nothing (each is what one column
 * reader of the reference decodes, file/reader.rs:252-260, 306-330); the batch runs every kernel
 * once over all their pages, so one row group, or several, costs the launches of one chunk. The
 * outs structs must stay valid until the pqg_sync that delivers them. */
int pqg_decode_chunks(pqg_ctx *ctx, uint32_t nchunks, const pqg_column *cols, const uint8_t *blob,
                      uint64_t blob_len, const pqg_page *const *pages, const uint32_t *npages,
                      pqg_output *outs, void *stream);

/* Wait for every decode enqueued on the ctx since the last pqg_sync, fill their outputs and
 * report the status of the first one (in issue order) that failed. On error *first_bad_page
 * names that decode's lowest failing page (the page the reference would fail on first). */
int pqg_sync(pqg_ctx *ctx, int *first_bad_page);
/* pqg_sync naming the failure fully: *bad_call = index of the failing decode call since the last
 * sync (0 = the first), *bad_chunk = its lowest failing chunk (0 for pqg_decode_chunk),
 * *bad_page = that chunk's lowest failing page. -1 when all succeeded. */
int pqg_sync_detail(pqg_ctx *ctx, int *bad_call, int *bad_chunk, int *bad_page);
/* Record assembly on the device (the layout TypedTripletIter builds per batch,
 * record/triplet.rs:300-318, over a whole decoded chunk): spaced[i] = the value of level i when
 * def_levels[i] == max_def (values = the decode's dense fixed-width values, value_size 1 / 4 / 8
 * / 12 bytes), zero bytes otherwise. All pointers are device memory and required (values too,
 * even when no level is non-null); enqueued on `stream` (NULL: the ctx's stream) after the
 * decode that produced them. */
int pqg_space_values(pqg_ctx *ctx, const int16_t *def_levels, uint64_t num_levels, int16_t max_def,
                     const void *values, int value_size, void *spaced, void *stream);
/* Averages over all decodes since pqg_reset_timings (timing must be enabled). */
int pqg_get_timings(pqg_ctx *ctx, pqg_timings *t);
int pqg_reset_timings(pqg_ctx *ctx);
const char *pqg_error_message(pqg_ctx *ctx);
/* The value-kernel families the last decode enqueued (diagnostics and tests: which path a page
 * shape takes), a mask of PQG_PATH_*. */
enum {
  PQG_PATH_PLAIN = 1,          /* fixed-width PLAIN copy */
  PQG_PATH_DICT_LEVEL = 2,     /* dictionary indices on the level path (LDS dictionary) */
  PQG_PATH_DICT_WINDOW = 4,    /* windowed dictionary gather, 257..65536 entries of 4 / 8 bytes */
  PQG_PATH_DICT_TILES = 8,     /* general dictionary tiles (L2 gather) */
  PQG_PATH_BYTES = 16,         /* byte arrays (PLAIN, dictionary, DELTA_LENGTH) */
  PQG_PATH_DELTA_BYTES = 32,   /* DELTA_BYTE_ARRAY slice rebuild */
  PQG_PATH_DELTA = 64,         /* DELTA_BINARY_PACKED */
  PQG_PATH_RLE_BOOL = 128      /* RLE booleans */
};
int pqg_ctx_last_paths(pqg_ctx *ctx, uint32_t *mask);

/* ---------------------------------------------------------------- row groups
 * The column chunks of one row group decoded together. The reference reads every column chunk
 * of a row group through its own page reader and column reader (file/reader.rs:252-260,
 * 306-330); they share nothing, so pqg_rg_decode is one pqg_decode_chunks of them on `stream`
 * (two row groups may be in flight: the ctx has two staging slots). `nstreams` is reserved: it
 * must be 1..16 (PQG_ERR_INVALID otherwise) and is otherwise ignored -- every decode runs on the
 * caller's stream, one batched launch sequence for all columns. pages[j] / npages[j] / outs[j] are column j's arguments of
 * pqg_decode_chunk, all pages in the one device blob. Asynchronous: pqg_rg_sync waits and fills
 * every outs[j]; it returns the first failing column's status (lowest index) and names that
 * column and its page. pages and outs (the arrays and the structs) must stay valid until that
 * sync. */
typedef struct pqg_rg_ctx pqg_rg_ctx;
int pqg_rg_ctx_create(int device, int nstreams, pqg_rg_ctx **out);
int pqg_rg_ctx_destroy(pqg_rg_ctx *g);
int pqg_rg_decode(pqg_rg_ctx *g, uint32_t ncols, const pqg_column *cols, const uint8_t *blob,
                  uint64_t blob_len, const pqg_page *const *pages, const uint32_t *npages,
                  pqg_output *outs, void *stream);
int pqg_rg_sync(pqg_rg_ctx *g, int *bad_column, int *bad_page);
/* pqg_rg_sync that also reports which pqg_rg_decode call (0 = the first since the last sync)
 * failed. With several row groups in flight the failure reported is the one the reference meets
 * first: the earliest failing row group, and in it the lowest failing column. */
int pqg_rg_sync_call(pqg_rg_ctx *g, int *bad_call, int *bad_column, int *bad_page);
const char *pqg_rg_error_message(pqg_rg_ctx *g);

/* ---------------------------------------------------------------- host-side reader
 * The parquet::file::reader surface kept on the host (src/file/reader.rs:51-90, 140-530):
 * footer + thrift-compact metadata, page headers, decompression (snappy, gzip), then the
 * GPU decode above. Column readers serve read_batch slices with the reference's contract
 * (column/reader.rs:159-265). */
typedef struct pqg_file_reader pqg_file_reader;
typedef struct pqg_column_reader pqg_column_reader;

int pqg_file_open(const char *path, pqg_file_reader **out);
int pqg_file_open_memory(const uint8_t *data, uint64_t len, pqg_file_reader **out);
void pqg_file_close(pqg_file_reader *r);
const char *pqg_file_error(pqg_file_reader *r);
int64_t pqg_file_num_rows(pqg_file_reader *r);
int pqg_file_num_row_groups(pqg_file_reader *r);
int pqg_file_num_columns(pqg_file_reader *r);
/* Leaf column descriptor (SchemaDescriptor::column): path is dot-joined. */
int pqg_file_column(pqg_file_reader *r, int col, pqg_column *out, char *path, size_t path_cap);
int64_t pqg_row_group_num_rows(pqg_file_reader *r, int rg);
/* Uncompressed pages of one column chunk (SerializedPageReader::get_next_page). Fills up
 * to `cap` page descriptors (offsets into an internal host blob that pqg_chunk_blob
 * returns); returns the page count or a negative status. */
int pqg_chunk_pages(pqg_file_reader *r, int rg, int col, pqg_page *pages, uint32_t cap);
int pqg_chunk_blob(pqg_file_reader *r, int rg, int col, const uint8_t **blob, uint64_t *len);

/* ColumnReaderImpl over the GPU decode: the chunk is decoded on `device` in one pass,
 * read_batch then copies slices to host buffers. def/rep may be NULL (read_batch(None)). */
int pqg_column_reader_open(pqg_file_reader *r, int rg, int col, pqg_ctx *ctx,
                           pqg_column_reader **out);
void pqg_column_reader_close(pqg_column_reader *cr);
/* Returns status; *values_read / *levels_read as read_batch's tuple. For BYTE_ARRAY/FLBA
 * `values` receives concatenated bytes (capacity values_bytes_cap) and `lengths` the
 * per-value byte lengths. */
int pqg_column_reader_read_batch(pqg_column_reader *cr, size_t batch_size, int16_t *def,
                                 int16_t *rep, void *values, uint64_t values_bytes_cap,
                                 uint32_t *lengths, size_t *values_read, size_t *levels_read);
/* read_batch with the reference's slice lengths (column/reader.rs:159-205): `def_cap` /
 * `rep_cap` levels (when def / rep are given) and `values_cap` values (BYTE_ARRAY/FLBA: entries of
 * `lengths`) clamp the batch and every page iteration as `def_levels.len()`, `rep_levels.len()`
 * and `values.len()` do; pqg_column_reader_read_batch is this call with every cap = batch_size.
 * def = NULL on a column with max_def > 0 reads iter_batch_size values per page iteration out of
 * step with the levels (:212-226, 247-250): PLAIN fixed width then ends in EOF and
 * PLAIN BYTE_ARRAY in PQG_ERR_PANIC once a page's non-null values are used up, the DELTA
 * encodings return short reads and then PQG_ERR_HANG (the reference's loop makes no progress);
 * dictionary and boolean pages read that far return PQG_ERR_NYI (the reference reads the
 * stream's padding bits there). */
int pqg_column_reader_read_batch_caps(pqg_column_reader *cr, size_t batch_size, int16_t *def,
                                      size_t def_cap, int16_t *rep, size_t rep_cap, void *values,
                                      size_t values_cap, uint64_t values_bytes_cap, uint32_t *lengths,
                                      size_t *values_read, size_t *levels_read);

/* ---------------------------------------------------------------- file -> device row groups
 * The product path of whole row groups, from the file to device (and host) memory, pipelined:
 * page headers of every column parsed and the payloads copied or decompressed (SNAPPY, GZIP) by
 * `host_threads` threads straight into pinned staging (SerializedPageReader::get_next_page,
 * file/reader.rs:420-522, for all of a row group's chunks, file/reader.rs:252-260, 306-330), one
 * async H2D copy, one batched decode of the row group's column chunks (pqg_decode_chunks), and
 * with PQG_RGR_HOST_OUTPUT async D2H copies of every output into pinned host buffers.
 * pqg_rgr_submit returns once the row group is staged and its copies and decode are enqueued; up
 * to two row groups may be in flight, so submitting g + 1 before waiting for g overlaps g + 1's
 * host work and H2D copy with g's decode. pqg_rgr_wait waits for the oldest row group in flight,
 * returns its status (the first failure the reference would meet reading its columns in order:
 * the lowest failing column, and in it the lowest failing page, be it a header / decompression
 * failure or a decode failure) and makes its outputs current for pqg_rgr_column. Current outputs
 * stay valid until the next pqg_rgr_wait. Staging, device blobs and outputs are kept across row
 * groups (grown, never shrunk). The file reader must outlive the pqg_rgr. */
typedef struct pqg_rgr pqg_rgr;
#define PQG_RGR_HOST_OUTPUT 1
typedef struct {
  const int16_t *def_levels; /* device; NULL when the column has no such levels */
  const int16_t *rep_levels;
  const void *values;        /* dense non-null values (BYTE_ARRAY/FLBA: concatenated bytes) */
  const int64_t *offsets;    /* BYTE_ARRAY/FLBA: num_values + 1 byte offsets */
  const int16_t *host_def_levels; /* pinned host copies (PQG_RGR_HOST_OUTPUT), else NULL */
  const int16_t *host_rep_levels;
  const void *host_values;
  const int64_t *host_offsets;
  uint64_t num_levels, num_values, num_bytes;
} pqg_rgr_output;
typedef struct {
  uint64_t row_groups;   /* submitted */
  uint64_t file_bytes;   /* column chunk bytes read from the file (compressed) */
  uint64_t staged_bytes; /* uncompressed page bytes copied H2D */
  uint64_t output_bytes; /* levels, values and offsets of waited row groups */
  double host_ms;        /* host time in submit: headers, copies / decompression, tables */
  double plan_ms;        /*   of which page headers */
  double fill_ms;        /*   of which page copies / decompression (the thread pool) */
  double enqueue_ms;     /* submit: H2D, decode and D2H enqueue */
  double sync_ms;        /* wait: for the decode */
  double d2h_wait_ms;    /* wait: for the D2H copies (PQG_RGR_HOST_OUTPUT) */
} pqg_rgr_stats;
int pqg_rgr_open(pqg_file_reader *r, int device, int host_threads, int flags, pqg_rgr **out);
int pqg_rgr_close(pqg_rgr *g);
int pqg_rgr_submit(pqg_rgr *g, int row_group);
int pqg_rgr_wait(pqg_rgr *g, int *row_group, int *bad_column, int *bad_page);
/* Outputs of column `col` of the current row group; returns the row group's status for a column at
 * or after its failing column (whose outputs are then partial), PQG_OK otherwise. */
int pqg_rgr_column(pqg_rgr *g, int col, pqg_rgr_output *out);
int pqg_rgr_get_stats(pqg_rgr *g, pqg_rgr_stats *out);
const char *pqg_rgr_error(pqg_rgr *g);

/* Record assembly's leaf iterator: TypedTripletIter (record/triplet.rs:168-330) over a column
 * reader. read_next (triplet.rs:270-294) advances one (definition level, repetition level,
 * value) triplet, refilling `batch_size` levels at a time through read_batch and spacing the
 * values onto the levels whose def == max_def (:300-318); *has_next = 0 when none is left.
 * def/rep levels of a column without them read as its max level (:246-262). value copies the
 * current value (BYTE_ARRAY/FLBA: its bytes; *len set) and returns PQG_ERR_PANIC on a null
 * slot, where the reference asserts (:236-243). The reader must outlive the iterator. */
typedef struct pqg_triplet_iter pqg_triplet_iter;
int pqg_triplet_iter_open(pqg_column_reader *cr, size_t batch_size, pqg_triplet_iter **out);
void pqg_triplet_iter_close(pqg_triplet_iter *it);
int pqg_triplet_iter_read_next(pqg_triplet_iter *it, int *has_next);
int pqg_triplet_iter_has_next(pqg_triplet_iter *it);
int16_t pqg_triplet_iter_def_level(pqg_triplet_iter *it);
int16_t pqg_triplet_iter_rep_level(pqg_triplet_iter *it);
int pqg_triplet_iter_is_null(pqg_triplet_iter *it);
int pqg_triplet_iter_value(pqg_triplet_iter *it, void *out, size_t cap, size_t *len);

/* ---------------------------------------------------------------- rows
 * Record assembly into rows: RowIter / ReaderIter over the reader tree TreeBuilder builds from the
 * file schema (record/reader.rs:38-717): optional, group, LIST (3-level and the legacy 2-level
 * forms), MAP / MAP_KEY_VALUE and unannotated repeated fields, leaf values converted by physical and
 * converted type (Field::convert_*, record/api.rs:449-555). Each leaf column chunk is decoded on
 * the GPU through a column reader (pqg_column_reader_open with `ctx`) and read through its triplet
 * iterator with `batch_size` levels per batch. row_group = -1 iterates every row group of the file
 * (RowIter::from_file), else that one (RowIter::from_row_group). */
typedef struct pqg_row_iter pqg_row_iter;
int pqg_row_iter_open(pqg_file_reader *r, int row_group, pqg_ctx *ctx, size_t batch_size, pqg_row_iter **out);
/* The same over a projection of the message's top-level fields, in the given order (fields named
 * that the schema lacks: PQG_ERR_GENERAL, "Root schema does not contain projection"). */
int pqg_row_iter_open_fields(pqg_file_reader *r, int row_group, pqg_ctx *ctx, size_t batch_size,
                             const char *const *fields, uint32_t nfields, pqg_row_iter **out);
void pqg_row_iter_close(pqg_row_iter *it);
/* The next row, rendered into buf (NUL-terminated): format 0 = the reference's Display text
 * (Row / Field fmt, record/api.rs:144-157, 557-666; dates and timestamps in UTC), 1 = JSON:
 * a row is [[name, field], ...], a field null or {"Kind": value} with Kind the Field variant name
 * (Group: fields as a row, List: [fields], Map: [[key, value], ...], Bytes: [bytes], Decimal: its
 * text). *has_row = 0 at the end. With cap too small: PQG_ERR_CAPACITY, *len = the text's length,
 * and the same row is returned by the next call. A failing column chunk ends the iteration with
 * its status (the reference panics there: read_next().unwrap(), reader.rs:400-401). */
int pqg_row_iter_next(pqg_row_iter *it, int format, char *buf, size_t cap, size_t *len, int *has_row);
const char *pqg_row_iter_error(pqg_row_iter *it);

#ifdef __cplusplus
}
#endif
#endif
