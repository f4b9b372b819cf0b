// file_reader.hpp — host-side parquet::file::reader surface (src/file/reader.rs:51-530):
// footer + thrift-compact FileMetaData, schema -> leaf column descriptors with max def/rep
// levels (schema/types.rs:737-793), and the SerializedPageReader loop (page headers,
// decompression, uncompressed page payloads). No decoding happens here: pages go to the GPU.
#pragma once
#include <stdint.h>

#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../../include/pqgpu.h"

namespace pqg {

struct SchemaNode {
  std::string name;
  int type = -1;            // physical type or -1 for groups
  int type_length = 0;
  int repetition = 0;       // 0 REQUIRED, 1 OPTIONAL, 2 REPEATED
  int num_children = 0;
  int converted_type = -1;
  int scale = 0, precision = 0;  // DECIMAL
};

struct LeafColumn {
  std::string path;
  int physical_type;
  int type_length;
  int16_t max_def, max_rep;
};

struct ColumnChunkMeta {
  int type = 0;
  int codec = 0;
  int64_t num_values = 0;
  int64_t total_compressed_size = 0;
  int64_t total_uncompressed_size = 0;
  int64_t data_page_offset = 0;
  bool has_dict_offset = false;
  int64_t dictionary_page_offset = 0;
  std::vector<int> encodings;
  std::vector<std::string> path;
};

struct RowGroupMeta {
  int64_t num_rows = 0;
  int64_t total_byte_size = 0;
  std::vector<ColumnChunkMeta> columns;
};

struct FileMeta {
  int32_t version = 0;
  int64_t num_rows = 0;
  std::string created_by;
  std::vector<SchemaNode> schema;
  std::vector<LeafColumn> leaves;
  std::vector<RowGroupMeta> row_groups;
};

struct PageHeaderInfo {
  int type = -1;
  int32_t uncompressed_size = 0, compressed_size = 0;
  // data page v1/v2, dictionary page
  int32_t num_values = 0, encoding = 0, def_encoding = 0, rep_encoding = 0;
  int32_t num_nulls = 0, num_rows = 0, def_len = 0, rep_len = 0;
  bool is_compressed = true, is_sorted = false;
  bool has_v1 = false, has_v2 = false, has_dict = false;
};

// Parses the footer and metadata; returns 0 or a PQG_ERR_* status with `err` set.
int parse_file_metadata(const uint8_t* data, uint64_t len, FileMeta& meta, std::string& err);
int parse_page_header(const uint8_t* p, uint64_t avail, PageHeaderInfo& h, uint64_t& used,
                      std::string& err);

// One page of a column chunk as found in the file: where its (possibly compressed) payload is
// and where it goes in the chunk's blob of uncompressed payloads (page.offset, 64-byte aligned).
struct PagePlan {
  const uint8_t* src;  // payload in the file (v2: level bytes, then the values)
  uint64_t prefix;     // data page v2: level bytes, stored uncompressed
  uint64_t clen;       // stored bytes after the prefix
  bool decompress;
  pqg_page page;       // offset relative to the chunk blob; nbytes uncompressed
};

// The page walk without the copies: headers parsed, pages planned (blob_len = the chunk blob's
// size with tail slack). fill_page then copies / decompresses one page into the blob; pages are
// independent, so a row group's pages fill in parallel.
int plan_chunk_pages(const uint8_t* file, uint64_t file_len, const ColumnChunkMeta& cc,
                     std::vector<PagePlan>& plan, uint64_t& blob_len, std::string& err);
int fill_page(const PagePlan& pp, int codec, uint8_t* chunk_blob, std::string& err);

// Reads every page of one column chunk (SerializedPageReader::get_next_page loop,
// file/reader.rs:420-522): the uncompressed payloads are appended to `blob` at 64-byte aligned
// offsets and described in `pages`.
int read_chunk_pages(const uint8_t* file, uint64_t file_len, const ColumnChunkMeta& cc,
                     std::vector<uint8_t>& blob, std::vector<pqg_page>& pages, std::string& err);

// Decompression (compression.rs:54-80): SNAPPY (raw), GZIP; other codecs -> NYI.
int decompress(int codec, const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_len,
               std::string& err);

struct ChunkPages {
  std::vector<uint8_t> blob;
  std::vector<pqg_page> pages;
  int status = 0;
  std::string err;
};

}  // namespace pqg

// SerializedFileReader (file/reader.rs:140-250): the file bytes (mapped, or owned for
// pqg_file_open_memory), its metadata, and the column chunks read so far by pqg_chunk_* /
// pqg_column_reader_open.
// Staging of the column readers of one file (pqg_column_reader_open): pinned page bytes, device
// blob and outputs, pinned output copies, and the stream they move on; grown, never shrunk.
struct ColumnStaging;

struct pqg_file_reader {
  ColumnStaging* staging = nullptr;
  std::vector<uint8_t> owned;
  void* map = nullptr;
  size_t map_len = 0;
  const uint8_t* data = nullptr;
  uint64_t len = 0;
  pqg::FileMeta meta;
  std::string err;
  std::map<std::pair<int, int>, std::unique_ptr<pqg::ChunkPages>> chunks;
  ~pqg_file_reader();
};
