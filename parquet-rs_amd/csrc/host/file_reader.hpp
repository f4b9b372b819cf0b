// file_reader.hpp — host-side parquet::file::reader surface (src/file/reader.rs:51-530):
// footer + thrift-compact FileMetaData, schema -> leaf column descriptors with max def/rep
// levels (schema/types.rs:737-793), and the SerializedPageReader loop (page headers,
// decompression, uncompressed page payloads). No decoding happens here: pages go to the GPU.
#pragma once
#include <stdint.h>

#include <string>
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

// Reads every page of one column chunk (SerializedPageReader::get_next_page loop,
// file/reader.rs:420-522): the uncompressed payloads are appended to `blob` at 64-byte aligned
// offsets and described in `pages`.
int read_chunk_pages(const uint8_t* file, uint64_t file_len, const ColumnChunkMeta& cc,
                     std::vector<uint8_t>& blob, std::vector<pqg_page>& pages, std::string& err);

// Decompression (compression.rs:54-80): SNAPPY (raw), GZIP; other codecs -> NYI.
int decompress(int codec, const uint8_t* in, uint64_t in_len, uint8_t* out, uint64_t out_len,
               std::string& err);

}  // namespace pqg
