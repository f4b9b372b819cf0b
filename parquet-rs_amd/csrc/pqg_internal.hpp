// pqg_internal.hpp — structures shared by the host driver (chunk_decoder.cpp) and the
// CDNA4 kernels (device/*.hip). Not part of the public C ABI (include/pqgpu.h).
#pragma once
#include <stdint.h>

#include <hip/hip_runtime.h>  // uint2

namespace pqg {

// Status codes: ParquetError kinds (src/errors.rs:24-51) plus the two outcomes the reference
// reaches on malformed input (a panic, an endless loop). Mirrors include/pqgpu.h.
enum Status : int32_t {
  ST_OK = 0,
  ST_GENERAL = 1,
  ST_NYI = 2,
  ST_EOF = 3,
  ST_PANIC = 4,  // reference would panic (assert!/bounds)
  ST_HANG = 5,   // reference would loop forever (rle.rs:414-425, column/reader.rs:182-262)
  ST_CAPACITY = 6,
  ST_INVALID_ARG = 7,
  ST_HIP = 8,
};

enum PhysType : int32_t {
  T_BOOLEAN = 0, T_INT32 = 1, T_INT64 = 2, T_INT96 = 3, T_FLOAT = 4, T_DOUBLE = 5,
  T_BYTE_ARRAY = 6, T_FLBA = 7
};

enum Enc : int32_t {
  E_PLAIN = 0, E_PLAIN_DICTIONARY = 2, E_RLE = 3, E_BIT_PACKED = 4, E_DELTA_BINARY_PACKED = 5,
  E_DELTA_LENGTH_BYTE_ARRAY = 6, E_DELTA_BYTE_ARRAY = 7, E_RLE_DICTIONARY = 8
};

enum PageType : int32_t { P_DATA = 0, P_INDEX = 1, P_DICTIONARY = 2, P_DATA_V2 = 3 };

enum LevelKind : uint8_t { LK_NONE = 0, LK_RLE = 1, LK_BIT_PACKED = 2 };

// Per-page working record in device memory. The host fills the first block from the page
// headers; the prepare kernel fills the stream layout; later kernels fill counts.
struct PageWork {
  // ---- host-filled
  uint64_t base;        // byte offset of the uncompressed payload inside the chunk blob
  uint32_t nbytes;      // payload length
  uint32_t num_values;  // header num_values (levels for data pages, entries for dict pages)
  uint64_t level_out;   // index of this page's first level in the level outputs
  int32_t page_type;
  int32_t encoding;
  int32_t def_encoding;
  int32_t rep_encoding;
  uint32_t def_len;     // v2
  uint32_t rep_len;     // v2
  uint32_t ltile0;      // first expand tile of this page (tiles of RUN_TILE levels)
  uint32_t ntiles;      // expand tiles of this page (0 for dictionary pages)
  // ---- prepare kernel
  uint32_t rep_off, rep_bytes;  // level streams, relative to base
  uint32_t def_off, def_bytes;
  uint32_t val_off, val_bytes;  // value section
  uint8_t rep_kind, def_kind, value_kind, pad0;
  int32_t status;
  // ---- levels kernel / scan
  uint64_t nonnull;     // values this page must yield (def == max_def count, or num_values)
  uint64_t value_out;   // index of this page's first value in its chunk's value output
  uint64_t byte_out;    // BYTE_ARRAY/FLBA: first byte of this page's values in the byte output
  uint64_t nbytes_out;  // BYTE_ARRAY/FLBA: bytes this page produces
  // ---- speculative PLAIN copy (ChunkWork::spec): the values the page's value section holds
  // (val_bytes / es, set by k_prepare) and their chunk-exclusive prefix (k_spec_scan)
  uint64_t spec_n;
  uint64_t spec_out;
  // ---- host-filled
  uint32_t chunk;       // the column chunk of the batch this page belongs to (ChunkWork index)
  // ---- level path: 1 when nbytes_out is the sum of the page's tile byte sums (k_ba_tsum adds
  // them): the byte-array dictionary emit writes entry indices only
  uint32_t tile_bytes;
};

// Chunk-level result, copied to pinned host memory at the end of a decode.
// Scalar state k_prepare sets before any other kernel of the decode runs (in place of memset
// launches): counters to a value, per-page flag arrays to 0, and the dictionary page check of
// fixed-width dictionaries (dict_es: value size, 0 = none; decoding.rs:282-288, :145-147).
struct PrepInit {
  uint32_t* word[8];
  uint32_t val[8];
  uint32_t* pzero[3];
  // level-path density probe (LevelTables::dense) of the def / rep streams, run by k_prepare's
  // wave right after it locates them; dense_zero: a stream kind's array cleared instead
  uint32_t* dense_def;
  uint32_t* dense_rep;
  uint32_t* dense_zero;
};

struct ChunkResult {
  uint64_t total_levels;
  uint64_t total_values;
  uint64_t total_bytes;
  uint64_t bad;            // lowest failing page (chunk-relative) and its status: (page << 32) | status;
                           // ~0 when clean
};

// Outputs per expand tile of the RLE/bit-packed hybrid decoder (device/pqg_runs.hpp).
constexpr uint32_t RUN_TILE = 4096;

// Run records kept per expand tile by the index pass (more runs: the expand pass re-walks the
// tile from its checkpoint).
constexpr uint32_t RUN_CAPT = 512;

// Walk checkpoint of one expand tile: the header of the run holding the tile's first output.
struct RunCkpt {
  uint32_t pos;    // stream-relative byte offset of the run header
  uint32_t first;  // page-relative index of the run's first output
};

// Everything the expand pass needs about one quarter tile (RUN_TILE / 4 outputs), gathered by
// k_quarter_desc (64 bytes).
struct QDesc {
  uint64_t S;        // absolute blob offset of the stream
  uint64_t out;      // global index of the stream's output 0 (page output base)
  uint32_t qlo, qhi; // page-relative outputs [qlo, qhi); qhi == 0: nothing to do
  uint32_t rec;      // first run record (index into RunTables::runs), RUN_REWALK: re-walk
  uint32_t nrec;     // run records overlapping the quarter
  uint32_t blo, bhi; // stream bytes holding the quarter's bit-packed payload (bhi == 0: none)
  uint32_t slen;     // stream bytes
  uint32_t w;        // bit width
  uint32_t kind;     // LK_RLE / LK_BIT_PACKED
  uint32_t page;
  uint32_t ckpos;    // re-walk: checkpoint header and its run's first output
  uint32_t ckfirst;
};
constexpr uint32_t RUN_REWALK = 0xFFFFFFFFu;

// Index-pass outputs of one stream kind, indexed by expand tile.
struct RunTables {
  RunCkpt* ck;      // [tiles + 1]
  uint2* runs;      // [tiles * RUN_CAPT]
  uint32_t* nruns;  // [tiles]
  QDesc* desc;      // [tiles * 4]
  uint32_t* qcount; // [tiles * 4] per quarter-tile counts (def levels == max_def; byte totals)
  uint32_t* pflag;  // [pages] PF_PAGE: stream decoded by the level path (pqg_levels.hip)
  uint32_t* nfall;  // streams the level path left to the tiled path (0: its kernels exit at once)
  uint32_t* hard;   // [2 + tiles]: windowed-gather tiles k_dict_win leaves to k_texpand_didx (counts, lists)
};

// DELTA_BINARY_PACKED index-pass outputs (device/pqg_delta.hip). Tiles of DELTA_TILE values
// per page; each tile keeps the records of the blocks its values need.
constexpr uint32_t DELTA_TILE = 4096;
constexpr uint32_t DELTA_BCAP = 64;   // block records per tile (more: per-page fallback kernel)
constexpr uint32_t DELTA_MBMAX = 16;  // mini-blocks per block on the tiled path

struct DeltaBlock {
  uint32_t wpos;      // stream offset of the block's mini-block width bytes
  uint32_t pos;       // stream offset of its first mini-block
  uint64_t min_delta;
  uint8_t w[DELTA_MBMAX];  // mini-block bit widths (the expand pass needs no second round trip)
};

struct DeltaPage {
  uint64_t first;     // first value (zigzag-decoded)
  uint32_t vpmb;      // values per mini-block
  uint32_t nmb;       // mini-blocks per block
  uint32_t tiled;     // 1: tiles/records valid; 0: decode with the per-page kernel
  uint32_t pad;
};

struct DeltaTables {
  DeltaPage* page;    // [npages]
  DeltaBlock* blocks; // [tiles * DELTA_BCAP]
  uint64_t* agg;      // [tiles] tile sums (decoupled look-back)
  uint64_t* inc;      // [tiles] inclusive prefixes
  uint32_t* flag;     // [tiles] epoch * 4 + {1 aggregate, 2 inclusive}
  uint64_t* dbg;      // diagnostics: per-page phase cycles of k_delta_page (PQG_DEBUG bit 5)
  uint32_t* nfall;    // pages k_delta_page left to the tiled path (0: its tile kernels exit at once)
};

// Level-path tables (device/pqg_levels.hip), per stream kind (def, rep, RLE booleans).
// One segment (lw_segw(w) windows of 1 KiB: ~16 KiB of one-bit levels, more for wider
// streams, whose runs are longer) of a sparse hybrid stream, walked by its own wave
// (pqg_levels.hip); it records at most LW_SCAP runs (room for a walk through two segments).
constexpr uint32_t LW_SEGW = 16;
constexpr uint32_t LW_SCAP = 64 * (2 * LW_SEGW + 2);
__host__ __device__ inline uint32_t lw_segw(uint32_t w) { return w <= 4 ? LW_SEGW : w <= 8 ? 4 * LW_SEGW : 16 * LW_SEGW; }
struct LvSeg {
  uint64_t out;       // outputs of the runs the segment's walk recorded
  uint64_t base_out;  // (page scan) outputs before the segment
  uint32_t runs;      // runs recorded
  uint32_t status;    // how the walk ended (LS_* in pqg_levels.hip)
  uint32_t next;      // LS_LANDED: the segment whose start the walk reached
  uint32_t lastpos;   // stream offset of the last recorded header
  uint32_t base_run;  // (page scan) runs before the segment
  uint32_t keep;      // (page scan) runs the page keeps (the last segment stops at the n-th output)
  uint32_t prevpos;   // (page scan) last header before the segment's first one (~0u: none)
  uint32_t flags;     // (page scan) 1: on the page's chain, 2: its last segment
  uint32_t tv, tc;    // a truncated last run: payload offset and output count
};

// Windows are 1 KiB of a page's stream; run records of walked pages are 64 per window + 128.
struct LevelTables {
  uint32_t* wbase;   // [pages + 1] first window of each page's stream (k_lv_plan)
  uint32_t* sbase;   // [pages + 1] first segment of each page's stream (k_lv_plan)
  uint32_t* bexit;   // [segments] where every chain entering a segment's first window leaves it
  LvSeg* seg;        // [segments]
  uint2* srec;       // [segments * LW_SCAP] runs recorded by each segment walk: (outputs before, info)
  uint32_t* spos;    // [segments * LW_SCAP] their header offsets
  uint32_t* wbase2;  // [pages + 1] the same over the pages the walker left to the window path
  uint32_t* wfirst;  // [windows + pages] walked pages: first run of each window, then the run count
  uint2* rec;        // [64 * (windows + 2 * pages)] walked pages' runs: (first output, info)
  uint2* tab;        // [windows * tstride] per window and entry offset: (exit offset, outputs)
  uint2* win;        // [windows] (true entry offset | LV_NONE, first output) (k_lv_stitch)
  uint16_t* bmp;     // [windows * 64] bit width 1: per segment of 16 bytes, the headers of the
                     // window's reference chain (k_lv_win), for k_lv_emit
  uint32_t* dense;   // [pages] 1: the stream's first 64 headers lie within 1 KiB (k_lv_probe): the
                     // window path takes it without a segment walk
  uint32_t* ctr;     // [16] last-workgroup tickets (zero between launches): [0] k_lv_segscan,
                     // [1] k_lv_fallback, [2] k_lv_plan
  uint32_t tstride;  // tab entries per window: lv_ent of the widest stream of the decode (the
                     // streams of a batch's chunks may differ in bit width)
  uint32_t* bail;    // PQG_DIAG builds, PQG_DEBUG 512: per page, where the level path handed it back
};

// RunTables::pflag values: stream decoded by the level path (pqg_levels.hip) — by its window
// kernels (PF_PAGE), after its page walker (PF_WALK) or, dense one-bit levels, by its chunk walks
// (pqg_lvd1.hpp, PF_D1) — or handed back by it to the general hybrid decoder (pqg_runs.hpp, PF_BAIL)
constexpr uint32_t PF_PAGE = 1u, PF_BAIL = 2u, PF_WALK = 3u, PF_D1 = 4u;
__host__ __device__ inline bool pf_level_path(uint32_t f) { return f == PF_PAGE || f == PF_WALK || f == PF_D1; }

struct ColumnParams {
  int32_t physical_type;
  int32_t type_length;
  int16_t max_def;
  int16_t max_rep;
  int32_t def_bit_width;
  int32_t rep_bit_width;
  int32_t want_def;  // def_levels output provided (read_batch(Some(def)))
  int32_t want_rep;
  int32_t debug;     // diagnostics switches (PQG_DEBUG), 0 in production
  uint32_t dict_maxw;  // widest dictionary index stream the hybrid-stream path takes
  uint64_t* dbgbuf;  // diagnostics: per-wave s_memtime phases (PQG_DEBUG bit 4)
};

// One column chunk of a decode (pqg_decode_chunk: one; pqg_decode_chunks: a batch of column
// chunks, e.g. every chunk of one or more row groups, decoded by one pass of every kernel). Its
// pages are [first_page, first_page + npages) of the decode's page table; outputs are the
// caller's, indexed by the pages' chunk-relative level_out / value_out / byte_out.
struct ChunkWork {
  ColumnParams cp;
  int16_t* def_out;
  int16_t* rep_out;
  uint8_t* val_out;      // fixed-width values / byte-array bytes
  int64_t* off_out;      // byte-array offsets
  uint64_t val_cap;      // bytes val_out holds
  uint64_t scr_base;     // byte arrays: first per-value slot of this chunk in the source/length scratch
  uint64_t dscr_base;    // byte arrays: first dictionary-entry slot in the dictionary scratch
  int32_t dict_page;     // page-table index of the chunk's dictionary page, or -1
  int32_t es;            // fixed value size in bytes (0: BYTE_ARRAY / FLBA)
  int32_t dict_es;       // k_prepare's fixed-width dictionary page check: value size, 0 = none
  uint32_t first_page;
  uint32_t npages;
  uint32_t lvdict;       // 1: its dictionary indices take the hybrid-stream (level) path
  uint32_t spec;         // 1: its PLAIN values are copied at speculative offsets beside the level decode
  uint32_t spec_bad;     // set by the value-offset scan when a speculative offset or count was wrong
  ChunkResult res;       // filled by the kernels, copied back after the decode
};

}  // namespace pqg
