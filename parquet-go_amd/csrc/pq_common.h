// pq_common.h — POD types shared by the host planner (pq_host.cpp) and the
// HIP kernels (pq_kernels.hip).  Everything here lives in HBM as flat arrays:
// one PageDesc per page of the batch (the descriptor table), one ColDesc per
// selected leaf, one PageInfo per page (written by the device).
#pragma once
#include <stdint.h>

namespace pq {

// parquet.Encoding (parquet/parquet.go:343-354)
enum : uint8_t { ENC_PLAIN = 0, ENC_PLAIN_DICT = 2, ENC_RLE = 3, ENC_BIT_PACKED = 4, ENC_DELTA_BP = 5,
                 ENC_DELTA_LBA = 6, ENC_DELTA_BA = 7, ENC_RLE_DICT = 8 };
// parquet.Type
enum : int32_t { T_BOOLEAN = 0, T_INT32 = 1, T_INT64 = 2, T_INT96 = 3, T_FLOAT = 4, T_DOUBLE = 5,
                 T_BYTE_ARRAY = 6, T_FLBA = 7 };

enum : uint8_t { PAGE_V1 = 0, PAGE_V2 = 1, PAGE_DICT = 2 };

// Where the uncompressed values section of a page comes from.
enum : uint8_t { BODY_RAW = 0,        // uncompressed: body == payload in the input buffer
                 BODY_SNAPPY = 1,     // snappy-decoded on the GPU into staging
                 BODY_HOST = 2,       // inflated on the host (gzip / user codec), uploaded into staging
                 BODY_GZIP = 3 };     // gzip-inflated on the GPU into staging (k_inflate, pq_inflate.hip)

// Error "stages" in the reference's order of evaluation.  The reference reads
// and initialises ALL pages of a chunk (phase 1, readPages chunk_reader.go:206)
// before decoding any (phase 2, readPageData :380), so a page's status key is
// (phase, page ordinal, stage); stages < STAGE_PHASE2 are phase 1.
enum : uint32_t {
  ST_HEADER = 1,      // host: nil/negative header fields, level encodings (page_v1.go:57-86)
  ST_V2_ENC = 2,      // host: V2 value encoding (page_v2.go:95-98)
  ST_V2_LEVELS = 3,   // host: V2 level bytes ReadFull (page_v2.go:103-108)
  ST_V2_SIZE = 4,     // host: V2 negative data size (chunk_reader.go:199-201)
  ST_DECOMPRESS = 5,  // device/host: newBlockReader (compress.go:102-122)
  ST_V1_ENC = 6,      // host: V1 value encoding (page_v1.go:95-97); dict: encoding check
  ST_REP_INIT = 7,    // device: V1 rep level length (hybrid_decoder.go:57-67)
  ST_DEF_INIT = 8,
  ST_VAL_INIT = 9,    // device: values init (type_dict.go:22-37, deltabp_decoder.go:197-246)
  ST_DICT_VALUES = 9, // device: dictionary page PLAIN decode (page_dict.go:54-61)
  ST_PHASE2 = 16,
  ST_REP = 16,        // decodePackedArray(rDecoder) page_v1.go:37
  ST_DEF = 17,
  ST_VALUES = 18,     // valuesDecoder.decodeValues page_v1.go:48-52
  // device-internal: a k_decode<3> part after the first met an error; the
  // page is decoded again whole (serially) by the redo launch, which replaces
  // this with the reference's status.  Above every real stage: a real status
  // from the page's first part wins the atomicMin.
  ST_REDO = 0x7FFF,
};
__host__ __device__ inline uint32_t make_status(uint32_t stage, uint32_t code) { return (stage << 16) | code; }
// device-internal code bit: a key-stream header error found by the run walk
// (k_prepare) is set at once with this bit, so that a dictionary-index error
// k_expand finds among the values before it (same stage, plain code) wins the
// atomicMin; the host masks it off (STATUS_CODE)
// Kernels that decode a tiled page's values after the run walk (k_expand_mix,
// k_expand_wg) must therefore gate on the DICTIONARY page's status, never on
// the data page's own: a data page already holding an E_LATE status still has
// its values before the bad header decoded, so an earlier dictionary-index
// error can win (tests/test_gpu_parity.py::test_dict_index_error_before_bad_header)
constexpr uint32_t E_LATE = 0x4000u;
constexpr uint32_t STATUS_CODE = 0x3fffu;
constexpr uint32_t STATUS_OK = 0xFFFFFFFFu;

struct PageDesc {
  uint64_t src;          // offset in the device input buffer of the page payload (after the header)
  uint64_t body;         // offset of the values section: staging (SNAPPY/HOST) or input buffer (RAW)
  int32_t comp_len;      // bytes fed to the codec (V2: compressed - level bytes)
  int32_t body_len;      // expected uncompressed values-section length
  int32_t num_values;    // header num_values (level entries); dictionary: entries
  int32_t col;           // ColDesc index
  int32_t dict;          // PageDesc index of this chunk's dictionary page, -1 if none
  int32_t rg;            // row group
  int32_t ord;           // page ordinal inside its chunk (error ordering)
  uint8_t kind;          // PAGE_V1 / PAGE_V2 / PAGE_DICT
  uint8_t enc;           // value encoding (PLAIN_DICT already mapped to RLE_DICT)
  uint8_t body_src;      // BODY_*
  uint8_t train;         // SNAPPY body that is only literals: copied by k_copy from the host plan
  int32_t v2_rep_len;    // V2: rep level bytes at src
  int32_t v2_def_len;    // V2: def level bytes at src + v2_rep_len
  int64_t level_base;    // first level entry of the page inside its column (flat slot base)
  int64_t dict_base;     // BYTE_ARRAY dictionary page: first entry in the dict offsets scratch
  int64_t run_base;      // tiled RLE_DICTIONARY page: first entry of its run table (k_runs -> k_expand)
  int32_t run_cap;       // run-table entries reserved for the page (runs + sentinel)
  int32_t tile_base;     // tiled page: first entry of its tile -> first-run index table
  int32_t job_base;      // tiled page: first entry of its job -> position table (page_jobs)
  int16_t alias_any;     // dictionary page: k_snappy may alias it at any alignment (LDS-group chunks)
  int16_t srec;          // tiled PLAIN page whose k_expand records the host wrote (no k_prepare work)
  int16_t lvl_bits;      // flat page (max_rep 0, no level output): its level scratch holds a bit per
                         // level (def == max_def), LSB first from the scratch's first word, not a byte
  int16_t pad_lb;
  int32_t part0;         // list page split into k_decode<3> parts: index of its first part (-1: none);
                         // k_levels counts its streams part by part into KArgs::part_pre
  int64_t lens_base;     // BYTE_ARRAY page scratch, 2 x num_values int32 (-1: none): DELTA_(LENGTH_)BYTE_ARRAY
                         // suffix / prefix lengths; PLAIN (offset, length) per value from k_prepare's walk
  int32_t sidx;          // index in the Snappy page list (-1: not decoded by k_snappy)
  int32_t swalk;         // long PLAIN BYTE_ARRAY page: index in the region-parallel length walk (-1: none)
  int64_t sp_base;       // flat dictionary-string page split into k_decode<2> parts: first entry of its
                         // string-byte prefix table (k_prepare: bytes of values [0, 256 s)); -1: none
  int64_t lvl_base;      // page with levels on k_prepare's count path: byte offset of its decoded
                         // levels in the level scratch (rep bytes if max_rep > 0, then def bytes,
                         // num_values each); -1: k_decode reads the level streams itself
};

// Tiled flat decode (k_prepare's run walk + k_expand).  The run walk records,
// per RUN_TILE values of a page, the run holding the first of them; a k_expand
// workgroup takes 4 waves x EX_WAVE_VALUES consecutive values of one page.
constexpr int RUN_TILE = 512;
constexpr int EX_WAVE_VALUES = 2048;
// Region-parallel length-prefix walk of long PLAIN BYTE_ARRAY pages
// (type_bytearray.go:24-45): the values section is cut into SW_R-byte regions;
// k_sw_regions walks every region from a candidate entry, k_sw_link confirms
// the chain region by region (re-walking a region whose candidate was not on
// it) and counts, k_sw_emit writes each value's (offset, length).
constexpr int SW_R = 256;            // bytes per region (one lane)
constexpr int SW_MIN = 64 * 1024;    // pages whose body is at least this long
struct SwPage {
  int32_t page;   // PageDesc index
  int32_t reg0;   // first region record
  int32_t nreg;   // regions (body_len / SW_R, rounded up)
  int32_t kind;   // 0: data page (lens scratch), 1: dictionary page (entry table)
};
struct SwReg {     // one region: [start, start + SW_R) of the values section
  int32_t c;       // k_sw_regions: candidate entry (values offset, -1: none); k_sw_link: the true entry
  int32_t x;       // the chain's exit (first entry at or past the region end)
  int32_t cnt;     // entries whose header starts in the region, before an error
  uint32_t err;    // first error on the chain (0: none), after cnt entries
  int64_t lsum;    // their string bytes
  int32_t base;    // k_sw_link: value index of the region's first entry (-1: nothing to emit)
  int32_t pad;
};
struct SwRes {     // per page, k_sw_link -> k_prepare / k_dict_prepare / k_sw_emit
  uint32_t err;    // the walk's error (0: none)
  int32_t n;       // entries read (the page's non-null values)
  int64_t sbytes;  // their string bytes
  int32_t treg;    // the region holding the n-th entry (k_sw_emit adds its part of sbytes)
  int32_t pad;
};
// k_reset: a device buffer zeroed at the start of every decode
// k_nest_count / k_nest_write (pq_nest.hip): the list structure of a column
// with max_rep >= 2 from its decoded levels.  Per level entry i, flag f_0 =
// rep == 0 (a row: a level-1 list starts) and f_k = rep <= k && def >=
// rdef[k] (an element of a level-k list, k = 1..max_rep; f_k also starts a
// level-(k+1) list).  Level k's offsets: at the j-th f_(k-1) entry, the
// number of f_k entries before it; its validity: def >= rdef[k] - 1.  The
// leaf slots (f_max_rep entries): validity def == max_def.
constexpr int NEST_MAXR = 8;
constexpr int NEST_CH = 4096;  // level entries a block
struct NestArgs {
  const uint8_t *def, *rep;
  int64_t n;
  int32_t max_rep, max_def;
  int32_t rdef[NEST_MAXR + 1];  // rdef[k]: def level of the k-th repeated ancestor
  int32_t *sums;                // per block: counts of f_0 .. f_max_rep
  int32_t *off;                 // level k's offsets at off + ostride * (k - 1)
  uint32_t *val;                // level k's validity at val + vstride * (k - 1); the leaf slots' at k = max_rep + 1
  int64_t ostride, vstride;
  int64_t *cnt;                 // totals of f_0 .. f_max_rep
  int32_t nblocks;
};

// k_inflate's arguments (pq_inflate.hip): the gzip pages, one wave each.
struct InflateArgs {
  const uint8_t *in;
  uint8_t *stage;
  const PageDesc *pages;
  uint32_t *status;
  const int32_t *list;
  int32_t n;
};

struct ZeroRange {
  uint32_t *ptr;
  uint64_t words;
};

// k_expand_ld: one workgroup per group of consecutive jobs of one column
// chunk, whose dictionary it holds in LDS (host-built)
constexpr int LD_WAVES_H = 4;             // waves of a k_expand_mix workgroup
constexpr int LD_LDS_MAX = 160 * 1024;    // LDS of one CU (gfx950)
constexpr int LD_MIX_MAX = 32 * 1024;     // k_expand_mix LDS per workgroup with a dictionary (default)
// k_expand_wg: chunks whose dictionary is past the mixed launch's LDS groups,
// up to WG_MAX_SLICES slices of a CU's LDS (a workgroup of 16 waves a CU);
// groups of WG_JOBS jobs by default
#ifndef PQ_WG_WAVES
#define PQ_WG_WAVES 16
#endif
constexpr int WG_WAVES = PQ_WG_WAVES;
constexpr uint32_t WG_SLICE = 160 * 1024;  // LDS bytes of a slice (the CU's LDS)
constexpr int WG_MAX_SLICES = 4;
constexpr int WG_JOBS = 64;
constexpr int PLAIN_STR_ITEM = 2048;      // k_plain_str: values per work item
constexpr int STR_PART = 2048;            // k_decode<2>: level entries per part of a split dictionary-string page
struct LdsGroup {
  int32_t job0, njobs;   // jobs [job0, job0 + njobs) of the launch order
  int32_t dpage;         // the chunk's dictionary page; -1: one job per wave, L1/L2 gathers
  int32_t dict_bytes;    // LDS bytes reserved for the dictionary (16-byte multiple)
  int32_t kspan;         // LDS bytes of staged key bytes per wave (1 KiB multiple)
  int32_t pad[3];
};

struct TileJob {         // one k_expand workgroup (host-built, XCD-affine order)
  uint8_t *out;          // the page's first output value
  int32_t page;          // PageDesc index
  int32_t dict;          // its dictionary page, -1 if none
  int32_t v0;            // first value of the job (page-relative)
  int32_t tf;            // tile_first index of the job's first value (RUN_TILE granularity)
  int32_t width;         // value bytes (4 / 8)
  int32_t pad;
};
// What k_expand needs about one job, written by k_prepare at the job's
// position in the launch order (one 64-byte scalar load).  A record is
// current only when `epoch` matches the decode's epoch: a page that failed
// before k_prepare leaves stale records, which k_expand skips.
struct ExRec {
  const uint8_t *vals;   // values section (PLAIN values; RLE_DICTIONARY: bit-width byte, then keys)
  const uint8_t *dict;   // dictionary values
  const uint2 *runs;     // the page's run table
  int32_t v0, lim;       // decode values [v0, lim) of the page (lim <= v0: nothing)
  int32_t bw;            // key bit width; -1: PLAIN
  int32_t nr;            // run entries (the sentinel is entry nr)
  int32_t first_run;     // run holding value v0
  int32_t byte_lo, byte_hi;  // key-stream bytes holding keys [v0, lim) (byte_hi exclusive, before slack)
  uint32_t dict_n;       // dictionary entries
  uint32_t epoch;
  int32_t val_len;       // values section bytes
};
static_assert(sizeof(ExRec) == 64, "one scalar load");
// ExRec::epoch of a record the host wrote once (a tiled PLAIN page: nothing
// about it depends on the data), current in every decode
constexpr uint32_t EPOCH_STATIC = 0xFFFFFFFFu;
__host__ __device__ inline bool rec_live(uint32_t rec_epoch, uint32_t epoch) {
  return rec_epoch == epoch || rec_epoch == EPOCH_STATIC;
}

// One RLE/bit-packed run of a key stream (hybrid_decoder.go:143-166), as
// written by k_runs: x = first value (page-relative) | RUN_RLE for an RLE run;
// y = the repeated value (RLE) or the byte offset of the run's packed data in
// the key stream (bit-packed).
constexpr uint32_t RUN_RLE = 0x80000000u;

struct ColDesc {
  int32_t ptype, width;        // physical type, bytes per value (0 = BYTE_ARRAY)
  int32_t max_def, max_rep, rep_def;
  int32_t page_begin, page_end; // pages of this column in the table (all row groups)
  int32_t flags;
  // outputs (device pointers)
  uint8_t *values;
  uint32_t *validity;
  int32_t *list_offsets;
  uint32_t *list_validity;
  int64_t *str_offsets;
  uint8_t *def_out, *rep_out;
  int64_t total_levels, total_slots, total_rows, total_str;
};
enum : int32_t { COL_NEEDS_COUNT = 1, COL_EMIT_LEVELS = 2 };

// Written by the device.  Offsets are relative to the level source (V1: the
// uncompressed body; V2: the payload) or to the body (values).
struct PageInfo {
  int32_t rep_off, rep_len;
  int32_t def_off, def_len;
  int32_t val_off, val_len;
  int32_t idx_bw;
  int32_t pad;
  int64_t rows, slots, non_null, str_bytes;  // counts (prepare)
  int64_t row_base, slot_base, str_base;     // exclusive scans over the column's pages
  int64_t alias1;  // k_snappy: 1 + input offset of the body when the block is one literal (0: none)
  int32_t cover;      // k_runs: values decodable before the first key-stream header error (n when none)
  uint32_t walk_err;  // k_runs: that header error (0: none); applied by k_level_check unless a
                      // dictionary error among the first `cover` values came first
  int32_t str_data;   // DELTA string pages: values-section offset of the first suffix byte
  int32_t str_cnt;    // DELTA string pages: decoded length entries (valuesCount)
};

}  // namespace pq
