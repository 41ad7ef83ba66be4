/*
 * pqgpu.h — C ABI of libpqgpu.so, the MI355X-native Parquet column-chunk decoder.
 *
 * This is the drop-in boundary for the read/decode path of kmatt/parquet-go
 * (module github.com/fraugster/parquet-go).  Plain pointers and sizes only; no
 * C++ or torch types cross it.  INTEGRATION.md shows the cgo binding a Go
 * maintainer would add on top of it.
 *
 * Entry points and the reference interface each one replaces:
 *
 *   pqg_register_block_compressor   RegisterBlockCompressor        compress.go:130-135
 *   pqg_get_registered_codecs       GetRegisteredBlockCompressors  compress.go:139-150
 *   pqg_decompress_block            BlockCompressor.DecompressBlock compress.go:24-27
 *                                   + newBlockReader size check     compress.go:102-122
 *   pqg_file_open_path / _buffer    NewFileReader + readFileMetaData file_reader.go:27, file_meta.go:14-62
 *   pqg_file_num_rows               FileReader.NumRows              file_reader.go:134
 *   pqg_file_row_group_count        FileReader.RowGroupCount        file_reader.go:129
 *   pqg_file_row_group_num_rows     FileReader.RowGroupNumRows      file_reader.go:60-67
 *   pqg_file_column_count/_info     SchemaReader.Columns, Column.MaxDefinitionLevel/
 *                                   MaxRepetitionLevel/FlatName     schema.go:70-101, :960-983
 *   pqg_file_find_column            SchemaReader.GetColumnByName    schema.go:977-983
 *   pqg_batch_create + _decode      FileReader.PreLoad/readRowGroup file_reader.go:51-57, :116;
 *                                   chunk_reader.go:404-431 (readChunk/readPages/readPageData)
 *   pqg_batch_column / _copy        ColumnStore values + levels     data_store.go:15-31, :158-203
 *
 * Threading: one pqg_ctx per GPU; contexts are independent; a ctx and the
 * batches made from it are used by one host thread at a time (the reference
 * FileReader is likewise not safe for concurrent use).  The codec registry is
 * process-global and guarded like compress.go:16-19 (reader lock held during a
 * host decompression call, so registered callbacks must be re-entrant).
 *
 * Errors: every call returns a pqg_status; pqg_last_error() returns the text.
 */
#ifndef PQGPU_H
#define PQGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: pqg_batch_stats_get takes the caller's sizeof(pqg_batch_stats) (the
 *    struct grew six doubles in version 1's lifetime; a size-less call could
 *    overrun an older caller's struct). */
#define PQGPU_ABI_VERSION 2

/* Status / error classes (same numbering as the oracle, oracle/pqref.h). */
typedef enum {
  PQG_OK = 0,
  PQG_ERR_ARG = 1,
  PQG_ERR_FORMAT = 2,       /* magic / footer length            file_meta.go:14-62 */
  PQG_ERR_THRIFT = 3,       /* compact-thrift decode            helpers.go:101-107 */
  PQG_ERR_SCHEMA = 4,       /* schema.go:789-1000 */
  PQG_ERR_CODEC = 5,        /* codec not registered             compress.go:90-100 */
  PQG_ERR_ENCODING = 6,     /* unsupported encoding             chunk_reader.go:58-196, :348-364 */
  PQG_ERR_SNAPPY = 7,       /* snappy ErrCorrupt */
  PQG_ERR_SIZE = 8,         /* size checks                      compress.go:108-119, chunk_reader.go:198-204 */
  PQG_ERR_PAGE = 9,         /* page header checks               page_v1.go:79-86, page_v2.go:73-89, page_dict.go:30-41 */
  PQG_ERR_EOF = 10,         /* level/value stream ended early */
  PQG_ERR_RLE = 11,         /* hybrid_decoder.go:127-129, :154-161 */
  PQG_ERR_DICT_INDEX = 12,  /* type_dict.go:51-53 */
  PQG_ERR_DELTA = 13,       /* deltabp_decoder.go header checks */
  PQG_ERR_BYTE_ARRAY = 14,  /* type_bytearray.go:31-36 */
  PQG_ERR_BITWIDTH = 15,    /* type_dict.go:28-30, deltabp_decoder.go:262-264 */
  PQG_ERR_NO_DICT = 16,     /* type_dict.go:40-42 */
  PQG_ERR_DEVICE = 17,      /* HIP runtime failure */
  PQG_ERR_COUNT = 18,       /* chunk_reader.go:389-391 */
  PQG_ERR_UNSUPPORTED = 19  /* outside the decoder's scope (BOOLEAN, DELTA_*_BYTE_ARRAY, ...) */
} pqg_status;

/* parquet.CompressionCodec (parquet/parquet.go:442-451) */
enum { PQG_CODEC_UNCOMPRESSED = 0, PQG_CODEC_SNAPPY = 1, PQG_CODEC_GZIP = 2, PQG_CODEC_LZO = 3,
       PQG_CODEC_BROTLI = 4, PQG_CODEC_LZ4 = 5, PQG_CODEC_ZSTD = 6, PQG_CODEC_LZ4_RAW = 7 };

/* parquet.Type (parquet/parquet.go) */
enum { PQG_BOOLEAN = 0, PQG_INT32 = 1, PQG_INT64 = 2, PQG_INT96 = 3, PQG_FLOAT = 4,
       PQG_DOUBLE = 5, PQG_BYTE_ARRAY = 6, PQG_FIXED_LEN_BYTE_ARRAY = 7 };

typedef struct pqg_ctx pqg_ctx;
typedef struct pqg_file pqg_file;
typedef struct pqg_batch pqg_batch;

/* ---- context ----------------------------------------------------------- */
int pqg_ctx_create(int device, pqg_ctx **out);
/* Destroys the context and releases the device's idle cached buffers. */
void pqg_ctx_destroy(pqg_ctx *ctx);
/* Device buffers of destroyed batches are kept per device for reuse (at most
   PQG_DEV_CACHE_MB, default min(1/8 of device memory, 8 GiB)); this frees the
   idle ones of `device` (-1: every device) for other allocators.  No
   reference counterpart (the Go reader allocates per page). */
int pqg_release_cache(int device);
/* HIP stream the context launches on (hipStream_t as void*). */
void *pqg_ctx_stream(pqg_ctx *ctx);
/* Copies the calling thread's / context's last error text into buf. */
int pqg_last_error(pqg_ctx *ctx, char *buf, size_t cap);
/* Number of HIP devices visible (0 when no GPU). */
int pqg_device_count(void);
int pqg_abi_version(void);

/* ---- codec registry (compress.go) -------------------------------------- */
/* Host decompressor callback: same contract as BlockCompressor.DecompressBlock,
 * with caller-owned output.  Return 0 and *out_len, or a nonzero pqg_status. */
typedef int (*pqg_decompress_fn)(void *user, const uint8_t *src, size_t src_len, uint8_t *dst, size_t dst_cap,
                                 size_t *out_len);
/* Register (or replace) a host decompressor for `codec`.  Passing fn == NULL
 * restores the built-in (UNCOMPRESSED: passthrough, SNAPPY: the GPU kernel,
 * GZIP: host zlib inflate). */
int pqg_register_block_compressor(int codec, pqg_decompress_fn fn, void *user);
/* Fills codecs[0..cap) with the registered codec ids; returns how many exist. */
int pqg_get_registered_codecs(int *codecs, int cap);
/* Decompress one block, with the caller-side size check of newBlockReader
 * (compress.go:117-119): the result must be exactly `expect_len` bytes, else
 * PQG_ERR_SIZE.  SNAPPY runs on the context's GPU; the others on the host. */
int pqg_decompress_block(pqg_ctx *ctx, int codec, const uint8_t *src, size_t src_len, uint8_t *dst, size_t dst_cap,
                         size_t expect_len, size_t *out_len);

/* ---- file (file_reader.go, file_meta.go, schema.go) --------------------- */
typedef struct {
  char name[512];           /* dotted flat name (Column.FlatName, schema.go:811-815) */
  int32_t physical_type;    /* PQG_INT32 ... */
  int32_t type_length;      /* FIXED_LEN_BYTE_ARRAY length */
  int32_t max_def;          /* Column.MaxDefinitionLevel */
  int32_t max_rep;          /* Column.MaxRepetitionLevel */
  int32_t rep_def;          /* definition level of the repeated ancestor (0 if none) */
  int32_t converted_type;   /* -1 if absent */
  int32_t unsigned_int;     /* INT32/INT64 read as unsigned (chunk_reader.go:29-50) */
  int32_t value_width;      /* bytes per decoded value (0 for BYTE_ARRAY) */
} pqg_column_info;

int pqg_file_open_path(const char *path, pqg_file **out);
/* Many files' footers parsed in parallel (a dataset of
 * many files before its row groups are sharded): out[i] is the opened file or
 * NULL; returns the first failing file's status (its index in *failed) or
 * PQG_OK.  threads <= 0: one per file up to the host's cores.  The reference
 * opens one file per NewFileReader (file_reader.go:27, file_meta.go:14-62). */
int pqg_file_open_many(const char *const *paths, int n, int threads, pqg_file **out, int *failed);
/* `data` must stay valid while the file is open unless `copy` is nonzero. */
int pqg_file_open_buffer(const uint8_t *data, size_t len, int copy, pqg_file **out);
void pqg_file_close(pqg_file *f);
int64_t pqg_file_num_rows(const pqg_file *f);
int pqg_file_row_group_count(const pqg_file *f);
int64_t pqg_file_row_group_num_rows(const pqg_file *f, int rg);
int64_t pqg_file_row_group_byte_size(const pqg_file *f, int rg); /* Σ chunk total_uncompressed_size */
/* Estimated decode cost of a row group on one GPU (relative units, ~ns) from
 * the footer and the dictionary page headers: uncompressed bytes, Snappy
 * input, and dictionary gathers priced by the index bit width.  The weight the
 * multi-GPU shard planner balances (no reference counterpart: the reader
 * decodes row groups one after another, file_reader.go:101-116). */
double pqg_file_row_group_cost(const pqg_file *f, int rg);
int pqg_file_column_count(const pqg_file *f);
int pqg_file_column_info(const pqg_file *f, int leaf, pqg_column_info *out);
int pqg_file_find_column(const pqg_file *f, const char *flat_name); /* leaf index or -1 */
/* Column selection like NewFileReader(r, columns...): a name selects the leaf
 * with that flat name, or every leaf under it (prefix + "."), schema.go:296-312.
 * Writes leaf indices into out[0..cap); returns the number selected. */
int pqg_file_select_columns(const pqg_file *f, const char *const *names, int nnames, int *out, int cap);
int pqg_file_last_error(const pqg_file *f, char *buf, size_t cap);

/* ---- batch: every page of row groups [rg_begin, rg_end) of the selected
 *      leaves, planned on the host into one descriptor table ----------------- */
typedef struct {
  /* device pointers (valid until pqg_batch_destroy) */
  void *values;         /* fixed width: slots * value_width (nulls zeroed); BYTE_ARRAY: string bytes */
  void *validity;       /* LSB-first bitmap over slots (def == max_def) */
  void *list_offsets;   /* int32[rows + 1], max_rep == 1 only */
  void *list_validity;  /* bitmap over rows (def >= rep_def - 1), max_rep == 1 only */
  void *str_offsets;    /* int64[slots + 1], BYTE_ARRAY only */
  void *def_levels;     /* uint8[levels] (only if PQG_BATCH_LEVELS) */
  void *rep_levels;     /* uint8[levels] (only if PQG_BATCH_LEVELS) */
  int64_t levels, slots, rows, str_bytes, non_null;
  int32_t value_width;
  int32_t leaf;
} pqg_column_view;

enum { PQG_BUF_VALUES = 0, PQG_BUF_VALIDITY = 1, PQG_BUF_LIST_OFFSETS = 2, PQG_BUF_LIST_VALIDITY = 3,
       PQG_BUF_STR_OFFSETS = 4, PQG_BUF_DEF = 5, PQG_BUF_REP = 6 };

/* batch flags */
enum {
  PQG_BATCH_LEVELS = 1,       /* also emit raw def/rep levels */
  PQG_BATCH_HOST_INFLATE = 2  /* inflate GZIP pages with zlib on the host while planning (default: k_inflate on the GPU) */
};

typedef struct {
  int64_t pages, data_pages, dict_pages, snappy_pages, host_inflated_pages;
  int64_t input_bytes;      /* B_in: stored page payload bytes (compressed values + levels + dictionaries) */
  int64_t staged_bytes;     /* uncompressed bytes the snappy kernel writes to HBM staging */
  int64_t output_bytes;     /* B_out: values + validity + offsets + string bytes */
  int64_t h2d_bytes;        /* bytes uploaded by pqg_batch_create */
  int64_t snappy_in_bytes;  /* compressed bytes of the Snappy pages (k_snappy's input) */
  int64_t dict_bytes;       /* uncompressed bytes of the dictionary pages */
  /* host time (ms) of pqg_batch_create's stages: page plan, device-cache
   * allocation, input upload (of which: gathering into the pinned ring, and
   * waiting for a ring buffer's previous DMA), output allocation + tables
   * (including a counting pass's launch, not its device time) */
  double create_plan_ms, create_alloc_ms, create_upload_ms, create_tables_ms;
  double upload_gather_ms, upload_wait_ms;
  int64_t gzip_device_pages;  /* GZIP pages inflated on the GPU (k_inflate) */
  int64_t gzip_in_bytes;      /* their compressed bytes */
} pqg_batch_stats;

int pqg_batch_create(pqg_ctx *ctx, pqg_file *f, int rg_begin, int rg_end, const int *leaves, int nleaves, int flags,
                     pqg_batch **out);
/* Launch the whole decode pipeline (asynchronous) on the batch's stream:
 * the context stream, except for slices of a pqg_stream, which may decode on a
 * second internal lane.  Order other device work after a decode with
 * pqg_batch_sync, or on pqg_batch_stream(b) — not on pqg_ctx_stream. */
int pqg_batch_decode(pqg_batch *b);
/* HIP stream (hipStream_t as void*) the batch's decodes are launched on. */
void *pqg_batch_stream(const pqg_batch *b);
/* Wait for the last decode and reduce the per-page status words: returns the
 * reference's first error (row group, leaf, page order) or PQG_OK. */
int pqg_batch_sync(pqg_batch *b);
int pqg_batch_error_location(const pqg_batch *b, int *rg, int *leaf, int *page);
int pqg_batch_column(const pqg_batch *b, int i, pqg_column_view *out);
/* Columns with max_rep >= 2 (List<...List<T>>; the reference's ColumnStore
 * keeps them as levels + values, data_store.go:158-203, schema.go:171-264):
 * the list structure, built on the GPU from the levels (kept for such
 * columns; pqg_column_view.def_levels / rep_levels).  level k = 1..max_rep:
 * the level-k lists' int32 offsets (count + 1 entries) into the level-(k+1)
 * lists — for k = max_rep into the leaf slots — and their validity bitmap
 * (LSB first; non-null iff def >= the k-th repeated ancestor's def level - 1);
 * level max_rep + 1: the leaf slots' validity (def == max_def: slot j holds the
 * next dense value), offsets NULL.  Device pointers, valid until the next
 * decode; *count from the last synced decode.  PQG_ERR_ARG for other columns
 * or levels, PQG_ERR_UNSUPPORTED past 8 repetition levels. */
int pqg_batch_column_nest(const pqg_batch *b, int i, int level, void **offsets, void **validity, int64_t *count);
/* Copy one of them to host memory: what 0 = offsets, 1 = validity. */
int pqg_batch_copy_nest(pqg_batch *b, int i, int level, int what, void *dst, size_t cap, size_t *nbytes);
/* Copy one output buffer of selected column i to host memory. */
int pqg_batch_copy(pqg_batch *b, int i, int buf_id, void *dst, size_t cap, size_t *nbytes);
/* Fills min(size, sizeof(pqg_batch_stats)) bytes of *out (pass sizeof(*out));
 * bytes past the library's struct are zeroed.  size must cover at least the
 * eleven int64 counters (the version-1 prefix): else PQG_ERR_ARG. */
int pqg_batch_stats_get(const pqg_batch *b, pqg_batch_stats *out, size_t size);
/* Device time (ms) per timed segment, averaged over the decodes issued since
 * the previous call (up to 64), from HIP events on the context stream.  By
 * default one segment brackets the decode phase (k_decode + k_expand); with
 * PQG_SEGMENT_TIMES=1 every phase is bracketed (events add launch gaps).
 * names/ms have room for `cap` entries; returns the number of segments. */
int pqg_batch_kernel_times(pqg_batch *b, const char **names, float *ms, int cap);
/* Record the timing events on every `every`-th decode only (1: every decode,
 * the default; 0: never).  Each event pair costs a few µs of launch gap, so a
 * throughput loop samples the kernel times instead of timing every pass. */
int pqg_batch_set_timing(pqg_batch *b, int every);
void pqg_batch_destroy(pqg_batch *b);

/* ---- stream: row groups [rg_begin, rg_end) in slices of rgs_per_slice row
 *      groups, pipelined.  Replaces the reader's row-group iteration
 *      (file_reader.go:101-116 NextRow / SkipRowGroup / PreLoad ->
 *      readRowGroup, chunk_reader.go:206-283): a host worker thread plans slice
 *      k + 1 and queues its H2D upload (the context's upload stream, pinned ring
 *      filled by PQG_UPLOAD_THREADS host threads) while the GPU decodes slice k.
 *      `depth` slices are built ahead (>= 1). ---------------------------------- */
typedef struct pqg_stream pqg_stream;
int pqg_stream_open(pqg_ctx *ctx, pqg_file *f, int rg_begin, int rg_end, const int *leaves, int nleaves, int flags,
                    int rgs_per_slice, int depth, pqg_stream **out);
/* The next slice: its decode is launched (asynchronous; pqg_batch_sync waits
 * and reports its first error) and *out is its batch, owned by the stream and
 * valid until the next pqg_stream_next / pqg_stream_close.  *out = NULL and
 * PQG_OK after the last slice; a slice whose planning failed returns that
 * error (the stream ends there). *rg_first: the slice's first row group. */
int pqg_stream_next(pqg_stream *s, pqg_batch **out, int *rg_first);
/* pqg_stream_open flag: the first two slices hold a quarter and a half of
 * rgs_per_slice row groups (at least one), so the first decode starts after a
 * short upload and the pipeline fills sooner; later slices hold rgs_per_slice.
 * Each slice's row groups: pqg_batch_row_groups. */
enum { PQG_STREAM_RAMP = 1 << 8 };
/* Row groups [*rg_begin, *rg_end) of a batch (a stream slice's range). */
int pqg_batch_row_groups(const pqg_batch *b, int *rg_begin, int *rg_end);
void pqg_stream_close(pqg_stream *s);

#ifdef __cplusplus
}
#endif
#endif /* PQGPU_H */
