/*
 * pqref — CPU ORACLE for the Parquet column-chunk decode path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is a plain-C, single-threaded restatement of
 * the reference decoder (kmatt/parquet-go, module github.com/fraugster/parquet-go)
 * used as the parity checker in tests/, __graft_entry__.smoke() and as the
 * `cpu_baseline` leg of bench.py.  The product path (libpqgpu.so + HIP kernels)
 * never links, loads or calls anything under oracle/.
 *
 * Parity pinning: the oracle is checked against (1) the reference's own
 * known-answer tables (bitpacking32_test.go:25-654, bitpacking64_test.go:25-1744,
 * transcribed into tests/golden/kat_bitpack.json by tests/golden/make_golden.py)
 * and (2) golden Parquet files written by pyarrow 25.0.0 with their decoded
 * outputs (tests/golden/ parquet files and npz expectations).  The Go reference itself cannot be
 * built here (no Go toolchain; see DESIGN.md "Oracle").
 *
 * Each function cites the reference file:line it restates.
 */
#ifndef PQREF_H
#define PQREF_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error classes.  Numeric values are the same contract as include/pqgpu.h
 * (tests/test_capi_symbols.py checks that they agree). */
enum {
  PQR_OK = 0,
  PQR_ERR_ARG = 1,
  PQR_ERR_FORMAT = 2,        /* magic / footer length (file_meta.go:14-62) */
  PQR_ERR_THRIFT = 3,        /* compact-thrift decode failure */
  PQR_ERR_SCHEMA = 4,        /* schema.go:789-1000 */
  PQR_ERR_CODEC = 5,         /* codec not registered (compress.go:90-100) */
  PQR_ERR_ENCODING = 6,      /* unsupported encoding (chunk_reader.go:58-196, :348-364) */
  PQR_ERR_SNAPPY = 7,        /* snappy ErrCorrupt (vendor/.../decode.go) */
  PQR_ERR_SIZE = 8,          /* compress.go:108-119, chunk_reader.go:198-204 */
  PQR_ERR_PAGE = 9,          /* page header checks (page_v1/v2/dict, chunk_reader.go:221-264) */
  PQR_ERR_EOF = 10,          /* a level/value stream ended early */
  PQR_ERR_RLE = 11,          /* hybrid_decoder.go:127-129,:154-161; helpers.go:326 */
  PQR_ERR_DICT_INDEX = 12,   /* type_dict.go:51-53 */
  PQR_ERR_DELTA = 13,        /* deltabp_decoder.go header checks */
  PQR_ERR_BYTE_ARRAY = 14,   /* type_bytearray.go:31-36 */
  PQR_ERR_BITWIDTH = 15,     /* type_dict.go:28-30, deltabp_decoder.go:262-264 */
  PQR_ERR_NO_DICT = 16,      /* type_dict.go:40-42 */
  PQR_ERR_DEVICE = 17,
  PQR_ERR_COUNT = 18,        /* chunk_reader.go:389-391 */
  PQR_ERR_UNSUPPORTED = 19   /* outside the oracle's scope (e.g. BOOLEAN, maxR>1 offsets) */
};

/* Parquet physical types (parquet/parquet.go Type enum). */
enum { PQR_BOOLEAN = 0, PQR_INT32 = 1, PQR_INT64 = 2, PQR_INT96 = 3, PQR_FLOAT = 4,
       PQR_DOUBLE = 5, PQR_BYTE_ARRAY = 6, PQR_FLBA = 7 };

typedef struct pqref_file pqref_file;
typedef struct pqref_result pqref_result;

typedef struct {
  char name[512];          /* dotted flat name (schema.go:811-815) */
  int32_t physical_type;
  int32_t type_length;
  int32_t max_def;         /* schema.go:800-802 */
  int32_t max_rep;         /* schema.go:804-806 */
  int32_t rep_def;         /* def level at the (single) repeated ancestor, 0 if none */
  int32_t converted_type;  /* -1 if absent */
  int32_t unsigned_int;    /* chunk_reader.go:29-50 unsigned flag */
} pqref_leaf;

int pqref_open(const uint8_t *buf, size_t len, pqref_file **out, char *err, size_t errcap);
void pqref_close(pqref_file *f);
int pqref_num_row_groups(const pqref_file *f);
int64_t pqref_rg_num_rows(const pqref_file *f, int rg);
int64_t pqref_num_rows(const pqref_file *f);
int pqref_num_leaves(const pqref_file *f);
int pqref_leaf_info(const pqref_file *f, int leaf, pqref_leaf *out);

/* Decode one leaf column over row groups [rg0, rg1) with reference page
 * semantics, then lay the result out Arrow-style (values spaced over slots,
 * nulls zeroed, validity bitmaps LSB-first, list offsets, string offsets). */
int pqref_decode(const pqref_file *f, int leaf, int rg0, int rg1, pqref_result **out);
/* ref-quirks mode (documentation only): for a
 * fixed-width leaf, the values the reference's row reader returns (its column
 * store's aliasing included): VALUES = one per defined level, VALIDITY bit =
 * not nil.  pqref.c documents the model. */
int pqref_decode_quirks(const pqref_file *f, int leaf, int rg0, int rg1, pqref_result **out);
void pqref_result_free(pqref_result *r);

/* Result accessors.  Buffer ids: */
enum { PQR_BUF_VALUES = 0, PQR_BUF_VALIDITY = 1, PQR_BUF_LIST_OFFSETS = 2,
       PQR_BUF_LIST_VALIDITY = 3, PQR_BUF_STR_OFFSETS = 4, PQR_BUF_DEF = 5, PQR_BUF_REP = 6 };
/* Counter ids: */
enum { PQR_CNT_LEVELS = 0, PQR_CNT_SLOTS = 1, PQR_CNT_ROWS = 2, PQR_CNT_NONNULL = 3,
       PQR_CNT_STR_BYTES = 4, PQR_CNT_PAGES = 5, PQR_CNT_VALUE_WIDTH = 6 };
int pqref_result_status(const pqref_result *r);
const char *pqref_result_error(const pqref_result *r);
int64_t pqref_result_count(const pqref_result *r, int which);
const void *pqref_result_buffer(const pqref_result *r, int which, size_t *nbytes);
/* Location of the first error: row group, page index within chunk (-1 = chunk-level). */
int pqref_result_error_rg(const pqref_result *r);
int pqref_result_error_page(const pqref_result *r);

/* Stand-alone primitives (for KAT and fuzz tests). */
int pqref_snappy_decode(const uint8_t *src, size_t n, uint8_t *dst, size_t cap, size_t *out_len);
void pqref_unpack8_32(const uint8_t *data, int width, int32_t out[8]);
void pqref_unpack8_64(const uint8_t *data, int width, int64_t out[8]);
/* Decode `count` values of an RLE/bit-packed hybrid stream (no length prefix). */
int pqref_hybrid_decode(const uint8_t *src, size_t n, int bit_width, int32_t *out, int64_t count);

#ifdef __cplusplus
}
#endif
#endif
