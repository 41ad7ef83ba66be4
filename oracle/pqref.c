/*
 * pqref.c — CPU ORACLE (test infrastructure only; see pqref.h header comment).
 *
 * A deliberately serial, allocation-happy restatement of the reference read
 * path.  Control flow mirrors the Go code so that error classes and their
 * order match: all pages of a chunk are read/initialised first (readPages,
 * chunk_reader.go:206-284), then decoded in order (readPageData,
 * chunk_reader.go:380-402).
 */
#include "pqref.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifdef PQREF_HAVE_ZLIB
#include <zlib.h>
#endif

/* ------------------------------------------------------------------------ */
/* small helpers                                                             */
/* ------------------------------------------------------------------------ */

typedef struct {
  uint8_t *p;
  size_t n, cap;
} bytebuf;

static void bb_reserve(bytebuf *b, size_t extra) {
  if (b->n + extra <= b->cap) return;
  size_t nc = b->cap ? b->cap : 256;
  while (nc < b->n + extra) nc *= 2;
  b->p = (uint8_t *)realloc(b->p, nc);
  b->cap = nc;
}
static void bb_put(bytebuf *b, const void *src, size_t k) {
  bb_reserve(b, k);
  if (k) memcpy(b->p + b->n, src, k);
  b->n += k;
}
static void bb_zero(bytebuf *b, size_t k) {
  bb_reserve(b, k);
  memset(b->p + b->n, 0, k);
  b->n += k;
}

/* A bytes.Reader: Read returns min(len, remaining) bytes and io.EOF only when
 * nothing remains (Go stdlib semantics relied on by hybrid_decoder.go:133-141). */
typedef struct {
  const uint8_t *p;
  size_t n, pos;
} rdr;

static size_t rd_read(rdr *r, uint8_t *dst, size_t k) {
  size_t avail = r->n - r->pos;
  if (k > avail) k = avail;
  if (k) memcpy(dst, r->p + r->pos, k);
  r->pos += k;
  return k;
}
/* io.ReadFull: 0 on success, PQR_ERR_EOF on short read. */
static int rd_full(rdr *r, uint8_t *dst, size_t k) {
  if (r->n - r->pos < k) {
    r->pos = r->n;
    return PQR_ERR_EOF;
  }
  if (dst) memcpy(dst, r->p + r->pos, k);
  r->pos += k;
  return 0;
}

/* binary.ReadUvarint (encoding/binary, Go 1.13): keeps reading while the
 * continuation bit is set; EOF from the reader is returned as is; overflow is
 * reported only when the terminating byte arrives (i > 9 || i == 9 && b > 1). */
static int rd_uvarint(rdr *r, uint64_t *out) {
  uint64_t x = 0;
  unsigned s = 0;
  for (int i = 0;; i++) {
    if (r->pos >= r->n) return PQR_ERR_EOF;
    uint8_t b = r->p[r->pos++];
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) return PQR_ERR_RLE; /* overflow */
      *out = x | ((uint64_t)b << (s & 63));
      return 0;
    }
    if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
}
/* readUVariant32 helpers.go:149-165 */
static int rd_uvarint32(rdr *r, int32_t *out, int range_err) {
  uint64_t v;
  int e = rd_uvarint(r, &v);
  if (e) return e == PQR_ERR_EOF ? PQR_ERR_EOF : range_err;
  if (v > 0x7fffffffULL) return range_err;
  *out = (int32_t)v;
  return 0;
}
/* binary.ReadVarint (zigzag) — readVariant64 helpers.go:199-206 */
static int rd_varint64(rdr *r, int64_t *out) {
  uint64_t u;
  int e = rd_uvarint(r, &u);
  if (e) return e;
  int64_t x = (int64_t)(u >> 1);
  if (u & 1) x = ~x;
  *out = x;
  return 0;
}

static uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

/* ------------------------------------------------------------------------ */
/* bit unpacking — bitbacking32.go / bitpacking64.go (LSB-first, as the      */
/* generator bitpack_gen.go:18-58 specifies)                                 */
/* ------------------------------------------------------------------------ */

void pqref_unpack8_32(const uint8_t *data, int width, int32_t out[8]) {
  for (int i = 0; i < 8; i++) {
    uint64_t v = 0;
    for (int b = 0; b < width; b++) {
      int bit = i * width + b;
      v |= (uint64_t)((data[bit >> 3] >> (bit & 7)) & 1) << b;
    }
    out[i] = (int32_t)(uint32_t)v;
  }
}

void pqref_unpack8_64(const uint8_t *data, int width, int64_t out[8]) {
  for (int i = 0; i < 8; i++) {
    uint64_t v = 0;
    for (int b = 0; b < width; b++) {
      int bit = i * width + b;
      v |= (uint64_t)((data[bit >> 3] >> (bit & 7)) & 1) << b;
    }
    out[i] = (int64_t)v;
  }
}

/* ------------------------------------------------------------------------ */
/* snappy — vendor/github.com/golang/snappy/decode.go:32-75, decode_other.go */
/* ------------------------------------------------------------------------ */

/* Returns 0 / PQR_ERR_SNAPPY.  `dst` may be NULL (validate only) or have
 * capacity `cap` < decoded length (then bytes beyond cap are dropped). */
static int snappy_decode_body(const uint8_t *src, size_t slen, uint8_t *dst, size_t dlen, size_t cap) {
  size_t d = 0, s = 0;
  while (s < slen) {
    size_t length, offset;
    uint8_t tag = src[s] & 3;
    if (tag == 0) { /* literal, decode_other.go:18-58 */
      uint32_t x = src[s] >> 2;
      if (x < 60) {
        s += 1;
      } else {
        size_t extra = x - 59; /* 1..4 bytes */
        s += 1 + extra;
        if (s > slen) return PQR_ERR_SNAPPY;
        x = 0;
        for (size_t k = 0; k < extra; k++) x |= (uint32_t)src[s - extra + k] << (8 * k);
      }
      length = (size_t)x + 1; /* length <= 0 impossible on 64-bit */
      if (length > dlen - d || length > slen - s) return PQR_ERR_SNAPPY;
      if (dst) {
        for (size_t k = 0; k < length; k++)
          if (d + k < cap) dst[d + k] = src[s + k];
      }
      d += length;
      s += length;
      continue;
    } else if (tag == 1) { /* copy1 */
      s += 2;
      if (s > slen) return PQR_ERR_SNAPPY;
      length = 4 + ((src[s - 2] >> 2) & 7);
      offset = ((size_t)(src[s - 2] & 0xe0) << 3) | src[s - 1];
    } else if (tag == 2) { /* copy2 */
      s += 3;
      if (s > slen) return PQR_ERR_SNAPPY;
      length = 1 + (src[s - 3] >> 2);
      offset = (size_t)src[s - 2] | (size_t)src[s - 1] << 8;
    } else { /* copy4 */
      s += 5;
      if (s > slen) return PQR_ERR_SNAPPY;
      length = 1 + (src[s - 5] >> 2);
      offset = (size_t)le32(src + s - 4);
    }
    if (offset == 0 || d < offset || length > dlen - d) return PQR_ERR_SNAPPY;
    if (dst) {
      for (size_t end = d + length; d != end; d++) /* forward, overlapping */
        if (d < cap) dst[d] = (d - offset < cap) ? dst[d - offset] : 0;
    } else {
      d += length;
    }
  }
  if (d != dlen) return PQR_ERR_SNAPPY;
  return 0;
}

/* snappy.Decode + the newBlockReader size check (compress.go:112-119). */
static int snappy_decode_checked(const uint8_t *src, size_t n, size_t expect, uint8_t **out) {
  rdr r = {src, n, 0};
  uint64_t v;
  if (rd_uvarint(&r, &v) != 0 || v > 0xffffffffULL) return PQR_ERR_SNAPPY; /* decodedLen */
  if (v != expect) {
    /* decode would still run into a dLen buffer; only the error class matters */
    int e = snappy_decode_body(src + r.pos, n - r.pos, NULL, (size_t)v, 0);
    return e ? e : PQR_ERR_SIZE;
  }
  uint8_t *dst = (uint8_t *)malloc(expect ? expect : 1);
  int e = snappy_decode_body(src + r.pos, n - r.pos, dst, (size_t)v, (size_t)v);
  if (e) {
    free(dst);
    return e;
  }
  *out = dst;
  return 0;
}

int pqref_snappy_decode(const uint8_t *src, size_t n, uint8_t *dst, size_t cap, size_t *out_len) {
  rdr r = {src, n, 0};
  uint64_t v;
  if (rd_uvarint(&r, &v) != 0 || v > 0xffffffffULL) return PQR_ERR_SNAPPY;
  *out_len = (size_t)v;
  if (v > cap) return snappy_decode_body(src + r.pos, n - r.pos, NULL, (size_t)v, 0) ? PQR_ERR_SNAPPY : PQR_ERR_SIZE;
  return snappy_decode_body(src + r.pos, n - r.pos, dst, (size_t)v, cap);
}

/* ------------------------------------------------------------------------ */
/* RLE / bit-packed hybrid — hybrid_decoder.go:30-166                        */
/* ------------------------------------------------------------------------ */

typedef struct {
  rdr r;
  int init;         /* hd.r != nil */
  int bw;
  int rle_size;     /* (bw+7)/8 */
  int32_t bp_run[8];
  uint32_t rle_count;
  int32_t rle_value;
  uint32_t bp_count;
  uint8_t bp_pos;
} hybrid;

static void hy_new(hybrid *h, int bw) {
  memset(h, 0, sizeof(*h));
  h->bw = bw;
  h->rle_size = (bw + 7) / 8;
}
static void hy_init(hybrid *h, const uint8_t *p, size_t n) {
  h->r.p = p;
  h->r.n = n;
  h->r.pos = 0;
  h->init = 1;
}

static int hy_read_header(hybrid *h) { /* :143-166 */
  int32_t hdr;
  int e = rd_uvarint32(&h->r, &hdr, PQR_ERR_RLE);
  if (e) return e;
  if (hdr & 1) {
    h->bp_count = (uint32_t)hdr >> 1;
    if (h->bp_count == 0) return PQR_ERR_RLE; /* "rle: empty bit-packed run" */
    h->bp_pos = 0;
  } else {
    h->rle_count = (uint32_t)hdr >> 1;
    if (h->rle_count == 0) return PQR_ERR_RLE; /* "rle: empty RLE run" */
    /* readRLERunValue :116-131 */
    uint8_t v[4] = {0, 0, 0, 0};
    size_t got = rd_read(&h->r, v, (size_t)h->rle_size);
    if (got == 0 && h->rle_size > 0) return PQR_ERR_EOF;
    if ((int)got != h->rle_size) return PQR_ERR_EOF; /* io.ErrUnexpectedEOF */
    uint32_t val = (uint32_t)v[0] | (uint32_t)v[1] << 8 | (uint32_t)v[2] << 16 | (uint32_t)v[3] << 24;
    h->rle_value = (int32_t)val;
    if (h->bw < 32 && (val >> h->bw) != 0) return PQR_ERR_RLE; /* value too large */
  }
  return 0;
}

static int hy_next(hybrid *h, int32_t *out) { /* :82-114 */
  if (h->bw == 0) {
    *out = 0;
    return 0;
  }
  if (!h->init) return PQR_ERR_EOF; /* "reader is not initialized" */
  if (h->rle_count == 0 && h->bp_count == 0 && h->bp_pos == 0) {
    int e = hy_read_header(h);
    if (e) return e;
  }
  if (h->rle_count > 0) {
    *out = h->rle_value;
    h->rle_count--;
  } else if (h->bp_count > 0 || h->bp_pos > 0) {
    if (h->bp_pos == 0) { /* readBitPackedRun :133-141 */
      uint8_t data[32];
      memset(data, 0, sizeof(data));
      size_t got = rd_read(&h->r, data, (size_t)h->bw);
      if (got == 0) return PQR_ERR_EOF;
      pqref_unpack8_32(data, h->bw, h->bp_run);
      h->bp_count--;
    }
    *out = h->bp_run[h->bp_pos];
    h->bp_pos = (uint8_t)((h->bp_pos + 1) % 8);
  } else {
    return PQR_ERR_EOF;
  }
  return 0;
}

int pqref_hybrid_decode(const uint8_t *src, size_t n, int bw, int32_t *out, int64_t count) {
  if (bw < 0 || bw > 32) return PQR_ERR_BITWIDTH;
  hybrid h;
  hy_new(&h, bw);
  hy_init(&h, src, n);
  for (int64_t i = 0; i < count; i++) {
    int e = hy_next(&h, &out[i]);
    if (e) return e;
  }
  return 0;
}

/* ------------------------------------------------------------------------ */
/* compact thrift (only what the reader needs; unknown fields skipped)       */
/* ------------------------------------------------------------------------ */

typedef struct {
  const uint8_t *p;
  size_t n, pos;
  int err;
  int depth;
} tproto;

enum { CT_STOP = 0, CT_TRUE = 1, CT_FALSE = 2, CT_BYTE = 3, CT_I16 = 4, CT_I32 = 5, CT_I64 = 6,
       CT_DOUBLE = 7, CT_BINARY = 8, CT_LIST = 9, CT_SET = 10, CT_MAP = 11, CT_STRUCT = 12 };

static uint8_t tp_byte(tproto *t) {
  if (t->pos >= t->n) {
    t->err = 1;
    return 0;
  }
  return t->p[t->pos++];
}
static uint64_t tp_uvar(tproto *t) {
  uint64_t x = 0;
  unsigned s = 0;
  for (int i = 0; i < 10; i++) {
    uint8_t b = tp_byte(t);
    if (t->err) return 0;
    x |= (uint64_t)(b & 0x7f) << s;
    if (!(b & 0x80)) return x;
    s += 7;
  }
  t->err = 1;
  return 0;
}
static int64_t tp_zz(tproto *t) {
  uint64_t u = tp_uvar(t);
  return (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
}
static void tp_skip(tproto *t, int type);
static void tp_skip_struct(tproto *t) {
  if (++t->depth > 64) {
    t->err = 1;
    return;
  }
  int16_t last = 0;
  while (!t->err) {
    uint8_t h = tp_byte(t);
    if (t->err || h == 0) break;
    int type = h & 0x0f;
    int delta = h >> 4;
    if (delta) last = (int16_t)(last + delta);
    else last = (int16_t)tp_zz(t);
    tp_skip(t, type);
  }
  t->depth--;
}
static void tp_list_header(tproto *t, int *etype, int64_t *size) {
  uint8_t h = tp_byte(t);
  int64_t sz = h >> 4;
  *etype = h & 0x0f;
  if (sz == 15) sz = (int64_t)tp_uvar(t);
  if (sz < 0 || sz > (int64_t)(t->n - t->pos) * 8 + 16) t->err = 1; /* sanity */
  *size = sz;
}
static void tp_skip(tproto *t, int type) {
  if (t->err) return;
  switch (type) {
    case CT_TRUE:
    case CT_FALSE:
      break;
    case CT_BYTE:
      tp_byte(t);
      break;
    case CT_I16:
    case CT_I32:
    case CT_I64:
      tp_uvar(t);
      break;
    case CT_DOUBLE:
      if (t->n - t->pos < 8) t->err = 1;
      else t->pos += 8;
      break;
    case CT_BINARY: {
      uint64_t l = tp_uvar(t);
      if (t->err || l > t->n - t->pos) t->err = 1;
      else t->pos += l;
      break;
    }
    case CT_LIST:
    case CT_SET: {
      int et;
      int64_t sz;
      tp_list_header(t, &et, &sz);
      for (int64_t i = 0; i < sz && !t->err; i++) {
        if (et == CT_TRUE || et == CT_FALSE) tp_byte(t);
        else tp_skip(t, et);
      }
      break;
    }
    case CT_MAP: {
      uint64_t sz = tp_uvar(t);
      if (sz == 0) break;
      uint8_t kv = tp_byte(t);
      if (sz > t->n - t->pos) {
        t->err = 1;
        break;
      }
      for (uint64_t i = 0; i < sz && !t->err; i++) {
        tp_skip(t, kv >> 4);
        tp_skip(t, kv & 0xf);
      }
      break;
    }
    case CT_STRUCT:
      tp_skip_struct(t);
      break;
    default:
      t->err = 1;
  }
}

/* iterate struct fields: returns field id, or 0 at stop / error */
static int tp_field(tproto *t, int16_t *last, int *type) {
  uint8_t h = tp_byte(t);
  if (t->err || h == 0) return 0;
  *type = h & 0x0f;
  int delta = h >> 4;
  if (delta) *last = (int16_t)(*last + delta);
  else *last = (int16_t)tp_zz(t);
  return *last == 0 ? -1 : *last; /* field id 0 is legal-but-unused: report -1 */
}
static int32_t tp_i32(tproto *t, int type) {
  if (type != CT_I32 && type != CT_I16 && type != CT_BYTE) {
    tp_skip(t, type);
    t->err = 1;
    return 0;
  }
  if (type == CT_BYTE) return (int8_t)tp_byte(t);
  return (int32_t)tp_zz(t);
}
static int64_t tp_i64(tproto *t, int type) {
  if (type != CT_I64 && type != CT_I32 && type != CT_I16) {
    tp_skip(t, type);
    t->err = 1;
    return 0;
  }
  return tp_zz(t);
}
static char *tp_string(tproto *t, int type) {
  if (type != CT_BINARY) {
    tp_skip(t, type);
    t->err = 1;
    return NULL;
  }
  uint64_t l = tp_uvar(t);
  if (t->err || l > t->n - t->pos) {
    t->err = 1;
    return NULL;
  }
  char *s = (char *)malloc(l + 1);
  memcpy(s, t->p + t->pos, l);
  s[l] = 0;
  t->pos += l;
  return s;
}

/* metadata structs (parquet/parquet.go) */
typedef struct {
  int has_type;
  int32_t type, type_length, repetition, num_children, converted;
  int has_rep, has_children;
  char *name;
  int int_unsigned; /* LogicalType.INTEGER && !IsSigned */
} sch_elem;

typedef struct {
  int32_t type, codec;
  int64_t num_values, total_uncompressed, total_compressed, data_page_offset, dict_page_offset;
  int has_dict_off;
  int has_meta;
  int has_file_path;
} col_chunk;

typedef struct {
  col_chunk *cols;
  int ncols;
  int64_t num_rows;
} row_group;

struct pqref_file {
  const uint8_t *buf;
  size_t len;
  sch_elem *schema;
  int nschema;
  row_group *rgs;
  int nrgs;
  int64_t num_rows;
  pqref_leaf *leaves;
  int nleaves;
};

static void read_int_type(tproto *t, int *is_unsigned) { /* IntType parquet.go:2311 */
  int16_t last = 0;
  int type, fid;
  int has_bw = 0, has_signed = 0, is_signed = 1;
  while ((fid = tp_field(t, &last, &type)) != 0 && !t->err) {
    if (fid == 1 && type == CT_BYTE) {
      tp_byte(t);
      has_bw = 1;
    } else if (fid == 2 && (type == CT_TRUE || type == CT_FALSE)) {
      is_signed = type == CT_TRUE;
      has_signed = 1;
    } else tp_skip(t, type);
  }
  if (!has_bw || !has_signed) t->err = 1;
  *is_unsigned = !is_signed;
}
static void read_logical_type(tproto *t, sch_elem *e) {
  int16_t last = 0;
  int type, fid;
  while ((fid = tp_field(t, &last, &type)) != 0 && !t->err) {
    if (fid == 10 && type == CT_STRUCT) {
      int u = 0;
      read_int_type(t, &u);
      e->int_unsigned = u;
    } else tp_skip(t, type);
  }
}
static void read_schema_elem(tproto *t, sch_elem *e) { /* SchemaElement parquet.go:3381 */
  memset(e, 0, sizeof(*e));
  e->converted = -1;
  int16_t last = 0;
  int type, fid;
  while ((fid = tp_field(t, &last, &type)) != 0 && !t->err) {
    switch (fid) {
      case 1: e->type = tp_i32(t, type); e->has_type = 1; break;
      case 2: e->type_length = tp_i32(t, type); break;
      case 3: e->repetition = tp_i32(t, type); e->has_rep = 1; break;
      case 4: free(e->name); e->name = tp_string(t, type); break;
      case 5: e->num_children = tp_i32(t, type); e->has_children = 1; break;
      case 6: e->converted = tp_i32(t, type); break;
      case 10:
        if (type == CT_STRUCT) read_logical_type(t, e);
        else tp_skip(t, type);
        break;
      default: tp_skip(t, type);
    }
  }
  if (!e->name) t->err = 1; /* Name is required */
}
static void read_col_meta(tproto *t, col_chunk *c) { /* ColumnMetaData parquet.go:6822 */
  int16_t last = 0;
  int type, fid;
  unsigned seen = 0;
  while ((fid = tp_field(t, &last, &type)) != 0 && !t->err) {
    switch (fid) {
      case 1: c->type = tp_i32(t, type); seen |= 1; break;
      case 2: tp_skip(t, type); seen |= 2; break;
      case 3: tp_skip(t, type); seen |= 4; break;
      case 4: c->codec = tp_i32(t, type); seen |= 8; break;
      case 5: c->num_values = tp_i64(t, type); seen |= 16; break;
      case 6: c->total_uncompressed = tp_i64(t, type); seen |= 32; break;
      case 7: c->total_compressed = tp_i64(t, type); seen |= 64; break;
      case 9: c->data_page_offset = tp_i64(t, type); seen |= 128; break;
      case 11: c->dict_page_offset = tp_i64(t, type); c->has_dict_off = 1; break;
      default: tp_skip(t, type);
    }
  }
  if (seen != 255) t->err = 1;
}
static void read_col_chunk(tproto *t, col_chunk *c) { /* ColumnChunk parquet.go:8042 */
  memset(c, 0, sizeof(*c));
  int16_t last = 0;
  int type, fid;
  int has_off = 0;
  while ((fid = tp_field(t, &last, &type)) != 0 && !t->err) {
    if (fid == 1) {
      char *s = tp_string(t, type);
      free(s);
      c->has_file_path = 1;
    } else if (fid == 2) {
      tp_i64(t, type);
      has_off = 1;
    } else if (fid == 3 && type == CT_STRUCT) {
      read_col_meta(t, c);
      c->has_meta = 1;
    } else tp_skip(t, type);
  }
  if (!has_off) t->err = 1;
}
static void read_row_group(tproto *t, row_group *g) { /* RowGroup parquet.go:8561 */
  memset(g, 0, sizeof(*g));
  int16_t last = 0;
  int type, fid;
  unsigned seen = 0;
  while ((fid = tp_field(t, &last, &type)) != 0 && !t->err) {
    if (fid == 1 && type == CT_LIST) {
      int et;
      int64_t sz;
      tp_list_header(t, &et, &sz);
      if (t->err || et != CT_STRUCT) {
        t->err = 1;
        break;
      }
      g->cols = (col_chunk *)calloc((size_t)sz + 1, sizeof(col_chunk));
      g->ncols = (int)sz;
      for (int64_t i = 0; i < sz && !t->err; i++) read_col_chunk(t, &g->cols[i]);
      seen |= 1;
    } else if (fid == 2) {
      tp_i64(t, type);
      seen |= 2;
    } else if (fid == 3) {
      g->num_rows = tp_i64(t, type);
      seen |= 4;
    } else tp_skip(t, type);
  }
  if (seen != 7) t->err = 1;
}
static void read_file_meta(tproto *t, pqref_file *f) { /* FileMetaData parquet.go:10564 */
  int16_t last = 0;
  int type, fid;
  unsigned seen = 0;
  while ((fid = tp_field(t, &last, &type)) != 0 && !t->err) {
    if (fid == 1) {
      tp_i32(t, type);
      seen |= 1;
    } else if (fid == 2 && type == CT_LIST) {
      int et;
      int64_t sz;
      tp_list_header(t, &et, &sz);
      if (t->err || et != CT_STRUCT) {
        t->err = 1;
        break;
      }
      f->schema = (sch_elem *)calloc((size_t)sz + 1, sizeof(sch_elem));
      f->nschema = (int)sz;
      for (int64_t i = 0; i < sz && !t->err; i++) read_schema_elem(t, &f->schema[i]);
      seen |= 2;
    } else if (fid == 3) {
      f->num_rows = tp_i64(t, type);
      seen |= 4;
    } else if (fid == 4 && type == CT_LIST) {
      int et;
      int64_t sz;
      tp_list_header(t, &et, &sz);
      if (t->err || et != CT_STRUCT) {
        t->err = 1;
        break;
      }
      f->rgs = (row_group *)calloc((size_t)sz + 1, sizeof(row_group));
      f->nrgs = (int)sz;
      for (int64_t i = 0; i < sz && !t->err; i++) read_row_group(t, &f->rgs[i]);
      seen |= 8;
    } else tp_skip(t, type);
  }
  if (seen != 15) t->err = 1;
}

/* PageHeader parquet.go:5794 and its sub-headers */
typedef struct {
  int32_t type, uncompressed, compressed;
  int has_dph, has_dict, has_v2;
  /* DataPageHeader :3953 */
  int32_t dp_num_values, dp_encoding, dp_def_enc, dp_rep_enc;
  /* DictionaryPageHeader :4303 */
  int32_t dict_num_values, dict_encoding;
  /* DataPageHeaderV2 :4522 */
  int32_t v2_num_values, v2_num_nulls, v2_num_rows, v2_encoding, v2_def_len, v2_rep_len;
  int v2_is_compressed;
} page_header;

static void read_page_header(tproto *t, page_header *h) {
  memset(h, 0, sizeof(*h));
  h->v2_is_compressed = 1;
  int16_t last = 0;
  int type, fid;
  unsigned seen = 0;
  while ((fid = tp_field(t, &last, &type)) != 0 && !t->err) {
    if (fid == 1) {
      h->type = tp_i32(t, type);
      seen |= 1;
    } else if (fid == 2) {
      h->uncompressed = tp_i32(t, type);
      seen |= 2;
    } else if (fid == 3) {
      h->compressed = tp_i32(t, type);
      seen |= 4;
    } else if (fid == 5 && type == CT_STRUCT) {
      int16_t l2 = 0;
      int ty2, f2;
      unsigned s2 = 0;
      while ((f2 = tp_field(t, &l2, &ty2)) != 0 && !t->err) {
        switch (f2) {
          case 1: h->dp_num_values = tp_i32(t, ty2); s2 |= 1; break;
          case 2: h->dp_encoding = tp_i32(t, ty2); s2 |= 2; break;
          case 3: h->dp_def_enc = tp_i32(t, ty2); s2 |= 4; break;
          case 4: h->dp_rep_enc = tp_i32(t, ty2); s2 |= 8; break;
          default: tp_skip(t, ty2);
        }
      }
      if (s2 != 15) t->err = 1;
      h->has_dph = 1;
    } else if (fid == 7 && type == CT_STRUCT) {
      int16_t l2 = 0;
      int ty2, f2;
      unsigned s2 = 0;
      while ((f2 = tp_field(t, &l2, &ty2)) != 0 && !t->err) {
        switch (f2) {
          case 1: h->dict_num_values = tp_i32(t, ty2); s2 |= 1; break;
          case 2: h->dict_encoding = tp_i32(t, ty2); s2 |= 2; break;
          default: tp_skip(t, ty2);
        }
      }
      if (s2 != 3) t->err = 1;
      h->has_dict = 1;
    } else if (fid == 8 && type == CT_STRUCT) {
      int16_t l2 = 0;
      int ty2, f2;
      unsigned s2 = 0;
      while ((f2 = tp_field(t, &l2, &ty2)) != 0 && !t->err) {
        switch (f2) {
          case 1: h->v2_num_values = tp_i32(t, ty2); s2 |= 1; break;
          case 2: h->v2_num_nulls = tp_i32(t, ty2); s2 |= 2; break;
          case 3: h->v2_num_rows = tp_i32(t, ty2); s2 |= 4; break;
          case 4: h->v2_encoding = tp_i32(t, ty2); s2 |= 8; break;
          case 5: h->v2_def_len = tp_i32(t, ty2); s2 |= 16; break;
          case 6: h->v2_rep_len = tp_i32(t, ty2); s2 |= 32; break;
          case 7:
            if (ty2 == CT_TRUE || ty2 == CT_FALSE) h->v2_is_compressed = ty2 == CT_TRUE;
            else tp_skip(t, ty2);
            break;
          default: tp_skip(t, ty2);
        }
      }
      if (s2 != 63) t->err = 1;
      h->has_v2 = 1;
    } else tp_skip(t, type);
  }
  if (seen != 7) t->err = 1;
}

/* ------------------------------------------------------------------------ */
/* file open: file_meta.go:14-62, schema.go:789-1000                         */
/* ------------------------------------------------------------------------ */

static void free_file(pqref_file *f) {
  if (!f) return;
  for (int i = 0; i < f->nschema; i++) free(f->schema[i].name);
  free(f->schema);
  for (int i = 0; i < f->nrgs; i++) free(f->rgs[i].cols);
  free(f->rgs);
  free(f->leaves);
  free(f);
}

/* readSchema/readGroupSchema/readColumnSchema: depth-first walk, leaves in
 * schema order, def/rep increments at :800-806. */
static int walk_schema(pqref_file *f, int *idx, const char *prefix, int d, int r, int rep_def, int depth) {
  if (depth > 64) return PQR_ERR_SCHEMA;
  if (*idx >= f->nschema) return PQR_ERR_SCHEMA;
  sch_elem *e = &f->schema[*idx];
  if (!e->name || e->name[0] == 0) return PQR_ERR_SCHEMA;
  if (!e->has_rep) return PQR_ERR_SCHEMA; /* "field RepetitionType is nil" */
  if (e->repetition != 0) d++;
  if (e->repetition == 2) {
    r++;
    rep_def = d;
  }
  char name[512];
  if (prefix[0]) snprintf(name, sizeof(name), "%s.%s", prefix, e->name);
  else snprintf(name, sizeof(name), "%s", e->name);
  (*idx)++;
  if (!e->has_children || e->num_children == 0) {
    if (!e->has_type) return PQR_ERR_SCHEMA;
    if (e->has_children && e->num_children == 0 && !e->has_type) return PQR_ERR_SCHEMA;
    f->leaves = (pqref_leaf *)realloc(f->leaves, sizeof(pqref_leaf) * (size_t)(f->nleaves + 1));
    pqref_leaf *L = &f->leaves[f->nleaves++];
    memset(L, 0, sizeof(*L));
    snprintf(L->name, sizeof(L->name), "%s", name);
    L->physical_type = e->type;
    L->type_length = e->type_length;
    L->max_def = d;
    L->max_rep = r;
    L->rep_def = rep_def;
    L->converted_type = e->converted;
    int uns = 0;
    if (e->type == PQR_INT32 && (e->converted == 11 || e->converted == 12 || e->converted == 13)) uns = 1;
    if (e->type == PQR_INT64 && e->converted == 14) uns = 1;
    if (e->int_unsigned) uns = 1;
    L->unsigned_int = uns;
    return 0;
  }
  for (int c = 0; c < e->num_children; c++) {
    int rc = walk_schema(f, idx, name, d, r, rep_def, depth + 1);
    if (rc) return rc;
  }
  return 0;
}

int pqref_open(const uint8_t *buf, size_t len, pqref_file **out, char *err, size_t errcap) {
  *out = NULL;
  if (len < 12 || memcmp(buf, "PAR1", 4) != 0) {
    if (err) snprintf(err, errcap, "invalid parquet file header");
    return PQR_ERR_FORMAT;
  }
  if (memcmp(buf + len - 4, "PAR1", 4) != 0) {
    if (err) snprintf(err, errcap, "invalid parquet file footer");
    return PQR_ERR_FORMAT;
  }
  int32_t fl = (int32_t)le32(buf + len - 8);
  if (fl <= 0 || (size_t)fl > len - 8) {
    if (err) snprintf(err, errcap, "invalid footer len %d", fl);
    return PQR_ERR_FORMAT;
  }
  pqref_file *f = (pqref_file *)calloc(1, sizeof(pqref_file));
  f->buf = buf;
  f->len = len;
  tproto t = {buf + len - 8 - fl, (size_t)fl, 0, 0, 0};
  read_file_meta(&t, f);
  if (t.err) {
    free_file(f);
    if (err) snprintf(err, errcap, "read file meta failed");
    return PQR_ERR_THRIFT;
  }
  /* makeSchema: schema[0] is the root; children are schema[1:] */
  if (f->nschema < 1) {
    free_file(f);
    if (err) snprintf(err, errcap, "empty schema");
    return PQR_ERR_SCHEMA;
  }
  int idx = 1;
  int nroot = f->schema[0].num_children;
  for (int c = 0; c < nroot; c++) {
    int rc = walk_schema(f, &idx, "", 0, 0, 0, 0);
    if (rc) {
      free_file(f);
      if (err) snprintf(err, errcap, "invalid schema");
      return rc;
    }
  }
  *out = f;
  return 0;
}

void pqref_close(pqref_file *f) { free_file(f); }
int pqref_num_row_groups(const pqref_file *f) { return f->nrgs; }
int64_t pqref_rg_num_rows(const pqref_file *f, int rg) { return (rg >= 0 && rg < f->nrgs) ? f->rgs[rg].num_rows : -1; }
int64_t pqref_num_rows(const pqref_file *f) { return f->num_rows; }
int pqref_num_leaves(const pqref_file *f) { return f->nleaves; }
int pqref_leaf_info(const pqref_file *f, int leaf, pqref_leaf *out) {
  if (leaf < 0 || leaf >= f->nleaves) return PQR_ERR_ARG;
  *out = f->leaves[leaf];
  return 0;
}

/* ------------------------------------------------------------------------ */
/* values decoders                                                           */
/* ------------------------------------------------------------------------ */

enum { ENC_PLAIN = 0, ENC_PLAIN_DICT = 2, ENC_RLE = 3, ENC_BIT_PACKED = 4, ENC_DELTA_BP = 5,
       ENC_DELTA_LBA = 6, ENC_DELTA_BA = 7, ENC_RLE_DICT = 8 };

static int value_width(const pqref_leaf *L) {
  switch (L->physical_type) {
    case PQR_INT32: case PQR_FLOAT: return 4;
    case PQR_INT64: case PQR_DOUBLE: return 8;
    case PQR_INT96: return 12;
    case PQR_FLBA: return L->type_length;
    case PQR_BOOLEAN: return 1; /* one byte (0 / 1) per value */
    default: return 0; /* BYTE_ARRAY: variable */
  }
}

/* dictionary as decoded values (page_dict.go:30-64) */
typedef struct {
  int present;
  int64_t n;
  uint8_t *fixed;        /* n * width */
  int64_t *str_off;      /* n + 1 (BYTE_ARRAY) */
  uint8_t *str_bytes;
} dictionary;

/* decoded page (dense), what readValues produces (page_v1.go:27-55) */
typedef struct {
  int64_t n;              /* num_values (level entries) */
  uint8_t *def, *rep;
  int64_t non_null;
  bytebuf vals;           /* fixed: non_null * width; BYTE_ARRAY: concatenated bytes */
  bytebuf lens;           /* BYTE_ARRAY: int64 lengths */
} dense_page;

typedef struct {
  /* page reader state after readPages (phase 1) */
  int is_v2;
  page_header h;
  int enc;
  uint8_t *body;          /* owned decompressed values section (V1: whole body) */
  size_t body_len;
  int own_body;
  /* level streams */
  hybrid rl, dl;
  int rl_const, dl_const;
  /* values stream */
  rdr vr;
  /* dict index state */
  hybrid keys;
  /* delta state */
  struct {
    int32_t block_size, mb_count, values_count, mb_value_count;
    int64_t prev, min_delta;
    uint8_t *widths;        /* mb_count bytes of the current block */
    int32_t cur_mb;
    uint8_t cur_w;
    int32_t mb_pos, position;
    int64_t group[8];
    int is32;
  } dl_state;
  /* DELTA_LENGTH_BYTE_ARRAY / DELTA_BYTE_ARRAY (type_bytearray.go:98-240) */
  int32_t *pre, *suf;     /* prefix lengths (DELTA_BYTE_ARRAY), suffix / value lengths */
  int32_t npre, nsuf, lpos;
  bytebuf prev;           /* previous value (DELTA_BYTE_ARRAY) */
} page_reader;

/* ---- DELTA_BINARY_PACKED: deltabp_decoder.go:14-334 ---- */
static int delta_read_mb_header(page_reader *p) { /* :248-271 / :95-121 */
  int64_t md;
  int e = rd_varint64(&p->vr, &md);
  if (e) return e == PQR_ERR_EOF ? PQR_ERR_EOF : PQR_ERR_DELTA;
  if (p->dl_state.is32 && (md > 0x7fffffffLL || md < -0x80000000LL)) return PQR_ERR_DELTA;
  p->dl_state.min_delta = md;
  int32_t m = p->dl_state.mb_count;
  /* make([]uint8, miniBlockCount) + io.ReadFull: any count; a count past the
     stream's end fails the read (allocated only when the bytes are there) */
  if ((size_t)m > p->vr.n - p->vr.pos) {
    p->vr.pos = p->vr.n;
    return PQR_ERR_EOF;
  }
  if (!p->dl_state.widths) {
    p->dl_state.widths = (uint8_t *)malloc((size_t)m);
    if (!p->dl_state.widths) return PQR_ERR_DELTA;
  }
  if (rd_full(&p->vr, p->dl_state.widths, (size_t)m)) return PQR_ERR_EOF;
  int maxw = p->dl_state.is32 ? 32 : 64;
  for (int32_t i = 0; i < m; i++)
    if (p->dl_state.widths[i] > maxw) return PQR_ERR_BITWIDTH;
  p->dl_state.cur_mb = 0;
  return 0;
}
static void delta_free(page_reader *p) {
  free(p->dl_state.widths);
  p->dl_state.widths = NULL;
}
static int delta_init(page_reader *p, int is32) { /* :197-246 */
  delta_free(p);
  memset(&p->dl_state, 0, sizeof(p->dl_state));
  p->dl_state.is32 = is32;
  int32_t bs, mc, vc;
  int e = rd_uvarint32(&p->vr, &bs, PQR_ERR_DELTA);
  if (e) return e;
  /* (bs <= 0 && bs%128 != 0) can never hold for a uvarint32 — reproduced as is */
  e = rd_uvarint32(&p->vr, &mc, PQR_ERR_DELTA);
  if (e) return e;
  if (mc <= 0 || bs % mc != 0) return PQR_ERR_DELTA;
  if (bs / mc == 0) return PQR_ERR_DELTA;
  e = rd_uvarint32(&p->vr, &vc, PQR_ERR_DELTA);
  if (e) return e;
  int64_t first;
  e = rd_varint64(&p->vr, &first);
  if (e) return e == PQR_ERR_EOF ? PQR_ERR_EOF : PQR_ERR_DELTA;
  if (is32 && (first > 0x7fffffffLL || first < -0x80000000LL)) return PQR_ERR_DELTA;
  p->dl_state.block_size = bs;
  p->dl_state.mb_count = mc;
  p->dl_state.mb_value_count = bs / mc;
  p->dl_state.values_count = vc;
  p->dl_state.prev = first;
  return delta_read_mb_header(p);
}
static int delta_next(page_reader *p, int64_t *out) { /* :273-334 */
  typeof(p->dl_state) *d = &p->dl_state;
  if (d->position >= d->values_count) return PQR_ERR_EOF;
  if (d->position % 8 == 0) {
    if (d->position % d->mb_value_count == 0) {
      if (d->cur_mb >= d->mb_count) {
        int e = delta_read_mb_header(p);
        if (e) return e;
      }
      d->cur_w = d->widths[d->cur_mb];
      d->mb_pos = 0;
      d->cur_mb++;
    }
    int32_t w = d->cur_w;
    uint8_t buf[64];
    if (rd_full(&p->vr, buf, (size_t)w)) return PQR_ERR_EOF;
    if (d->is32) {
      int32_t g[8];
      pqref_unpack8_32(buf, w, g);
      for (int i = 0; i < 8; i++) d->group[i] = g[i];
    } else {
      pqref_unpack8_64(buf, w, d->group);
    }
    d->mb_pos += w;
    if (d->position + 8 >= d->values_count) {
      int32_t sl = (d->mb_value_count / 8) * w - d->mb_pos;
      if (sl < 0) return PQR_ERR_DELTA;
      /* padding skips: errors ignored, reads harmless for a values section that ends the page */
      size_t skip = (size_t)sl;
      p->vr.pos = (p->vr.n - p->vr.pos < skip) ? p->vr.n : p->vr.pos + skip;
      for (int32_t i = d->cur_mb; i < d->mb_count; i++) {
        int32_t w2 = d->widths[d->cur_mb]; /* sic: index cur_mb (D5) */
        if (w2 != 0) {
          size_t s2 = (size_t)((d->mb_value_count / 8) * w2);
          p->vr.pos = (p->vr.n - p->vr.pos < s2) ? p->vr.n : p->vr.pos + s2;
        }
      }
    }
  }
  int64_t ret = d->prev;
  if (d->is32) {
    uint32_t nv = (uint32_t)(int32_t)d->prev + (uint32_t)(int32_t)d->group[d->position % 8] + (uint32_t)(int32_t)d->min_delta;
    d->prev = (int32_t)nv;
  } else {
    uint64_t nv = (uint64_t)d->prev + (uint64_t)d->group[d->position % 8] + (uint64_t)d->min_delta;
    d->prev = (int64_t)nv;
  }
  d->position++;
  *out = ret;
  return 0;
}

/* decodeInt32 over a fresh deltaBitPackDecoder32 on the page reader
   (helpers.go:119-129, deltabp_decoder.go:14-175): every valuesCount value is
   decoded, the reader left where the decoder's reads and padding skips leave it */
static int delta_lengths(page_reader *p, int32_t **out, int32_t *count) {
  *out = NULL;
  *count = 0;
  int e = delta_init(p, 1);
  if (e) return e;
  int32_t vc = p->dl_state.values_count;
  size_t cap = 0;
  int32_t *a = NULL;
  for (int32_t i = 0; i < vc; i++) {
    int64_t v;
    e = delta_next(p, &v);
    if (e) {
      free(a);
      return e;
    }
    if ((size_t)i >= cap) { /* grown as decoded: a corrupt count fails before a huge allocation */
      cap = cap ? 2 * cap : 1024;
      a = (int32_t *)realloc(a, cap * sizeof(int32_t));
    }
    a[i] = (int32_t)v;
  }
  *out = a;
  *count = vc;
  return 0;
}

/* ------------------------------------------------------------------------ */
/* page reading (phase 1) and decoding (phase 2)                             */
/* ------------------------------------------------------------------------ */

/* newBlockReader compress.go:102-122 */
static int block_reader(const pqref_file *f, size_t off, size_t chunk_end, int codec, int32_t csize, int32_t usize,
                        uint8_t **out, size_t *out_len, int *own) {
  if (csize < 0 || usize < 0) return PQR_ERR_SIZE; /* createDataReader chunk_reader.go:199-201 */
  if (off > f->len || (size_t)csize > f->len - off) return PQR_ERR_SIZE; /* short read :108-110 */
  (void)chunk_end;
  const uint8_t *src = f->buf + off;
  if (codec == 0) { /* UNCOMPRESSED */
    if (csize != usize) return PQR_ERR_SIZE;
    *out = (uint8_t *)src;
    *out_len = (size_t)csize;
    *own = 0;
    return 0;
  }
  if (codec == 1) { /* SNAPPY */
    uint8_t *dst = NULL;
    int e = snappy_decode_checked(src, (size_t)csize, (size_t)usize, &dst);
    if (e) return e;
    *out = dst;
    *out_len = (size_t)usize;
    *own = 1;
    return 0;
  }
#ifdef PQREF_HAVE_ZLIB
  if (codec == 2) { /* GZIP via zlib (Go compress/gzip equivalent; parity unpinned) */
    uint8_t *dst = (uint8_t *)malloc(usize ? (size_t)usize : 1);
    z_stream zs;
    memset(&zs, 0, sizeof(zs));
    if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) {
      free(dst);
      return PQR_ERR_CODEC;
    }
    zs.next_in = (Bytef *)src;
    zs.avail_in = (uInt)csize;
    zs.next_out = dst;
    zs.avail_out = (uInt)usize;
    int rc = inflate(&zs, Z_FINISH);
    size_t got = (size_t)usize - zs.avail_out;
    inflateEnd(&zs);
    if (rc != Z_STREAM_END) {
      free(dst);
      return rc == Z_BUF_ERROR ? PQR_ERR_SIZE : PQR_ERR_CODEC;
    }
    if (got != (size_t)usize) {
      free(dst);
      return PQR_ERR_SIZE;
    }
    *out = dst;
    *out_len = got;
    *own = 1;
    return 0;
  }
#endif
  return PQR_ERR_CODEC;
}

static int supported_value_encoding(const pqref_leaf *L, int enc, int has_dict) {
  (void)has_dict;
  if (enc == ENC_PLAIN_DICT) enc = ENC_RLE_DICT; /* chunk_reader.go:145-147 */
  switch (L->physical_type) {
    case PQR_BYTE_ARRAY:
      return enc == ENC_PLAIN || enc == ENC_RLE_DICT || enc == ENC_DELTA_LBA || enc == ENC_DELTA_BA ? 0 : PQR_ERR_ENCODING;
    case PQR_FLBA:
      return enc == ENC_PLAIN || enc == ENC_RLE_DICT || enc == ENC_DELTA_BA ? 0 : PQR_ERR_ENCODING;
    case PQR_FLOAT:
    case PQR_DOUBLE:
    case PQR_INT96:
      return enc == ENC_PLAIN || enc == ENC_RLE_DICT ? 0 : PQR_ERR_ENCODING;
    case PQR_INT32:
    case PQR_INT64:
      return enc == ENC_PLAIN || enc == ENC_RLE_DICT || enc == ENC_DELTA_BP ? 0 : PQR_ERR_ENCODING;
    case PQR_BOOLEAN: /* getBooleanValuesDecoder chunk_reader.go:58-69; dictionaries of booleans are not built */
      return enc == ENC_PLAIN || enc == ENC_RLE ? 0 : enc == ENC_RLE_DICT ? PQR_ERR_UNSUPPORTED : PQR_ERR_ENCODING;
  }
  return PQR_ERR_ENCODING;
}

static int bits_len16(int v) {
  int n = 0;
  while (v) {
    n++;
    v >>= 1;
  }
  return n;
}

/* values init (valuesDecoder.init) */
static int values_init(page_reader *p, const pqref_leaf *L) {
  int enc = p->enc == ENC_PLAIN_DICT ? ENC_RLE_DICT : p->enc;
  if (enc == ENC_RLE_DICT) { /* type_dict.go:22-37 */
    uint8_t w;
    if (rd_full(&p->vr, &w, 1)) return PQR_ERR_EOF;
    if (w > 32) return PQR_ERR_BITWIDTH;
    hy_new(&p->keys, w);
    hy_init(&p->keys, p->vr.p + p->vr.pos, p->vr.n - p->vr.pos);
    return 0;
  }
  if (enc == ENC_DELTA_BP) return delta_init(p, L->physical_type == PQR_INT32);
  if ((enc == ENC_DELTA_LBA && L->physical_type == PQR_BYTE_ARRAY) ||
      (enc == ENC_DELTA_BA && (L->physical_type == PQR_BYTE_ARRAY || L->physical_type == PQR_FLBA))) {
    /* FIXED_LEN_BYTE_ARRAY DELTA_BYTE_ARRAY: the same byteArrayDeltaDecoder
       (getFixedLenByteArrayValuesDecoder chunk_reader.go:86-96);
       byteArrayDeltaDecoder.init :186-209 (prefix lengths, then the suffixes'
       DELTA_LENGTH stream); byteArrayDeltaLengthDecoder.init :98-108 */
    int e;
    if (enc == ENC_DELTA_BA) {
      e = delta_lengths(p, &p->pre, &p->npre);
      if (e) return e;
    }
    e = delta_lengths(p, &p->suf, &p->nsuf);
    if (e) return e;
    if (enc == ENC_DELTA_BA && p->npre != p->nsuf) return PQR_ERR_BYTE_ARRAY; /* "different number of suffixes and prefixes" */
    p->lpos = 0;
    return 0;
  }
  if (enc == ENC_RLE && L->physical_type == PQR_BOOLEAN) {
    /* booleanRLEDecoder.init type_boolean.go:101-104: hybridDecoder(1).initSize
       (hybrid_decoder.go:57-67): u32 LE size, then a LimitReader over the rest */
    uint8_t lb[4];
    if (rd_full(&p->vr, lb, 4)) return PQR_ERR_EOF;
    size_t sz = le32(lb);
    size_t take = p->vr.n - p->vr.pos < sz ? p->vr.n - p->vr.pos : sz;
    hy_new(&p->keys, 1);
    hy_init(&p->keys, p->vr.p + p->vr.pos, take);
    return 0;
  }
  return 0; /* PLAIN decoders just keep the reader */
}

/* decodeValues for notNull values (phase 2) */
static int values_decode(page_reader *p, const pqref_leaf *L, const dictionary *dict, int64_t count, dense_page *dp) {
  int enc = p->enc == ENC_PLAIN_DICT ? ENC_RLE_DICT : p->enc;
  int w = value_width(L);
  if (enc == ENC_RLE_DICT) {
    if (!dict || !dict->present) {
      /* dictDecoder with nil values: size 0 → every key is out of range */
      if (count > 0) {
        int32_t k;
        int e = hy_next(&p->keys, &k);
        return e ? e : PQR_ERR_DICT_INDEX;
      }
      return 0;
    }
    for (int64_t i = 0; i < count; i++) {
      int32_t k;
      int e = hy_next(&p->keys, &k);
      if (e) return e;
      if (k < 0 || (int64_t)k >= dict->n) return PQR_ERR_DICT_INDEX;
      if (L->physical_type == PQR_BYTE_ARRAY) {
        int64_t a = dict->str_off[k], b = dict->str_off[k + 1];
        int64_t len = b - a;
        bb_put(&dp->lens, &len, 8);
        bb_put(&dp->vals, dict->str_bytes + a, (size_t)len);
      } else {
        bb_put(&dp->vals, dict->fixed + (size_t)k * (size_t)w, (size_t)w);
      }
    }
    return 0;
  }
  if (enc == ENC_DELTA_BP) {
    for (int64_t i = 0; i < count; i++) {
      int64_t v;
      int e = delta_next(p, &v);
      if (e) return e;
      if (L->physical_type == PQR_INT32) {
        int32_t v32 = (int32_t)v;
        bb_put(&dp->vals, &v32, 4);
      } else {
        bb_put(&dp->vals, &v, 8);
      }
    }
    return 0;
  }
  if (L->physical_type == PQR_BOOLEAN) {
    if (enc == ENC_RLE) { /* booleanRLEDecoder.decodeValues type_boolean.go:106-117 */
      for (int64_t i = 0; i < count; i++) {
        int32_t b;
        int e = hy_next(&p->keys, &b);
        if (e) return e;
        uint8_t v = b == 1;
        bb_put(&dp->vals, &v, 1);
      }
      return 0;
    }
    /* booleanPlainDecoder.decodeValues type_boolean.go:43-68: one byte per 8
       values, LSB first (unpack8int32_1), read only while values remain */
    for (int64_t i = 0; i < count; i += 8) {
      uint8_t byte;
      if (rd_full(&p->vr, &byte, 1)) return PQR_ERR_EOF;
      for (int j = 0; j < 8 && i + j < count; j++) {
        uint8_t v = (byte >> j) & 1;
        bb_put(&dp->vals, &v, 1);
      }
    }
    return 0;
  }
  if (enc == ENC_DELTA_LBA || enc == ENC_DELTA_BA) {
    for (int64_t i = 0; i < count; i++) {
      /* byteArrayDeltaLengthDecoder.next :111-123 */
      if (p->lpos >= p->nsuf) return PQR_ERR_EOF;
      int32_t size = p->suf[p->lpos];
      if (size < 0) return PQR_ERR_BYTE_ARRAY; /* the reference panics in make([]byte, size) */
      if (p->vr.n - p->vr.pos < (size_t)size) return PQR_ERR_EOF; /* io.ReadFull: "there is no byte left" */
      const uint8_t *suffix = p->vr.p + p->vr.pos;
      p->vr.pos += (size_t)size;
      p->lpos++;
      int64_t len;
      if (enc == ENC_DELTA_LBA) {
        len = size;
        bb_put(&dp->lens, &len, 8);
        bb_put(&dp->vals, suffix, (size_t)size);
        continue;
      }
      /* byteArrayDeltaDecoder.decodeValues :211-240 */
      int32_t pl = p->pre[p->lpos - 1];
      if ((int64_t)pl + size < 0) return PQR_ERR_BYTE_ARRAY; /* make with a negative capacity panics */
      if ((int64_t)p->prev.n < (int64_t)pl) return PQR_ERR_BYTE_ARRAY; /* "invalid prefix len" */
      bytebuf v = {0};
      if (pl > 0) bb_put(&v, p->prev.p, (size_t)pl);
      bb_put(&v, suffix, (size_t)size);
      len = (int64_t)v.n;
      if (L->physical_type == PQR_FLBA) {
        /* a fixed-size slot holds type_length bytes: a value of another length
           (the reference keeps it as a []byte) cannot be laid out -- the one
           documented deviation */
        if (len != (int64_t)w) {
          free(v.p);
          return PQR_ERR_BYTE_ARRAY;
        }
      } else {
        bb_put(&dp->lens, &len, 8);
      }
      bb_put(&dp->vals, v.p, v.n);
      free(p->prev.p);
      p->prev = v;
    }
    return 0;
  }
  /* PLAIN */
  if (L->physical_type == PQR_BYTE_ARRAY) { /* type_bytearray.go:24-55 */
    for (int64_t i = 0; i < count; i++) {
      uint8_t lb[4];
      if (rd_full(&p->vr, lb, 4)) return PQR_ERR_EOF;
      int32_t l = (int32_t)le32(lb);
      if (l < 0) return PQR_ERR_BYTE_ARRAY;
      if (p->vr.n - p->vr.pos < (size_t)l) return PQR_ERR_EOF;
      int64_t len = l;
      bb_put(&dp->lens, &len, 8);
      bb_put(&dp->vals, p->vr.p + p->vr.pos, (size_t)l);
      p->vr.pos += (size_t)l;
    }
    return 0;
  }
  if (w <= 0) return PQR_ERR_UNSUPPORTED;
  /* binary.Read per value (type_int32.go:23-37 etc.) */
  for (int64_t i = 0; i < count; i++) {
    if (p->vr.n - p->vr.pos < (size_t)w) return PQR_ERR_EOF;
    bb_put(&dp->vals, p->vr.p + p->vr.pos, (size_t)w);
    p->vr.pos += (size_t)w;
  }
  return 0;
}

/* dictionary page (page_dict.go:30-64) */
static int read_dict_page(const pqref_file *f, const pqref_leaf *L, const page_header *h, size_t off, int codec,
                          dictionary *dict) {
  if (!h->has_dict) return PQR_ERR_PAGE;
  if (h->dict_num_values < 0) return PQR_ERR_PAGE;
  if (h->dict_encoding != ENC_PLAIN && h->dict_encoding != ENC_PLAIN_DICT) return PQR_ERR_ENCODING;
  uint8_t *body;
  size_t blen;
  int own;
  int e = block_reader(f, off, 0, codec, h->compressed, h->uncompressed, &body, &blen, &own);
  if (e) return e;
  rdr r = {body, blen, 0};
  int64_t n = h->dict_num_values;
  dict->n = n;
  dict->present = 1;
  if (L->physical_type == PQR_BYTE_ARRAY) {
    dict->str_off = (int64_t *)malloc(sizeof(int64_t) * (size_t)(n + 1));
    bytebuf bytes = {0};
    dict->str_off[0] = 0;
    for (int64_t i = 0; i < n && !e; i++) {
      uint8_t lb[4];
      if (rd_full(&r, lb, 4)) {
        e = PQR_ERR_EOF;
        break;
      }
      int32_t l = (int32_t)le32(lb);
      if (l < 0) {
        e = PQR_ERR_BYTE_ARRAY;
        break;
      }
      if (r.n - r.pos < (size_t)l) {
        e = PQR_ERR_EOF;
        break;
      }
      bb_put(&bytes, r.p + r.pos, (size_t)l);
      r.pos += (size_t)l;
      dict->str_off[i + 1] = dict->str_off[i] + l;
    }
    dict->str_bytes = bytes.p;
  } else {
    int w = value_width(L);
    if (w <= 0 || L->physical_type == PQR_BOOLEAN) e = PQR_ERR_UNSUPPORTED; /* boolean dictionaries: not built */
    else if ((size_t)n * (size_t)w > blen) e = PQR_ERR_EOF;
    else {
      dict->fixed = (uint8_t *)malloc((size_t)n * (size_t)w + 1);
      memcpy(dict->fixed, body, (size_t)n * (size_t)w);
    }
  }
  if (own) free(body);
  return e;
}

/* phase 1 for a data page: p.init + p.read (page_v1.go:57-108, page_v2.go:56-129) */
static int read_data_page(const pqref_file *f, const pqref_leaf *L, const page_header *h, size_t off, int codec,
                          page_reader *p) {
  int maxr_bw = bits_len16(L->max_rep), maxd_bw = bits_len16(L->max_def);
  p->rl_const = L->max_rep == 0;
  p->dl_const = L->max_def == 0;
  hy_new(&p->rl, maxr_bw);
  hy_new(&p->dl, maxd_bw);
  if (h->type == 0) { /* DATA_PAGE */
    p->is_v2 = 0;
    /* init: nil header check and level encodings (chunk_reader.go:348-364) */
    if (!h->has_dph) return PQR_ERR_PAGE;
    if (!p->rl_const && h->dp_rep_enc != ENC_RLE) return PQR_ERR_ENCODING;
    if (!p->dl_const && h->dp_def_enc != ENC_RLE) return PQR_ERR_ENCODING;
    /* read */
    if (h->dp_num_values < 0) return PQR_ERR_PAGE;
    int e = block_reader(f, off, 0, codec, h->compressed, h->uncompressed, &p->body, &p->body_len, &p->own_body);
    if (e) return e;
    p->enc = h->dp_encoding;
    e = supported_value_encoding(L, p->enc, 1);
    if (e) return e;
    rdr br = {p->body, p->body_len, 0};
    /* rDecoder.initSize then dDecoder.initSize (hybrid_decoder.go:57-67, buffered) */
    if (!p->rl_const && maxr_bw > 0) {
      uint8_t lb[4];
      if (rd_full(&br, lb, 4)) return PQR_ERR_EOF;
      size_t sz = le32(lb);
      size_t take = br.n - br.pos < sz ? br.n - br.pos : sz;
      hy_init(&p->rl, br.p + br.pos, take);
      br.pos += take;
    }
    if (!p->dl_const && maxd_bw > 0) {
      uint8_t lb[4];
      if (rd_full(&br, lb, 4)) return PQR_ERR_EOF;
      size_t sz = le32(lb);
      size_t take = br.n - br.pos < sz ? br.n - br.pos : sz;
      hy_init(&p->dl, br.p + br.pos, take);
      br.pos += take;
    }
    p->vr = br;
    return values_init(p, L);
  }
  if (h->type == 3) { /* DATA_PAGE_V2 */
    p->is_v2 = 1;
    if (!h->has_v2) return PQR_ERR_PAGE;
    if (h->v2_num_values < 0) return PQR_ERR_PAGE;
    if (h->v2_rep_len < 0 || h->v2_def_len < 0) return PQR_ERR_PAGE;
    p->enc = h->v2_encoding;
    int e = supported_value_encoding(L, p->enc, 1);
    if (e) return e;
    int32_t lsize = h->v2_rep_len + h->v2_def_len;
    if (lsize > 0) {
      if (off > f->len || (size_t)lsize > f->len - off) return PQR_ERR_EOF;
      const uint8_t *lv = f->buf + off;
      if (h->v2_rep_len > 0 && !p->rl_const) hy_init(&p->rl, lv, (size_t)h->v2_rep_len);
      if (h->v2_def_len > 0 && !p->dl_const) hy_init(&p->dl, lv + h->v2_rep_len, (size_t)h->v2_def_len);
    }
    /* is_compressed is ignored by the reference (page_v2.go:123; D4) */
    e = block_reader(f, off + (size_t)(lsize > 0 ? lsize : 0), 0, codec, h->compressed - lsize, h->uncompressed - lsize,
                     &p->body, &p->body_len, &p->own_body);
    if (e) return e;
    p->vr.p = p->body;
    p->vr.n = p->body_len;
    p->vr.pos = 0;
    return values_init(p, L);
  }
  return PQR_ERR_PAGE; /* "DATA_PAGE or DATA_PAGE_V2 type supported" */
}

/* phase 2: readValues (page_v1.go:27-55) */
static int decode_data_page(page_reader *p, const pqref_leaf *L, const dictionary *dict, dense_page *dp) {
  int64_t n = p->is_v2 ? p->h.v2_num_values : p->h.dp_num_values;
  dp->n = n;
  dp->def = (uint8_t *)calloc((size_t)n + 1, 1);
  dp->rep = (uint8_t *)calloc((size_t)n + 1, 1);
  if (n == 0) return 0;
  for (int64_t i = 0; i < n; i++) {
    int32_t v = 0;
    if (!p->rl_const) {
      int e = hy_next(&p->rl, &v);
      if (e) return e;
    }
    dp->rep[i] = (uint8_t)v;
  }
  int64_t nn = 0;
  for (int64_t i = 0; i < n; i++) {
    int32_t v = 0;
    if (!p->dl_const) {
      int e = hy_next(&p->dl, &v);
      if (e) return e;
    }
    dp->def[i] = (uint8_t)v;
    if (v == L->max_def) nn++;
  }
  dp->non_null = nn;
  if (nn != 0) return values_decode(p, L, dict, nn, dp);
  return 0;
}

/* ------------------------------------------------------------------------ */
/* column decode + Arrow layout                                              */
/* ------------------------------------------------------------------------ */

struct pqref_result {
  int status;
  char err[256];
  int err_rg, err_page;
  int64_t counts[8];
  bytebuf bufs[8];
};

static void set_err(pqref_result *r, int code, int rg, int page, const char *fmt, ...) {
  if (r->status) return;
  r->status = code;
  r->err_rg = rg;
  r->err_page = page;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(r->err, sizeof(r->err), fmt, ap);
  va_end(ap);
}

static void bit_set(bytebuf *b, int64_t i) { b->p[i >> 3] |= (uint8_t)(1u << (i & 7)); }

/* readChunk + readPages, phase 1 (chunk_reader.go:206-346, :314-346): the
 * dictionary page decoded into *dict, every data page initialised (p.init +
 * p.read) into *pages_out; errors into R (the first one ends the chunk) */
static void read_chunk_pages(const pqref_file *f, const pqref_leaf *L, int leaf, int rg, pqref_result *R,
                             dictionary *dict, page_reader **pages_out, int *npages_out) {
  *pages_out = NULL;
  *npages_out = 0;
  {
    const row_group *G = &f->rgs[rg];
    if (leaf >= G->ncols) {
      set_err(R, PQR_ERR_PAGE, rg, -1, "column index %d is out of bounds", leaf);
      return;
    }
    const col_chunk *C = &G->cols[leaf];
    /* readChunk chunk_reader.go:314-346 */
    if (C->has_file_path) {
      set_err(R, PQR_ERR_PAGE, rg, -1, "nyi: data is in another file");
      return;
    }
    if (!C->has_meta) {
      set_err(R, PQR_ERR_PAGE, rg, -1, "missing meta data");
      return;
    }
    if (C->type != L->physical_type) {
      set_err(R, PQR_ERR_PAGE, rg, -1, "wrong type in Column chunk metadata");
      return;
    }
    int64_t offset = C->has_dict_off ? C->dict_page_offset : C->data_page_offset;
    if (offset < 0 || (uint64_t)offset > f->len) {
      set_err(R, PQR_ERR_SIZE, rg, -1, "seek out of range");
      return;
    }
    /* readPages :206-284 — phase 1 over all pages */
    int64_t pos = offset, count = 0;
    page_reader *pages = NULL;
    int npages = 0, page_idx = 0;
    while (C->total_compressed - count > 0) {
      tproto t = {f->buf + pos, f->len - (size_t)pos, 0, 0, 0};
      page_header h;
      read_page_header(&t, &h);
      if (t.err) {
        set_err(R, PQR_ERR_THRIFT, rg, page_idx, "page header");
        break;
      }
      pos += (int64_t)t.pos;
      count += (int64_t)t.pos;
      int32_t csz = h.compressed;
      if (h.type == 2) { /* DICTIONARY_PAGE */
        if (dict->present) {
          set_err(R, PQR_ERR_PAGE, rg, page_idx, "there should be only one dictionary");
          break;
        }
        if (!h.has_dict) {
          set_err(R, PQR_ERR_PAGE, rg, page_idx, "null DictionaryPageHeader");
          break;
        }
        if (L->physical_type == PQR_FLBA && L->type_length <= 0) { /* getDictValuesDecoder :20-24 */
          set_err(R, PQR_ERR_SCHEMA, rg, page_idx, "nil type len");
          break;
        }
        int e = read_dict_page(f, L, &h, (size_t)pos, C->codec, dict);
        if (e) {
          set_err(R, e, rg, page_idx, "dictionary page");
          break;
        }
        if (csz > 0) {
          pos += csz;
          count += csz;
        }
        /* seek back to data_page_offset if the dictionary did not end there (:243-249) */
        if (C->has_dict_off && C->dict_page_offset != pos) {
          count += C->data_page_offset - pos;
          pos = C->data_page_offset;
          if (pos < 0 || (uint64_t)pos > f->len) {
            set_err(R, PQR_ERR_SIZE, rg, page_idx, "seek");
            break;
          }
        }
        page_idx++;
        continue;
      }
      if (h.type != 0 && h.type != 3) {
        set_err(R, PQR_ERR_PAGE, rg, page_idx, "DATA_PAGE or DATA_PAGE_V2 type supported");
        break;
      }
      pages = (page_reader *)realloc(pages, sizeof(page_reader) * (size_t)(npages + 1));
      page_reader *p = &pages[npages];
      memset(p, 0, sizeof(*p));
      p->h = h;
      npages++;
      int e = read_data_page(f, L, &h, (size_t)pos, C->codec, p);
      if (e) {
        set_err(R, e, rg, page_idx, "data page read");
        break;
      }
      if (csz > 0) {
        pos += csz;
        count += csz;
      } else if (csz < 0) {
        set_err(R, PQR_ERR_SIZE, rg, page_idx, "negative size");
        break;
      }
      page_idx++;
      if ((uint64_t)pos > f->len) {
        set_err(R, PQR_ERR_SIZE, rg, page_idx, "chunk beyond file end");
        break;
      }
    }
    *pages_out = pages;
    *npages_out = npages;
  }
}

int pqref_decode(const pqref_file *f, int leaf, int rg0, int rg1, pqref_result **out) {
  pqref_result *R = (pqref_result *)calloc(1, sizeof(pqref_result));
  R->err_rg = -1;
  R->err_page = -1;
  *out = R;
  if (leaf < 0 || leaf >= f->nleaves || rg0 < 0 || rg1 > f->nrgs || rg0 > rg1) {
    set_err(R, PQR_ERR_ARG, -1, -1, "bad arguments");
    return R->status;
  }
  const pqref_leaf *L = &f->leaves[leaf];
  int w = value_width(L);
  int is_ba = L->physical_type == PQR_BYTE_ARRAY;
  R->counts[PQR_CNT_VALUE_WIDTH] = is_ba ? 0 : w;

  /* gather dense per-page results for all row groups */
  bytebuf levels_def = {0}, levels_rep = {0}, dense_vals = {0}, dense_lens = {0};
  int64_t total_levels = 0, total_nonnull = 0, total_pages = 0;

  for (int rg = rg0; rg < rg1 && !R->status; rg++) {
    dictionary dict;
    memset(&dict, 0, sizeof(dict));
    page_reader *pages = NULL;
    int npages = 0;
    read_chunk_pages(f, L, leaf, rg, R, &dict, &pages, &npages);
    /* phase 2: readPageData :380-402 */
    int data_idx = 0;
    for (int i = 0; i < npages && !R->status; i++) {
      dense_page dp;
      memset(&dp, 0, sizeof(dp));
      int e = decode_data_page(&pages[i], L, &dict, &dp);
      if (e) {
        /* map data-page ordinal back to page index (dictionary page first, if any) */
        set_err(R, e, rg, i + (dict.present ? 1 : 0), "read values");
      } else {
        bb_put(&levels_def, dp.def, (size_t)dp.n);
        bb_put(&levels_rep, dp.rep, (size_t)dp.n);
        total_levels += dp.n;
        total_nonnull += dp.non_null;
        bb_put(&dense_vals, dp.vals.p, dp.vals.n);
        bb_put(&dense_lens, dp.lens.p, dp.lens.n);
      }
      free(dp.def);
      free(dp.rep);
      free(dp.vals.p);
      free(dp.lens.p);
      data_idx++;
    }
    total_pages += npages;
    for (int i = 0; i < npages; i++) {
      if (pages[i].own_body) free(pages[i].body);
      free(pages[i].pre);
      free(pages[i].suf);
      free(pages[i].prev.p);
      delta_free(&pages[i]);
    }
    free(pages);
    free(dict.fixed);
    free(dict.str_off);
    free(dict.str_bytes);
  }

  if (!R->status) {
    /* Arrow layout */
    int64_t n = total_levels;
    const uint8_t *def = levels_def.p, *rep = levels_rep.p;
    int64_t slots = 0, rows = 0;
    int maxd = L->max_def, maxr = L->max_rep;
    if (maxr == 0) {
      slots = n;
      rows = n;
    } else if (maxr == 1) {
      for (int64_t i = 0; i < n; i++) {
        if (rep[i] == 0) rows++;
        if (def[i] >= L->rep_def) slots++;
      }
    } else {
      slots = total_nonnull; /* dense only for deeper nesting */
    }
    R->counts[PQR_CNT_LEVELS] = n;
    R->counts[PQR_CNT_SLOTS] = slots;
    R->counts[PQR_CNT_ROWS] = rows;
    R->counts[PQR_CNT_NONNULL] = total_nonnull;
    R->counts[PQR_CNT_PAGES] = total_pages;
    bb_put(&R->bufs[PQR_BUF_DEF], def, (size_t)n);
    bb_put(&R->bufs[PQR_BUF_REP], rep, (size_t)n);
    bytebuf *V = &R->bufs[PQR_BUF_VALUES], *VB = &R->bufs[PQR_BUF_VALIDITY];
    bb_zero(VB, (size_t)((slots + 7) / 8));
    if (is_ba) {
      bytebuf *SO = &R->bufs[PQR_BUF_STR_OFFSETS];
      int64_t acc = 0;
      bb_put(SO, &acc, 8);
      int64_t k = 0, boff = 0;
      const int64_t *lens = (const int64_t *)dense_lens.p;
      int64_t s = 0;
      for (int64_t i = 0; i < n; i++) {
        int slot = maxr == 0 ? 1 : (maxr == 1 ? def[i] >= L->rep_def : def[i] == maxd);
        if (!slot) continue;
        if (def[i] == maxd) {
          bit_set(VB, s);
          bb_put(V, dense_vals.p + boff, (size_t)lens[k]);
          boff += lens[k];
          acc += lens[k];
          k++;
        }
        bb_put(SO, &acc, 8);
        s++;
      }
      R->counts[PQR_CNT_STR_BYTES] = acc;
    } else {
      int64_t k = 0, s = 0;
      for (int64_t i = 0; i < n; i++) {
        int slot = maxr == 0 ? 1 : (maxr == 1 ? def[i] >= L->rep_def : def[i] == maxd);
        if (!slot) continue;
        if (def[i] == maxd) {
          bit_set(VB, s);
          bb_put(V, dense_vals.p + (size_t)k * (size_t)w, (size_t)w);
          k++;
        } else {
          bb_zero(V, (size_t)w);
        }
        s++;
      }
    }
    if (maxr == 1) {
      bytebuf *LO = &R->bufs[PQR_BUF_LIST_OFFSETS], *LV = &R->bufs[PQR_BUF_LIST_VALIDITY];
      bb_zero(LV, (size_t)((rows + 7) / 8));
      int32_t acc = 0;
      int64_t r = -1;
      for (int64_t i = 0; i < n; i++) {
        if (rep[i] == 0) {
          r++;
          bb_put(LO, &acc, 4);
          if (def[i] >= L->rep_def - 1) bit_set(LV, r);
        }
        if (def[i] >= L->rep_def) acc++;
      }
      bb_put(LO, &acc, 4);
    }
  }
  free(levels_def.p);
  free(levels_rep.p);
  free(dense_vals.p);
  free(dense_lens.p);
  return R->status;
}

/* ------------------------------------------------------------------------ */
/* ref-quirks mode: the values the reference's row reader returns            */
/* ------------------------------------------------------------------------ */
/* Documentation only: the column store the
 * reference fills per row group and reads back row by row, for fixed-width
 * leaves.
 *  - readPageData appends every page's whole `data` slice — numValues slots,
 *    only [:notNull] filled, the rest nil — to the store
 *    (chunk_reader.go:380-402, :397); ColumnStore.get hands the k-th defined
 *    level the store's k-th slot (data_store.go:158-203, dictStore.getNextValue
 *    type_dict.go:114-121).  A page with nulls therefore shifts every later
 *    page's values by its null count, and hands nil to defined levels (D1).
 *  - The store is reset per row group with its capacity kept
 *    (ColumnStore.reset data_store.go:59, dictStore.init type_dict.go:72); the
 *    dictionary page decodes into that backing array when it is large enough
 *    (chunk_reader.go:234-235, page_dict.go:50-53), and the data pages' in-place
 *    appends then overwrite the dictionary entries later pages look up (D2).
 * The store's capacity is modelled as Go's append growth (go 1.13 rules:
 * double below 1024 elements, else 1.25x; large allocations rounded to 8 KiB
 * pages of 16-byte interfaces; the small size classes are not modelled).
 * With row groups of equal size every append after the first row group is in
 * place, whatever the growth rule.
 * Output: BUF_VALUES = one value per defined level (def == max_def) in level
 * order, BUF_VALIDITY = bit k set when that value is not nil; counts LEVELS
 * and NONNULL. */
static int64_t go_grow(int64_t old_cap, int64_t old_len, int64_t need) {
  int64_t c = old_cap, dbl = old_cap + old_cap;
  if (need > dbl) c = need;
  else if (old_len < 1024) c = dbl;
  else
    while (c < need) c += c / 4;
  if (c * 16 > 32768) c = ((c * 16 + 8191) / 8192) * 8192 / 16;
  return c;
}

int pqref_decode_quirks(const pqref_file *f, int leaf, int rg0, int rg1, pqref_result **out) {
  pqref_result *R = (pqref_result *)calloc(1, sizeof(pqref_result));
  R->err_rg = -1;
  R->err_page = -1;
  *out = R;
  if (leaf < 0 || leaf >= f->nleaves || rg0 < 0 || rg1 > f->nrgs || rg0 > rg1) {
    set_err(R, PQR_ERR_ARG, -1, -1, "bad arguments");
    return R->status;
  }
  const pqref_leaf *L = &f->leaves[leaf];
  const int w = value_width(L);
  if (L->physical_type == PQR_BYTE_ARRAY || L->physical_type == PQR_BOOLEAN || w <= 0) {
    set_err(R, PQR_ERR_UNSUPPORTED, -1, -1, "quirks mode: fixed-width leaves only");
    return R->status;
  }
  R->counts[PQR_CNT_VALUE_WIDTH] = w;
  /* the store's backing array: values + nil flags, len / cap in elements */
  uint8_t *sv = NULL, *snil = NULL;
  int64_t slen = 0, scap = 0;
  bytebuf outv = {0}, outnil = {0};
  int64_t nout = 0, nlev = 0;
  for (int rg = rg0; rg < rg1 && !R->status; rg++) {
    slen = 0; /* reset: values[:0], capacity kept */
    dictionary dict;
    memset(&dict, 0, sizeof(dict));
    page_reader *pages = NULL;
    int npages = 0;
    read_chunk_pages(f, L, leaf, rg, R, &dict, &pages, &npages);
    /* the dictionary's entries: the store's array when it holds them (then
       later in-place appends overwrite them), else their own array */
    const uint8_t *dv = dict.fixed, *dnil = NULL;
    uint8_t *own_nil = NULL;
    int aliased = 0;
    if (!R->status && dict.present && dict.n > 0 && scap >= dict.n) {
      memcpy(sv, dict.fixed, (size_t)dict.n * (size_t)w);
      memset(snil, 0, (size_t)dict.n);
      dv = sv;
      dnil = snil;
      aliased = 1;
    }
    /* levels of the row group, for the row reader */
    bytebuf rdef = {0};
    for (int i = 0; i < npages && !R->status; i++) {
      page_reader *p = &pages[i];
      int64_t n = p->is_v2 ? p->h.v2_num_values : p->h.dp_num_values;
      uint8_t *def = (uint8_t *)calloc((size_t)n + 1, 1);
      int e = 0;
      /* readValues: levels, then the first notNull values (page_v1.go:27-55) */
      for (int64_t k = 0; k < n && !e; k++) {
        int32_t v = 0;
        if (!p->rl_const) e = hy_next(&p->rl, &v);
      }
      int64_t nn = 0;
      for (int64_t k = 0; k < n && !e; k++) {
        int32_t v = 0;
        if (!p->dl_const) e = hy_next(&p->dl, &v);
        def[k] = (uint8_t)v;
        nn += v == L->max_def;
      }
      uint8_t *data = (uint8_t *)calloc((size_t)(n + 1) * (size_t)w, 1), *dnl = (uint8_t *)malloc((size_t)n + 1);
      memset(dnl, 1, (size_t)n + 1); /* make([]interface{}, n): nil until filled */
      if (!e && nn > 0) {
        int enc = p->enc == ENC_PLAIN_DICT ? ENC_RLE_DICT : p->enc;
        if (enc == ENC_RLE_DICT) { /* dictDecoder.decodeValues type_dict.go:39-59, on the current entries */
          if (!dict.present) {
            int32_t k;
            e = hy_next(&p->keys, &k);
            if (!e) e = PQR_ERR_DICT_INDEX;
          }
          for (int64_t k = 0; k < nn && !e; k++) {
            int32_t key;
            e = hy_next(&p->keys, &key);
            if (e) break;
            if (key < 0 || (int64_t)key >= dict.n) {
              e = PQR_ERR_DICT_INDEX;
              break;
            }
            memcpy(data + (size_t)k * (size_t)w, dv + (size_t)key * (size_t)w, (size_t)w);
            dnl[k] = dnil ? dnil[key] : 0;
          }
        } else {
          dense_page dp;
          memset(&dp, 0, sizeof(dp));
          e = values_decode(p, L, &dict, nn, &dp);
          if (!e) {
            memcpy(data, dp.vals.p, (size_t)nn * (size_t)w);
            memset(dnl, 0, (size_t)nn);
          }
          free(dp.vals.p);
          free(dp.lens.p);
        }
      }
      if (e) {
        set_err(R, e, rg, i + (dict.present ? 1 : 0), "read values");
      } else {
        /* s.values.values = append(s.values.values, data...) (chunk_reader.go:397) */
        if (slen + n > scap) {
          int64_t nc = go_grow(scap, slen, slen + n);
          uint8_t *nv = (uint8_t *)malloc((size_t)nc * (size_t)w + 1), *nnl = (uint8_t *)malloc((size_t)nc + 1);
          if (slen) {
            memcpy(nv, sv, (size_t)slen * (size_t)w);
            memcpy(nnl, snil, (size_t)slen);
          }
          if (aliased) { /* the dictionary keeps the old array: freeze its entries */
            own_nil = (uint8_t *)malloc((size_t)dict.n + 1);
            memcpy(dict.fixed, sv, (size_t)dict.n * (size_t)w);
            memcpy(own_nil, snil, (size_t)dict.n);
            dv = dict.fixed;
            dnil = own_nil;
            aliased = 0;
          }
          free(sv);
          free(snil);
          sv = nv;
          snil = nnl;
          scap = nc;
        }
        memcpy(sv + (size_t)slen * (size_t)w, data, (size_t)n * (size_t)w);
        memcpy(snil + slen, dnl, (size_t)n);
        slen += n;
        bb_put(&rdef, def, (size_t)n);
      }
      free(def);
      free(data);
      free(dnl);
    }
    /* the row reader: the k-th defined level takes the store's k-th slot */
    if (!R->status) {
      int64_t vpos = 0;
      for (size_t k = 0; k < rdef.n; k++) {
        nlev++;
        if (rdef.p[k] < L->max_def) continue;
        if (vpos >= slen) { /* getNextValue: "out of range" */
          set_err(R, PQR_ERR_COUNT, rg, -1, "out of range");
          break;
        }
        bb_put(&outv, sv + (size_t)vpos * (size_t)w, (size_t)w);
        uint8_t nil = snil[vpos];
        bb_put(&outnil, &nil, 1);
        vpos++;
        nout++;
      }
    }
    free(rdef.p);
    free(own_nil);
    for (int i = 0; i < npages; i++) {
      if (pages[i].own_body) free(pages[i].body);
      free(pages[i].pre);
      free(pages[i].suf);
      free(pages[i].prev.p);
      delta_free(&pages[i]);
    }
    free(pages);
    free(dict.fixed);
    free(dict.str_off);
    free(dict.str_bytes);
  }
  if (!R->status) {
    R->counts[PQR_CNT_LEVELS] = nlev;
    R->counts[PQR_CNT_NONNULL] = nout;
    bb_put(&R->bufs[PQR_BUF_VALUES], outv.p, outv.n);
    bytebuf *VB = &R->bufs[PQR_BUF_VALIDITY];
    bb_zero(VB, (size_t)((nout + 7) / 8));
    for (int64_t k = 0; k < nout; k++)
      if (!outnil.p[k]) bit_set(VB, k);
  }
  free(outv.p);
  free(outnil.p);
  free(sv);
  free(snil);
  return R->status;
}

void pqref_result_free(pqref_result *r) {
  if (!r) return;
  for (int i = 0; i < 8; i++) free(r->bufs[i].p);
  free(r);
}
int pqref_result_status(const pqref_result *r) { return r->status; }
const char *pqref_result_error(const pqref_result *r) { return r->err; }
int64_t pqref_result_count(const pqref_result *r, int which) { return (which >= 0 && which < 8) ? r->counts[which] : -1; }
const void *pqref_result_buffer(const pqref_result *r, int which, size_t *nbytes) {
  if (which < 0 || which >= 8) {
    *nbytes = 0;
    return NULL;
  }
  *nbytes = r->bufs[which].n;
  return r->bufs[which].p;
}
int pqref_result_error_rg(const pqref_result *r) { return r->err_rg; }
int pqref_result_error_page(const pqref_result *r) { return r->err_page; }
