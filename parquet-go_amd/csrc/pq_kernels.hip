// pq_kernels.hip — the MI355X decode pipeline for one batch of pages.
//
//   k_snappy        wave per Snappy page: payload -> HBM staging          (compress.go:102-122 + snappy)
//   k_dict_prepare  wave per dictionary page: PLAIN dictionary check,
//                   BYTE_ARRAY entry table                               (page_dict.go:30-64)
//   k_prepare       wave per data page: level/value stream layout, values
//                   init, and (lists / strings) level counts             (page_v1.go:79-108, page_v2.go:73-129)
//   k_scan          block per column: exclusive scans of rows/slots/bytes over pages
//   k_decode        wave per data page: levels -> validity / list offsets,
//                   values (PLAIN / RLE_DICTIONARY / DELTA_BINARY_PACKED / BYTE_ARRAY)
//                                                                        (page_v1.go:27-55, chunk_reader.go:380-402)
//
// Launch shape: 256-thread workgroups, one page per wave, so a launch keeps
// thousands of independent serial header walks in flight; every global value
// access is lane-consecutive (coalesced), run headers come from a register
// window (pq_device.h).  Nothing here is a contraction, so no MFMA.
#include <hip/hip_runtime.h>

#include "pq_common.h"
#include "pq_device.h"

namespace pq {

struct KArgs {
  const uint8_t *in;      // input buffer: every selected column chunk's bytes
  uint8_t *stage;         // staging: uncompressed values sections
  const PageDesc *pages;
  PageInfo *info;
  uint32_t *status;       // per page, (stage << 16 | code), STATUS_OK when clean
  ColDesc *cols;
  uint64_t *dict_ent;     // BYTE_ARRAY dictionary entries: (offset << 32) | length
  const int32_t *list;    // page indices handled by this launch
  int32_t nlist;
  int32_t ncols;
};

__device__ __forceinline__ void set_status(uint32_t *status, int page, uint32_t stage, uint32_t code) {
  if (lane_id() == 0) atomicMin(&status[page], make_status(stage, code));
}
__device__ __forceinline__ uint32_t page_status(const uint32_t *status, int page) {
  return ufirst(__atomic_load_n(&status[page], __ATOMIC_RELAXED));
}

__device__ __forceinline__ const uint8_t *body_ptr(const KArgs &a, const PageDesc &d) {
  return d.body_src == BODY_RAW ? a.in + d.body : a.stage + d.body;
}

// ===========================================================================
// K1: Snappy (vendor/github.com/golang/snappy/decode.go:55-75, decode_other.go:14-101)
// ===========================================================================
constexpr int RING = 8192;  // per-wave LDS history (bytes)
constexpr int RING_MASK = RING - 1;
constexpr int SNAPPY_WAVES = 4;

__global__ __launch_bounds__(256) void k_snappy(KArgs a) {
  __shared__ uint8_t ring_all[SNAPPY_WAVES][RING];
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  const int gi = blockIdx.x * SNAPPY_WAVES + wv;
  if (gi >= a.nlist) return;
  const int page = ufirst(a.list[gi]);
  const PageDesc d = a.pages[page];
  if (page_status(a.status, page) < make_status(ST_DECOMPRESS, 0)) return;
  uint8_t *ring = ring_all[wv];

  const int64_t lsize = d.kind == PAGE_V2 ? (int64_t)d.v2_rep_len + d.v2_def_len : 0;
  const uint8_t *src = a.in + d.src + lsize;
  const int64_t slen = d.comp_len;
  uint8_t *dst = a.stage + d.body;
  const int64_t expect = d.body_len;

  Win W;
  W.reset();
  // decodedLen: binary.Uvarint over the block (n <= 0 or > 0xffffffff -> ErrCorrupt)
  int64_t s = 0;
  uint64_t dlen = 0;
  {
    uint32_t sh = 0;
    bool ok = false;
    for (int i = 0; s < slen; i++) {
      uint32_t b = W.byte_at(src + s);
      s++;
      if (b < 0x80) {
        if (i > 9 || (i == 9 && b > 1)) break;
        dlen |= (uint64_t)b << (sh & 63);
        ok = true;
        break;
      }
      if (sh < 64) dlen |= (uint64_t)(b & 0x7f) << sh;
      sh += 7;
    }
    if (!ok || dlen > 0xffffffffull) {
      set_status(a.status, page, ST_DECOMPRESS, E_SNAPPY);
      return;
    }
  }
  // when the decoded length disagrees with the page header we still run the
  // decoder (validate only, no stores) to tell ErrCorrupt from a size mismatch
  const bool write = dlen == (uint64_t)expect;
  const int64_t dl = (int64_t)dlen;
  int64_t dpos = 0;
  uint32_t err = E_OK;
  while (s < slen) {
    uint32_t tag = W.byte_at(src + s);
    int64_t length, offset;
    if ((tag & 3) == 0) {  // literal
      uint32_t x = tag >> 2;
      if (x < 60) {
        s += 1;
      } else {
        int extra = (int)x - 59;
        s += 1 + extra;
        if (s > slen) {
          err = E_SNAPPY;
          break;
        }
        x = 0;
        for (int k = 0; k < extra; k++) x |= W.byte_at(src + s - extra + k) << (8 * k);
      }
      length = (int64_t)x + 1;
      if (length > dl - dpos || length > slen - s) {
        err = E_SNAPPY;
        break;
      }
      if (write) {
        const int64_t ring_from = length - RING;  // only the tail needs to enter the history
        for (int64_t k = 0; k < length; k += 256) {
#pragma unroll
          for (int j = 0; j < 4; j++) {
            int64_t idx = k + j * 64 + lane;
            if (idx < length) {
              uint8_t b = src[s + idx];
              dst[dpos + idx] = b;
              if (idx >= ring_from) ring[(dpos + idx) & RING_MASK] = b;
            }
          }
        }
      }
      dpos += length;
      s += length;
      continue;
    }
    if ((tag & 3) == 1) {  // copy1
      s += 2;
      if (s > slen) {
        err = E_SNAPPY;
        break;
      }
      uint32_t b1 = W.byte_at(src + s - 1);
      length = 4 + ((tag >> 2) & 7);
      offset = ((int64_t)(tag & 0xe0) << 3) | b1;
    } else if ((tag & 3) == 2) {  // copy2
      s += 3;
      if (s > slen) {
        err = E_SNAPPY;
        break;
      }
      length = 1 + (tag >> 2);
      offset = (int64_t)(W.byte_at(src + s - 2) | (W.byte_at(src + s - 1) << 8));
    } else {  // copy4
      s += 5;
      if (s > slen) {
        err = E_SNAPPY;
        break;
      }
      length = 1 + (tag >> 2);
      offset = (int64_t)W.u32_at(src + s - 4);
    }
    if (offset <= 0 || dpos < offset || length > dl - dpos) {
      err = E_SNAPPY;
      break;
    }
    if (write) {
      // forward, possibly self-overlapping copy of <= 64 bytes
      uint8_t b = 0;
      bool act = lane < length;
      int64_t from = dpos - offset + (offset >= length ? (int64_t)lane : (int64_t)lane % offset);
      if (offset <= RING) {
        if (act) b = ring[from & RING_MASK];
      } else {
        // far copy: make this wave's earlier stores visible, read through L2
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        if (act) {
          const uint32_t *wp = (const uint32_t *)((uintptr_t)(dst + from) & ~(uintptr_t)3);
          uint32_t word = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          b = (uint8_t)(word >> (((uintptr_t)(dst + from) & 3) * 8));
        }
      }
      if (act) {
        dst[dpos + lane] = b;
        ring[(dpos + lane) & RING_MASK] = b;
      }
    }
    dpos += length;
  }
  if (err == E_OK && dpos != dl) err = E_SNAPPY;
  if (err == E_OK && !write) err = E_SIZE;  // compress.go:117-119
  if (err) set_status(a.status, page, ST_DECOMPRESS, err);
}

// ===========================================================================
// K2: dictionary pages (page_dict.go:30-64)
// ===========================================================================
__global__ __launch_bounds__(256) void k_dict_prepare(KArgs a) {
  const int gi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gi >= a.nlist) return;
  const int lane = lane_id();
  const int page = ufirst(a.list[gi]);
  const PageDesc d = a.pages[page];
  if (page_status(a.status, page) != STATUS_OK) return;
  const ColDesc c = a.cols[d.col];
  const uint8_t *body = body_ptr(a, d);
  const int64_t n = d.num_values, len = d.body_len;
  if (c.ptype != T_BYTE_ARRAY) {
    if (n * (int64_t)c.width > len) set_status(a.status, page, ST_DICT_VALUES, E_EOF);
    return;
  }
  // serial length-prefix walk (type_bytearray.go:24-45); lane j of each
  // 64-entry group collects its entry and stores it coalesced
  Win W;
  W.reset();
  int64_t pos = 0;
  for (int64_t base = 0; base < n; base += 64) {
    int cnt = (int)min<int64_t>(64, n - base);
    uint64_t mine = 0;
    for (int j = 0; j < cnt; j++) {
      if (pos + 4 > len) {
        set_status(a.status, page, ST_DICT_VALUES, E_EOF);
        return;
      }
      int32_t l = (int32_t)W.u32_at(body + pos);
      if (l < 0) {
        set_status(a.status, page, ST_DICT_VALUES, E_BYTE_ARRAY);
        return;
      }
      if (pos + 4 + l > len) {
        set_status(a.status, page, ST_DICT_VALUES, E_EOF);
        return;
      }
      if (lane == j) mine = ((uint64_t)(pos + 4) << 32) | (uint32_t)l;
      pos += 4 + l;
    }
    if (lane < cnt) a.dict_ent[d.dict_base + base + lane] = mine;
  }
}

// ===========================================================================
// Page stream layout shared by k_prepare and k_decode
// ===========================================================================
struct PageStreams {
  const uint8_t *lvl;   // level source (V1: body, V2: payload)
  const uint8_t *body;  // values section
  int64_t rep_off, rep_len, def_off, def_len, val_off, val_len;
};

// V1: [u32 len][rep RLE] [u32 len][def RLE] values  (page_v1.go:99-107, hybrid_decoder.go:57-67)
// V2: rep bytes, def bytes raw in the payload; values section decompressed separately
__device__ uint32_t layout(const KArgs &a, const PageDesc &d, const ColDesc &c, PageStreams &ps, uint32_t &stage) {
  ps.body = body_ptr(a, d);
  const int64_t blen = d.body_len;
  if (d.kind == PAGE_V1) {
    ps.lvl = ps.body;
    int64_t pos = 0;
    Win W;
    W.reset();
    ps.rep_off = ps.rep_len = ps.def_off = ps.def_len = 0;
    if (c.max_rep > 0) {
      stage = ST_REP_INIT;
      if (blen - pos < 4) return E_EOF;
      int64_t sz = W.u32_at(ps.body + pos);
      pos += 4;
      int64_t take = min(sz, blen - pos);
      ps.rep_off = pos;
      ps.rep_len = take;
      pos += take;
    }
    if (c.max_def > 0) {
      stage = ST_DEF_INIT;
      if (blen - pos < 4) return E_EOF;
      int64_t sz = W.u32_at(ps.body + pos);
      pos += 4;
      int64_t take = min(sz, blen - pos);
      ps.def_off = pos;
      ps.def_len = take;
      pos += take;
    }
    ps.val_off = pos;
    ps.val_len = blen - pos;
  } else {
    ps.lvl = a.in + d.src;
    // a level stream of length 0 stays uninitialised (page_v2.go:110-120)
    ps.rep_off = 0;
    ps.rep_len = d.v2_rep_len > 0 ? d.v2_rep_len : -1;
    ps.def_off = d.v2_rep_len;
    ps.def_len = d.v2_def_len > 0 ? d.v2_def_len : -1;
    ps.val_off = 0;
    ps.val_len = blen;
  }
  return E_OK;
}

__device__ __forceinline__ int bits_len(int v) { return v ? 32 - __clz(v) : 0; }

// ===========================================================================
// K3: data page prepare
// ===========================================================================
__global__ __launch_bounds__(256) void k_prepare(KArgs a) {
  const int gi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gi >= a.nlist) return;
  const int lane = lane_id();
  const int page = ufirst(a.list[gi]);
  const PageDesc d = a.pages[page];
  PageInfo *pi = &a.info[page];
  if (page_status(a.status, page) != STATUS_OK) return;
  if (d.dict >= 0 && page_status(a.status, d.dict) != STATUS_OK) return;  // reported first anyway
  const ColDesc c = a.cols[d.col];
  PageStreams ps;
  uint32_t stage = ST_REP_INIT;
  uint32_t e = layout(a, d, c, ps, stage);
  if (e) {
    set_status(a.status, page, stage, e);
    return;
  }
  // values init
  int32_t idx_bw = 0;
  if (d.enc == ENC_RLE_DICT) {  // type_dict.go:22-37
    if (ps.val_len < 1) {
      set_status(a.status, page, ST_VAL_INIT, E_EOF);
      return;
    }
    idx_bw = ps.body[ps.val_off];
    if (idx_bw > 32) {
      set_status(a.status, page, ST_VAL_INIT, E_BITWIDTH);
      return;
    }
  } else if (d.enc == ENC_DELTA_BP) {
    Delta dd;
    e = dd.init(ps.body + ps.val_off, ps.val_len, c.ptype == T_INT32);
    if (e) {
      set_status(a.status, page, ST_VAL_INIT, e);
      return;
    }
  }
  if (lane == 0) {
    pi->rep_off = (int32_t)ps.rep_off;
    pi->rep_len = (int32_t)ps.rep_len;
    pi->def_off = (int32_t)ps.def_off;
    pi->def_len = (int32_t)ps.def_len;
    pi->val_off = (int32_t)ps.val_off;
    pi->val_len = (int32_t)ps.val_len;
    pi->idx_bw = idx_bw;
  }
  if (!(c.flags & COL_NEEDS_COUNT)) return;

  // counts for lists / strings: decode the level streams (phase 2 stages)
  const int n = d.num_values;
  Hyb rep, def;
  rep.init(ps.lvl + ps.rep_off, ps.rep_len, bits_len(c.max_rep));
  def.init(ps.lvl + ps.def_off, ps.def_len, bits_len(c.max_def));
  int64_t rows = 0, slots = 0, nn = 0;
  for (int e0 = 0; e0 < n && c.max_rep > 0; e0 += 64) {
    int cnt = min(64, n - e0);
    uint32_t r;
    e = rep.next(cnt, r);
    if (e) {
      set_status(a.status, page, ST_REP, e);
      return;
    }
    rows += __popcll(ballot(lane < cnt && r == 0));
  }
  for (int e0 = 0; e0 < n; e0 += 64) {
    int cnt = min(64, n - e0);
    uint32_t dl = 0;
    if (c.max_def > 0) {
      e = def.next(cnt, dl);
      if (e) {
        set_status(a.status, page, ST_DEF, e);
        return;
      }
    }
    bool act = lane < cnt;
    nn += __popcll(ballot(act && (int)dl == c.max_def));
    slots += __popcll(ballot(act && (c.max_rep == 0 || (int)dl >= c.rep_def)));
  }
  if (c.max_rep == 0) rows = n;
  // string bytes of the non-null values
  int64_t sbytes = 0;
  if (c.ptype == T_BYTE_ARRAY && nn > 0) {
    if (d.enc == ENC_PLAIN) {
      Win W;
      W.reset();
      const uint8_t *vp = ps.body + ps.val_off;
      int64_t pos = 0, vlen = ps.val_len;
      for (int64_t i = 0; i < nn; i++) {
        if (pos + 4 > vlen) {
          set_status(a.status, page, ST_VALUES, E_EOF);
          return;
        }
        int32_t l = (int32_t)W.u32_at(vp + pos);
        if (l < 0) {
          set_status(a.status, page, ST_VALUES, E_BYTE_ARRAY);
          return;
        }
        if (pos + 4 + l > vlen) {
          set_status(a.status, page, ST_VALUES, E_EOF);
          return;
        }
        sbytes += l;
        pos += 4 + l;
      }
    } else if (d.enc == ENC_RLE_DICT) {
      if (d.dict < 0) {
        // dictDecoder with no dictionary: the first key is out of range
        Hyb keys;
        keys.init(ps.body + ps.val_off + 1, ps.val_len - 1, idx_bw);
        uint32_t k;
        e = keys.next(1, k);
        set_status(a.status, page, ST_VALUES, e ? e : E_DICT);
        return;
      }
      const PageDesc dd = a.pages[d.dict];
      const int64_t dn = dd.num_values;
      Hyb keys;
      keys.init(ps.body + ps.val_off + 1, ps.val_len - 1, idx_bw);
      int64_t acc = 0;
      for (int64_t k0 = 0; k0 < nn; k0 += 64) {
        int cnt = (int)min<int64_t>(64, nn - k0);
        uint32_t k;
        e = keys.next(cnt, k);
        if (e) {
          set_status(a.status, page, ST_VALUES, e);
          return;
        }
        bool act = lane < cnt;
        if (ballot(act && (int64_t)k >= dn)) {
          set_status(a.status, page, ST_VALUES, E_DICT);
          return;
        }
        int64_t l = act ? (int64_t)(a.dict_ent[dd.dict_base + k] & 0xffffffffu) : 0;
        acc += wave_incl_scan64(l);  // every lane adds the same total below
        acc = (int64_t)ufirst64((int64_t)shfl64((uint64_t)acc, 63));
      }
      sbytes = acc;
    } else {
      set_status(a.status, page, ST_VALUES, E_UNSUPPORTED);
      return;
    }
  }
  if (lane == 0) {
    pi->rows = rows;
    pi->slots = slots;
    pi->non_null = nn;
    pi->str_bytes = sbytes;
  }
}

// ===========================================================================
// K4: per-column exclusive scans over pages (one block per column)
// ===========================================================================
__global__ __launch_bounds__(256) void k_scan(KArgs a) {
  __shared__ int64_t sh[3][256];
  __shared__ int64_t carry[3];
  const int col = blockIdx.x;
  ColDesc *c = &a.cols[col];
  const int t = threadIdx.x;
  if (t < 3) carry[t] = 0;
  __syncthreads();
  const bool counted = (c->flags & COL_NEEDS_COUNT) != 0;
  for (int b = c->page_begin; b < c->page_end; b += 256) {
    int p = b + t;
    int64_t v[3] = {0, 0, 0};
    bool data = p < c->page_end && a.pages[p].kind != PAGE_DICT;
    if (data) {
      if (counted) {
        v[0] = a.info[p].rows;
        v[1] = a.info[p].slots;
        v[2] = a.info[p].str_bytes;
      } else {
        v[0] = v[1] = a.pages[p].num_values;
      }
    }
    for (int k = 0; k < 3; k++) sh[k][t] = v[k];
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
      int64_t x[3];
      for (int k = 0; k < 3; k++) x[k] = t >= off ? sh[k][t - off] : 0;
      __syncthreads();
      for (int k = 0; k < 3; k++) sh[k][t] += x[k];
      __syncthreads();
    }
    if (data) {
      a.info[p].row_base = carry[0] + sh[0][t] - v[0];
      a.info[p].slot_base = carry[1] + sh[1][t] - v[1];
      a.info[p].str_base = carry[2] + sh[2][t] - v[2];
    }
    __syncthreads();
    if (t < 3) carry[t] += sh[t][255];
    __syncthreads();
  }
  if (t == 0) {
    c->total_rows = carry[0];
    c->total_slots = carry[1];
    c->total_str = carry[2];
    if (c->list_offsets) c->list_offsets[carry[0]] = (int32_t)carry[1];
    if (c->str_offsets) c->str_offsets[0] = 0;
  }
}

// ===========================================================================
// K5: data page decode
// ===========================================================================
__device__ __forceinline__ void store_value(uint8_t *out, int64_t slot, int w, uint64_t v, const uint8_t *srcbytes) {
  if (w == 4) {
    *(uint32_t *)(out + slot * 4) = (uint32_t)v;
  } else if (w == 8) {
    *(uint64_t *)(out + slot * 8) = v;
  } else {
    uint8_t *o = out + slot * (int64_t)w;
    if (srcbytes) {
      for (int k = 0; k < w; k++) o[k] = srcbytes[k];
    } else {
      for (int k = 0; k < w; k++) o[k] = 0;
    }
  }
}

__device__ __forceinline__ void or_bits(uint32_t *bm, int64_t bit0, uint64_t bits, int count, bool exclusive_word) {
  // bits for positions [bit0, bit0 + count); LSB-first.  Only lane 0 stores.
  if (lane_id() != 0 || count == 0) return;
  if (count < 64) bits &= (1ull << count) - 1;
  int64_t w = bit0 >> 5;
  int sh = (int)(bit0 & 31);
  uint64_t lo = bits << sh;
  uint32_t hi = sh ? (uint32_t)(bits >> (64 - sh)) : 0u;
  if (exclusive_word && sh == 0 && count == 64) {
    *(uint64_t *)(bm + w) = bits;  // a full, 64-bit aligned word owned by this chunk
    return;
  }
  if ((uint32_t)lo) atomicOr(&bm[w], (uint32_t)lo);
  if ((uint32_t)(lo >> 32)) atomicOr(&bm[w + 1], (uint32_t)(lo >> 32));
  if (hi) atomicOr(&bm[w + 2], hi);
}

__global__ __launch_bounds__(256) void k_decode(KArgs a) {
  const int gi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gi >= a.nlist) return;
  const int lane = lane_id();
  const int page = ufirst(a.list[gi]);
  if (page_status(a.status, page) != STATUS_OK) return;
  const PageDesc d = a.pages[page];
  if (d.dict >= 0 && page_status(a.status, d.dict) != STATUS_OK) return;
  const ColDesc c = a.cols[d.col];
  const PageInfo pi = a.info[page];
  const int n = d.num_values;
  if (n == 0) return;

  const uint8_t *lvl = d.kind == PAGE_V1 ? body_ptr(a, d) : a.in + d.src;
  const uint8_t *body = body_ptr(a, d);
  const uint8_t *vals = body + pi.val_off;
  const int64_t vlen = pi.val_len;
  const int w = c.width;
  const bool flat = c.max_rep == 0;
  const bool is_ba = c.ptype == T_BYTE_ARRAY;

  Hyb rep, def;
  rep.init(lvl + pi.rep_off, pi.rep_len, bits_len(c.max_rep));
  def.init(lvl + pi.def_off, pi.def_len, bits_len(c.max_def));

  // value decoders
  Hyb keys;
  Delta dz;
  const PageDesc *dp = d.dict >= 0 ? &a.pages[d.dict] : nullptr;
  const uint8_t *dict_vals = nullptr;
  int64_t dict_n = 0, dict_base = 0;
  if (d.enc == ENC_RLE_DICT) {
    keys.init(vals + 1, vlen - 1, pi.idx_bw);
    if (dp) {
      dict_vals = body_ptr(a, *dp);
      dict_n = dp->num_values;
      dict_base = dp->dict_base;
    }
  } else if (d.enc == ENC_DELTA_BP) {
    dz.init(vals, vlen, c.ptype == T_INT32);
  }
  uint64_t delta_prev = (uint64_t)dz.first;
  Win SW;  // string-length window (PLAIN BYTE_ARRAY)
  SW.reset();
  int64_t spos = 0;

  const int64_t slot_base = flat ? d.level_base : pi.slot_base;
  int64_t e0 = 0, slot_run = 0, row_run = 0, nn_run = 0, str_run = pi.str_base;
  uint32_t err = E_OK, err_stage = 0;

  while (e0 < n) {
    // first chunk of a flat page ends on a 64-slot boundary so that later
    // chunks own whole 64-bit validity words
    int cnt = (int)min<int64_t>(n - e0, flat ? 64 - ((slot_base + e0) & 63) : 64);
    const bool act = lane < cnt;
    uint32_t r = 0, dl = 0;
    if (c.max_rep > 0) {
      err = rep.next(cnt, r);
      if (err) {
        err_stage = ST_REP;
        break;
      }
    }
    if (c.max_def > 0) {
      err = def.next(cnt, dl);
      if (err) {
        err_stage = ST_DEF;
        break;
      }
    }
    const bool valid = act && (int)dl == c.max_def;
    const bool slot = act && (flat || (int)dl >= c.rep_def);
    const uint64_t vmask = ballot(valid);
    const uint64_t smask = ballot(slot);
    const int m = __popcll(vmask);
    const int vr = rank_in(vmask);   // dense rank among valid lanes
    const int sr = rank_in(smask);   // rank among slot lanes
    const int64_t myslot = slot_base + slot_run + sr;

    if (c.flags & COL_EMIT_LEVELS) {
      if (act) {
        c.def_out[d.level_base + e0 + lane] = (uint8_t)dl;
        c.rep_out[d.level_base + e0 + lane] = (uint8_t)r;
      }
    }
    if (!flat) {  // list rows start where rep == 0 (data_store.go:188-202)
      const uint64_t rmask = ballot(act && r == 0);
      if (act && r == 0) {
        int64_t row = pi.row_base + row_run + rank_in(rmask);
        c.list_offsets[row] = (int32_t)myslot;
        if ((int)dl >= c.rep_def - 1) atomicOr(&c.list_validity[row >> 5], 1u << (row & 31));
      }
      row_run += __popcll(rmask);
    }

    // ---- values for the m valid lanes (dense index nn_run + vr) ----
    uint64_t v = 0;
    const uint8_t *vsrc = nullptr;  // for widths other than 4 / 8
    int64_t slen_mine = 0, soff_mine = 0;
    if (m > 0) {
      if (d.enc == ENC_PLAIN && !is_ba) {
        if ((nn_run + m) * (int64_t)w > vlen) {
          err = E_EOF;
          err_stage = ST_VALUES;
          break;
        }
        if (valid) {
          const uint8_t *vp = vals + (nn_run + vr) * (int64_t)w;
          if (w == 4) v = load_u32_unaligned(vp);
          else if (w == 8) v = load_u64_unaligned(vp);
          else vsrc = vp;
        }
      } else if (d.enc == ENC_RLE_DICT) {
        uint32_t k;
        err = keys.next(m, k);
        if (err) {
          err_stage = ST_VALUES;
          break;
        }
        uint32_t key = shfl32(k, valid ? vr : 0);
        if (!dp) {
          err = E_DICT;
          err_stage = ST_VALUES;
          break;
        }
        if (ballot(valid && (int64_t)key >= dict_n)) {
          err = E_DICT;
          err_stage = ST_VALUES;
          break;
        }
        if (valid) {
          if (is_ba) {
            uint64_t ent = a.dict_ent[dict_base + key];
            soff_mine = (int64_t)(ent >> 32);
            slen_mine = (int64_t)(ent & 0xffffffffu);
            vsrc = dict_vals;
          } else {
            const uint8_t *vp = dict_vals + (int64_t)key * w;
            if (w == 4) v = load_u32_unaligned(vp);
            else if (w == 8) v = load_u64_unaligned(vp);
            else vsrc = vp;
          }
        }
      } else if (d.enc == ENC_DELTA_BP) {
        uint64_t dv;
        err = dz.next(m, dv);
        if (err) {
          err_stage = ST_VALUES;
          break;
        }
        if (lane >= m) dv = 0;
        uint64_t incl = wave_incl_scan_u64(dv);
        uint64_t excl = incl - dv;
        uint64_t val = delta_prev + excl;
        uint64_t tot = shfl64(incl, 63);
        v = shfl64(val, valid ? vr : 0);
        delta_prev += tot;
        if (c.ptype == T_INT32) v &= 0xffffffffull;
      } else if (d.enc == ENC_PLAIN && is_ba) {
        // serial length walk (type_bytearray.go:24-45)
        uint64_t ent = 0;
        for (int j = 0; j < m; j++) {
          if (spos + 4 > vlen) {
            err = E_EOF;
            break;
          }
          int32_t l = (int32_t)SW.u32_at(vals + spos);
          if (l < 0) {
            err = E_BYTE_ARRAY;
            break;
          }
          if (spos + 4 + l > vlen) {
            err = E_EOF;
            break;
          }
          if (lane == j) ent = ((uint64_t)(spos + 4) << 32) | (uint32_t)l;
          spos += 4 + l;
        }
        if (err) {
          err_stage = ST_VALUES;
          break;
        }
        ent = shfl64(ent, valid ? vr : 0);
        if (valid) {
          soff_mine = (int64_t)(ent >> 32);
          slen_mine = (int64_t)(ent & 0xffffffffu);
          vsrc = vals;
        }
      } else {
        err = E_UNSUPPORTED;
        err_stage = ST_VALUES;
        break;
      }
    }

    if (is_ba) {
      // offsets over slots (nulls have zero length), then byte copies
      int64_t l = valid ? slen_mine : 0;
      int64_t incl = wave_incl_scan64(slot ? l : 0);
      int64_t start = str_run + incl - l;
      if (slot) c.str_offsets[myslot + 1] = str_run + incl;
      if (valid) {
        const uint8_t *sp = vsrc + soff_mine;
        uint8_t *op = c.values + start;
        for (int64_t k = 0; k < l; k++) op[k] = sp[k];
      }
      str_run += (int64_t)shfl64((uint64_t)incl, 63);
    } else {
      if (slot) {
        if (w == 4 || w == 8) store_value(c.values, myslot, w, valid ? v : 0, nullptr);
        else store_value(c.values, myslot, w, 0, valid ? vsrc : nullptr);
      }
    }
    if (c.max_def > 0) {
      if (flat) {
        or_bits(c.validity, slot_base + slot_run, vmask, cnt, true);
      } else if (valid) {
        atomicOr(&c.validity[myslot >> 5], 1u << (myslot & 31));
      }
    }
    slot_run += __popcll(smask);
    nn_run += m;
    e0 += cnt;
  }

  // a later-found level error can outrank this one: k_level_check re-walks
  // the earlier level streams (the reference decodes all rep levels, then all
  // def levels, then the values, page_v1.go:37-52)
  if (err) {
    set_status(a.status, page, err_stage, err);
  }
}

// level-error precedence pass: for pages that failed in k_decode at the
// values or def stage, finish decoding the earlier level streams to see if
// the reference would have failed there first.
__global__ __launch_bounds__(256) void k_level_check(KArgs a) {
  const int gi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (gi >= a.nlist) return;
  const int page = ufirst(a.list[gi]);
  uint32_t st = page_status(a.status, page);
  if (st == STATUS_OK || (st >> 16) <= ST_REP) return;
  const PageDesc d = a.pages[page];
  const ColDesc c = a.cols[d.col];
  const PageInfo pi = a.info[page];
  const int n = d.num_values;
  const uint8_t *lvl = d.kind == PAGE_V1 ? body_ptr(a, d) : a.in + d.src;
  if (c.max_rep > 0) {
    Hyb rep;
    rep.init(lvl + pi.rep_off, pi.rep_len, bits_len(c.max_rep));
    for (int e0 = 0; e0 < n; e0 += 64) {
      uint32_t r;
      uint32_t e = rep.next(min(64, n - e0), r);
      if (e) {
        set_status(a.status, page, ST_REP, e);
        return;
      }
    }
  }
  if ((st >> 16) > ST_DEF && c.max_def > 0) {
    Hyb def;
    def.init(lvl + pi.def_off, pi.def_len, bits_len(c.max_def));
    for (int e0 = 0; e0 < n; e0 += 64) {
      uint32_t r;
      uint32_t e = def.next(min(64, n - e0), r);
      if (e) {
        set_status(a.status, page, ST_DEF, e);
        return;
      }
    }
  }
}

}  // namespace pq

// ---------------------------------------------------------------------------
// host-side launchers (called from pq_host.cpp)
// ---------------------------------------------------------------------------
extern "C" {

struct pq_launch_args {
  const uint8_t *in;
  uint8_t *stage;
  const void *pages;
  void *info;
  uint32_t *status;
  void *cols;
  uint64_t *dict_ent;
  const int32_t *list;
  int32_t nlist;
  int32_t ncols;
};

static pq::KArgs to_k(const pq_launch_args *p) {
  pq::KArgs k;
  k.in = p->in;
  k.stage = p->stage;
  k.pages = (const pq::PageDesc *)p->pages;
  k.info = (pq::PageInfo *)p->info;
  k.status = p->status;
  k.cols = (pq::ColDesc *)p->cols;
  k.dict_ent = p->dict_ent;
  k.list = p->list;
  k.nlist = p->nlist;
  k.ncols = p->ncols;
  return k;
}

int pq_launch(int which, const pq_launch_args *p, hipStream_t s) {
  pq::KArgs k = to_k(p);
  if (which == 4) {
    if (k.ncols <= 0) return 0;
    hipLaunchKernelGGL(pq::k_scan, dim3(k.ncols), dim3(256), 0, s, k);
    return hipGetLastError() == hipSuccess ? 0 : 17;
  }
  if (k.nlist <= 0) return 0;
  dim3 grid((k.nlist + 3) / 4), block(256);
  switch (which) {
    case 0: hipLaunchKernelGGL(pq::k_snappy, grid, block, 0, s, k); break;
    case 1: hipLaunchKernelGGL(pq::k_dict_prepare, grid, block, 0, s, k); break;
    case 2: hipLaunchKernelGGL(pq::k_prepare, grid, block, 0, s, k); break;
    case 3: hipLaunchKernelGGL(pq::k_decode, grid, block, 0, s, k); break;
    case 5: hipLaunchKernelGGL(pq::k_level_check, grid, block, 0, s, k); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 17;
}

}  // extern "C"
