// pq_device.h — wave-level stream decoders for gfx950 (CDNA4, wave64).
//
// Every decoder below is driven by ONE wavefront: its state is wave-uniform
// (it lives in SGPRs), headers are parsed serially from a 256-byte register
// window (4 bytes per lane, read back with v_readlane), and the values of a
// run are produced 64 at a time, one per lane.  Kernels give each page to one
// wave and keep many pages in flight per CU to hide the serial header walks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pq_common.h"

namespace pq {

// error codes (same numbering as include/pqgpu.h)
enum : uint32_t { E_OK = 0, E_SNAPPY = 7, E_SIZE = 8, E_PAGE = 9, E_EOF = 10, E_RLE = 11, E_DICT = 12, E_DELTA = 13,
                  E_BYTE_ARRAY = 14, E_BITWIDTH = 15, E_NO_DICT = 16, E_UNSUPPORTED = 19 };

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
__device__ __forceinline__ uint32_t ufirst(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int64_t ufirst64(int64_t x) {
  uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(uint64_t)x);
  uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int rank_in(uint64_t mask) {  // number of set bits below this lane
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}
__device__ __forceinline__ uint32_t shfl32(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
  uint32_t lo = shfl32((uint32_t)v, src), hi = shfl32((uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ int32_t wave_incl_scan32_impl(int32_t v) {
  int lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int32_t o = (int32_t)shfl32((uint32_t)v, lane >= d ? lane - d : lane);
    if (lane >= d) v += o;
  }
  return v;
}
// inclusive wave prefix sum
__device__ __forceinline__ int64_t wave_incl_scan64(int64_t v) {
  int lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int64_t o = (int64_t)shfl64((uint64_t)v, lane >= d ? lane - d : lane);
    if (lane >= d) v += o;
  }
  return v;
}
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {  // wrapping
  int lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t o = shfl64(v, lane >= d ? lane - d : lane);
    if (lane >= d) v += o;
  }
  return v;
}
// exclusive wave prefix sum; *total receives the wave total (uniform)
__device__ __forceinline__ int32_t wave_excl_scan32(int32_t v, int32_t *total) {
  int32_t incl = wave_incl_scan32_impl(v);
  *total = (int32_t)__builtin_amdgcn_readlane((uint32_t)incl, 63);
  return incl - v;
}
__device__ __forceinline__ int32_t wave_incl_scan32(int32_t v) {
  int lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int32_t o = (int32_t)shfl32((uint32_t)v, lane >= d ? lane - d : lane);
    if (lane >= d) v += o;
  }
  return v;
}

// Unaligned little-endian loads built from aligned dwords (buffers are padded
// so reading up to 12 bytes past any stream end stays inside the allocation).
__device__ __forceinline__ uint64_t load_u64_unaligned(const uint8_t *a) {
  uintptr_t ai = (uintptr_t)a;
  const uint32_t *q = (const uint32_t *)(ai & ~(uintptr_t)3);
  uint32_t sh = (uint32_t)(ai & 3) * 8;
  uint64_t lo = ((uint64_t)q[1] << 32) | q[0];
  uint64_t hi = q[2];
  return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}
__device__ __forceinline__ uint32_t load_u32_unaligned(const uint8_t *a) {
  uintptr_t ai = (uintptr_t)a;
  const uint32_t *q = (const uint32_t *)(ai & ~(uintptr_t)3);
  uint32_t sh = (uint32_t)(ai & 3) * 8;
  uint64_t v = ((uint64_t)q[1] << 32) | q[0];
  return (uint32_t)(v >> sh);
}

// LSB-first bit unpacking (bitbacking32.go / bitpacking64.go).  Bytes at or
// beyond `len` read as zero, like the zero-filled short group in
// hybrid_decoder.go:133-141.
__device__ __forceinline__ uint32_t unpack_u32(const uint8_t *p, int64_t len, int64_t bitpos, int bw) {
  if (bw == 0) return 0;
  int64_t byte = bitpos >> 3;
  int sh = (int)(bitpos & 7);
  uint64_t v = load_u64_unaligned(p + byte) >> sh;
  uint32_t val = (uint32_t)v & (bw == 32 ? 0xffffffffu : ((1u << bw) - 1));
  int64_t avail = (len - byte) * 8 - sh;
  if (avail < bw) val = avail <= 0 ? 0u : (val & ((1u << avail) - 1));
  return val;
}
__device__ __forceinline__ uint64_t unpack_u64(const uint8_t *p, int64_t len, int64_t bitpos, int bw) {
  if (bw == 0) return 0;
  int64_t byte = bitpos >> 3;
  int sh = (int)(bitpos & 7);
  uint64_t lo = load_u64_unaligned(p + byte);
  uint64_t v = lo >> sh;
  if (sh && bw + sh > 64) {
    uint64_t hi = (uint64_t)p[byte + 8];
    v |= hi << (64 - sh);
  }
  uint64_t val = bw == 64 ? v : (v & ((1ull << bw) - 1));
  int64_t avail = (len - byte) * 8 - sh;
  if (avail < bw) val = avail <= 0 ? 0ull : (val & ((1ull << avail) - 1));
  return val;
}

// 256-byte register window over a byte stream (uniform cursor).
struct Win {
  const uint8_t *ab;  // aligned absolute base of the window
  uint32_t w;         // this lane's 4 bytes
  __device__ __forceinline__ void reset() { ab = (const uint8_t *)(uintptr_t)1; }
  __device__ __forceinline__ uint32_t byte_at(const uint8_t *a) {
    uint64_t off = (uint64_t)(a - ab);
    if (off >= 252) {  // keep 4 bytes of slack so a u32 read never straddles the window end
      ab = (const uint8_t *)((uintptr_t)a & ~(uintptr_t)3);
      w = ((const uint32_t *)ab)[lane_id()];
      off = (uint64_t)(a - ab);
    }
    uint32_t word = __builtin_amdgcn_readlane(w, (int)(off >> 2));
    return (word >> ((off & 3) * 8)) & 0xffu;
  }
  __device__ __forceinline__ uint32_t u32_at(const uint8_t *a) {
    uint64_t off = (uint64_t)(a - ab);
    if (off >= 252) {
      ab = (const uint8_t *)((uintptr_t)a & ~(uintptr_t)3);
      w = ((const uint32_t *)ab)[lane_id()];
      off = (uint64_t)(a - ab);
    }
    uint32_t i = (uint32_t)(off >> 2), s = (uint32_t)(off & 3) * 8;
    uint32_t lo = __builtin_amdgcn_readlane(w, (int)i);
    uint32_t hi = __builtin_amdgcn_readlane(w, (int)(i + 1));
    return s ? (lo >> s) | (hi << (32 - s)) : lo;
  }
};

// Go 1.13 binary.ReadUvarint over a bounded stream (helpers.go:149-165 uses it).
// Returns E_OK, E_EOF (stream ended) or E_RLE-class overflow (caller maps).
__device__ __forceinline__ uint32_t read_uvarint(Win &W, const uint8_t *p, int64_t len, int64_t &pos, uint64_t &out,
                                                 bool &overflow) {
  uint64_t x = 0;
  uint32_t s = 0;
  overflow = false;
  for (int i = 0;; i++) {
    if (pos >= len) return E_EOF;
    uint32_t b = W.byte_at(p + pos);
    pos++;
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) {
        overflow = true;
        return E_RLE;
      }
      out = x | ((uint64_t)b << (s & 63));
      return E_OK;
    }
    if (s < 64) x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
}

// ---------------------------------------------------------------------------
// RLE / bit-packed hybrid stream (hybrid_decoder.go:30-166)
// ---------------------------------------------------------------------------
struct Hyb {
  const uint8_t *p;
  int64_t len;     // < 0: stream not initialised ("reader is not initialized")
  int64_t pos;     // next header
  int64_t rem;     // values left in the current run
  int64_t data;    // bit-packed: first data byte of the run
  int64_t vi;      // bit-packed: next value index inside the run
  uint32_t rle_val;
  int32_t bw;
  int32_t rle;
  int32_t got;     // values the last next4 / next produced (before an error: the ones the
                   // reference read successfully, value by value, hybrid_decoder.go:82-114)
  Win W;

  __device__ __forceinline__ void init(const uint8_t *ptr, int64_t n, int bitw) {
    p = ptr;
    len = n;
    pos = 0;
    rem = 0;
    data = 0;
    vi = 0;
    rle_val = 0;
    bw = bitw;
    rle = 0;
    got = 0;
    W.reset();
  }

  // readRunHeader :143-166 (+ readRLERunValue :116-131)
  __device__ uint32_t header() {
    if (len < 0) return E_EOF;
    uint64_t h;
    bool ovf;
    uint32_t e = read_uvarint(W, p, len, pos, h, ovf);
    if (e) return e;
    if (h > 0x7fffffffull) return E_RLE;  // "int32 out of range"
    uint32_t hdr = (uint32_t)h;
    if (hdr & 1) {
      int64_t g = hdr >> 1;
      if (g == 0) return E_RLE;  // empty bit-packed run
      rle = 0;
      rem = g * 8;
      data = pos;
      vi = 0;
      pos = data + g * (int64_t)bw;
    } else {
      int64_t c = hdr >> 1;
      if (c == 0) return E_RLE;  // empty RLE run
      int sz = (bw + 7) >> 3;
      if (pos >= len) return E_EOF;
      if (pos + sz > len) return E_EOF;  // io.ErrUnexpectedEOF
      uint32_t v = 0;
      for (int k = 0; k < sz; k++) v |= W.byte_at(p + pos + k) << (8 * k);
      pos += sz;
      if (bw < 32 && (v >> bw) != 0) return E_RLE;  // "RLE run value is too large"
      rle = 1;
      rem = c;
      rle_val = v;
    }
    return E_OK;
  }

  // Produce the next n (<= 256) values, four per lane: value j goes to lane
  // j >> 2, element j & 3.
  // Bit-packed values [vi, vi + take) of the current run that the reference can
  // read: every 8-value group must start inside the stream (a short last group
  // is zero-filled, readBitPackedRun :133-141).
  __device__ __forceinline__ int readable(int take) const {
    const int64_t last_group = (vi + take - 1) >> 3;
    if (data + last_group * bw < len) return take;
    const int64_t groups = len > data ? (len - data + bw - 1) / bw : 0;  // groups starting inside
    return (int)max<int64_t>(0, min<int64_t>((int64_t)take, groups * 8 - vi));
  }

  __device__ uint32_t next4(int n, uint32_t (&out)[4]) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 0; k < 4; k++) out[k] = 0;
    got = 0;
    if (bw == 0) {
      got = n;
      return E_OK;
    }
    while (got < n) {
      if (rem == 0) {
        uint32_t e = header();
        if (e) return e;
      }
      int take = (int)min<int64_t>(rem, (int64_t)(n - got));
      if (rle) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
          int j = 4 * lane + k;
          if (j >= got && j < got + take) out[k] = rle_val;
        }
      } else {
        const int ok = readable(take);
        const int64_t bit0 = data * 8 + (vi - got) * (int64_t)bw;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          int j = 4 * lane + k;
          if (j >= got && j < got + ok) out[k] = unpack_u32(p, len, bit0 + (int64_t)j * bw, bw);
        }
        if (ok < take) {  // a group starting at the end of the stream: io.EOF
          got += ok;
          return E_EOF;
        }
        vi += take;
      }
      rem -= take;
      got += take;
    }
    return E_OK;
  }

  // Produce the next n (<= 64) values: lane l < n receives value l.
  __device__ uint32_t next(int n, uint32_t &out) {
    int lane = lane_id();
    out = 0;
    got = 0;
    if (bw == 0) {  // hybrid_decoder.go:84-86
      got = n;
      return E_OK;
    }
    while (got < n) {
      if (rem == 0) {
        uint32_t e = header();
        if (e) return e;
      }
      int take = (int)min<int64_t>(rem, (int64_t)(n - got));
      bool mine = lane >= got && lane < got + take;
      if (rle) {
        if (mine) out = rle_val;
      } else {
        // every bit-packed group needed must start inside the stream (:133-141)
        const int ok = readable(take);
        if (lane >= got && lane < got + ok) out = unpack_u32(p, len, data * 8 + (vi + (lane - got)) * (int64_t)bw, bw);
        if (ok < take) {
          got += ok;
          return E_EOF;
        }
        vi += take;
      }
      rem -= take;
      got += take;
    }
    return E_OK;
  }
};

// ---------------------------------------------------------------------------
// DELTA_BINARY_PACKED (deltabp_decoder.go:14-334); lanes receive delta+minDelta
// ---------------------------------------------------------------------------
struct Delta {
  const uint8_t *p;
  int64_t len, pos;
  int32_t block_size, mb_count, mbvc, total;
  int64_t first, min_delta;
  int32_t cur_mb;       // miniblocks started in the current block
  int32_t mb_w;         // width of the current miniblock
  int64_t mb_data;      // first data byte of the current miniblock
  int32_t mb_vi;        // values consumed in the current miniblock (== mbvc: exhausted)
  int32_t position;     // deltas consumed
  uint32_t widths;      // lane j: width of miniblock j of the current block
  int32_t is32;
  Win W;

  __device__ uint32_t read_mb_header() {  // :248-271
    uint64_t u;
    bool ovf;
    uint32_t e = read_uvarint(W, p, len, pos, u, ovf);
    if (e) return e == E_EOF ? E_EOF : E_DELTA;
    int64_t md = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
    if (is32 && (md > 0x7fffffffll || md < -0x80000000ll)) return E_DELTA;
    min_delta = md;
    if (pos + mb_count > len) return E_EOF;  // io.ReadFull of the widths
    int lane = lane_id();
    uint32_t wv = lane < mb_count ? p[pos + lane] : 0u;
    pos += mb_count;
    uint32_t maxw = is32 ? 32u : 64u;
    if (ballot(lane < mb_count && wv > maxw)) return E_BITWIDTH;
    widths = wv;
    cur_mb = 0;
    return E_OK;
  }

  // init :197-246 (block header + first miniblock header)
  __device__ uint32_t init(const uint8_t *ptr, int64_t n, bool i32) {
    p = ptr;
    len = n;
    pos = 0;
    is32 = i32;
    W.reset();
    uint64_t u;
    bool ovf;
    uint32_t e = read_uvarint(W, p, len, pos, u, ovf);
    if (e || u > 0x7fffffffull) return e == E_EOF ? E_EOF : E_DELTA;
    block_size = (int32_t)u;
    e = read_uvarint(W, p, len, pos, u, ovf);
    if (e || u > 0x7fffffffull) return e == E_EOF ? E_EOF : E_DELTA;
    mb_count = (int32_t)u;
    if (mb_count <= 0 || block_size % mb_count != 0) return E_DELTA;
    mbvc = block_size / mb_count;
    if (mbvc == 0) return E_DELTA;
    e = read_uvarint(W, p, len, pos, u, ovf);
    if (e || u > 0x7fffffffull) return e == E_EOF ? E_EOF : E_DELTA;
    total = (int32_t)u;
    e = read_uvarint(W, p, len, pos, u, ovf);
    if (e) return e == E_EOF ? E_EOF : E_DELTA;
    first = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
    if (is32 && (first > 0x7fffffffll || first < -0x80000000ll)) return E_DELTA;
    // a non-multiple-of-8 miniblock or >64 miniblocks is outside the spec and this decoder
    if ((mbvc & 7) != 0 || mb_count > 64) return E_UNSUPPORTED;
    e = read_mb_header();
    if (e) return e;
    mb_vi = mbvc;  // no miniblock started yet
    cur_mb = 0;
    position = 0;
    return E_OK;
  }

  // four per lane: value j of the next n (<= 256) goes to lane j >> 2, element j & 3
  __device__ uint32_t next4(int n, uint64_t (&out)[4]) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 0; k < 4; k++) out[k] = 0;
    if (position + n > total) return E_EOF;
    int got = 0;
    while (got < n) {
      if (mb_vi >= mbvc) {
        if (cur_mb >= mb_count) {
          uint32_t e = read_mb_header();
          if (e) return e;
        }
        mb_w = (int32_t)__builtin_amdgcn_readlane(widths, cur_mb);
        mb_data = pos;
        pos = mb_data + (int64_t)(mbvc >> 3) * mb_w;
        cur_mb++;
        mb_vi = 0;
      }
      const int take = min(mbvc - mb_vi, n - got);
      int64_t last_group = (mb_vi + take - 1) >> 3;
      if (mb_data + (last_group + 1) * mb_w > len) return E_EOF;
      const int64_t bit0 = mb_data * 8 + (int64_t)(mb_vi - got) * mb_w;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        int j = 4 * lane + k;
        if (j >= got && j < got + take) out[k] = unpack_u64(p, len, bit0 + (int64_t)j * mb_w, mb_w) + (uint64_t)min_delta;
      }
      mb_vi += take;
      position += take;
      got += take;
    }
    return E_OK;
  }

  // lanes l < n receive (delta[position + l] + min_delta) as a wrapping 64-bit value
  __device__ uint32_t next(int n, uint64_t &out) {
    int lane = lane_id();
    out = 0;
    if (position + n > total) return E_EOF;  // d.position >= d.valuesCount
    int got = 0;
    while (got < n) {
      if (mb_vi >= mbvc) {  // start a miniblock (:280-295)
        if (cur_mb >= mb_count) {
          uint32_t e = read_mb_header();
          if (e) return e;
        }
        mb_w = (int32_t)__builtin_amdgcn_readlane(widths, cur_mb);
        mb_data = pos;
        pos = mb_data + (int64_t)(mbvc >> 3) * mb_w;
        cur_mb++;
        mb_vi = 0;
      }
      int take = min(mbvc - mb_vi, n - got);
      int64_t last_group = (mb_vi + take - 1) >> 3;
      if (mb_data + (last_group + 1) * mb_w > len) return E_EOF;  // io.ReadFull of a group
      if (lane >= got && lane < got + take) {
        uint64_t d = unpack_u64(p, len, mb_data * 8 + (int64_t)(mb_vi + lane - got) * mb_w, mb_w);
        out = d + (uint64_t)min_delta;
      }
      mb_vi += take;
      position += take;
      got += take;
    }
    return E_OK;
  }
};

// decodeInt32 over a deltaBitPackDecoder32 that reads the values section from
// offset `pos` (helpers.go:119-129, deltabp_decoder.go:14-175), as the
// DELTA_(LENGTH_)BYTE_ARRAY decoders do at init (type_bytearray.go:98-108,
// :186-209): every one of the stream's valuesCount values is decoded (errors
// are init errors), the first `cap` are stored to `out`, and `pos` is left
// where the reference's reader is left — the end of the last miniblock started
// (the padding read of :150-155), then the skips of the remaining miniblocks
// at the width of miniblock currentMiniBlock (:156-163, D5), clamped to the
// section (io.ReadFull errors ignored).
__device__ inline uint32_t delta_len_stream(const uint8_t *p, int64_t len, int64_t &pos, int32_t *out, int32_t cap,
                                            int32_t &count) {
  Delta dz;
  uint32_t e = dz.init(p + pos, len - pos, true);
  if (e) return e;
  count = dz.total;
  uint32_t prev = (uint32_t)dz.first;
  const int lane = lane_id();
  for (int32_t v0 = 0; v0 < count; v0 += 256) {
    const int m = min(256, count - v0);
    uint64_t dv[4];
    e = dz.next4(m, dv);
    if (e) return e;
    // value j = first + the (wrapping int32) deltas before it
    const uint32_t loc = (uint32_t)dv[0] + (uint32_t)dv[1] + (uint32_t)dv[2] + (uint32_t)dv[3];
    uint32_t incl = loc;  // wrapping inclusive scan over lanes
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t o = shfl32(incl, lane >= d ? lane - d : lane);
      if (lane >= d) incl += o;
    }
    uint32_t val = prev + (incl - loc);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int32_t j = v0 + 4 * lane + k;
      if (4 * lane + k < m && j < cap) out[j] = (int32_t)val;
      val += (uint32_t)dv[k];
    }
    prev += (uint32_t)__builtin_amdgcn_readlane(incl, 63);
  }
  int64_t fin = dz.pos;
  if (count > 0 && dz.cur_mb < dz.mb_count) {
    const int32_t w = (int32_t)__builtin_amdgcn_readlane(dz.widths, dz.cur_mb);
    fin += (int64_t)(dz.mb_count - dz.cur_mb) * (dz.mbvc >> 3) * w;
  }
  pos += min<int64_t>(fin, len - pos);
  return E_OK;
}

}  // namespace pq
