// pq_device.h — wave-level stream decoders for gfx950 (CDNA4, wave64).
//
// Every decoder below is driven by ONE wavefront: its state is wave-uniform
// (it lives in SGPRs), headers are parsed serially from a 256-byte register
// window (4 bytes per lane, read back with v_readlane), and the values of a
// run are produced 64 at a time, one per lane.  Kernels give each page to one
// wave and keep many pages in flight per CU to hide the serial header walks.
#pragma once
#include <type_traits>
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
// 64-bit values rebuilt from readlane words.  __builtin_amdgcn_readlane
// returns int: OR-ing a low word whose bit 31 is set into a 64-bit value
// without going through uint32_t sign-extends it over the high word (the
// round-1 deferred-literal fault and the round-5 k_expand_wg run-table fault).
// Every site that rebuilds a pointer or an int64 from lane words uses these.
// readlane_u64(v, lo_lane, hi_lane): v a 32-bit lane word, the value's low word
// in lane lo_lane and its high word in lane hi_lane (a lane-distributed record)
template <class T>
__device__ __forceinline__ uint64_t readlane_u64(T v, int lo_lane, int hi_lane) {
  static_assert(std::is_same<T, uint32_t>::value, "lane words are uint32_t");
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)v, lo_lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)v, hi_lane);
  return ((uint64_t)hi << 32) | (uint64_t)lo;
}
// readlane64(v, lane): lane `lane`'s value of a 64-bit per-lane register
template <class T>
__device__ __forceinline__ uint64_t readlane64(T v, int lane) {
  static_assert(sizeof(T) == 8 && (std::is_integral<T>::value || std::is_pointer<T>::value), "a 64-bit operand");
  const uint64_t x = (uint64_t)v;
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), lane);
  return ((uint64_t)hi << 32) | (uint64_t)lo;
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
// Wave-wide scans by DPP row shifts and row broadcasts: VALU moves between
// lanes, ~6 instructions a scan, instead of six ds_bpermute round trips
// through the LDS crossbar (~100 cycles each under load).  Called with every
// lane of the wave active.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
// v from the lane CTRL names, 0 where there is none (row_shr past the row
// start) and in the rows outside ROWS: no lane masks, so no per-step
// v_cndmask and no loop-invariant mask registers (k_snappy spilled them)
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp_z(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xf, true);
}
template <bool MAX>
__device__ __forceinline__ uint32_t wave_incl_dpp(uint32_t v) {
#ifdef PQ_SNAP_GUARD
  // a lane outside EXEC would read as 0 and cut the prefix at it: the guard
  // build reports any call from a partial wave (tests/test_gpu_guard.py)
  if (__builtin_amdgcn_read_exec() != ~0ull && lane_id() == (int)__builtin_ctzll(__builtin_amdgcn_read_exec()))
    printf("PQ_CHK scan: exec %llx\n", (unsigned long long)__builtin_amdgcn_read_exec());
#endif
  // (0 is the identity of both + and unsigned max)
#define PQ_STEP(C, R)                \
  do {                               \
    const uint32_t t = dpp_z<C, R>(v); \
    v = MAX ? max(v, t) : v + t;     \
  } while (0)
  PQ_STEP(0x111, 0xf);  // row_shr:1
  PQ_STEP(0x112, 0xf);  // row_shr:2
  PQ_STEP(0x114, 0xf);  // row_shr:4
  PQ_STEP(0x118, 0xf);  // row_shr:8
  PQ_STEP(0x142, 0xa);  // row_bcast:15 into rows 1 and 3
  PQ_STEP(0x143, 0xc);  // row_bcast:31 into rows 2 and 3
#undef PQ_STEP
  return v;
}
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint64_t dpp_z64(uint64_t v) {
  return ((uint64_t)dpp_z<CTRL, ROWS>((uint32_t)(v >> 32)) << 32) | dpp_z<CTRL, ROWS>((uint32_t)v);
}
__device__ __forceinline__ uint64_t wave_incl_add64_dpp(uint64_t v) {
#ifdef PQ_SNAP_GUARD
  if (__builtin_amdgcn_read_exec() != ~0ull && lane_id() == (int)__builtin_ctzll(__builtin_amdgcn_read_exec()))
    printf("PQ_CHK scan64: exec %llx\n", (unsigned long long)__builtin_amdgcn_read_exec());
#endif
  v += dpp_z64<0x111>(v);
  v += dpp_z64<0x112>(v);
  v += dpp_z64<0x114>(v);
  v += dpp_z64<0x118>(v);
  v += dpp_z64<0x142, 0xa>(v);
  v += dpp_z64<0x143, 0xc>(v);
  return v;
}
__device__ __forceinline__ int32_t wave_incl_scan32_impl(int32_t v) { return (int32_t)wave_incl_dpp<false>((uint32_t)v); }
// inclusive wave prefix sum
__device__ __forceinline__ int64_t wave_incl_scan64(int64_t v) { return (int64_t)wave_incl_add64_dpp((uint64_t)v); }
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) { return wave_incl_add64_dpp(v); }  // wrapping
// wave sum (uniform)
__device__ __forceinline__ int32_t wave_sum32(int32_t v) {
  return (int32_t)__builtin_amdgcn_readlane(wave_incl_dpp<false>((uint32_t)v), 63);
}
__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
  return (int64_t)readlane64(wave_incl_add64_dpp((uint64_t)v), 63);
}
// exclusive wave prefix sum; *total receives the wave total (uniform)
__device__ __forceinline__ int32_t wave_excl_scan32(int32_t v, int32_t *total) {
  int32_t incl = wave_incl_scan32_impl(v);
  *total = (int32_t)__builtin_amdgcn_readlane((uint32_t)incl, 63);
  return incl - v;
}
__device__ __forceinline__ int32_t wave_incl_scan32(int32_t v) { return wave_incl_scan32_impl(v); }

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

// In-order bitmap writer (wave-uniform state): bits are appended in value
// order; every word is stored once, whole, when its 32 bits are known (the
// partial word in `carry` until then), so a level bitmap costs its own size
// in writes — no zeroing pass, no atomics.
struct BitOut {
  uint32_t *g;     // the bitmap
  int64_t pos;     // bits appended
  uint32_t carry;  // bits [pos & ~31, pos) of word pos >> 5
  // append the n <= 64 low bits of b
  __device__ __forceinline__ void put64(uint64_t b, int n) {
    if (n <= 0) return;
    const int sh = (int)(pos & 31);
    b &= n == 64 ? ~0ull : ((1ull << n) - 1);
    const uint64_t lo = (uint64_t)carry | (b << sh);
    const uint32_t hiw = sh ? (uint32_t)(b >> (64 - sh)) : 0u;
    const int tot = sh + n;
    const int64_t w = pos >> 5;
    const int l = lane_id();
    if ((l == 0 && tot >= 32) || (l == 1 && tot >= 64)) g[w + l] = l ? (uint32_t)(lo >> 32) : (uint32_t)lo;
    carry = tot >= 64 ? hiw : tot >= 32 ? (uint32_t)(lo >> 32) : (uint32_t)lo;
    pos += n;
  }
  // append n copies of one bit value
  __device__ __forceinline__ void fill(int64_t n, bool one) {
    const int sh = (int)(pos & 31);
    if (sh) {
      const int k = (int)min<int64_t>(n, 32 - sh);
      put64(one ? ~0ull : 0ull, k);
      n -= k;
    }
    if (n <= 0) return;
    const int64_t w0 = pos >> 5, nw = n >> 5;
    for (int64_t w = lane_id(); w < nw; w += 64) g[w0 + w] = one ? 0xffffffffu : 0u;
    pos += nw * 32;
    n -= nw * 32;
    carry = one && n ? (1u << n) - 1u : 0u;
    pos += n;
  }
  // the last, partial word
  __device__ __forceinline__ void finish() {
    if ((pos & 31) && lane_id() == 0) g[pos >> 5] = carry;
  }
};

// ---------------------------------------------------------------------------
// RLE / bit-packed hybrid stream (hybrid_decoder.go:30-166)
// ---------------------------------------------------------------------------
// TABLE = false: the serial header walk only (no run table, and none of its
// registers: k_decode, whose register budget is tight).
template <bool TABLE>
struct HybT {
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
  // Run table (streams of short runs): up to 64 whole runs parsed at once,
  // lane m holding run m — its first value (relative to t_base), kind and
  // RLE value or bit-packed data offset.  The header chain inside the
  // 256-byte window is found by pointer jumping (every byte position parsed
  // as a header, lane m lands on header m), so a stream of short runs costs
  // one window step per 64 runs instead of a serial header walk per run.
  // Anything unusual (a header or payload past the stream, an oversized
  // varint, an empty run) ends the table before it: the serial path reads it
  // with the reference's exact errors.
  int64_t vdone;   // values produced since init
  int64_t t_base;  // value index of table run 0
  int64_t t_end;   // value index after the table (t_end == vdone: no table)
  int32_t t_n;     // runs in the table
  int32_t t_try;   // build a table at the next header (short runs lately)
  int32_t tr_s;    // lane m < t_n: run m's first value - t_base
  uint32_t tr_v;   // RLE value, or bit-packed data offset in the stream
  int32_t tr_k;    // 1 RLE, 0 bit-packed

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
    vdone = t_base = t_end = 0;
    t_n = 0;
    t_try = 1;
    tr_s = 0x7fffffff;
    tr_v = 0;
    tr_k = 0;
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
    // serial runs: a short one suggests more (try the table at the next header)
    t_try = rem < 64;
    return E_OK;
  }

  // one window position i (relative to W.ab, i < 248) parsed as a run header:
  // returns the position after its run (relative to W.ab; 0x7fffffff:
  // not a whole, well-formed run inside the stream), its value count, and
  // its RLE value / bit-packed data offset (relative to W.ab)
  __device__ __forceinline__ int32_t parse_at(int i, int32_t &cnt, uint32_t &val, int32_t &kind, int32_t &hdr_len) const {
    const int q = i >> 2, sb = i & 3;
    const uint32_t d0 = shfl32(W.w, q), d1 = shfl32(W.w, q + 1 < 64 ? q + 1 : 63), d2 = shfl32(W.w, q + 2 < 64 ? q + 2 : 63);
    const uint32_t x0 = __builtin_amdgcn_alignbyte(d1, d0, sb), x1 = __builtin_amdgcn_alignbyte(d2, d1, sb);
    const uint64_t B = ((uint64_t)x1 << 32) | x0;  // bytes i .. i + 7
    const uint32_t b0 = x0 & 0xff, b1 = (x0 >> 8) & 0xff, b2 = (x0 >> 16) & 0xff, b3 = x0 >> 24, b4 = x1 & 0xff;
    const int hl = b0 < 0x80 ? 1 : b1 < 0x80 ? 2 : b2 < 0x80 ? 3 : b3 < 0x80 ? 4 : 5;
    const uint64_t h = (uint64_t)(b0 & 0x7f) | ((uint64_t)(b1 & 0x7f) << 7) * (hl > 1) |
                       ((uint64_t)(b2 & 0x7f) << 14) * (hl > 2) | ((uint64_t)(b3 & 0x7f) << 21) * (hl > 3) |
                       ((uint64_t)b4 << 28) * (hl > 4);
    const int sz = (bw + 7) >> 3;
    bool ok = !(hl == 5 && b4 >= 0x08) && h <= 0x7fffffffull && (h >> 1) != 0;
    const bool bp = h & 1;
    const int64_t g = (int64_t)(h >> 1);
    int64_t nx;
    uint32_t v = 0;
    if (bp) {
      nx = (int64_t)i + hl + g * bw;
      cnt = g <= (1 << 22) ? (int32_t)(g * 8) : (1 << 25);
      v = (uint32_t)(i + hl);
    } else {
      nx = (int64_t)i + hl + sz;
      ok &= hl + sz <= 8;
      const uint64_t rv = B >> (8 * hl);
      v = sz == 0 ? 0u : (uint32_t)(rv & (sz >= 4 ? 0xffffffffull : ((1ull << (8 * sz)) - 1)));
      ok &= bw >= 32 || (v >> bw) == 0;
      cnt = g <= (1 << 25) ? (int32_t)g : (1 << 25);
    }
    // the whole run lies inside the stream
    ok &= (int64_t)(W.ab - p) + nx <= len;
    val = v;
    kind = bp ? 0 : 1;
    hdr_len = hl;
    return ok ? (int32_t)nx : 0x7fffffff;
  }

  // build a table of the runs from header `pos` (0: none, serial path)
  __device__ __forceinline__ int build_table() {
    const int lane = lane_id();
    if (pos >= len || len < 0) return 0;
    if ((uint64_t)(p + pos - W.ab) > 8) {
      W.ab = (const uint8_t *)((uintptr_t)(p + pos) & ~(uintptr_t)3);
      W.w = ((const uint32_t *)W.ab)[lane];
    }
    const int h0 = (int)(p + pos - W.ab);
    // J_0 over positions 4 lane + k: the next header, 256 = none
    uint32_t j01 = 0, j23 = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int i = 4 * lane + k;
      int32_t c, kd, hl;
      uint32_t v;
      const int32_t nx0 = parse_at(i < 248 ? i : 0, c, v, kd, hl);
      const int32_t nx = i < 248 ? nx0 : 0x7fffffff;
      const uint32_t J = nx < 248 ? (uint32_t)nx : 256u;
      if (k == 0) j01 = J;
      if (k == 1) j01 |= J << 16;
      if (k == 2) j23 = J;
      if (k == 3) j23 |= J << 16;
    }
    auto gather = [&](uint32_t x) -> uint32_t {  // J_b(x), x <= 256
      const int l = (int)(x >> 2) & 63;
      const uint32_t a = shfl32(j01, l), b = shfl32(j23, l);
      const uint32_t w = (x & 2) ? b : a;
      const uint32_t r = (x & 1) ? (w >> 16) : (w & 0xffff);
      return x >= 256 ? 256u : r;
    };
    uint32_t at = (uint32_t)h0;  // lane m: header m
#pragma unroll
    for (int b = 0; b < 6; b++) {
      const uint32_t hop = gather(at);
      if ((lane >> b) & 1) at = hop;
      if (b < 5) {
        const uint32_t n0 = gather(j01 & 0xffff), n1 = gather(j01 >> 16), n2 = gather(j23 & 0xffff), n3 = gather(j23 >> 16);
        j01 = n0 | (n1 << 16);
        j23 = n2 | (n3 << 16);
      }
    }
    // my run (a header every hop before me is whole and well-formed)
    int32_t c = 0, kd = 0, hl = 0;
    uint32_t v = 0;
    // (every lane parses: a masked lane's window dword would not reach the shuffles)
    const int32_t nx = parse_at(at < 248 ? (int)at : 0, c, v, kd, hl);
    const bool valid = at < 248 && nx != 0x7fffffff;
    const uint64_t vm = ballot(valid);
    int R = ~vm ? (int)__builtin_ctzll(~vm) : 64;  // leading runs
    // a huge run ends the table (its count was clamped)
    const uint64_t big = ballot(lane < R && c >= (1 << 25));
    if (big) R = min(R, (int)__builtin_ctzll(big));
    if (R == 0) return 0;
    int32_t tot = 0;
    const int32_t st = wave_excl_scan32(lane < R ? c : 0, &tot);
    tr_s = lane < R ? st : 0x7fffffff;
    tr_k = kd;
    tr_v = kd ? v : (uint32_t)((int64_t)(W.ab - p) + (int64_t)v);
    t_n = R;
    t_base = vdone;
    t_end = vdone + tot;
    pos = (int64_t)(W.ab - p) + (int64_t)__builtin_amdgcn_readlane(nx, R - 1);
    t_try = tot < 64 * R;  // keep building while the runs stay short
    return R;
  }

  // value number rel (relative to t_base) of the table
  __device__ __forceinline__ uint32_t table_value(int32_t rel) const {
    int r = 0;
#pragma unroll
    for (int st = 32; st >= 1; st >>= 1) {
      const int32_t s2 = (int32_t)shfl32((uint32_t)tr_s, r + st < 64 ? r + st : 63);
      if (r + st < t_n && s2 <= rel) r += st;
    }
    const int32_t s0 = (int32_t)shfl32((uint32_t)tr_s, r);
    const uint32_t v = shfl32(tr_v, r);
    const int32_t k = (int32_t)shfl32((uint32_t)tr_k, r);
    const int64_t bitpos = (int64_t)v * 8 + (int64_t)(rel - s0) * bw;
    const uint64_t o = (uint64_t)(p + (bitpos >> 3) - W.ab);
    const bool inwin = o + 8 <= 256;
    // every lane takes part in the window's shuffles (a masked lane's
    // register does not reach ds_bpermute); a position past the window (the
    // last run's tail) is read from memory
    const uint32_t wv = win_unpack(inwin ? bitpos : (int64_t)(W.ab - p) * 8);
    if (k) return v;
    return inwin ? wv : unpack_u32(p, len, bitpos, bw);
  }

  // values rel .. rel + 3 of the table (the caller masks those past its end):
  // one binary search, then the next runs' starts checked value by value
  __device__ __forceinline__ void table_value4(int32_t rel, uint32_t (&out)[4]) const {
    int r = 0;
#pragma unroll
    for (int st = 32; st >= 1; st >>= 1) {
      const int32_t s2 = (int32_t)shfl32((uint32_t)tr_s, r + st < 64 ? r + st : 63);
      if (r + st < t_n && s2 <= rel) r += st;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      // runs hold >= 1 value: at most one step per value
      const int32_t sn = (int32_t)shfl32((uint32_t)tr_s, r + 1 < 64 ? r + 1 : 63);
      if (i > 0 && r + 1 < t_n && sn <= rel + i) r++;
      const int32_t s0 = (int32_t)shfl32((uint32_t)tr_s, r);
      const uint32_t v = shfl32(tr_v, r);
      const int32_t k = (int32_t)shfl32((uint32_t)tr_k, r);
      const int64_t bitpos = (int64_t)v * 8 + (int64_t)(rel + i - s0) * bw;
      const uint64_t o = (uint64_t)(p + (bitpos >> 3) - W.ab);
      const bool inwin = o + 8 <= 256;
      const uint32_t wv = win_unpack(inwin ? bitpos : (int64_t)(W.ab - p) * 8);
      out[i] = k ? v : inwin ? wv : unpack_u32(p, len, bitpos, bw);
    }
  }

  // Bit-packed values of the current run from the register window: the bytes
  // [lo, hi) of the stream are made resident (one refill, a 256-byte load)
  // when they fit; false when they do not (wide values: the caller reads
  // memory).  One global load per window instead of one per run: level
  // streams of short runs waited on a load per run.
  __device__ __forceinline__ bool window_covers(int64_t lo, int64_t hi) {
    if (hi - lo > 248) return false;
    const uint64_t o0 = (uint64_t)(p + lo - W.ab), o1 = (uint64_t)(p + hi - W.ab);
    if (o0 < 256 && o1 <= 256) return true;
    W.ab = (const uint8_t *)((uintptr_t)(p + lo) & ~(uintptr_t)3);
    W.w = ((const uint32_t *)W.ab)[lane_id()];
    return true;
  }
  // value at stream bit `bitpos` (bw bits, LSB first) from the window; bytes
  // at or beyond len read as zero (unpack_u32)
  __device__ __forceinline__ uint32_t win_unpack(int64_t bitpos) const {
    const int64_t byte = bitpos >> 3;
    const uint32_t off = (uint32_t)(uint64_t)(p + byte - W.ab);  // <= 248
    const int li = (int)(off >> 2) & 63;
    const uint32_t d0 = shfl32(W.w, li), d1 = shfl32(W.w, li + 1 < 64 ? li + 1 : 63);
    const uint64_t v = (((uint64_t)d1 << 32) | d0) >> ((off & 3) * 8 + (uint32_t)(bitpos & 7));
    uint32_t val = (uint32_t)v & (bw == 32 ? 0xffffffffu : ((1u << bw) - 1));
    const int64_t avail = (len - byte) * 8 - (bitpos & 7);
    if (avail < bw) val = avail <= 0 ? 0u : (val & ((1u << avail) - 1));
    return val;
  }

  // Bit-packed values [vi, vi + take) of the current run that the reference can
  // read: every 8-value group must start inside the stream (a short last group
  // is zero-filled, readBitPackedRun :133-141).
  __device__ __forceinline__ int readable(int take) const {
    const int64_t last_group = (vi + take - 1) >> 3;
    if (data + last_group * bw < len) return take;
    const int64_t groups = len > data ? (len - data + bw - 1) / bw : 0;  // groups starting inside
    return (int)max<int64_t>(0, min<int64_t>((int64_t)take, groups * 8 - vi));
  }

  // Produce the next n (<= 256) values, PER values a lane: value j goes to
  // lane j / PER, element j % PER (next4: PER 4, n <= 256; next: PER 1, n <= 64).
  template <int PER>
  __device__ __forceinline__ uint32_t produce(int n, uint32_t (&out)[PER]) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 0; k < PER; k++) out[k] = 0;
    got = 0;
    if (bw == 0) {  // hybrid_decoder.go:84-86
      got = n;
      vdone += n;
      return E_OK;
    }
    while (got < n) {
      if (rem == 0) {
        if (TABLE && t_end <= vdone && t_try) build_table();
        if (TABLE && t_end > vdone) {  // from the table
          const int take = (int)min<int64_t>(t_end - vdone, (int64_t)(n - got));
          const int32_t rel0 = (int32_t)(vdone - t_base) - got;
#pragma unroll
          for (int k = 0; k < PER; k++) {
            const int j = PER * lane + k;
            const bool in = j >= got && j < got + take;
            const uint32_t v = table_value(rel0 + (in ? j : got));
            if (in) out[k] = v;
          }
          got += take;
          vdone += take;
          continue;
        }
        uint32_t e = header();
        if (e) return e;
      }
      int take = (int)min<int64_t>(rem, (int64_t)(n - got));
      if (rle) {
#pragma unroll
        for (int k = 0; k < PER; k++) {
          int j = PER * lane + k;
          if (j >= got && j < got + take) out[k] = rle_val;
        }
      } else {
        const int ok = readable(take);
        const int64_t bit0 = data * 8 + (vi - got) * (int64_t)bw;
        if (window_covers(data + ((vi * bw) >> 3), data + (((vi + take) * bw + 7) >> 3) + 8)) {
#pragma unroll
          for (int k = 0; k < PER; k++) {
            const int j = PER * lane + k;
            const bool in = j >= got && j < got + ok;
            const uint32_t v = win_unpack(bit0 + (int64_t)(in ? j : got) * bw);  // every lane shuffles
            if (in) out[k] = v;
          }
        } else {
#pragma unroll
          for (int k = 0; k < PER; k++) {
            int j = PER * lane + k;
            if (j >= got && j < got + ok) out[k] = unpack_u32(p, len, bit0 + (int64_t)j * bw, bw);
          }
        }
        if (ok < take) {  // a group starting at the end of the stream: io.EOF
          got += ok;
          vdone += ok;
          return E_EOF;
        }
        vi += take;
      }
      rem -= take;
      got += take;
      vdone += take;
    }
    return E_OK;
  }

  // bit-packed values [lo, hi) of the run whose value 0 is at stream bit b0
  // (lo, hi relative to the run), counted: == A into cA, >= B into cB; with
  // dst (the run's value 0), each stored as a byte
  // (with bo: one bit a value, set when it equals A, appended in order)
  template <bool BITS = false>
  __device__ __forceinline__ void count_packed(int64_t b0, int64_t lo, int64_t hi, uint32_t A, uint32_t B, int64_t &cA,
                                               int64_t &cB, uint8_t *dst, BitOut *bo = nullptr) {
    const int lane = lane_id();
    for (int64_t j0 = lo; j0 < hi; j0 += 64) {
      const int64_t j = j0 + lane;
      const bool in = j < hi;
      const int64_t last = min<int64_t>(j0 + 64, hi) - 1;
      uint32_t v;
      const int64_t blo = (b0 + j0 * bw) >> 3, bhi = ((b0 + (last + 1) * bw + 7) >> 3) + 8;
      if (window_covers(blo, bhi)) v = win_unpack(b0 + (in ? j : j0) * bw);
      else v = in ? unpack_u32(p, len, b0 + j * bw, bw) : 0u;
      const uint64_t ma = ballot(in && v == A);
      cA += __popcll(ma);
      cB += __popcll(ballot(in && v >= B));
      if (dst && in) dst[j] = (uint8_t)v;
      if (BITS) bo->put64(ma, (int)(last + 1 - j0));
    }
  }
  // RLE value v for values [lo, hi) of dst
  __device__ __forceinline__ static void fill_run(uint8_t *dst, int64_t lo, int64_t hi, uint32_t v) {
    for (int64_t j = lo + lane_id(); j < hi; j += 64) dst[j] = (uint8_t)v;
  }

  // analysis builds (-DPQ_LEVELS_SERIAL_FILL): the run-at-a-time fill
  __device__ __forceinline__ static bool lvl_serial_fill() {
#ifdef PQ_LEVELS_SERIAL_FILL
    return true;
#else
    return false;
#endif
  }
  // Consume the next n values (any n), counting those == A (cA) and >= B
  // (cB): the count path of k_prepare, no value leaves the run table (RLE
  // runs count whole).  Errors as next4 would report reading them.  With
  // dst, value i (since init) is also stored at dst[i] (one byte).
  // With BITS (bo instead of dst), value i is bit i of a bitmap: set when it
  // equals A (flat pages: def == max_def, all k_decode needs).
  template <bool BITS = false>
  __device__ uint32_t count2(int64_t n, uint32_t A, uint32_t B, int64_t &cA, int64_t &cB, uint8_t *dst = nullptr,
                             BitOut *bo = nullptr) {
    const int lane = lane_id();
    if (n <= 0) return E_OK;
    if (bw == 0) {  // all zeros
      cA += A == 0 ? n : 0;
      cB += B == 0 ? n : 0;
      if (dst) fill_run(dst, vdone, vdone + n, 0u);
      if (BITS) bo->fill(n, A == 0);
      vdone += n;
      return E_OK;
    }
    int64_t left = n;
    while (left > 0) {
      if (rem == 0) {
        if (TABLE && t_end <= vdone && t_try) build_table();
        if (TABLE && t_end > vdone) {
          const int64_t take = min<int64_t>(t_end - vdone, left);
          const int32_t rel0 = (int32_t)(vdone - t_base), rel1 = rel0 + (int32_t)take;
          const int32_t nxt = (int32_t)shfl32((uint32_t)tr_s, lane + 1 < 64 ? lane + 1 : 63);
          const int32_t e = lane + 1 < t_n ? nxt : (int32_t)(t_end - t_base);
          const bool mine = lane < t_n;
          if (BITS && bw == 1) {
            // bit width 1 (max_def 1): a bit-packed run's data bytes are the
            // bitmap's bits themselves (LSB first), an RLE run of A a range of
            // set bits — lane j builds output word j of a pass (its first run
            // by a binary search over the lanes' run starts, then run by run),
            // instead of a table search per value
            int32_t la = 0;
            const int64_t A0 = t_base + rel0, A1 = t_base + rel1;  // this part, absolute values
            const int64_t wa = A0 >> 5;
            const int64_t nwd = ((A1 - 1) >> 5) - wa + 1;
            const int32_t tlast = (int32_t)(t_end - t_base);
            for (int64_t w0 = 0; w0 < nwd; w0 += 64) {
              const int64_t W = wa + w0 + lane;
              const bool act = w0 + lane < nwd;
              const int32_t v0 = (int32_t)(max(W * 32, A0) - t_base), v1 = (int32_t)(min(W * 32 + 32, A1) - t_base);
              int r = 0;
#pragma unroll
              for (int st = 32; st >= 1; st >>= 1) {
                const int32_t s2 = (int32_t)shfl32((uint32_t)tr_s, r + st < 64 ? r + st : 63);
                if (r + st < t_n && s2 <= v0) r += st;
              }
              uint32_t word = 0;
              int32_t v = v0;
              // (every lane takes part in the shuffles; a lane past the part idles)
              for (int it = 0; it < 32; it++) {
                const bool go = act && v < v1;
                if (!ballot(go)) break;
                const int32_t s0 = (int32_t)shfl32((uint32_t)tr_s, r);
                const int32_t sn = (int32_t)shfl32((uint32_t)tr_s, r + 1 < 64 ? r + 1 : 63);
                const int32_t s1 = r + 1 < t_n ? sn : tlast;
                const uint32_t tv = shfl32(tr_v, r);
                const int32_t tk = (int32_t)shfl32((uint32_t)tr_k, r);
                if (go) {
                  const int32_t e2 = min(s1, v1);
                  const int n2 = e2 - v;
                  const uint32_t m = n2 >= 32 ? 0xffffffffu : ((1u << n2) - 1u);
                  uint32_t x;
                  if (tk) {
                    x = tv == A ? m : 0u;
                  } else {
                    const int64_t q = (int64_t)tv * 8 + (v - s0);
                    x = (uint32_t)(load_u64_unaligned(p + (q >> 3)) >> (q & 7)) & m;
                  }
                  word |= x << (int)((t_base + v) & 31);
                  v = e2;
                  r++;
                }
              }
              la += __builtin_popcount(word);
              // whole words stored; the part's first word completes the
              // writer's carry, its last (partial) word becomes the carry
              const bool first = act && w0 + lane == 0, lastw = act && w0 + lane == nwd - 1;
              if (first) word |= bo->carry;
              const bool partial_end = lastw && (A1 & 31) != 0;
              if (act && !partial_end) bo->g[W] = word;
              const uint64_t pe = ballot(partial_end);
              if (pe) bo->carry = __builtin_amdgcn_readlane(word, (int)__builtin_ctzll(pe));
              else if (ballot(lastw)) bo->carry = 0u;
            }
            bo->pos = A1;
            cA += wave_sum32(la);
            cB += take;  // (bitmaps are for flat pages: B = 0, every value counts)
            vdone += take;
            left -= take;
            continue;
          }
          if (BITS) {
            // every value by its own lane as below (4 a lane), a nibble a lane,
            // words assembled over 8 lanes; lanes start at a 32-value boundary
            int32_t la = 0, lb = 0;
            const int32_t a0 = rel0 - (int32_t)((t_base + rel0) & 31);
            for (int32_t q0 = a0; q0 < rel1; q0 += 256) {
              const int32_t q = q0 + 4 * lane;
              uint32_t v4[4];
              table_value4(q < rel0 ? rel0 : (q < rel1 ? q : rel0), v4);  // every lane takes part
              uint32_t nib = 0;
#pragma unroll
              for (int i = 0; i < 4; i++) {
                const bool in = q + i >= rel0 && q + i < rel1;
                const int k = q < rel0 ? q + i - rel0 : i;
                const uint32_t v = k >= 0 && k < 4 ? v4[k] : 0u;
                la += in && v == A;
                lb += in && v >= B;
                nib |= (in && v == A ? 1u : 0u) << i;
              }
              uint32_t word = nib << (4 * (lane & 7));
              word |= __shfl_xor(word, 1);
              word |= __shfl_xor(word, 2);
              word |= __shfl_xor(word, 4);
              const int32_t g0 = q0 + 32 * (lane >> 3);  // the group's first value
              const bool own = (lane & 7) == 0 && g0 < rel1 && g0 + 32 > rel0;
              if (own && g0 < rel0) word |= bo->carry;  // the part's first word: the bits before it
              const bool partial_end = own && g0 + 32 > rel1;
              if (own && !partial_end) bo->g[(t_base + g0) >> 5] = word;
              const uint64_t pe = ballot(partial_end);
              if (pe) bo->carry = __builtin_amdgcn_readlane(word, (int)__builtin_ctzll(pe));
              else if (ballot(own && g0 + 32 == rel1)) bo->carry = 0u;
            }
            bo->pos = t_base + rel1;
            cA += wave_sum32(la);
            cB += wave_sum32(lb);
            vdone += take;
            left -= take;
            continue;
          }
          if (dst && !lvl_serial_fill()) {
            // every value of the table's part by its own lane (run found by
            // a binary search over the lanes' run starts, table_value), one
            // coalesced byte store per 64 values — instead of a fill or
            // unpack loop per run, one run at a time (C4's definition
            // streams: ~15 values a run)
            int32_t la = 0, lb = 0;
#ifdef PQ_LEVELS_LANE1  // analysis build: one value a lane (C4 4.05 vs 3.96 ms with 4 a lane)
            for (int32_t q0 = rel0; q0 < rel1; q0 += 64) {
              const int32_t q = q0 + lane;
              const bool in = q < rel1;
              const uint32_t v = table_value(in ? q : rel0);  // every lane takes part in the shuffles
              if (in) dst[t_base + q] = (uint8_t)v;
              la += in && v == A;
              lb += in && v >= B;
            }
#else
            // 4 values a lane, 4-aligned in memory (whole dword stores)
            const int32_t a0 = rel0 - (int32_t)((uintptr_t)(dst + t_base + rel0) & 3);
            for (int32_t q0 = a0; q0 < rel1; q0 += 256) {
              const int32_t q = q0 + 4 * lane;
              uint32_t v4[4];
              table_value4(q < rel0 ? rel0 : (q < rel1 ? q : rel0), v4);  // every lane takes part
              uint32_t word = 0;
              bool all = true;
#pragma unroll
              for (int i = 0; i < 4; i++) {
                const bool in = q + i >= rel0 && q + i < rel1;
                all &= in;
                // (a lane that starts below rel0 searched from rel0: value q + i is v4[q + i - rel0])
                const int k = q < rel0 ? q + i - rel0 : i;
                const uint32_t v = k >= 0 && k < 4 ? v4[k] : 0u;
                word |= (v & 0xffu) << (8 * i);
                la += in && v == A;
                lb += in && v >= B;
              }
              if (all) {
                *(uint32_t *)(dst + t_base + q) = word;
              } else {
#pragma unroll
                for (int i = 0; i < 4; i++)
                  if (q + i >= rel0 && q + i < rel1) dst[t_base + q + i] = (uint8_t)(word >> (8 * i));
              }
            }
#endif
            cA += wave_sum32(la);
            cB += wave_sum32(lb);
            vdone += take;
            left -= take;
            continue;
          }
          const int32_t lo = max(tr_s, rel0), hi = min(e, rel1);
          const int64_t c = mine && hi > lo ? (int64_t)(hi - lo) : 0;
          // RLE runs: whole counts, summed over the wave
          int64_t ra = mine && tr_k && tr_v == A ? c : 0, rb = mine && tr_k && tr_v >= B ? c : 0;
#pragma unroll
          for (int d = 32; d >= 1; d >>= 1) {
            ra += (int64_t)shfl64((uint64_t)ra, lane ^ d);
            rb += (int64_t)shfl64((uint64_t)rb, lane ^ d);
          }
          cA += ufirst64(ra);
          cB += ufirst64(rb);
          if (dst) {  // RLE runs' bytes, a run at a time
            uint64_t rm = ballot(mine && tr_k && c > 0);
            while (rm) {
              const int m = (int)__builtin_ctzll(rm);
              rm &= rm - 1;
              const int32_t lm = __builtin_amdgcn_readlane(lo, m), hm = __builtin_amdgcn_readlane(hi, m);
              fill_run(dst, t_base + lm, t_base + hm, __builtin_amdgcn_readlane(tr_v, m));
            }
          }
          // bit-packed runs: their values, 64 at a time
          uint64_t bpm = ballot(mine && !tr_k && c > 0);
          while (bpm) {
            const int m = (int)__builtin_ctzll(bpm);
            bpm &= bpm - 1;
            const int32_t sm = __builtin_amdgcn_readlane(tr_s, m), lm = __builtin_amdgcn_readlane(lo, m),
                          hm = __builtin_amdgcn_readlane(hi, m);
            const uint32_t dm = __builtin_amdgcn_readlane(tr_v, m);
            count_packed((int64_t)dm * 8, lm - sm, hm - sm, A, B, cA, cB, dst ? dst + t_base + sm : nullptr);
          }
          vdone += take;
          left -= take;
          continue;
        }
        uint32_t er = header();
        if (er) return er;
      }
      const int64_t take = min<int64_t>(rem, left);
      if (rle) {
        cA += rle_val == A ? take : 0;
        cB += rle_val >= B ? take : 0;
        if (dst) fill_run(dst, vdone, vdone + take, rle_val);
        if (BITS) bo->fill(take, rle_val == A);
      } else {
        const int ok = readable((int)min<int64_t>(take, 1 << 30));
        count_packed<BITS>(data * 8, vi, vi + ok, A, B, cA, cB, dst ? dst + vdone - vi : nullptr, bo);
        if (ok < take) {
          vdone += ok;
          return E_EOF;
        }
        vi += take;
      }
      rem -= take;
      left -= take;
      vdone += take;
    }
    return E_OK;
  }

  // Consume the next k values without producing them (a k_decode part that
  // starts mid-page seeks its key stream here).  Runs are stepped over by
  // their headers; after a bit-packed run, a train of identical headers (an
  // encoder's stream of high-entropy keys) is accepted up to 64 runs a step,
  // lane j checking the header one stride j further.  Returns an error where
  // reading the values would fail (the caller then leaves the page to a
  // whole-page decode that reports the reference's error).
  __device__ uint32_t skip(int64_t k) {
    const int lane = lane_id();
    if (bw == 0 || k <= 0) {
      vdone += k > 0 ? k : 0;
      return E_OK;
    }
    while (k > 0) {
      if (rem == 0) {
        const int64_t h0 = pos;
        const uint32_t e = header();
        if (e) return e;
        if (!rle && rem < k) {
          // this run is skipped whole; try the train of identical headers after it
          const int64_t hl = data - h0, g = rem >> 3, stride = hl + g * (int64_t)bw;
          const int64_t c = pos + (int64_t)lane * stride;  // candidate header of run + 1 + lane
          bool ok = (int64_t)(lane + 1) * rem < k - rem + 1 && c + stride <= len;
          if (ok)
            for (int q = 0; q < (int)hl; q++) ok &= p[c + q] == p[h0 + q];
          const uint64_t okm = ballot(ok);
          const int m = ~okm ? (int)__builtin_ctzll(~okm) : 64;
          if (m > 0) {
            pos += (int64_t)m * stride;
            k -= (int64_t)m * rem;
            vdone += (int64_t)m * rem;
          }
        }
      }
      const int64_t take = min<int64_t>(rem, k);
      if (!rle) {
        const int ok = readable((int)take);
        if (ok < take) return E_EOF;
        vi += take;
      }
      rem -= take;
      k -= take;
      vdone += take;
    }
    return E_OK;
  }

  // Produce the next n (<= 256) values, four per lane: value j goes to lane
  // j >> 2, element j & 3.
  __device__ __forceinline__ uint32_t next4(int n, uint32_t (&out)[4]) { return produce<4>(n, out); }

  // Produce the next n (<= 64) values: lane l < n receives value l.
  __device__ __forceinline__ uint32_t next(int n, uint32_t &out) {
    uint32_t o[1];
    const uint32_t e = produce<1>(n, o);
    out = o[0];
    return e;
  }
};
using Hyb = HybT<true>;     // run tables (k_prepare's count path, k_level_check)
using HybS = HybT<false>;   // serial (k_decode)

// ---------------------------------------------------------------------------
// DELTA_BINARY_PACKED (deltabp_decoder.go:14-334); lanes receive delta+minDelta
// ---------------------------------------------------------------------------
struct Delta {
  const uint8_t *p;
  int64_t len, pos;
  int32_t block_size, mb_count, mbvc, total;
  // the reference reads 8 values a group and starts a miniblock only where the
  // value position is a multiple of both 8 and mbvc (:121-136): every adv =
  // lcm(8, mbvc) values, all read at one width; adv == mbvc for the
  // spec-conformant multiples of 8
  int32_t adv;
  int64_t first, min_delta;
  int32_t cur_mb;       // miniblocks started in the current block
  int32_t mb_w;         // width of the current miniblock
  int64_t mb_data;      // first data byte of the current miniblock
  int32_t mb_vi;        // values consumed in the current miniblock (== adv: exhausted)
  int32_t mb_v0;        // value position where the current miniblock started
  int32_t position;     // deltas consumed
  uint32_t widths;      // mb_count <= 64: lane j holds the width of miniblock j of the current block
  int64_t wpos;         // mb_count > 64: stream offset of the current block's widths (read on demand)
  int32_t is32;
  Win W;

  __device__ __forceinline__ int32_t width_of(int32_t j) {
    return mb_count <= 64 ? (int32_t)__builtin_amdgcn_readlane(widths, j) : (int32_t)W.byte_at(p + wpos + j);
  }

  __device__ uint32_t read_mb_header() {  // :248-271
    uint64_t u;
    bool ovf;
    uint32_t e = read_uvarint(W, p, len, pos, u, ovf);
    if (e) return e == E_EOF ? E_EOF : E_DELTA;
    int64_t md = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
    if (is32 && (md > 0x7fffffffll || md < -0x80000000ll)) return E_DELTA;
    min_delta = md;
    if (pos + mb_count > len) return E_EOF;  // io.ReadFull of the widths
    const int lane = lane_id();
    const uint32_t maxw = is32 ? 32u : 64u;
    if (mb_count <= 64) {
      // the widths from the register window (usually resident after the
      // varint): no global round trip of its own per block
      uint32_t wv = 0u;
      for (int q = 0; q < mb_count; q++) {
        const uint32_t b = W.byte_at(p + pos + q);
        if (lane == q) wv = b;
      }
      if (ballot(lane < mb_count && wv > maxw)) return E_BITWIDTH;
      widths = wv;
    } else {
      // any number of miniblocks (:97-106): every width checked, 64 a load
      for (int32_t q0 = 0; q0 < mb_count; q0 += 64) {
        const uint32_t b = q0 + lane < mb_count ? (uint32_t)p[pos + q0 + lane] : 0u;
        if (ballot(b > maxw)) return E_BITWIDTH;
      }
      wpos = pos;
    }
    pos += mb_count;
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
    {
      const int64_t g = (mbvc & 7) == 0 ? 8 : (mbvc & 3) == 0 ? 4 : (mbvc & 1) == 0 ? 2 : 1;  // gcd(8, mbvc)
      const int64_t l = (int64_t)mbvc * (8 / g);
      adv = (int32_t)min<int64_t>(l, 0x7ffffff8ll);  // past any int32 position: one miniblock for the page
    }
    e = read_uvarint(W, p, len, pos, u, ovf);
    if (e || u > 0x7fffffffull) return e == E_EOF ? E_EOF : E_DELTA;
    total = (int32_t)u;
    e = read_uvarint(W, p, len, pos, u, ovf);
    if (e) return e == E_EOF ? E_EOF : E_DELTA;
    first = (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
    if (is32 && (first > 0x7fffffffll || first < -0x80000000ll)) return E_DELTA;
    e = read_mb_header();
    if (e) return e;
    mb_vi = adv;  // no miniblock started yet
    mb_v0 = 0;
    mb_data = pos;
    mb_w = 0;
    cur_mb = 0;
    position = 0;
    return E_OK;
  }

  // A miniblock starts at the current position (:123-136).
  __device__ __forceinline__ uint32_t start_mb() {
    if (cur_mb >= mb_count) {
      uint32_t e = read_mb_header();
      if (e) return e;
    }
    mb_w = width_of(cur_mb);
    mb_data = pos;
    pos = mb_data + (int64_t)(adv >> 3) * mb_w;
    cur_mb++;
    mb_vi = 0;
    mb_v0 = position;
    return E_OK;
  }

  // The checks of the groups of values [position, position + take) of the
  // current miniblock: io.ReadFull of each group (:138-143), then, at the
  // group holding the last header value, the padding length of :150-155
  // ((mbvc / 8) * w minus the bytes read in this miniblock; < 0 -> error:
  // only a miniblock whose size is not a multiple of 8 gets there).
  __device__ __forceinline__ uint32_t check_groups(int take) {
    const int64_t last_group = (mb_vi + take - 1) >> 3;
    if (mb_data + (last_group + 1) * mb_w > len) return E_EOF;
    if (total > 0) {
      const int32_t pchk = (total - 1) & ~7;  // the only group with position + 8 >= total
      if (pchk >= position && pchk < position + take && mb_w > 0 &&
          (int64_t)((pchk - mb_v0) >> 3) + 1 > (int64_t)(mbvc >> 3))
        return E_DELTA;
    }
    return E_OK;
  }

  // four per lane: value j of the next n (<= 256) goes to lane j >> 2, element j & 3
  // The step's miniblocks are walked first (headers only: each lane notes
  // where its values' bits are), then every value is unpacked with all loads
  // in flight together (one dependent round trip for the step, not one per
  // miniblock).
  template <bool BATCH = true>
  __device__ uint32_t next4(int n, uint64_t (&out)[4]) {
    const int lane = lane_id();
    int32_t bk[4], wk[4];
    int64_t mdk[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      out[k] = 0;
      bk[k] = -1;
      wk[k] = 0;
      mdk[k] = 0;
    }
    if (position + n > total) return E_EOF;
    int got = 0;
    while (got < n) {
      if (mb_vi >= adv) {
        uint32_t e = start_mb();
        if (e) return e;
      }
      const int take = min(adv - mb_vi, n - got);
      uint32_t e = check_groups(take);
      if (e) return e;
      const int64_t bit0 = mb_data * 8 + (int64_t)(mb_vi - got) * mb_w;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        int j = 4 * lane + k;
        if (j >= got && j < got + take) {
          if (BATCH) {
            bk[k] = (int32_t)(bit0 + (int64_t)j * mb_w);  // pages < 256 MiB
            wk[k] = mb_w;
            mdk[k] = min_delta;
          } else {  // fewer registers (a register-bound caller): unpacked here
            out[k] = unpack_u64(p, len, bit0 + (int64_t)j * mb_w, mb_w) + (uint64_t)min_delta;
          }
        }
      }
      mb_vi += take;
      position += take;
      got += take;
    }
    if (BATCH) {
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (bk[k] >= 0) out[k] = unpack_u64(p, len, bk[k], wk[k]) + (uint64_t)mdk[k];
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
      if (mb_vi >= adv) {  // start a miniblock (:280-295)
        uint32_t e = start_mb();
        if (e) return e;
      }
      int take = min(adv - mb_vi, n - got);
      uint32_t e = check_groups(take);
      if (e) return e;
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
  // the padding read of :150-155 ends the current miniblock at (mbvc / 8) * w
  // bytes past its data (checked >= the bytes read by check_groups)
  int64_t fin = count > 0 ? dz.mb_data + (int64_t)(dz.mbvc >> 3) * dz.mb_w : dz.pos;
  if (count > 0 && dz.cur_mb < dz.mb_count) {
    const int32_t w = dz.width_of(dz.cur_mb);
    fin += (int64_t)(dz.mb_count - dz.cur_mb) * (dz.mbvc >> 3) * w;
  }
  pos += min<int64_t>(fin, len - pos);
  return E_OK;
}

}  // namespace pq
