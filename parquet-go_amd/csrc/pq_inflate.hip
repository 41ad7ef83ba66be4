// pq_inflate.hip — GZIP pages inflated on the GPU (k_inflate), one wave a page.
//
// The reference inflates a GZIP page with Go's compress/gzip
// (compress.go:63-76, gzipCompressor.DecompressBlock, called from
// newBlockReader compress.go:102-122); this library's host path is zlib
// (pq_host.cpp gzip_inflate: inflateInit2(16 + MAX_WBITS), one
// inflate(Z_FINISH) into a buffer of the header's uncompressed size), and the
// oracle is the same zlib call.  k_inflate reproduces that call's OUTCOME on
// every input — the bytes, and which of PQG_ERR_CODEC (Z_DATA_ERROR) /
// PQG_ERR_SIZE (Z_BUF_ERROR: input ended or output full; or a short result)
// the page gets — by evaluating the checks in zlib 1.2.11's order:
//   * gzip header (RFC 1952 2.3): magic, CM == 8, reserved flags, MTIME /
//     XFL / OS, FEXTRA, FNAME, FCOMMENT, FHCRC (the header's CRC-16);
//   * DEFLATE blocks (RFC 1951): stored (LEN / NLEN), fixed, dynamic (HLIT <=
//     286, HDIST <= 30, the code-length code complete, repeat codes inside the
//     set, end-of-block present, literal/length and distance codes neither
//     over-subscribed nor incomplete — one 1-bit code excepted, as zlib's
//     inflate_table allows); invalid symbols (286/287, distance 30/31, an
//     unused code); a distance beyond the output so far; the output limit
//     checked before the distance (zlib's MATCH state);
//   * a missing bit is PQG_ERR_SIZE wherever zlib would wait for input;
//   * trailer: CRC-32 of the output, then ISIZE; then the size compare.
// Trailing bytes after the member are ignored (zlib returns Z_STREAM_END).
//
// Layout: one wave per page, everything the decoder decides is wave-uniform
// (SGPRs); the per-wave LDS holds the whole 32 KiB window as a ring (no
// distance ever leaves LDS), the root lookup tables (literal/length 10 bits,
// distance 9 bits; longer codes decoded canonically from per-length counts
// kept in VGPR lanes) and the code lengths.  The ring is flushed to staging
// 1 KiB at a time (16 bytes a lane), and the CRC-32 is folded in per flush
// (each lane's 16 bytes, shifted by x^(8 n) mod P into place, XOR-reduced).
// 39.9 KiB of LDS a wave: four waves a CU.
#include <hip/hip_runtime.h>

#include "pq_common.h"
#include "pq_device.h"

namespace pq {
namespace {

constexpr int GZ_RING = 32768;  // RFC 1951 3.2.5: distances <= 32768
constexpr int GZ_LB = 10, GZ_DB = 9;
constexpr int GZ_FLUSH = 1024;
constexpr uint32_t CRC_POLY = 0xEDB88320u;
constexpr uint32_t E_CODEC = 5;  // PQG_ERR_CODEC (include/pqgpu.h)

enum : uint32_t { Y_LIT = 0, Y_SYM = 1, Y_EOB = 2, Y_BAD = 3, Y_SLOW = 4 };
// table entry: value [0,16) | code bits [16,20) | extra bits [20,24) | kind [24,27)
__device__ __forceinline__ uint32_t ent(uint32_t kind, uint32_t val, uint32_t bits, uint32_t extra) {
  return val | bits << 16 | extra << 20 | kind << 24;
}
__device__ __forceinline__ uint32_t e_val(uint32_t e) { return e & 0xffffu; }
__device__ __forceinline__ uint32_t e_bits(uint32_t e) { return (e >> 16) & 15u; }
__device__ __forceinline__ uint32_t e_extra(uint32_t e) { return (e >> 20) & 15u; }
__device__ __forceinline__ uint32_t e_kind(uint32_t e) { return (e >> 24) & 7u; }

// Table kinds (zlib inflate_table's CODES / LENS / DISTS)
enum { K_CODES = 0, K_LENS = 1, K_DISTS = 2 };

// The entry of symbol s of a code of kind K: literal/length symbols carry
// their length base and extra bits (RFC 1951 3.2.5), distance symbols theirs.
template <int K>
__device__ __forceinline__ uint32_t sym_entry(uint32_t s, uint32_t L) {
  if (K == K_CODES) return ent(Y_SYM, s, L, 0);
  if (K == K_LENS) {
    if (s < 256) return ent(Y_LIT, s, L, 0);
    if (s == 256) return ent(Y_EOB, 0, L, 0);
    if (s > 285) return ent(Y_BAD, 0, L, 0);
    const uint32_t i = s - 257;
    if (i < 8) return ent(Y_SYM, 3 + i, L, 0);
    if (i == 28) return ent(Y_SYM, 258, L, 0);
    const uint32_t x = (i >> 2) - 1;
    return ent(Y_SYM, ((4 + (i & 3)) << x) + 3, L, x);
  }
  if (s >= 30) return ent(Y_BAD, 0, L, 0);
  if (s < 4) return ent(Y_SYM, s + 1, L, 0);
  const uint32_t x = (s >> 1) - 1;
  return ent(Y_SYM, ((2 + (s & 1)) << x) + 1, L, x);
}

struct GzLds {
  uint8_t ring[GZ_RING];
  uint32_t lt[1 << GZ_LB];  // literal/length root table
  uint32_t dt[1 << GZ_DB];  // distance root table (the code-length code's, 7 bits, while lengths are read)
  uint16_t lsorted[288];    // symbols by (length, value): codes longer than the root
  uint16_t dsorted[32];
  uint8_t lens[320];        // code lengths: literal/length [0, nlen), distance [nlen, nlen + ndist)
};

// Per-length code facts for the canonical decode of long codes, one length a
// lane (lane L): count, first code, first position in the sorted symbols.
struct Canon {
  uint32_t cnt, first, offs;
};

// Build the root table of a code from its lengths (RFC 1951 3.2.2), with
// zlib inflate_table's acceptance rules: over-subscribed never; incomplete
// only for a literal/length or distance code whose longest code is 1 bit; a
// code with no symbols builds (every entry invalid, 1 bit — for the
// code-length code zlib's entry then reads as length 0, as here).  Returns
// false for a rejected set.  Whole wave; LDS only.
template <int K, int ROOT>
__device__ bool build_table(const uint8_t *lens, int n, uint32_t *tab, uint16_t *sorted, Canon &cv) {
  const int lane = lane_id();
  constexpr int ROWS = K == K_LENS ? 5 : 1;  // n <= 288, 32, 19
  uint32_t Lr[ROWS];
#pragma unroll
  for (int r = 0; r < ROWS; r++) {
    const int s = lane + 64 * r;
    Lr[r] = s < n ? (uint32_t)lens[s] : 0u;
  }
  uint32_t cnt[16];
  cnt[0] = 0;
#pragma unroll
  for (int l = 1; l < 16; l++) {
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < ROWS; r++) c += (uint32_t)__builtin_popcountll(ballot(Lr[r] == (uint32_t)l));
    cnt[l] = c;
  }
  int mx = 0;
#pragma unroll
  for (int l = 1; l < 16; l++)
    if (cnt[l]) mx = l;
  constexpr int NT = 1 << ROOT;
  if (mx == 0) {
    const uint32_t e = K == K_CODES ? ent(Y_SYM, 0, 1, 0) : ent(Y_BAD, 0, 1, 0);
    for (int j = lane; j < NT; j += 64) tab[j] = e;
    cv.cnt = 0;
    cv.first = 0;
    cv.offs = 0;
    __syncthreads();
    return true;
  }
  int left = 1;
#pragma unroll
  for (int l = 1; l < 16; l++) {
    left <<= 1;
    left -= (int)cnt[l];
    if (left < 0) return false;  // over-subscribed
  }
  if (left > 0 && (K == K_CODES || mx != 1)) return false;  // incomplete
  uint32_t first[16], offs[16], base[16];
  {
    uint32_t code = 0, o = 0;
#pragma unroll
    for (int l = 1; l < 16; l++) {
      code = (code + cnt[l - 1]) << 1;
      first[l] = code;
      offs[l] = o;
      o += cnt[l];
      base[l] = 0;
    }
  }
  cv.cnt = 0;
  cv.first = 0;
  cv.offs = 0;
#pragma unroll
  for (int l = 1; l < 16; l++)
    if (lane == l) {
      cv.cnt = cnt[l];
      cv.first = first[l];
      cv.offs = offs[l];
    }
  if (left > 0) {  // the one unused 1-bit code: invalid, 1 bit
    for (int j = lane; j < NT; j += 64) tab[j] = ent(Y_BAD, 0, 1, 0);
  }
#pragma unroll
  for (int r = 0; r < ROWS; r++) {
    const uint32_t L = Lr[r];
    const uint32_t s = (uint32_t)(lane + 64 * r);
    uint32_t code = 0;
#pragma unroll
    for (int l = 1; l < 16; l++) {
      const uint64_t m = ballot(L == (uint32_t)l);
      if (L == (uint32_t)l) {
        const uint32_t rank = base[l] + (uint32_t)rank_in(m);
        code = first[l] + rank;
        sorted[offs[l] + rank] = (uint16_t)s;
      }
      base[l] += (uint32_t)__builtin_popcountll(m);
    }
    if (L != 0) {
      const uint32_t rev = __builtin_bitreverse32(code) >> (32 - L);
      if (L <= (uint32_t)ROOT) {
        const uint32_t e = sym_entry<K>(s, L);
        for (uint32_t j = rev; j < (uint32_t)NT; j += 1u << L) tab[j] = e;
      } else {
        tab[rev & (NT - 1)] = ent(Y_SLOW, 0, ROOT, 0);
      }
    }
  }
  __syncthreads();
  return true;
}

// A code longer than the root: extend the root bits one at a time until a
// length's code range holds it (canonical codes, RFC 1951 3.2.2).  The entry's
// bit count is the code's length (the caller checks it against the bits left).
template <int K, int ROOT>
__device__ __forceinline__ uint32_t slow_decode(uint64_t bb, const uint16_t *sorted, const Canon &cv) {
  uint32_t code = __builtin_bitreverse32((uint32_t)bb & ((1u << ROOT) - 1)) >> (32 - ROOT);
  for (int L = ROOT + 1; L < 16; L++) {
    code = (code << 1) | (uint32_t)((bb >> (L - 1)) & 1u);
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cv.cnt, L);
    const uint32_t f = (uint32_t)__builtin_amdgcn_readlane((int)cv.first, L);
    if (code - f < c) {
      const uint32_t o = (uint32_t)__builtin_amdgcn_readlane((int)cv.offs, L);
      return sym_entry<K>(ufirst(sorted[o + code - f]), (uint32_t)L);
    }
  }
  return ent(Y_BAD, 0, 15, 0);  // (not reached for an accepted code)
}

// CRC-32 (ISO-HDLC, reflected 0xEDB88320): GF(2) products for shifting a CRC
// over appended zero bytes (the combine of RFC 1952's CRC of concatenated
// pieces: crc(A B) = crc(A) * x^(8 |B|) mod P  xor  crc(B)).
__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 0; i < 32; i++) {
    if (a & (0x80000000u >> i)) p ^= b;
    b = (b & 1u) ? (b >> 1) ^ CRC_POLY : b >> 1;
  }
  return p;
}
__device__ __forceinline__ uint32_t x8n(uint32_t nbytes) {  // x^(8 nbytes) mod P
  uint32_t p = 0x80000000u, t = 1u << 23;                 // x^0, x^8
  while (nbytes) {
    if (nbytes & 1u) p = multmodp(t, p);
    nbytes >>= 1;
    if (nbytes) t = multmodp(t, t);
  }
  return p;
}
__device__ __forceinline__ uint32_t crc_bytes(uint32_t c, uint32_t w, int nbytes) {  // c: running, uninverted
  for (int k = 0; k < nbytes; k++) {
    c ^= (w >> (8 * k)) & 0xffu;
#pragma unroll
    for (int b = 0; b < 8; b++) c = (c >> 1) ^ (CRC_POLY & (0u - (c & 1u)));
  }
  return c;
}
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v ^= (uint32_t)__shfl_xor((int)v, m);
  return v;
}

// The page's compressed bytes through two 256-byte register windows (4 bytes
// a lane): the next window is loaded when the decoder enters the current one,
// so a refill is two v_readlane, never a load wait.  Offsets are relative to
// p0, the page start rounded down to 4 bytes; windows may read up to 512
// bytes past the page (the input buffer's 4 KiB readable slack covers the end).
struct GzIn {
  const uint32_t *p0;
  int64_t wb;  // window base (multiple of 256)
  uint32_t w0, w1;
  __device__ __forceinline__ void at(int64_t base) {
    wb = base;
    w0 = p0[(wb >> 2) + lane_id()];
    w1 = p0[(wb >> 2) + 64 + lane_id()];
  }
  __device__ __forceinline__ uint32_t u32(int64_t o) {  // bytes [o, o + 4), o >= 0
    int64_t d = o - wb;
    if (d >= 256) {
      if (d < 512) {
        wb += 256;
        w0 = w1;
        w1 = p0[(wb >> 2) + 64 + lane_id()];
      } else {
        at(o & ~(int64_t)255);
      }
      d = o - wb;
    } else if (d < 0) {
      at(o & ~(int64_t)255);
      d = o - wb;
    }
    const int i = (int)(d >> 2), sh = (int)(d & 3) * 8;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)w0, i);
    const uint32_t hi = i < 63 ? (uint32_t)__builtin_amdgcn_readlane((int)w0, i + 1)
                               : (uint32_t)__builtin_amdgcn_readlane((int)w1, 0);
    return sh ? (lo >> sh) | (hi << (32 - sh)) : lo;
  }
};

// Fixed Huffman code lengths (RFC 1951 3.2.6): literal/length 0-143: 8,
// 144-255: 9, 256-279: 7, 280-287: 8; distance 0-31: 5.
__device__ __forceinline__ void fixed_lens(uint8_t *lens) {
  for (int s = lane_id(); s < 320; s += 64) {
    uint32_t L = s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : s < 288 ? 8 : 5;
    lens[s] = (uint8_t)L;
  }
  __syncthreads();
}

__global__ __launch_bounds__(64) void k_inflate(InflateArgs a) {
  __shared__ __attribute__((aligned(16))) GzLds S;
  const int lane = lane_id();
  const int page = (int)ufirst((uint32_t)a.list[blockIdx.x]);
  const PageDesc d = a.pages[page];
  if (ufirst(__atomic_load_n(&a.status[page], __ATOMIC_RELAXED)) < make_status(ST_DECOMPRESS, 0)) return;
  const int64_t lsize = d.kind == PAGE_V2 ? (int64_t)d.v2_rep_len + d.v2_def_len : 0;
  const uint8_t *src = a.in + d.src + lsize;
  const int64_t n = d.comp_len;
  uint8_t *dst = a.stage + d.body;
  const int64_t cap = d.body_len;
  const int64_t s0 = (int64_t)((uintptr_t)src & 3);
  GzIn in;
  in.p0 = (const uint32_t *)(src - s0);
  in.at(0);
  // bit reader (RFC 1951 3.1.1: bits from the least significant end)
  uint64_t bb = 0;
  int nb = 0;
  int64_t ip = 0;  // next stream byte not yet in bb
  auto refill = [&]() {
    if (nb <= 32) {
      if (ip + 4 <= n) {
        bb |= (uint64_t)in.u32(ip + s0) << nb;
        ip += 4;
        nb += 32;
      } else {
        while (ip < n && nb <= 56) {
          bb |= (uint64_t)(in.u32(ip + s0) & 0xffu) << nb;
          ip++;
          nb += 8;
        }
      }
    }
  };
  auto take = [&](int k) -> uint32_t {  // k <= nb, k <= 32
    const uint32_t v = (uint32_t)bb & (uint32_t)((1ull << k) - 1);
    bb >>= k;
    nb -= k;
    return v;
  };
  auto byte_at = [&](int64_t i) -> uint32_t { return in.u32(i + s0) & 0xffu; };

  uint32_t err = 0;
  // ---- gzip header (RFC 1952 2.3.1; zlib inflate.c HEAD .. HCRC) ----
  int64_t p = 0;
  uint32_t flg = 0;
  do {
    if (n < 2) { err = E_SIZE; break; }
    if (byte_at(0) != 0x1f || byte_at(1) != 0x8b) { err = E_CODEC; break; }
    if (n < 4) { err = E_SIZE; break; }
    if (byte_at(2) != 8) { err = E_CODEC; break; }
    flg = byte_at(3);
    if (flg & 0xe0) { err = E_CODEC; break; }
    p = 10;  // MTIME, XFL, OS
    if (n < p) { err = E_SIZE; break; }
    if (flg & 4) {  // FEXTRA
      if (n < p + 2) { err = E_SIZE; break; }
      const int64_t xlen = (int64_t)(byte_at(p) | byte_at(p + 1) << 8);
      p += 2 + xlen;
      if (n < p) { err = E_SIZE; break; }
    }
    for (uint32_t f = 8; f <= 16 && !err; f <<= 1) {  // FNAME, FCOMMENT: zero-terminated
      if (!(flg & f)) continue;
      for (;;) {
        if (p >= n) { err = E_SIZE; break; }
        if (byte_at(p++) == 0) break;
      }
    }
    if (err) break;
    if (flg & 2) {  // FHCRC: low 16 bits of the CRC-32 of the header bytes so far
      if (n < p + 2) { err = E_SIZE; break; }
      uint32_t c = 0xffffffffu;
      for (int64_t i = 0; i < p; i++) c = crc_bytes(c, byte_at(i), 1);
      c = ~c;
      if ((c & 0xffffu) != (byte_at(p) | byte_at(p + 1) << 8)) { err = E_CODEC; break; }
      p += 2;
    }
  } while (0);
  ip = p;

  // CRC shift of this lane's 16 bytes inside a 1 KiB flush, and of a flush
  const uint32_t x_lane = x8n((uint32_t)(16 * (63 - lane)));
  const uint32_t x_flush = x8n(GZ_FLUSH);
  uint32_t crc = 0;  // CRC-32 of the flushed bytes
  int64_t o = 0, f = 0;
  auto flush = [&]() {  // [f, f + 1024) from the ring to staging
    const uint4 v = *(const uint4 *)&S.ring[(f + lane * 16) & (GZ_RING - 1)];
    *(uint4 *)(dst + f + lane * 16) = v;
    uint32_t c = 0xffffffffu;
    c = crc_bytes(c, v.x, 4);
    c = crc_bytes(c, v.y, 4);
    c = crc_bytes(c, v.z, 4);
    c = crc_bytes(c, v.w, 4);
    const uint32_t part = wave_xor(multmodp(x_lane, ~c));
    crc = multmodp(x_flush, crc) ^ ufirst(part);
    f += GZ_FLUSH;
  };

  bool last = false;
  int tabs = 0;  // tables in LDS: 0 none, 1 fixed, 2 dynamic
  Canon lcv{0, 0, 0}, dcv{0, 0, 0};
  while (!err && !last) {
    // ---- block header (RFC 1951 3.2.3) ----
    refill();
    if (nb < 3) { err = E_SIZE; break; }
    last = take(1) != 0;
    const uint32_t type = take(2);
    if (type == 3) { err = E_CODEC; break; }
    if (type == 0) {  // stored (3.2.4)
      take(nb & 7);
      refill();
      if (nb < 32) { err = E_SIZE; break; }
      const uint32_t w = take(32);
      if ((w & 0xffffu) != ((w >> 16) ^ 0xffffu)) { err = E_CODEC; break; }
      int64_t len = w & 0xffffu;
      ip -= nb >> 3;  // unread the whole bytes still in the bit buffer
      bb = 0;
      nb = 0;
      if (len == 0) continue;
      if (o >= cap || ip >= n) { err = E_SIZE; break; }
      const bool fits = ip + len <= n && o + len <= cap;
      if (!fits) { err = E_SIZE; break; }  // (zlib copies what fits, then Z_BUF_ERROR)
      while (len > 0) {
        const int64_t k = len < GZ_FLUSH ? len : GZ_FLUSH;
#pragma unroll
        for (int q = 0; q < 16; q++) {
          const int64_t j = (int64_t)lane * 16 + q;
          if (j < k) S.ring[(o + j) & (GZ_RING - 1)] = src[ip + j];
        }
        o += k;
        ip += k;
        len -= k;
        while (o - f >= GZ_FLUSH) flush();
      }
      continue;
    }
    if (type == 1) {  // fixed codes (3.2.6)
      if (tabs != 1) {
        fixed_lens(S.lens);
        build_table<K_LENS, GZ_LB>(S.lens, 288, S.lt, S.lsorted, lcv);
        build_table<K_DISTS, GZ_DB>(S.lens + 288, 32, S.dt, S.dsorted, dcv);
        tabs = 1;
      }
    } else {  // dynamic codes (3.2.7)
      tabs = 2;
      refill();
      if (nb < 14) { err = E_SIZE; break; }
      const int nlen = (int)take(5) + 257, ndist = (int)take(5) + 1, ncode = (int)take(4) + 4;
      if (nlen > 286 || ndist > 30) { err = E_CODEC; break; }
      // the code-length code's lengths, in the order of 3.2.7
      uint32_t cl = 0;  // length of order position `lane` (lanes 0..18)
      for (int i = 0; i < ncode; i++) {
        refill();
        if (nb < 3) { err = E_SIZE; break; }
        const uint32_t v = take(3);
        if (lane == i) cl = v;
      }
      if (err) break;
      {
        // order: 16 17 18 0 8 7 9 6 10 5 11 4 12 3 13 2 14 1 15
        const uint64_t ord = 0x0f010e020d030c04ull;  // positions 11..18 -> symbols (a byte each, low first)
        uint32_t sym;
        switch (lane) {
          case 0: sym = 16; break;
          case 1: sym = 17; break;
          case 2: sym = 18; break;
          case 3: sym = 0; break;
          case 4: sym = 8; break;
          case 5: sym = 7; break;
          case 6: sym = 9; break;
          case 7: sym = 6; break;
          case 8: sym = 10; break;
          case 9: sym = 5; break;
          case 10: sym = 11; break;
          default: sym = lane < 19 ? (uint32_t)((ord >> (8 * (lane - 11))) & 255u) : 0u; break;
        }
        if (lane < 19) S.lens[sym] = (uint8_t)cl;
        __syncthreads();
      }
      Canon ccv;
      if (!build_table<K_CODES, 7>(S.lens, 19, S.dt, S.dsorted, ccv)) { err = E_CODEC; break; }
      // the literal/length and distance code lengths (3.2.7; zlib CODELENS)
      const int total = nlen + ndist;
      int have = 0;
      uint32_t prev = 0;
      __syncthreads();
      while (have < total) {
        refill();
        const uint32_t e = ufirst(S.dt[(uint32_t)bb & 127u]);
        const int L = (int)e_bits(e);
        if (L > nb) { err = E_SIZE; break; }
        const uint32_t sym = e_val(e);
        if (sym < 16) {
          take(L);
          if (lane == 0) S.lens[have] = (uint8_t)sym;
          have++;
          prev = sym;
          continue;
        }
        const int xb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
        if (L + xb > nb) { err = E_SIZE; break; }
        take(L);
        if (sym == 16 && have == 0) { err = E_CODEC; break; }
        const uint32_t v = sym == 16 ? prev : 0u;
        const int rep = (sym == 16 ? 3 : sym == 17 ? 3 : 11) + (int)take(xb);
        if (have + rep > total) { err = E_CODEC; break; }
        for (int j = lane; j < rep; j += 64) S.lens[have + j] = (uint8_t)v;
        have += rep;
        prev = v;
      }
      if (err) break;
      __syncthreads();
      if (ufirst(S.lens[256]) == 0) { err = E_CODEC; break; }  // no end-of-block code
      if (!build_table<K_LENS, GZ_LB>(S.lens, nlen, S.lt, S.lsorted, lcv)) { err = E_CODEC; break; }
      if (!build_table<K_DISTS, GZ_DB>(S.lens + nlen, ndist, S.dt, S.dsorted, dcv)) { err = E_CODEC; break; }
    }
    // ---- Huffman-coded data (3.2.5; zlib LEN .. MATCH) ----
    for (;;) {
      refill();
      uint32_t e = ufirst(S.lt[(uint32_t)bb & ((1u << GZ_LB) - 1)]);
      if (e_kind(e) == Y_SLOW) e = slow_decode<K_LENS, GZ_LB>(bb, S.lsorted, lcv);
      const int L = (int)e_bits(e);
      if (L > nb) { err = E_SIZE; break; }
      take(L);
      const uint32_t kind = e_kind(e);
      if (kind == Y_LIT) {
        if (o >= cap) { err = E_SIZE; break; }
        if (lane == 0) S.ring[o & (GZ_RING - 1)] = (uint8_t)e_val(e);
        o++;
        if (o - f >= GZ_FLUSH) flush();
        continue;
      }
      if (kind == Y_EOB) break;
      if (kind != Y_SYM) { err = E_CODEC; break; }  // 286 / 287, an unused code
      const int lx = (int)e_extra(e);
      if (lx > nb) { err = E_SIZE; break; }
      const int64_t len = (int64_t)e_val(e) + take(lx);
      refill();
      uint32_t g = ufirst(S.dt[(uint32_t)bb & ((1u << GZ_DB) - 1)]);
      if (e_kind(g) == Y_SLOW) g = slow_decode<K_DISTS, GZ_DB>(bb, S.dsorted, dcv);
      const int dL = (int)e_bits(g);
      if (dL > nb) { err = E_SIZE; break; }
      take(dL);
      if (e_kind(g) != Y_SYM) { err = E_CODEC; break; }  // 30 / 31, an unused code
      const int dx = (int)e_extra(g);
      if (dx > nb) { err = E_SIZE; break; }
      const int64_t dist = (int64_t)e_val(g) + take(dx);
      if (o >= cap) { err = E_SIZE; break; }            // MATCH: no room left
      if (dist > o) { err = E_CODEC; break; }     // too far back
      if (o + len > cap) { err = E_SIZE; break; }       // partial copy, then no room
      // the copy, 64 bytes a step: sources [o - dist, o) (periodic when dist < len)
      for (int64_t k0 = 0; k0 < len; k0 += 64) {
        const int64_t k = k0 + lane;
        if (k < len) {
          const int64_t sp = o - dist + (dist >= len ? k : (int64_t)((uint32_t)k % (uint32_t)dist));
          const uint8_t b = S.ring[sp & (GZ_RING - 1)];
          S.ring[(o + k) & (GZ_RING - 1)] = b;
        }
      }
      o += len;
      if (o - f >= GZ_FLUSH) flush();
    }
  }
  if (!err) {
    // the last partial flush and the CRC of the whole output
    const int64_t r = o - f;  // < 1024
    const int64_t j0 = f + (int64_t)lane * 16;
    const int64_t k = r - (int64_t)lane * 16 > 16 ? 16 : (r - (int64_t)lane * 16 > 0 ? r - (int64_t)lane * 16 : 0);
    uint32_t c = 0xffffffffu;
    for (int64_t q = 0; q < k; q++) {
      const uint8_t b = S.ring[(j0 + q) & (GZ_RING - 1)];
      dst[j0 + q] = b;
      c = crc_bytes(c, b, 1);
    }
    const int64_t after = r - (int64_t)lane * 16 - k;  // bytes after this lane's piece
    const uint32_t mine = k > 0 ? multmodp(x8n((uint32_t)(after > 0 ? after : 0)), ~c) : 0u;
    crc = multmodp(x8n((uint32_t)r), crc) ^ ufirst(wave_xor(mine));
    // trailer (RFC 1952 2.3.1: CRC32, ISIZE; zlib CHECK, LENGTH)
    take(nb & 7);
    ip -= nb >> 3;
    bb = 0;
    nb = 0;
    if (ip + 4 > n) {
      err = E_SIZE;
    } else {
      const uint32_t want = in.u32(ip + s0);
      if (want != crc) {
        err = E_CODEC;
      } else if (ip + 8 > n) {
        err = E_SIZE;
      } else if (in.u32(ip + 4 + s0) != (uint32_t)o) {
        err = E_CODEC;
      } else if (o != cap) {
        err = E_SIZE;  // newBlockReader's size check (compress.go:116-118)
      }
    }
  }
  if (err && lane == 0) atomicMin(&a.status[page], make_status(ST_DECOMPRESS, err));
}

}  // namespace
}  // namespace pq

extern "C" int pq_launch_inflate(const pq::InflateArgs *a, hipStream_t s) {
  if (a->n <= 0) return 0;
  hipLaunchKernelGGL(pq::k_inflate, dim3((unsigned)a->n), dim3(64), 0, s, *a);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
