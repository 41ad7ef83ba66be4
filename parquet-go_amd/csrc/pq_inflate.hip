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

// Diagnostic build (-DPQ_GZ_STAMPS, tools/gzip_rate.py with PQGPU_LIB): the
// first page's s_memtime cycles per phase and event counts, printed by lane 0.
#ifdef PQ_GZ_STAMPS
#define GZ_T(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define GZ_ADD(i, t) gz_acc[i] += __builtin_amdgcn_s_memtime() - (t)
#define GZ_CNT(i) gz_cnt[i]++
#else
#define GZ_T(v)
#define GZ_ADD(i, t)
#define GZ_CNT(i)
#endif

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
__device__ __forceinline__ bool build_table(const uint8_t *lens, int n, uint32_t *tab, uint16_t *sorted, Canon &cv) {
  // (per-length values live in VGPR lanes, lane l for length l, and the
  // loops over lengths are not unrolled: the decoder's state stays in SGPRs)
  const int lane = lane_id();
  constexpr int ROWS = K == K_LENS ? 5 : 1;  // n <= 288, 32, 19
  uint32_t Lr[ROWS];
#pragma unroll
  for (int r = 0; r < ROWS; r++) {
    const int s = lane + 64 * r;
    Lr[r] = s < n ? (uint32_t)lens[s] : 0u;
  }
  uint32_t cntv = 0;
  int mx = 0;
#pragma unroll 1
  for (int l = 1; l < 16; l++) {
    uint32_t c = 0;
#pragma unroll
    for (int r = 0; r < ROWS; r++) c += (uint32_t)__builtin_popcountll(ballot(Lr[r] == (uint32_t)l));
    c = ufirst(c);
    if (c) mx = l;
    if (lane == l) cntv = c;
  }
  constexpr int NT = 1 << ROOT;
  cv.cnt = 0;
  cv.first = 0;
  cv.offs = 0;
  if (mx == 0) {
    const uint32_t e = K == K_CODES ? ent(Y_SYM, 0, 1, 0) : ent(Y_BAD, 0, 1, 0);
    for (int j = lane; j < NT; j += 64) tab[j] = e;
    __syncthreads();
    return true;
  }
  int left = 1;
  uint32_t code = 0, o = 0, prevc = 0;
#pragma unroll 1
  for (int l = 1; l < 16; l++) {
    const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cntv, l);
    left = (left << 1) - (int)c;
    if (left < 0) return false;  // over-subscribed
    code = (code + prevc) << 1;
    if (lane == l) {
      cv.first = code;
      cv.offs = o;
    }
    o += c;
    prevc = c;
  }
  if (left > 0 && (K == K_CODES || mx != 1)) return false;  // incomplete
  cv.cnt = cntv;
  if (left > 0) {  // the one unused 1-bit code: invalid, 1 bit
    for (int j = lane; j < NT; j += 64) tab[j] = ent(Y_BAD, 0, 1, 0);
  }
  uint32_t basev = 0;  // lane l: symbols of length l ranked so far
#pragma unroll
  for (int r = 0; r < ROWS; r++) {
    const uint32_t L = Lr[r];
    const uint32_t s = (uint32_t)(lane + 64 * r);
    uint32_t scode = 0;
#pragma unroll 1
    for (int l = 1; l < 16; l++) {
      const uint64_t m = ballot(L == (uint32_t)l);
      if (m) {
        const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)basev, l);
        if (L == (uint32_t)l) {
          const uint32_t rank = base + (uint32_t)rank_in(m);
          scode = (uint32_t)__builtin_amdgcn_readlane((int)cv.first, l) + rank;
          sorted[(uint32_t)__builtin_amdgcn_readlane((int)cv.offs, l) + rank] = (uint16_t)s;
        }
        if (lane == l) basev = base + (uint32_t)__builtin_popcountll(m);
      }
    }
    if (L != 0) {
      const uint32_t rev = __builtin_bitreverse32(scode) >> (32 - L);
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
#pragma unroll 1
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

// The page's compressed bytes through 256-byte register windows (4 bytes a
// lane; window k = bytes [256 k, 256 k + 256) from p0, the page start rounded
// down to 4 bytes): c holds the current window, x the next, and p the one
// after is in flight — entering a window moves x and p down (p was issued a
// whole window earlier, so the move's wait is normally already met) and
// issues the next load.  Windows may read up to 768 bytes past the page: the
// input buffer's 4 KiB readable slack covers the end.
//
// The bit reader on top (RFC 1951 3.1.1: bits from the least significant
// end) keeps 33..64 bits in bb; a refill inside the current window is two
// v_readlane and a 64-bit funnel shift.  All of it is wave-uniform (SGPRs).
struct Bits {
  const uint32_t *p0;
  int s0, n;        // page start's offset in its aligned word; compressed length
  int kc, base;     // current window, its first byte (256 kc)
  uint32_t c, x, p;
  uint64_t bb = 0;  // bits not yet consumed (zeros above nb)
  int nb = 0;
  int ip = 0;       // next stream byte not yet in bb
  __device__ __forceinline__ uint32_t load(int k) { return p0[k * 64 + lane_id()]; }
  __device__ __forceinline__ void at(int k) {
    kc = k;
    base = k << 8;
    c = load(k);
    x = load(k + 1);
    p = load(k + 2);
  }
  __device__ __forceinline__ uint32_t u32_far(int pos) {  // any pos (window moves)
    const int k = pos >> 8;
    if (k != kc) {
      if (k == kc + 1) {
        c = x;
        x = p;
        p = load(k + 2);
        kc = k;
        base = k << 8;
      } else {
        at(k);
      }
    }
    const int w = (pos - base) >> 2;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)c, w);
    const uint32_t hi = w < 63 ? (uint32_t)__builtin_amdgcn_readlane((int)c, w + 1)
                               : (uint32_t)__builtin_amdgcn_readlane((int)x, 0);
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> ((pos & 3) * 8));
  }
  __device__ __forceinline__ uint32_t u32(int pos) {  // bytes [pos, pos + 4) from p0
    const uint32_t rel = (uint32_t)(pos - base);
    if (rel < 252u) {
      const int w = (int)(rel >> 2);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)c, w);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)c, w + 1);
      return (uint32_t)((((uint64_t)hi << 32) | lo) >> ((pos & 3) * 8));
    }
    return u32_far(pos);
  }
  __device__ __forceinline__ void refill() {
    if (nb <= 32) {
      if (ip + 4 <= n) {
        bb |= (uint64_t)u32(ip + s0) << nb;
        ip += 4;
        nb += 32;
      } else {
        while (ip < n && nb <= 56) {
          bb |= (uint64_t)(u32(ip + s0) & 0xffu) << nb;
          ip++;
          nb += 8;
        }
      }
    }
  }
  __device__ __forceinline__ uint32_t take(int k) {  // k <= nb, k <= 32
    const uint32_t v = (uint32_t)bb & (uint32_t)((1ull << k) - 1);
    bb >>= k;
    nb -= k;
    return v;
  }
  __device__ __forceinline__ uint32_t byte_at(int i) { return u32(i + s0) & 0xffu; }
};

// [f, f + 1024) from the ring to staging, and its CRC-32 folded into crc
__device__ __forceinline__ void flush(const uint8_t *ring, uint8_t *dst, int lane, int &f, uint32_t &crc,
                                      uint32_t x_lane, uint32_t x_flush) {
  const uint4 v = *(const uint4 *)&ring[(f + lane * 16) & (GZ_RING - 1)];
  *(uint4 *)(dst + f + lane * 16) = v;
  uint32_t c = 0xffffffffu;
  c = crc_bytes(c, v.x, 4);
  c = crc_bytes(c, v.y, 4);
  c = crc_bytes(c, v.z, 4);
  c = crc_bytes(c, v.w, 4);
  const uint32_t part = wave_xor(multmodp(x_lane, ~c));
  crc = multmodp(x_flush, crc) ^ ufirst(part);
  f += GZ_FLUSH;
}

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
  // (every field read into SGPRs: a uniform value left in a VGPR drags the
  // whole decoder's scalar state into VALU code)
  const int64_t lsize = ufirst(d.kind) == PAGE_V2 ? (int64_t)(int32_t)ufirst((uint32_t)d.v2_rep_len) +
                                                         (int64_t)(int32_t)ufirst((uint32_t)d.v2_def_len)
                                                   : 0;
  const uint8_t *src = a.in + (uint64_t)ufirst64((int64_t)d.src) + lsize;
  const int n = (int32_t)ufirst((uint32_t)d.comp_len);
  uint8_t *dst = a.stage + (uint64_t)ufirst64((int64_t)d.body);
  const int cap = (int32_t)ufirst((uint32_t)d.body_len);
  const int s0 = (int)((uintptr_t)src & 3);
  Bits R;
  R.p0 = (const uint32_t *)(src - s0);
  R.s0 = s0;
  R.n = n;
  R.at(0);

  uint32_t err = 0;
  // ---- gzip header (RFC 1952 2.3.1; zlib inflate.c HEAD .. HCRC) ----
  int p = 0;
  uint32_t flg = 0;
  do {
    if (n < 2) { err = E_SIZE; break; }
    if (R.byte_at(0) != 0x1f || R.byte_at(1) != 0x8b) { err = E_CODEC; break; }
    if (n < 4) { err = E_SIZE; break; }
    if (R.byte_at(2) != 8) { err = E_CODEC; break; }
    flg = R.byte_at(3);
    if (flg & 0xe0) { err = E_CODEC; break; }
    p = 10;  // MTIME, XFL, OS
    if (n < p) { err = E_SIZE; break; }
    if (flg & 4) {  // FEXTRA
      if (n < p + 2) { err = E_SIZE; break; }
      const int xlen = (int)(R.byte_at(p) | R.byte_at(p + 1) << 8);
      p += 2 + xlen;
      if (n < p) { err = E_SIZE; break; }
    }
    for (uint32_t fl = 8; fl <= 16 && !err; fl <<= 1) {  // FNAME, FCOMMENT: zero-terminated
      if (!(flg & fl)) continue;
      for (;;) {
        if (p >= n) { err = E_SIZE; break; }
        if (R.byte_at(p++) == 0) break;
      }
    }
    if (err) break;
    if (flg & 2) {  // FHCRC: low 16 bits of the CRC-32 of the header bytes so far
      if (n < p + 2) { err = E_SIZE; break; }
      uint32_t c = 0xffffffffu;
      for (int i = 0; i < p; i++) c = crc_bytes(c, R.byte_at(i), 1);
      c = ~c;
      if ((c & 0xffffu) != (R.byte_at(p) | R.byte_at(p + 1) << 8)) { err = E_CODEC; break; }
      p += 2;
    }
  } while (0);
  R.ip = p;

  // CRC shift of this lane's 16 bytes inside a 1 KiB flush, and of a flush
#ifdef PQ_GZ_STAMPS
  uint64_t gz_acc[6] = {0, 0, 0, 0, 0, 0}, gz_cnt[6] = {0, 0, 0, 0, 0, 0};
  const uint64_t gz_t0 = __builtin_amdgcn_s_memtime();
#endif
  const uint32_t x_lane = x8n((uint32_t)(16 * (63 - lane)));
  const uint32_t x_flush = x8n(GZ_FLUSH);
  uint32_t crc = 0;  // CRC-32 of the flushed bytes
  int o = 0, f = 0;
  // literals not yet in the ring: lane i holds the byte of position o - q + i
  uint32_t lbuf = 0;
  int q = 0;
  auto put_lits = [&]() {
    if (lane < q) S.ring[(o - q + lane) & (GZ_RING - 1)] = (uint8_t)lbuf;
    q = 0;
  };

  bool last = false;
  int tabs = 0;  // tables built: 0 none, 1 fixed, 2 dynamic
  Canon lcv{0, 0, 0}, dcv{0, 0, 0};
  // the root tables in VGPRs (entry i: lane i & 63 of register i >> 6): a
  // lookup is s_set_gpr_idx + v_readlane, no LDS round trip
  uint32_t ltv[1 << (GZ_LB - 6)], dtv[1 << (GZ_DB - 6)];
  while (!err && !last) {
    // ---- block header (RFC 1951 3.2.3) ----
    R.refill();
    if (R.nb < 3) { err = E_SIZE; break; }
    last = R.take(1) != 0;
    const uint32_t type = R.take(2);
    if (type == 3) { err = E_CODEC; break; }
    if (type == 0) {  // stored (3.2.4)
      R.take(R.nb & 7);
      R.refill();
      if (R.nb < 32) { err = E_SIZE; break; }
      const uint32_t w = R.take(32);
      if ((w & 0xffffu) != ((w >> 16) ^ 0xffffu)) { err = E_CODEC; break; }
      int len = (int)(w & 0xffffu);
      R.ip -= R.nb >> 3;  // unread the whole bytes still in the bit buffer
      R.bb = 0;
      R.nb = 0;
      if (len == 0) continue;
      if (R.ip + len > n || o + len > cap) { err = E_SIZE; break; }  // (zlib copies what fits, then Z_BUF_ERROR)
      while (len > 0) {
        const int k = len < GZ_FLUSH ? len : GZ_FLUSH;
#pragma unroll
        for (int t = 0; t < 16; t++) {
          const int j = lane * 16 + t;
          if (j < k) S.ring[(o + j) & (GZ_RING - 1)] = src[R.ip + j];
        }
        o += k;
        R.ip += k;
        len -= k;
        while (o - f >= GZ_FLUSH) flush(S.ring, dst, lane, f, crc, x_lane, x_flush);
      }
      continue;
    }
    if (type == 1) {  // fixed codes (3.2.6)
      if (tabs != 1) {
        fixed_lens(S.lens);
        build_table<K_LENS, GZ_LB>(S.lens, 288, S.lt, S.lsorted, lcv);
        build_table<K_DISTS, GZ_DB>(S.lens + 288, 32, S.dt, S.dsorted, dcv);
#pragma unroll
        for (int j = 0; j < (1 << (GZ_LB - 6)); j++) ltv[j] = S.lt[j * 64 + lane];
#pragma unroll
        for (int j = 0; j < (1 << (GZ_DB - 6)); j++) dtv[j] = S.dt[j * 64 + lane];
        tabs = 1;
      }
    } else {  // dynamic codes (3.2.7)
      GZ_T(gz_tb);
      GZ_CNT(0);
      tabs = 2;
      R.refill();
      if (R.nb < 14) { err = E_SIZE; break; }
      const int nlen = (int)R.take(5) + 257, ndist = (int)R.take(5) + 1, ncode = (int)R.take(4) + 4;
      if (nlen > 286 || ndist > 30) { err = E_CODEC; break; }
      // the code-length code's lengths, in the order of 3.2.7
      uint32_t cl = 0;  // length of order position `lane` (lanes 0..18)
      for (int i = 0; i < ncode; i++) {
        R.refill();
        if (R.nb < 3) { err = E_SIZE; break; }
        const uint32_t v = R.take(3);
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
        R.refill();
        const uint32_t e = ufirst(S.dt[(uint32_t)R.bb & 127u]);
        const int L = (int)e_bits(e);
        if (L > R.nb) { err = E_SIZE; break; }
        const uint32_t sym = e_val(e);
        if (sym < 16) {
          R.take(L);
          if (lane == 0) S.lens[have] = (uint8_t)sym;
          have++;
          prev = sym;
          continue;
        }
        const int xb = sym == 16 ? 2 : sym == 17 ? 3 : 7;
        if (L + xb > R.nb) { err = E_SIZE; break; }
        R.take(L);
        if (sym == 16 && have == 0) { err = E_CODEC; break; }
        const uint32_t v = sym == 16 ? prev : 0u;
        const int rep = (sym == 16 ? 3 : sym == 17 ? 3 : 11) + (int)R.take(xb);
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
#pragma unroll
      for (int j = 0; j < (1 << (GZ_LB - 6)); j++) ltv[j] = S.lt[j * 64 + lane];
#pragma unroll
      for (int j = 0; j < (1 << (GZ_DB - 6)); j++) dtv[j] = S.dt[j * 64 + lane];
      GZ_ADD(0, gz_tb);
    }
    // ---- Huffman-coded data (3.2.5; zlib LEN .. MATCH) ----
    for (;;) {
      // literals in a tight loop (one exit, no stores: a literal goes to its
      // lane of lbuf); anything else — a length or end-of-block code, a code
      // past the root table, missing bits, a full output, a full lbuf, a
      // flush due — leaves it, undecoded, for the general path below
      // (e >> 16 is a literal's code length, and >= 256 for any other
      // kind, so one compare against nb catches both; lim folds the output
      // limit, a full lbuf and a flush due into one bound on o)
      uint32_t e;
      {
        const int lim = (int)ufirst((uint32_t)min(cap, min(f + GZ_FLUSH, o - q + 64)));
        GZ_T(gz_tl);
        for (;;) {
          GZ_CNT(1);
          R.refill();
          const uint32_t li = (uint32_t)R.bb & ((1u << GZ_LB) - 1);
          e = (uint32_t)__builtin_amdgcn_readlane((int)ltv[li >> 6], (int)(li & 63));
          const int L = (int)(e >> 16);
          if (L > R.nb || o >= lim) break;
          R.bb >>= L;
          R.nb -= L;
          lbuf = lane == q ? (e & 0xffu) : lbuf;
          q++;
          o++;
          // a second literal without the refill check (the exits are only
          // taken at the top, after a refill)
          const uint32_t li2 = (uint32_t)R.bb & ((1u << GZ_LB) - 1);
          const uint32_t e2 = (uint32_t)__builtin_amdgcn_readlane((int)ltv[li2 >> 6], (int)(li2 & 63));
          const int L2 = (int)(e2 >> 16);
          if (L2 > R.nb || o >= lim) continue;
          R.bb >>= L2;
          R.nb -= L2;
          lbuf = lane == q ? (e2 & 0xffu) : lbuf;
          q++;
          o++;
        }
        GZ_ADD(1, gz_tl);
      }
      if (q == 64 || o - f >= GZ_FLUSH) {
        GZ_T(gz_fl);
        GZ_CNT(2);
        put_lits();
        if (o - f >= GZ_FLUSH) flush(S.ring, dst, lane, f, crc, x_lane, x_flush);
        GZ_ADD(2, gz_fl);
        continue;
      }
      GZ_T(gz_gp);
      GZ_CNT(3);
      if (e_kind(e) == Y_SLOW) e = slow_decode<K_LENS, GZ_LB>(R.bb, S.lsorted, lcv);
      const int L = (int)e_bits(e);
      if (L > R.nb) { err = E_SIZE; break; }
      R.take(L);
      const uint32_t kind = e_kind(e);
      if (kind == Y_LIT) {  // (q < 64 and no flush due here: the tight loop handled those)
        if (o >= cap) { err = E_SIZE; break; }
        lbuf = lane == q ? e_val(e) : lbuf;
        q++;
        o++;
        continue;
      }
      if (kind == Y_EOB) break;
      if (kind != Y_SYM) { err = E_CODEC; break; }  // 286 / 287, an unused code
      GZ_CNT(4);
      const int lx = (int)e_extra(e);
      if (lx > R.nb) { err = E_SIZE; break; }
      const int len = (int)e_val(e) + (int)R.take(lx);
      R.refill();
      const uint32_t di = (uint32_t)R.bb & ((1u << GZ_DB) - 1);
      uint32_t g = (uint32_t)__builtin_amdgcn_readlane((int)dtv[di >> 6], (int)(di & 63));
      if (e_kind(g) == Y_SLOW) g = slow_decode<K_DISTS, GZ_DB>(R.bb, S.dsorted, dcv);
      const int dL = (int)e_bits(g);
      if (dL > R.nb) { err = E_SIZE; break; }
      R.take(dL);
      if (e_kind(g) != Y_SYM) { err = E_CODEC; break; }  // 30 / 31, an unused code
      const int dx = (int)e_extra(g);
      if (dx > R.nb) { err = E_SIZE; break; }
      const int dist = (int)e_val(g) + (int)R.take(dx);
      if (o >= cap) { err = E_SIZE; break; }        // MATCH: no room left
      if (dist > o) { err = E_CODEC; break; }       // too far back
      if (o + len > cap) { err = E_SIZE; break; }   // partial copy, then no room
      put_lits();
      // the copy, 64 bytes a step: sources [o - dist, o) (periodic when dist < len)
      if (dist >= len) {
        for (int k0 = 0; k0 < len; k0 += 64) {
          const int k = k0 + lane;
          if (k < len) S.ring[(o + k) & (GZ_RING - 1)] = S.ring[(o - dist + k) & (GZ_RING - 1)];
        }
      } else {
        for (int k0 = 0; k0 < len; k0 += 64) {
          const int k = k0 + lane;
          if (k < len) {
            const int sp = o - dist + (int)((uint32_t)k % (uint32_t)dist);
            S.ring[(o + k) & (GZ_RING - 1)] = S.ring[sp & (GZ_RING - 1)];
          }
        }
      }
      o += len;
      if (o - f >= GZ_FLUSH) flush(S.ring, dst, lane, f, crc, x_lane, x_flush);
      GZ_ADD(3, gz_gp);
    }
    put_lits();
  }
  if (!err) {
    // the last partial flush and the CRC of the whole output
    const int r = o - f;  // < 1024
    const int j0 = f + lane * 16;
    const int k = r - lane * 16 > 16 ? 16 : (r - lane * 16 > 0 ? r - lane * 16 : 0);
    uint32_t c = 0xffffffffu;
    for (int t = 0; t < k; t++) {
      const uint8_t b = S.ring[(j0 + t) & (GZ_RING - 1)];
      dst[j0 + t] = b;
      c = crc_bytes(c, b, 1);
    }
    const int after = r - lane * 16 - k;  // bytes after this lane's piece
    const uint32_t mine = k > 0 ? multmodp(x8n((uint32_t)(after > 0 ? after : 0)), ~c) : 0u;
    crc = multmodp(x8n((uint32_t)r), crc) ^ ufirst(wave_xor(mine));
    // trailer (RFC 1952 2.3.1: CRC32, ISIZE; zlib CHECK, LENGTH)
    R.take(R.nb & 7);
    R.ip -= R.nb >> 3;
    R.bb = 0;
    R.nb = 0;
    if (R.ip + 4 > n) {
      err = E_SIZE;
    } else {
      const uint32_t want = R.u32(R.ip + s0);
      if (want != crc) {
        err = E_CODEC;
      } else if (R.ip + 8 > n) {
        err = E_SIZE;
      } else if (R.u32(R.ip + 4 + s0) != (uint32_t)o) {
        err = E_CODEC;
      } else if (o != cap) {
        err = E_SIZE;  // newBlockReader's size check (compress.go:116-118)
      }
    }
  }
  if (err && lane == 0) atomicMin(&a.status[page], make_status(ST_DECOMPRESS, err));
#ifdef PQ_GZ_STAMPS
  if (blockIdx.x == 0 && lane == 0)
    printf("GZSTAMP out %d in %d total %llu tables %llu/%llu litloop %llu/%llu flush %llu/%llu general %llu/%llu copies %llu\n",
           o, n, (unsigned long long)(__builtin_amdgcn_s_memtime() - gz_t0), (unsigned long long)gz_acc[0],
           (unsigned long long)gz_cnt[0], (unsigned long long)gz_acc[1], (unsigned long long)gz_cnt[1],
           (unsigned long long)gz_acc[2], (unsigned long long)gz_cnt[2], (unsigned long long)gz_acc[3],
           (unsigned long long)gz_cnt[3], (unsigned long long)gz_cnt[4]);
#endif
}

}  // namespace
}  // namespace pq

extern "C" int pq_launch_fail_which, pq_launch_fail_err;  // pq_kernels.hip

extern "C" int pq_launch_inflate(const pq::InflateArgs *a, hipStream_t s) {
  if (a->n <= 0) return 0;
  hipLaunchKernelGGL(pq::k_inflate, dim3((unsigned)a->n), dim3(64), 0, s, *a);
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  pq_launch_fail_which = 40;  // (launch id of k_inflate in error messages)
  pq_launch_fail_err = (int)e;
  return 17;
}
