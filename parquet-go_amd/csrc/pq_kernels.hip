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

#include <type_traits>

#include "pq_common.h"
#include "pq_device.h"

namespace pq {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// global-address-space accessors for addresses held as integers (keeps the
// compiler on global_load / global_store instead of flat)
typedef __attribute__((address_space(1))) const uint32_t g_u32;
typedef __attribute__((address_space(1))) const uint64_t g_u64;

__device__ __forceinline__ uint32_t gld32(uintptr_t p) { return *(g_u32 *)p; }
__device__ __forceinline__ uint64_t gld64(uintptr_t p) { return *(g_u64 *)p; }
__device__ __forceinline__ void gst32(uintptr_t p, uint32_t v) { *(__attribute__((address_space(1))) uint32_t *)p = v; }
__device__ __forceinline__ void gst64(uintptr_t p, uint64_t v) { *(__attribute__((address_space(1))) uint64_t *)p = v; }
__device__ __forceinline__ void gst128(uintptr_t p, uint4 v) {
  u32x4 x = {v.x, v.y, v.z, v.w};
  *(__attribute__((address_space(1))) u32x4 *)p = x;
}

struct CopyJob {  // dst[0, len) = src[0, len), both in device memory
  const uint8_t *src;
  uint8_t *dst;
  int64_t len;
};

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
  CopyJob *jobs;          // long Snappy literals deferred to k_copy, in per-page regions
  uint32_t *njobs;        // per Snappy-list position: jobs written this decode
  uint32_t max_jobs;      // total job slots
  const int32_t *job_base;   // per Snappy-list position: first slot of its region
  const int32_t *job_owner;  // per slot: Snappy-list position that owns it
  uint64_t *dbg;          // diagnostic build only (-DPQ_STAMPS): per-wave k_expand stamps
  uint64_t *dbg2;         // diagnostic build only: per-page k_prepare stamps / values
  uint64_t *dbg3;         // diagnostic build only: run-walk iteration stamps of page 1
  uint2 *runs;            // k_runs -> k_expand: run tables (PageDesc.run_base)
  int2 *tile_info;        // per RUN_TILE values: {first run, byte of its first key} (PageDesc.tile_base)
  int32_t ex_lds;         // k_expand: staged key bytes per wave (dynamic LDS)
  ExRec *recs;            // k_prepare -> k_expand: one record per job (launch order)
  const int32_t *page_jobs;  // per tiled page (PageDesc.job_base): positions of its jobs
  uint32_t epoch;         // this decode's record epoch
  uint32_t *copy_cnt;     // deferred literals registered this decode: [epoch & 1] (the other is reset)
  int32_t *copy_idx;      // their job slots, compact (k_snappy -> k_copy)
  const int64_t *hjobs;   // literal-train pages' copies from the host plan: (d_in offset, d_stage offset, len, 0)
  int32_t nhjobs;
  uint32_t *status_next;  // k_level_check: the next decode's status array, set to status0 (null: k_reset does it)
  const SwPage *sw_pages;  // region-parallel length walk: pages, region records, results, (page, chunk) items
  SwReg *sw_regs;
  SwRes *sw_res;
  const int2 *sw_items;
  int32_t n_sw_items, n_sw_pages, sw_page0;  // (a launch's part: pages [sw_page0, + n_sw_pages))
  int32_t *lens;          // DELTA string pages: suffix lengths [0, nv), prefix lengths [nv, 2 nv)
  uint8_t *lvl;           // decoded levels of count-path pages (PageDesc::lvl_base), k_prepare -> k_decode
  const uint32_t *status0;  // k_reset: every page's initial status (host planning errors)
  const ZeroRange *zr;      // k_reset: buffers zeroed per decode (validity bitmaps)
  int32_t nzr, npages;
  const TileJob *tiles;   // k_expand: one workgroup per entry
  const LdsGroup *lgroups;  // k_expand_ld: one workgroup per entry
  const uint8_t *in_end, *stage_end;  // allocation ends (PQ_SNAP_GUARD build)
  // Snappy segments (pages longer than SNAP_SEG are decoded by several waves)
  const int2 *sitems;     // k_snappy work items {Snappy-list position, segment}
  int32_t nitems;
  int32_t nwalk;          // k_snappy_walk / fallback: pages in `walk`
  const int32_t *walk;    // Snappy-list positions of the segmented pages
  const int32_t *seg_base;  // per Snappy-list position: first entry in segs (nseg = next - this)
  int64_t *segs;          // per segment: stream offset of its first token (k_snappy_walk)
  uint32_t *seg_flag;     // per Snappy-list position: 0 segments ok, 1 serial fallback, 2 nothing to do
  const int32_t *parts;   // k_decode<3> / <2>: (page, first level, end level) per wave, instead of `list`
  int32_t redo;           // k_decode<3> / <2>: the pages left at ST_REDO by their parts, decoded whole
  int64_t *str_pre;       // split k_decode<2> pages: string bytes before every 256 values (k_prepare)
  const int32_t *part_tab;  // list-page parts (as `parts`), for k_levels
  int32_t *part_pre;        // per part: rows, slots, values before it (4 ints; PageDesc::part0)
};

#ifdef PQ_STAMPS
// per-wave s_memrealtime (100 MHz) stamps, slot (blockIdx * 4 + wave) * 8:
// [0] the kernel's start, [i] (1..5) time accumulated over the wave's jobs
// from the previous stamp to stamp i, [6] the last stamp (the wave's end),
// [7] jobs (counted at stamp 1)
#define STAMP(i)                                                                              \
  do {                                                                                        \
    if (a.dbg && lane_id() == 0) {                                                            \
      const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                   \
      uint64_t *sl_ = a.dbg + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8;              \
      if ((i) == 0) {                                                                         \
        sl_[0] = t_;                                                                          \
        sl_[7] = 0;                                                                           \
        for (int q_ = 1; q_ < 6; q_++) sl_[q_] = 0;                                           \
      } else {                                                                                \
        sl_[(i)] += t_ - sl_[6];                                                              \
        if ((i) == 1) sl_[7] += 1;                                                            \
      }                                                                                       \
      sl_[6] = t_;                                                                            \
    }                                                                                         \
  } while (0)
// k_expand_wg: the same slots per wave of its 16-wave workgroups
#define WSTAMP(i)                                                                             \
  do {                                                                                        \
    if (a.dbg && lane_id() == 0) {                                                            \
      const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                   \
      uint64_t *sl_ = a.dbg + ((size_t)blockIdx.x * WG_WAVES + (threadIdx.x >> 6)) * 8;       \
      if ((i) == 0) {                                                                         \
        sl_[0] = t_;                                                                          \
        sl_[7] = 0;                                                                           \
        for (int q_ = 1; q_ < 6; q_++) sl_[q_] = 0;                                           \
      } else {                                                                                \
        sl_[(i)] += t_ - sl_[6];                                                              \
        if ((i) == 2) sl_[7] += 1;                                                            \
      }                                                                                       \
      sl_[6] = t_;                                                                            \
    }                                                                                         \
  } while (0)
#define PSTAMP(page, i, v)                              \
  do {                                                   \
    if (a.dbg2 && lane_id() == 0) a.dbg2[(size_t)(page) * 8 + (i)] = (v); \
  } while (0)
#else
#define WSTAMP(i) \
  do {                 \
  } while (0)
#define PSTAMP(page, i, v) \
  do {                     \
  } while (0)
#define STAMP(i) \
  do {           \
  } while (0)
#endif

__device__ __forceinline__ void set_status(uint32_t *status, int page, uint32_t stage, uint32_t code) {
  if (lane_id() == 0) atomicMin(&status[page], make_status(stage, code));
}
__device__ __forceinline__ uint32_t page_status(const uint32_t *status, int page) {
  return ufirst(__atomic_load_n(&status[page], __ATOMIC_RELAXED));
}

// Values section of page `idx`.  A Snappy block that is a single literal is
// its own content: k_snappy then leaves it in place (PageInfo.alias1) instead
// of copying it to staging.
__device__ __forceinline__ const uint8_t *body_ptr(const KArgs &a, const PageDesc &d, int idx) {
  if (d.body_src == BODY_RAW) return a.in + d.body;
  if (d.body_src == BODY_SNAPPY) {
    const int64_t al = a.info[idx].alias1;
    if (al) return a.in + (al - 1);
  }
  return a.stage + d.body;
}

// ===========================================================================
// K1: Snappy (vendor/github.com/golang/snappy/decode.go:55-75, decode_other.go:14-101)
// ===========================================================================
#ifndef PQ_RING
#define PQ_RING 4096
#endif
#ifndef PQ_PF_EARLY
#define PQ_PF_EARLY 1  // k_snappy: the next batch's window prefetched right after the token chain (0: after the far copies)
#endif
#ifndef PQ_SNAP_TOKEN
#define PQ_SNAP_TOKEN 1  // k_snappy: token-parallel output when the batch allows it (0: the per-byte chase always)
#endif
#ifndef SNAP_DEP_MAX
#define SNAP_DEP_MAX 64  // copies overlapping their own batch written one after another (more: per-byte chase)
#endif
#ifndef PQ_SNAP_B16
#define PQ_SNAP_B16 1  // k_snappy: short tokens stored as byte pairs (0: a byte at a time)
#endif
#ifndef SNAP_TOK_SHORT
#define SNAP_TOK_SHORT 16  // token-parallel output: longer literals / near copies take the whole wave each
#endif
#ifndef PQ_FAR_DEFER
#define PQ_FAR_DEFER 1  // k_snappy: short far copies' loads overlap the token tables (0: written at once)
#endif
#ifndef PQ_SNAPPY_WPE
#define PQ_SNAPPY_WPE 6
#endif
// per-wave LDS history (bytes): 4 KB keeps six waves per SIMD resident (older
// bytes: HBM).  Measured (C3 / C5 step, ms): 4 KB at 6 waves 5.26 / 24.4;
// 8 KB at 4 waves 6.24 / 28.7; 16 KB at 2 waves 8.40 / 39.7; 2 KB at 7 waves
// 5.10 / 24.8, at 8 waves (10 VGPRs spilled) 5.17 / 25.7 — occupancy first.
constexpr int RING = PQ_RING;
constexpr int RING_MASK = RING - 1;
constexpr int SNAPPY_WAVES = 4;

// Literal run: dst[dpos, dpos+len) = s[0, len).  The staging page base is
// 16-byte aligned, so after a <16-byte head every lane stores whole 16-byte
// chunks (1 KiB per wave instruction); the source is read as aligned dwords
// and funnel-shifted (v_alignbyte) by the uniform source/destination skew.
// Only the last RING bytes also enter the LDS history.
// A far copy reads back this wave's own staged output.  Stores of the same CU
// are visible to its loads through the CU's L1 once complete (the workgroup
// fence before the far copies waits for them; a workgroup acquire needs no L1
// invalidate), so the loads are plain global loads — served by L1 / the XCD's
// L2 — instead of device-scope ones, which on gfx950 miss the L2 and went to
// the Infinity Cache / HBM for every copy (C3: k_snappy's FETCH was 11x its
// compressed input).  PQ_FAR_AGENT (analysis) restores device scope.
template <class T>
__device__ __forceinline__ T far_ld(const T *p) {
#ifdef PQ_FAR_AGENT
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  return *(const __attribute__((address_space(1))) T *)p;
#endif
}

__device__ __forceinline__ void copy_literal(const uint8_t *s, uint8_t *dst, int64_t dpos, int64_t len, uint8_t *ring,
                                             int lane) {
  uint8_t *D = dst + dpos;
  const int64_t ring_from = dpos + len - RING;  // page offsets >= ring_from go to the history
  int64_t head = (int64_t)((16 - ((uintptr_t)D & 15)) & 15);
  if (head > len) head = len;
  if (lane < head) {
    uint8_t b = s[lane];
    D[lane] = b;
    if (dpos + lane >= ring_from) ring[(dpos + lane) & RING_MASK] = b;
  }
  const int64_t body = (len - head) >> 4;
  const uint8_t *S = s + head;
  uint8_t *D16 = D + head;
  const int64_t q0 = dpos + head;  // page offset of the first 16-byte chunk (multiple of 16)
  const uint32_t skew = (uint32_t)((uintptr_t)S & 3);
  const uint32_t *SA = (const uint32_t *)((uintptr_t)S & ~(uintptr_t)3);
  for (int64_t c = lane; c < body; c += 128) {
    int64_t c2 = c + 64;
    uint4 a = *(const uint4 *)(SA + 4 * c);
    uint32_t a4 = SA[4 * c + 4];
    uint4 b = make_uint4(0, 0, 0, 0);
    uint32_t b4 = 0;
    if (c2 < body) {
      b = *(const uint4 *)(SA + 4 * c2);
      b4 = SA[4 * c2 + 4];
    }
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(a.y, a.x, skew);
    o.y = __builtin_amdgcn_alignbyte(a.z, a.y, skew);
    o.z = __builtin_amdgcn_alignbyte(a.w, a.z, skew);
    o.w = __builtin_amdgcn_alignbyte(a4, a.w, skew);
    *(uint4 *)(D16 + 16 * c) = o;
    if (q0 + 16 * c + 16 > ring_from) *(uint4 *)(ring + ((q0 + 16 * c) & RING_MASK)) = o;
    if (c2 < body) {
      uint4 p;
      p.x = __builtin_amdgcn_alignbyte(b.y, b.x, skew);
      p.y = __builtin_amdgcn_alignbyte(b.z, b.y, skew);
      p.z = __builtin_amdgcn_alignbyte(b.w, b.z, skew);
      p.w = __builtin_amdgcn_alignbyte(b4, b.w, skew);
      *(uint4 *)(D16 + 16 * c2) = p;
      if (q0 + 16 * c2 + 16 > ring_from) *(uint4 *)(ring + ((q0 + 16 * c2) & RING_MASK)) = p;
    }
  }
  const int64_t done = head + body * 16;
  const int64_t tail = len - done;
  if (lane < tail) {
    uint8_t b = s[done + lane];
    D[done + lane] = b;
    ring[(dpos + done + lane) & RING_MASK] = b;
  }
}

// Wave copy of len bytes between arbitrary addresses: 16-byte aligned stores
// after a short head, funnel-shifted dword loads (no LDS history).
__device__ __forceinline__ void copy_bytes_wave(const uint8_t *s, uint8_t *D, int64_t len, int lane) {
  int64_t head = (int64_t)((16 - ((uintptr_t)D & 15)) & 15);
  if (head > len) head = len;
  if (lane < head) D[lane] = s[lane];
  const int64_t body = (len - head) >> 4;
  const uint8_t *S = s + head;
  uint8_t *D16 = D + head;
  const uint32_t skew = (uint32_t)((uintptr_t)S & 3);
  const uint32_t *SA = (const uint32_t *)((uintptr_t)S & ~(uintptr_t)3);
  for (int64_t c = lane; c < body; c += 64) {
    uint4 x = *(const uint4 *)(SA + 4 * c);
    uint32_t x4 = SA[4 * c + 4];
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(x.y, x.x, skew);
    o.y = __builtin_amdgcn_alignbyte(x.z, x.y, skew);
    o.z = __builtin_amdgcn_alignbyte(x.w, x.z, skew);
    o.w = __builtin_amdgcn_alignbyte(x4, x.w, skew);
    *(uint4 *)(D16 + 16 * c) = o;
  }
  const int64_t done = head + body * 16;
  if (lane < len - done) D[done + lane] = s[done + lane];
}

// Put the last min(len, RING) bytes of a deferred literal into the history
// (16-byte LDS stores from funnel-shifted dword loads; done lazily, only when
// a copy token follows the literal).
__device__ __forceinline__ void ring_fill(const uint8_t *s, int64_t dpos, int64_t len, uint8_t *ring, int lane) {
  const int64_t from = len > RING ? len - RING : 0;     // literal offset of the first history byte
  const int64_t q_end = dpos + len;
  int64_t q0 = (dpos + from + 15) & ~(int64_t)15;        // first 16-byte aligned page offset
  // unaligned head bytes
  if (lane < q0 - (dpos + from) && dpos + from + lane < q_end) ring[(dpos + from + lane) & RING_MASK] = s[from + lane];
  const int64_t nchunks = (q_end - q0) >> 4;
  for (int64_t c = lane; c < nchunks; c += 64) {
    const uint8_t *sp = s + (q0 + 16 * c - dpos);
    const uint32_t skew = (uint32_t)((uintptr_t)sp & 3);
    const uint32_t *sa = (const uint32_t *)((uintptr_t)sp & ~(uintptr_t)3);
    uint4 x = *(const uint4 *)sa;
    uint32_t x4 = sa[4];
    uint4 o;
    o.x = __builtin_amdgcn_alignbyte(x.y, x.x, skew);
    o.y = __builtin_amdgcn_alignbyte(x.z, x.y, skew);
    o.z = __builtin_amdgcn_alignbyte(x.w, x.z, skew);
    o.w = __builtin_amdgcn_alignbyte(x4, x.w, skew);
    *(uint4 *)(ring + ((q0 + 16 * c) & RING_MASK)) = o;
  }
  const int64_t t0 = q0 + nchunks * 16;
  if (t0 + lane < q_end) ring[(t0 + lane) & RING_MASK] = s[t0 + lane - dpos];
}

constexpr int64_t BIG_LITERAL = 16 * 1024;  // longer literals are copied by k_copy (many workgroups)
constexpr int MAX_DEFER = 64;  // one entry per lane

// ---- batched short tokens --------------------------------------------------
// A run of copies and short literals (the body of a compressible block) is
// decoded SB_TOK tokens at a time instead of one token per wave iteration:
//  1. 512 compressed bytes are staged in LDS; each lane classifies the 4 tag
//     positions it holds (token size + output length, 16 bits each);
//  2. the token chain is walked on the scalar unit (two v_readlane per hop),
//     token k's position written to lane k;
//  3. lane k decodes token k, checks it (decode_other.go:14-101 order: header
//     inside src, literal/copy length <= remaining dst, 0 < offset <= d) and an
//     exclusive scan gives every token's output position;
//  4. every output byte of the batch is resolved by its own lane: the byte's
//     token comes from a token-start bitmap (+ per-word prefix counts); a copy
//     byte maps to dst[start - offset + (r mod offset)] and is chased back
//     until it lands in a literal or before the batch (LDS history, or the
//     staged output / a deferred literal's payload when older than RING);
//  5. the bytes enter the history; whole 16-byte chunks go to HBM.
constexpr int SB_TOK = 64;    // tokens per batch (one per lane)
constexpr int SB_OUT = 1024;  // output bytes per batch (token-start bitmap: 32 words)
constexpr int SB_WIN = 512;   // compressed bytes staged per batch (walk covers the first 256)

struct SnapLds {  // per wave
#ifdef PQ_SNAP_STAMPS
  uint64_t acc[8];  // diagnostic build: shader cycles per batch phase, batches
  uint64_t tprev;
#endif
  uint32_t win[SB_WIN / 4 + 4];
  union {
    struct {
      uint4 tok[SB_TOK];        // {out_rel, len | literal << 31 | prefilled << 30, literal: window byte / copy: offset, 0}
      uint2 bmc[SB_OUT / 32];   // token-start bits, tokens starting in earlier words
    };
    uint16_t jt[280];           // token chain: entry addresses of J_b over window positions 0..256 (jt_off)
  };
};

// diagnostic build (-DPQ_SNAP_STAMPS, tools/diag_snappy.py): shader cycles of
// each phase of a batch, accumulated per wave and written per page to dbg2
#ifdef PQ_SNAP_STAMPS
#define SNAP_T(i)                                                  \
  do {                                                             \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();              \
    if (lane == 0) {                                               \
      if ((i) >= 0) L.acc[(i) < 0 ? 0 : (i)] += t_ - L.tprev;      \
      L.tprev = t_;                                                \
    }                                                              \
  } while (0)
#elif defined(PQ_SNAP_MARKS)
#define SNAP_T(i) asm volatile(";SNAPMARK " #i)
#else
#define SNAP_T(i) \
  do {            \
  } while (0)
#endif

#ifndef PQ_K5_WPE
#define PQ_K5_WPE 3  // k_decode<5> (parts of list pages: level scratch, PLAIN / dictionary values): waves per SIMD
#endif
#ifndef PQ_K4_WPE
#define PQ_K4_WPE 8  // k_decode<4> (flat required dictionary strings): waves per SIMD
#endif

// diagnostic build (-DPQ_DEC_STAMPS, tools/diag_decode.py): k_decode<2>'s
// shader cycles per step phase, accumulated per wave, added to dbg2 per page
#ifdef PQ_DEC_STAMPS
#define DEC_T(i)                                               \
  do {                                                         \
    if (KIND == 1 || KIND == 2 || KIND == 4 || KIND == 5) {                 \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();        \
      if ((i) >= 0) dacc[(i) < 0 ? 0 : (i)] += t_ - dprev;     \
      dprev = t_;                                              \
    }                                                          \
  } while (0)
#else
#define DEC_T(i) \
  do {           \
  } while (0)
#endif

#ifdef PQ_SNAP_GUARD
#define PQ_CHK(c, id, u, v, onfail)                                                                   \
  do {                                                                                                \
    if (c) {                                                                                          \
      printf("PQ_CHK %d: %llx %llx\n", id, (unsigned long long)(u), (unsigned long long)(v));        \
      onfail;                                                                                         \
    }                                                                                                 \
  } while (0)
#define SNAP_GUARD(c, id, u, v)                                                                      \
  do {                                                                                               \
    if (c) printf("SNAP_GUARD %d: %lld %lld (dpos %lld dl %lld s %lld)\n", id, (long long)(u),        \
                  (long long)(v), (long long)dpos, (long long)dl, (long long)s);                     \
  } while (0)
#else
#define PQ_CHK(c, id, u, v, onfail) \
  do {                              \
  } while (0)
#define SNAP_GUARD(c, id, u, v) \
  do {                          \
  } while (0)
#endif

__device__ __forceinline__ uint32_t snappy_tok_class(uint32_t tag) {
  // token size in the stream (low byte) | output length << 8; 0: long literal
  const uint32_t t = tag & 3, x = tag >> 2;
  if (t == 0) return x >= 60 ? 0u : (x + 2) | ((x + 1) << 8);
  if (t == 1) return 2u | ((4 + (x & 7)) << 8);
  return (t == 2 ? 3u : 5u) | ((1 + x) << 8);
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// LDS byte addresses (address space 3): the chain table holds them, so a hop
// is one ds_read_u16 with no address arithmetic, and byte copies add
// immediate offsets to them.  (A workgroup's LDS addresses start at 0 and
// k_snappy's stay below 64 KiB.)
#define PQ_LDS __attribute__((address_space(3)))
__device__ __forceinline__ uint32_t lds_addr(const void *p) { return (uint32_t)(uintptr_t)(const PQ_LDS void *)p; }
__device__ __forceinline__ uint32_t lds_u8(uint32_t a) { return *(const PQ_LDS uint8_t *)(uintptr_t)a; }
__device__ __forceinline__ uint32_t lds_u16(uint32_t a) { return *(const PQ_LDS uint16_t *)(uintptr_t)a; }
__device__ __forceinline__ uint32_t lds_u32(uint32_t a) { return *(const PQ_LDS uint32_t *)(uintptr_t)a; }
__device__ __forceinline__ void lds_st8(uint32_t a, uint32_t v) { *(PQ_LDS uint8_t *)(uintptr_t)a = (uint8_t)v; }
__device__ __forceinline__ void lds_st16(uint32_t a, uint32_t v) { *(PQ_LDS uint16_t *)(uintptr_t)a = (uint16_t)v; }
__device__ __forceinline__ void lds_st64(uint32_t a, uint32_t lo, uint32_t hi) {  // a: 8-byte aligned
  *(PQ_LDS uint64_t *)(uintptr_t)a = ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ void lds_st32(uint32_t a, uint32_t v) { *(PQ_LDS uint32_t *)(uintptr_t)a = v; }

// Tag table of k_snappy (one per workgroup, LDS), a u16 per tag: the stream
// bytes of a short token (a literal's tag and payload, a copy's header; 255
// for a long literal's tag) | its output length << 8 (0: long literal) —
// decode_other.go:27-86's cases as one lookup instead of a branch per case.
constexpr int SNAP_LUT = 512;
__device__ __forceinline__ void snappy_lut_init(uint8_t *lut, int tag) {
  const uint32_t t = (uint32_t)tag & 3, x = (uint32_t)tag >> 2;
  uint32_t need, len;
  if (t == 0) {
    need = x >= 60 ? 255u : x + 2;
    len = x >= 60 ? 0u : x + 1;
  } else if (t == 1) {
    need = 2;
    len = 4 + (x & 7);
  } else {
    need = t == 2 ? 3u : 5u;
    len = x + 1;
  }
  // one u16 a tag (stream bytes | output length << 8): one ds_read_u16 a
  // token instead of two byte reads at independent random banks
  *(uint16_t *)(lut + 2 * tag) = (uint16_t)(need | (len << 8));
}

// The chain table's byte offset of window position p: PQ_JT_PAD bytes after
// every 64 positions.  Lane l's reads of a round land near position 4 l + c,
// so lanes l and l + 16 of a 32-lane group hit one bank; a pad of 8 shifts
// each 64-position block by two banks (the lanes' 8-byte stores stay 8-byte
// aligned).  Measured (round 6, analysis variants): C3 3.218 ms unpadded vs
// 3.255 padded, C5 16.14 vs 16.19 — the jump rounds are not bound by these
// conflicts, so the default is no pad.
#ifndef PQ_JT_PAD
#define PQ_JT_PAD 0
#endif
__device__ __forceinline__ uint32_t jt_off(uint32_t p) { return 2 * p + PQ_JT_PAD * (p >> 6); }
__device__ __forceinline__ uint32_t jt_pos(uint32_t off) {  // inverse of jt_off (off <= jt_off(256))
  const uint32_t blk = (uint32_t)(off >= 128 + PQ_JT_PAD) + (uint32_t)(off >= 2 * (128 + PQ_JT_PAD)) +
                       (uint32_t)(off >= 3 * (128 + PQ_JT_PAD)) + (uint32_t)(off >= 4 * (128 + PQ_JT_PAD));
  return (off - PQ_JT_PAD * blk) >> 1;
}

// One batch starting at the short token at s.  Returns false on a corrupt
// token (err set); advances s / dpos / F otherwise.  `lut`: the tag tables.
__device__ __forceinline__ bool snappy_batch(SnapLds &L, uint8_t *ring, uint32_t lut, const uint8_t *src, int64_t slen,
                                             uint8_t *dst, int64_t dl, int64_t seg_lo, bool write, int64_t &s,
                                             int64_t &dpos, int64_t &F, uint32_t &err, const uint8_t *pend_src,
                                             int64_t pend_dpos, int64_t &pend_len, int ndefer, int64_t def_dst,
                                             int64_t def_len, uint64_t def_src, int lane, const uint8_t *in_end,
                                             int64_t &pf_s, int64_t &pf_F, uint32_t &pg0, uint32_t &pg1, uint32_t &pg2) {
  SNAP_T(-1);
  // 1. stage the window (aligned base; `sh` = position of byte s); the
  // previous batch prefetched it into pg0..pg2 when it ended at s
  const uintptr_t abase = (uintptr_t)(src + s) & ~(uintptr_t)3;
  const int sh = (int)((uintptr_t)(src + s) & 3);
  const uint32_t *ga = (const uint32_t *)abase;
  PQ_CHK(in_end && abase + 528 > (uintptr_t)in_end, 10, abase, in_end, err = E_SNAPPY; return false);
  uint32_t g0, g1, g2;
  // staged output known written: loads and stores retire in order (one
  // vmcnt), so waiting for the window's loads retired every store issued
  // before them — the flushes up to pf_F for the prefetch, F for a fresh load
  int64_t F_safe = F;
  if (pf_s == s) {
    g0 = pg0;
    g1 = pg1;
    g2 = pg2;
    F_safe = pf_F;
  } else {
    g0 = ga[lane];
    g1 = ga[lane + 64];
    g2 = lane < 4 ? ga[lane + 128] : 0u;
  }
  pf_s = -1;
  L.win[lane] = g0;
  L.win[lane + 64] = g1;
  if (lane < 4) L.win[lane + 128] = g2;
  const uint32_t wb = lds_addr(L.win);  // window byte 0
  const uint32_t tb = lds_addr(L.jt);      // chain table (u16): the entry of position i at tb + jt_off(i)
  const uint32_t stop = tb + jt_off(256);  // position 256: the chain's end (its entry points at itself)
  // J_0 of this lane's positions 4 lane + j (the bytes of its window dword):
  // the entry address of the position after a token starting there.  Token
  // sizes SWAR over the 4 tags: a literal x + 2, copies 2 / 3 / 5 by a byte
  // permute (a long literal's tag reads 62..65 here; the decode below cuts
  // the batch at it)
  const uint32_t t4 = g0 & 0x03030303u, x4 = (g0 >> 2) & 0x3f3f3f3fu;
  const uint32_t mlit = __builtin_amdgcn_perm(0u, 0x000000ffu, t4);  // 0xff where a literal
  const uint32_t need4 = ((x4 + 0x02020202u) & mlit) | (__builtin_amdgcn_perm(0u, 0x05030200u, t4) & ~mlit);
  uint32_t J[4];
#pragma unroll
  for (int j = 0; j < 4; j++) J[j] = tb + jt_off(min(4 * (uint32_t)lane + j + ((need4 >> (8 * j)) & 0xffu), 256u));
  const uint32_t jl = tb + jt_off(4 * (uint32_t)lane);  // this lane's four entries (8-byte aligned)
  lds_st64(jl, J[0] | (J[1] << 16), J[2] | (J[3] << 16));
  if (lane == 0) lds_st16(stop, stop);
  SNAP_T(0);
  // 2. the token chain by pointer jumping, in place: J_b+1 = J_b o J_b (a
  // round's reads are all issued before its writes; the wave's LDS accesses
  // run in order); lane m applies J_b for the set bits b of m starting at
  // sh, so it lands on the m-th token
  wave_lds_sync();
  uint32_t P = tb + jt_off((uint32_t)sh);
#pragma unroll
  for (int b = 0; b < 6; b++) {
    const uint32_t hop = lds_u16(P);
    if (b < 5) {
      uint32_t n[4];
#pragma unroll
      for (int j = 0; j < 4; j++) n[j] = lds_u16(J[j]);
#pragma unroll
      for (int j = 0; j < 4; j++) J[j] = n[j];
      lds_st64(jl, n[0] | (n[1] << 16), n[2] | (n[3] << 16));
    }
    if ((lane >> b) & 1) P = hop;
    if (b < 5) wave_lds_sync();
  }
  // 3. decode token `lane` (its tag from the tables, its offset from the 5
  // bytes at it) and check it (decode_other.go:14-101 order: header inside
  // src, length <= remaining dst, 0 < offset <= d)
  const int64_t lim64 = (int64_t)sh + (slen - s) - 1;  // last position inside the block
  const uint32_t lim = lim64 < 255 ? (uint32_t)lim64 : 255u;
  const uint32_t pos = jt_pos(P - tb);
  const uint32_t pa = wb + pos;
  const uint32_t tag = lds_u8(pa);
  const uint32_t nl = lds_u16(lut + 2 * tag);
  const uint32_t need = nl & 0xffu, len0 = nl >> 8;
  const uint32_t d0 = lds_u32(pa & ~3u), d1 = lds_u32((pa & ~3u) + 4);
  const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, pa & 3u), hi = __builtin_amdgcn_alignbyte(0u, d1, pa & 3u);
  const uint32_t t = tag & 3;
  const bool lit = t == 0;
  const uint32_t c1 = ((tag >> 5) << 8) | ((lo >> 8) & 0xffu);  // tagCopy1
  const uint32_t c2 = (lo >> 8) & 0xffffu;                      // tagCopy2
  const uint32_t c4 = __builtin_amdgcn_alignbyte(hi, lo, 1u);   // tagCopy4
  // literal: window position of its bytes / copy: offset
  const uint32_t x = lit ? pos + 1 : t == 1 ? c1 : t == 2 ? c2 : c4;
  const bool valid = pos <= lim && len0 != 0;
  const int64_t rem64 = slen - s, room64 = dl - dpos;
  const int32_t rem = rem64 < 0x40000000 ? (int32_t)rem64 : 0x40000000;  // stream bytes from s
  const int32_t room = room64 < 0x40000000 ? (int32_t)room64 : 0x40000000;
  const int32_t tend = (int32_t)pos - sh + (int32_t)need;  // the token's end, from s
  const uint32_t vlen = valid ? len0 : 0u;
  const int32_t incl = (int32_t)wave_incl_dpp<false>(vlen);
  // the leading lanes: tokens that fit the batch and start before the end of
  // the output (of the segment: a later token belongs to the next one)
  const uint64_t okm = ballot(valid && incl <= SB_OUT && incl - (int32_t)vlen < room);
  const int ntok = ~okm ? (int)__builtin_ctzll(~okm) : 64;
  if (ntok == 0) {  // output complete but tokens remain, or a token crosses the segment end
    err = E_SNAPPY;
    return false;
  }
  const int T = (int)__builtin_amdgcn_readlane(incl, ntok - 1);
  const int cur = (int)__builtin_amdgcn_readlane(tend, ntok - 1) + sh;
  if (PQ_PF_EARLY) {
    // the next batch's window, prefetched as soon as this batch's end is
    // known: its loads overlap this batch's decode, far copies and output
    const int64_t sn = s + (cur - sh);
    if (sn < slen) {
      const uint32_t *gn = (const uint32_t *)((uintptr_t)(src + sn) & ~(uintptr_t)3);
      pg0 = gn[lane];
      pg1 = gn[lane + 64];
      pg2 = lane < 4 ? gn[lane + 128] : 0u;
      pf_s = sn;
      pf_F = F;
    }
  }
  SNAP_T(1);
  const bool act = lane < ntok;
  const uint32_t len = act ? len0 : 0u;
  const int32_t out_rel = incl - (int32_t)len;
  const uint32_t back = (uint32_t)(dpos - seg_lo);  // output before the batch (< 2^31: a page's size is an int32)
  if (ballot(act && (tend > rem || incl > room || (!lit && (x == 0 || x > back + (uint32_t)out_rel))))) {
    err = E_SNAPPY;
    return false;
  }
  const int32_t total = T;
  SNAP_T(2);
  if (write) {
    if (pend_len) {  // the history must hold the last deferred literal's tail
      ring_fill(pend_src, pend_dpos, pend_len, ring, lane);
      pend_len = 0;
    }
    // 4. far copies first: a copy token whose whole source is older than the
    // history (staged output of earlier batches, or a deferred literal's
    // payload) is loaded by its own lane and written to the history at its
    // output position, all such loads in flight together
    const int64_t near_lo = dpos + T - RING;  // older bytes may be overwritten by this batch
    const uint32_t b32 = (uint32_t)dpos;      // (ring positions: low 32 bits suffice)
    const bool far = act && !lit && x > (uint32_t)(out_rel + RING - T);  // source starts before near_lo
    bool pre = false, fdefer = false;
    uint64_t fq0 = 0, fq1 = 0;
    int fsh = 0;
    if (ballot(far)) {
      const int64_t S = dpos + out_rel - (int64_t)x;  // absolute source start
      // this wave's earlier staging stores must be visible to the loads below
      // (unless every source lies in output known written)
      if (ballot(far && S + (int64_t)len > F_safe)) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      pre = far && x >= len && S + (int64_t)len <= near_lo;
      uintptr_t fsrc = pre ? (uintptr_t)(dst + S) : 0;
      bool in_payload = false;
      for (int k2 = 0; k2 < ndefer; k2++) {  // every lane active: readlane of the deferred-literal table
        const int64_t kd = (int64_t)readlane64(def_dst, k2);
        const int64_t kl = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)def_len, k2);
        const uint64_t ks = readlane64(def_src, k2);
        if (pre && S < kd + kl && S + (int64_t)len > kd) {
          if (S >= kd && S + (int64_t)len <= kd + kl) {
            fsrc = (uintptr_t)ks + (uintptr_t)(S - kd);
            in_payload = true;
          } else {
            pre = false;  // straddles a deferred literal: byte by byte below
          }
        }
      }
      if (pre && PQ_FAR_DEFER && (int)(fsrc & 7) + (int)len <= 16) {
        // a short far copy (two aligned qwords): loads issued now, bytes
        // written to the history with the short tokens', so the round trip
        // overlaps the steps between
        const uintptr_t b8 = fsrc & ~(uintptr_t)7;
        const uint64_t *qp = (const uint64_t *)b8;
        fq0 = in_payload ? qp[0] : far_ld(qp);
        if ((int)(fsrc & 7) + (int)len > 8)
          fq1 = in_payload ? qp[1] : far_ld(qp + 1);
        fsh = (int)(fsrc & 7);
        fdefer = true;
      } else if (pre) {
        // <= 64 source bytes: up to 9 aligned qwords of staged output (far_ld)
        const uintptr_t b8 = fsrc & ~(uintptr_t)7;
        const int sh8 = (int)(fsrc & 7);
        const int64_t o = dpos + out_rel;
#pragma unroll
        for (int w = 0; w < 9; w++) {
          if (w * 8 >= sh8 + (int)len) break;
          const uint64_t *qp = (const uint64_t *)(b8 + 8 * (uintptr_t)w);
          const uint64_t v = in_payload ? *qp : far_ld(qp);
#pragma unroll
          for (int bb = 0; bb < 8; bb++) {
            const int i2 = w * 8 + bb - sh8;
            if (i2 >= 0 && i2 < (int)len) ring[(o + i2) & RING_MASK] = (uint8_t)(v >> (8 * bb));
          }
        }
      }
    }
    // prefetch the next batch's window (its loads overlap this batch's output)
    if (!PQ_PF_EARLY) {
      const int64_t sn = s + (cur - sh);
      if (sn < slen) {
        const uint32_t *gn = (const uint32_t *)((uintptr_t)(src + sn) & ~(uintptr_t)3);
        pg0 = gn[lane];
        pg1 = gn[lane + 64];
        pg2 = lane < 4 ? gn[lane + 128] : 0u;
        pf_s = sn;
        pf_F = F;
      }
    }
    SNAP_T(3);
    const uint8_t *winb = (const uint8_t *)L.win;
    // Token-parallel output (PQ_SNAP_TOKEN): when every copy's source is
    // either already in the history (older than the batch: `near`), or was
    // prefilled / is being loaded (`pre`), or lies partly inside the batch
    // (`dep`), the tokens are written by their own lanes — literals from the
    // window, near copies history to history, short far copies from their
    // loaded qwords, all at once — and then the dep copies one after another
    // in token order, a byte a lane (an overlapping copy by pattern: byte r
    // from S + r mod offset).  No token table, no start bitmap, no per-byte
    // chase.
    const bool nearc = act && !lit && !far && x >= (uint32_t)out_rel + len;
    const bool depc = act && !lit && !far && x < (uint32_t)out_rel + len;
    const uint64_t depm = ballot(depc);
    const bool fast = PQ_SNAP_TOKEN && !ballot(far && !pre);
    if (fast) {
      const uint32_t rb = lds_addr(ring);
      const uint32_t ro = (b32 + (uint32_t)out_rel) & RING_MASK;  // ring position of the token's output
      // LDS address of the token's source bytes: the window, the history, or
      // (a short far copy) its two qwords parked in the token-table area
      uint32_t sa = lit ? wb + x : rb + ((b32 + (uint32_t)out_rel - x) & RING_MASK);
      if (fdefer) {
        L.tok[lane] = make_uint4((uint32_t)fq0, (uint32_t)(fq0 >> 32), (uint32_t)fq1, (uint32_t)(fq1 >> 32));
        sa = lds_addr(&L.tok[lane]) + (uint32_t)fsh;
      }
      // tokens of up to SNAP_TOK_SHORT bytes by their own lanes (all of a
      // step's reads before its writes: one LDS round trip a step); longer
      // ones (long literals) one after another by the whole wave
      const bool shortc = act && (lit || nearc || fdefer) && len <= SNAP_TOK_SHORT;
      const uint32_t mylen = shortc ? len : 0u;
      const uint32_t da = rb + ro;
      // a source or destination range that runs past the end of the ring
      const bool wrap = shortc && (ro + len > RING || (!lit && !fdefer && (sa - rb) + len > RING));
      if (!ballot(wrap)) {
#if PQ_SNAP_B16
        // the source as aligned dwords, funnel-shifted (v_alignbyte) to the
        // token's bytes and again to the destination's 2-byte alignment; a
        // head byte to an even address, then byte pairs (ds_write_b16 /
        // _d16_hi), then a tail byte: at most 10 store steps a token
        // instead of 16 byte stores
        const uint32_t s4 = sa & ~3u, hb = da & 1u;
        uint32_t w[6];
#pragma unroll
        for (int i = 0; i < 6; i++) w[i] = lds_u32(s4 + 4 * i);  // (bytes past the token: unused)
        const uint32_t tail = lds_u8(sa + (mylen ? mylen - 1 : 0));
        uint32_t r[5], v[4];
#pragma unroll
        for (int i = 0; i < 5; i++) r[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sa & 3u);  // token bytes 4 i ..
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = __builtin_amdgcn_alignbyte(r[i + 1], r[i], hb);  // token bytes hb + 4 i ..
        if (hb && mylen) lds_st8(da, r[0]);
#pragma unroll
        for (int h = 0; h < 2; h++) {
          if (h > 0 && !ballot(mylen > hb + 8u)) break;
#pragma unroll
          for (int p = 4 * h; p < 4 * h + 4; p++)
            if (hb + 2u * p + 2u <= mylen) lds_st16(da + hb + 2 * p, (p & 1) ? v[p >> 1] >> 16 : v[p >> 1]);
        }
        if (mylen > hb && ((mylen - hb) & 1u)) lds_st8(da + mylen - 1, tail);
#else
        // (analysis build PQ_SNAP_B16=0: the byte stores this replaced)
        const uint32_t s4 = sa & ~3u;
#pragma unroll
        for (int h = 0; h < SNAP_TOK_SHORT / 8; h++) {
          if (h > 0 && !ballot(mylen > 8u * h)) break;
          const uint32_t w0 = lds_u32(s4 + 8 * h), w1 = lds_u32(s4 + 8 * h + 4), w2 = lds_u32(s4 + 8 * h + 8);
          const uint32_t r0 = __builtin_amdgcn_alignbyte(w1, w0, sa & 3u), r1 = __builtin_amdgcn_alignbyte(w2, w1, sa & 3u);
#pragma unroll
          for (int i = 0; i < 8; i++)
            if (8u * h + i < mylen) lds_st8(da + 8 * h + i, (i < 4 ? r0 : r1) >> (8 * (i & 3)));
        }
#endif
      } else {
        for (uint32_t i = 0; i < SNAP_TOK_SHORT; i++) {
          if (!ballot(i < mylen)) break;
          if (i < mylen) {
            const uint32_t sb = lit || fdefer ? sa + i : rb + ((sa - rb + i) & RING_MASK);
            lds_st8(rb + ((ro + i) & RING_MASK), lds_u8(sb));
          }
        }
      }
      for (uint64_t lm = ballot(act && (lit || nearc) && len > SNAP_TOK_SHORT); lm; lm &= lm - 1) {
        const int k = (int)__builtin_ctzll(lm);
        const uint32_t ok = b32 + (uint32_t)__builtin_amdgcn_readlane(out_rel, k);
        const uint32_t lk = (uint32_t)__builtin_amdgcn_readlane((int)len, k);
        const uint32_t xk = (uint32_t)__builtin_amdgcn_readlane((int)x, k);
        const bool litk = __builtin_amdgcn_readlane((int)lit, k) != 0;
        if ((uint32_t)lane < lk) ring[(ok + lane) & RING_MASK] = litk ? winb[xk + lane] : ring[(ok - xk + lane) & RING_MASK];
      }
      wave_lds_sync();
      SNAP_T(4);
      for (uint64_t dm = depm; dm; dm &= dm - 1) {
        const int k = (int)__builtin_ctzll(dm);
        const uint32_t ok = b32 + (uint32_t)__builtin_amdgcn_readlane(out_rel, k);
        const uint32_t lk = (uint32_t)__builtin_amdgcn_readlane((int)len, k);
        const uint32_t xk = (uint32_t)__builtin_amdgcn_readlane((int)x, k);
        uint32_t r = (uint32_t)lane;
        if (xk < lk) r = (uint32_t)lane % xk;  // (uniform branch) a repeated pattern
        if ((uint32_t)lane < lk) ring[(ok + lane) & RING_MASK] = ring[(ok - xk + r) & RING_MASK];
        wave_lds_sync();
      }
    } else {
    // token table + start bitmap
    if (act) L.tok[lane] = make_uint4((uint32_t)out_rel, len | (lit ? 0x80000000u : 0u) | (pre ? 0x40000000u : 0u), x, 0u);
    if (lane < SB_OUT / 32) L.bmc[lane] = make_uint2(0u, 0u);
    wave_lds_sync();
    if (act) __hip_atomic_fetch_or(&L.bmc[out_rel >> 5].x, 1u << (out_rel & 31), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
    wave_lds_sync();
    const uint32_t bits = lane < SB_OUT / 32 ? L.bmc[lane].x : 0u;
    int32_t tot2;
    const int32_t before = wave_excl_scan32((int32_t)__builtin_popcount(bits), &tot2);
    if (lane < SB_OUT / 32) L.bmc[lane].y = (uint32_t)before;
    if (fdefer) {  // the deferred far copies' bytes (their loads overlapped the tables)
      const int64_t o = dpos + out_rel;
#pragma unroll
      for (int i2 = 0; i2 < 16; i2++) {
        if (i2 >= (int)len) break;
        const int bi = fsh + i2;
        ring[(o + i2) & RING_MASK] = (uint8_t)((bi < 8 ? fq0 >> (8 * bi) : fq1 >> (8 * (bi - 8))) & 0xffu);
      }
    }
    wave_lds_sync();
    SNAP_T(4);
    // 5. every output byte by its own lane, 64 bytes per pass: a copy byte is
    // chased back to a literal, a prefilled far copy, a byte resolved by an
    // earlier pass (already in the history), or a byte before the batch
    for (int it = 0; it * 64 < T; it++) {
      const int j = lane + 64 * it;
      if (j < T) {
        int q = j;
        uint8_t b = 0;
        for (;;) {
          const uint2 e = L.bmc[q >> 5];
          const int k = (int)e.y + __builtin_popcount(e.x & (0xffffffffu >> (31 - (q & 31)))) - 1;
          SNAP_GUARD(k < 0 || k >= ntok, 3, k, q);
          const uint4 t = L.tok[k];
          const int r = q - (int)t.x;
          if (t.y >> 31) {
            SNAP_GUARD(t.z + r >= 528u, 4, t.z, r);
            b = winb[t.z + r];
            break;
          }
          if (t.y & 0x40000000u) {  // far copy, prefilled
            b = ring[(dpos + q) & RING_MASK];
            break;
          }
          const uint32_t tl = t.y & 0x3fffffffu, off = t.z;
          const int q2 = (int)t.x - (int)off + (int)(off >= tl ? (uint32_t)r : (uint32_t)r % off);
          if (q2 >= 0) {
            if (q2 < 64 * it) {  // resolved by an earlier pass
              b = ring[(dpos + q2) & RING_MASK];
              break;
            }
            q = q2;
            continue;
          }
          const int64_t p = dpos + q2;
          if (p >= near_lo) {
            b = ring[p & RING_MASK];
          } else {
            // rare: one byte of a copy that straddles the history edge or a
            // deferred literal
            uintptr_t from = (p >= 0 && p < F) ? (uintptr_t)(dst + p) : 0;
            bool payload = false;
            for (int k2 = 0; k2 < ndefer; k2++) {
              const int64_t kd = (int64_t)readlane64(def_dst, k2);
              const int64_t kl = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)def_len, k2);
              if (p >= kd && p < kd + kl) {
                const uint64_t ks = readlane64(def_src, k2);
                from = (uintptr_t)ks + (uintptr_t)(p - kd);
                payload = true;
              }
            }
            PQ_CHK(from && payload && (from < (uintptr_t)src || from >= (uintptr_t)(src + slen)), 11, from, p, from = 0);
            PQ_CHK(from && !payload && (from < (uintptr_t)dst || from >= (uintptr_t)(dst + dl)), 12, from, p, from = 0);
            if (from) {
              if (payload) {
                b = *(const uint8_t *)from;
              } else {
                const uint32_t word = far_ld((const uint32_t *)(from & ~(uintptr_t)3));
                b = (uint8_t)(word >> ((from & 3) * 8));
              }
            }
          }
          break;
        }
        ring[(dpos + j) & RING_MASK] = b;
      }
      wave_lds_sync();
    }
    }  // (per-byte path)
    wave_lds_sync();
    SNAP_T(5);
    // 6. to HBM: bytes up to the next 16-byte boundary (F is unaligned after
    // a long literal), then whole 16-byte chunks up to floor16(dpos + T)
    // (dst is 16-byte aligned)
    const int64_t end = dpos + T;
    int64_t a16 = (F + 15) & ~(int64_t)15;
    if (a16 > end) a16 = end;
    SNAP_GUARD(a16 - F > 64 || a16 > dl, 1, a16, F);
    if (lane < a16 - F) dst[F + lane] = ring[(F + lane) & RING_MASK];
    F = a16;
    const int64_t e16 = end & ~(int64_t)15;
    if ((F & 15) == 0)
      for (int64_t c = F + 16 * (int64_t)lane; c < e16; c += 1024) {
      const uint4 v = *(const uint4 *)(ring + (c & RING_MASK));
      *(uint4 *)(dst + c) = v;
    }
    SNAP_GUARD(e16 > dl, 5, e16, dl);
    if (e16 > F) F = e16;
    SNAP_T(6);
  }
#ifdef PQ_SNAP_STAMPS
  if (lane == 0) L.acc[7] += 1;
#endif
  dpos += total;
  s += cur - sh;
  return true;
}

// Work modes of k_snappy.  A page whose body is longer than SNAP_SEG is cut at
// every SNAP_SEG-th output byte: Snappy encoders compress 64 KiB blocks
// independently (google snappy's kBlockSize, golang/snappy's maxBlockSize),
// so a token starts there and no copy reaches back across it.  k_snappy_walk
// finds those tokens; each segment is then its own work item.  A stream
// without that structure (or a corrupt one) falls back to the serial
// one-wave-per-page decode (SNAP_FALLBACK), which is exact for any stream.
constexpr int64_t SNAP_SEG = 65536;
enum { SNAP_ITEMS = 0, SNAP_FALLBACK = 1 };

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PQ_SNAPPY_WPE))) void k_snappy(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t ring_all[SNAPPY_WAVES][RING];
  __shared__ SnapLds sl_all[SNAPPY_WAVES];
  __shared__ __attribute__((aligned(4))) uint8_t snap_lut[SNAP_LUT];
  snappy_lut_init(snap_lut, (int)threadIdx.x);  // (256 threads: one tag each)
  __syncthreads();
  const int lane = lane_id();
  const int wv = (int)ufirst(threadIdx.x >> 6);  // wave-uniform (keeps per-wave state in SGPRs)
  const int wi = blockIdx.x * SNAPPY_WAVES + wv;
  if (MODE == SNAP_ITEMS && blockIdx.x == 0 && threadIdx.x == 0) a.copy_cnt[(a.epoch + 1) & 1] = 0;  // the next decode's list
  int gi, seg_k = 0;
  bool seg = false;
  if (MODE == SNAP_FALLBACK) {
    if (wi >= a.nwalk) return;
    gi = ufirst(a.walk[wi]);
    if (__hip_atomic_load(&a.seg_flag[gi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 1u) return;
  } else {
    if (wi >= a.nitems) return;
    const int2 it = a.sitems[wi];
    gi = ufirst(it.x);
    seg_k = ufirst(it.y);
    seg = a.seg_base[gi + 1] - a.seg_base[gi] > 1;
    // written by k_snappy_walk in the previous launch: read at device scope
    if (seg && __hip_atomic_load(&a.seg_flag[gi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return;
  }
  const int page = ufirst(a.list[gi]);
  const PageDesc d = a.pages[page];
  if (!seg && a.max_jobs > 0 && lane == 0) a.njobs[gi] = 0u;  // no deferred jobs unless written below
  if (page_status(a.status, page) < make_status(ST_DECOMPRESS, 0)) return;
  uint8_t *ring = ring_all[wv];
  SnapLds &L = sl_all[wv];
#ifdef PQ_SNAP_STAMPS
  if (lane < 8) L.acc[lane] = 0;
  const uint64_t t_page0 = __builtin_amdgcn_s_memtime();
#endif

  const int64_t lsize = d.kind == PAGE_V2 ? (int64_t)d.v2_rep_len + d.v2_def_len : 0;
  const uint8_t *src = a.in + d.src + lsize;
  const int64_t slen = d.comp_len;
  uint8_t *dst = a.stage + d.body;
  const int64_t expect = d.body_len;
  PQ_CHK(a.in_end && (src < a.in || src + slen > a.in_end), 13, (uintptr_t)src, slen, return);
  PQ_CHK(a.stage_end && (dst < a.stage || dst + expect > a.stage_end), 14, (uintptr_t)dst, expect, return);

  Win W;
  W.reset();
  int64_t s = 0, seg_lo = 0, dl;
  bool write;
  if (seg) {
    // k_snappy_walk checked the preamble (decoded length == page size) and
    // found the segment's first token
    s = __hip_atomic_load(&a.segs[a.seg_base[gi] + seg_k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s = (int64_t)ufirst64(s);
    seg_lo = (int64_t)seg_k * SNAP_SEG;
    dl = min(seg_lo + SNAP_SEG, expect);
    write = true;
  } else {
    // decodedLen: binary.Uvarint over the block (n <= 0 or > 0xffffffff -> ErrCorrupt)
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
    write = dlen == (uint64_t)expect;
    dl = (int64_t)dlen;
    // a block that is exactly one literal is its own content: leave it in place
    if (write && lane == 0) a.info[page].alias1 = 0;
    // (a dictionary page only when 8-byte aligned — L1/L2 gathers read aligned
    // entries — unless its chunk copies it into LDS, which funnel-shifts)
    if (write && dl > 0 && s < slen) {
      uint32_t tag = W.byte_at(src + s);
      if ((tag & 3) == 0) {
        uint32_t x = tag >> 2;
        int64_t hs = 1;
        bool ok = true;
        if (x >= 60) {
          int extra = (int)x - 59;
          hs = 1 + extra;
          if (s + hs > slen) ok = false;
          else {
            x = 0;
            for (int k = 0; k < extra; k++) x |= W.byte_at(src + s + 1 + k) << (8 * k);
          }
        }
        // (never for a page whose k_expand records the host wrote: they read
        // staging, so the block must be staged)
        if (ok && (int64_t)x + 1 == dl && s + hs + dl == slen && !d.srec &&
            (d.kind != PAGE_DICT || d.alias_any || ((d.src + lsize + s + hs) & 7) == 0)) {
          if (lane == 0) a.info[page].alias1 = 1 + (int64_t)(d.src + lsize + s + hs);
          return;
        }
      }
    }
  }
  int64_t dpos = seg_lo;
  int64_t F = seg_lo;  // staged output below F is in HBM; [F, dpos) only in the history
  uint32_t err = E_OK;
  int ndefer = 0;                      // deferred literals: lane k holds entry k
  const uint8_t *pend_src = nullptr;   // last deferred literal whose tail is not yet in the history
  int64_t pend_dpos = 0, pend_len = 0;
  int64_t def_dst = 0, def_len = 0;
  uint64_t def_src = 0;
  int64_t pf_s = -1;  // stream position of the window prefetched into pg0..pg2
  int64_t pf_F = 0;   // staged output flushed when that prefetch was issued
  uint32_t pg0 = 0, pg1 = 0, pg2 = 0;
  while (s < slen && (!seg || dpos < dl)) {
    const uint32_t tag = pf_s == s ? (__builtin_amdgcn_readlane(pg0, 0) >> (8 * ((uintptr_t)(src + s) & 3))) & 0xffu
                                   : W.byte_at(src + s);
    if ((tag & 3) != 0 || (tag >> 2) < 60) {
      // ---- short tokens (copies, literals <= 60 bytes): one batch of up to
      // SB_TOK tokens / SB_OUT output bytes per pass (snappy_batch)
      if (!snappy_batch(L, ring, lds_addr(snap_lut), src, slen, dst, dl, seg_lo, write, s, dpos, F, err, pend_src,
                        pend_dpos, pend_len, ndefer, def_dst, def_len, def_src, lane, a.in_end, pf_s, pf_F, pg0, pg1, pg2))
        break;
      continue;
    }
    // ---- long literal (tag >= 60 << 2): whole-wave copy or deferred to k_copy
    if (write && F < dpos) {  // bytes of the last batch still only in the history
      SNAP_GUARD(dpos - F > 64, 6, dpos, F);
      if (lane < dpos - F) dst[F + lane] = ring[(F + lane) & RING_MASK];
      F = dpos;
    }
    int64_t length;
    {
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
        bool deferred = false;
        if (!seg && length >= BIG_LITERAL && ndefer < MAX_DEFER && a.max_jobs > 0) {
          // deterministic slot in this page's region (sized by the host: body_len / BIG_LITERAL)
          const uint32_t slot = (uint32_t)(a.job_base[gi] + ndefer);
          const uint32_t region_end = (gi + 1 < a.nlist) ? (uint32_t)a.job_base[gi + 1] : a.max_jobs;
          if (slot < region_end) {
            if (lane == 0) a.jobs[slot] = CopyJob{src + s, dst + dpos, length};
            // remember it: far copies that land inside read the literal from the payload
            if (lane == ndefer) {
              def_dst = dpos;
              def_len = length;
              def_src = (uint64_t)(uintptr_t)(src + s);
            }
            ndefer++;
            pend_src = src + s;  // history filled lazily, if a copy follows
            pend_dpos = dpos;
            pend_len = length;
            deferred = true;
          }
        }
        if (!deferred) {
          if (pend_len) {  // history must hold the deferred literal's tail before newer bytes land
            ring_fill(pend_src, pend_dpos, pend_len, ring, lane);
            pend_len = 0;
          }
          PQ_CHK(dpos + length > dl || s + length > slen, 15, dpos + length, s + length, return);
          copy_literal(src + s, dst, dpos, length, ring, lane);
        }
      }
      dpos += length;
      s += length;
      if (write && pend_len == length && pend_dpos + length == dpos) {
        // speculative skip: an incompressible region is a train of identical
        // maximal literals (same tag bytes, same length); lane k checks the
        // k-th next token and the matching prefix is deferred in one step
        const int64_t hs = (int64_t)((tag >> 2) < 60 ? 1 : 1 + (int)(tag >> 2) - 59);
        const int64_t stride = hs + length;
        const int64_t cs = s + (int64_t)lane * stride;  // candidate tag position
        const uint32_t region_end = (gi + 1 < a.nlist) ? (uint32_t)a.job_base[gi + 1] : a.max_jobs;
        bool ok = ndefer + lane < MAX_DEFER && (uint32_t)(a.job_base[gi] + ndefer + lane) < region_end &&
                  cs + stride <= slen && dpos + (int64_t)(lane + 1) * length <= dl;
        if (ok) {
          const uint8_t *t0 = src + s - stride;  // the accepted token's tag
          for (int q = 0; q < hs; q++) ok &= src[cs + q] == t0[q];
        }
        const uint64_t okm = ballot(ok);
        const int m = ~okm ? (int)__builtin_ctzll(~okm) : 64;
        if (m > 0) {
          if (lane < m) {
            a.jobs[a.job_base[gi] + ndefer + lane] = CopyJob{src + cs + hs, dst + dpos + (int64_t)lane * length, length};
          }
          // deferred-literal table: lane ndefer + k holds candidate k
          const int k = lane - ndefer;
          if (k >= 0 && k < m) {
            def_dst = dpos + (int64_t)k * length;
            def_len = length;
            def_src = (uint64_t)(uintptr_t)(src + s + (int64_t)k * stride + hs);
          }
          ndefer += m;
          pend_src = src + s + (int64_t)(m - 1) * stride + hs;
          pend_dpos = dpos + (int64_t)(m - 1) * length;
          pend_len = length;
          dpos += (int64_t)m * length;
          s += (int64_t)m * stride;
        }
      }
      if (write) F = dpos;
      continue;
    }
  }
  if (err == E_OK && dpos != dl) err = E_SNAPPY;
  if (err == E_OK && write)
    for (int64_t p = F + lane; p < dl; p += 64) dst[p] = ring[p & RING_MASK];
  if (err == E_OK && !write) err = E_SIZE;  // compress.go:117-119
  if (seg) {
    // the last segment must end the stream exactly (decode_other.go:16-99
    // rejects tokens or bytes after the decoded length)
    if (err == E_OK && seg_k == a.seg_base[gi + 1] - a.seg_base[gi] - 1 && s != slen) err = E_SNAPPY;
    // a segment that does not decode on its own: the page is decoded again
    // serially (which also finds the exact error of a corrupt stream)
    if (err && lane == 0) atomicMax(&a.seg_flag[gi], 1u);
    err = E_OK;
  }
  if (!seg && a.max_jobs > 0 && lane == 0) a.njobs[gi] = err ? 0u : (uint32_t)ndefer;
  if (!err && ndefer > 0) {  // register the page's deferred literals in the compact list
    uint32_t base = 0;
    if (lane == 0) base = atomicAdd(&a.copy_cnt[a.epoch & 1], (uint32_t)ndefer);
    base = __builtin_amdgcn_readfirstlane(base);
    if (lane < ndefer) a.copy_idx[base + lane] = a.job_base[gi] + lane;
  }
  if (err) set_status(a.status, page, ST_DECOMPRESS, err);
#ifdef PQ_SNAP_STAMPS
  // per page (segments add up): phase cycles and batches; wave lifetimes
  if (a.dbg2 && lane < 8) atomicAdd((unsigned long long *)&a.dbg2[(size_t)page * 8 + lane], (unsigned long long)L.acc[lane]);
  if (a.dbg && lane == 0) {
    atomicAdd((unsigned long long *)&a.dbg[(size_t)page * 4 + 0], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_page0));
    atomicMax((unsigned long long *)&a.dbg[(size_t)page * 4 + 1], (unsigned long long)(__builtin_amdgcn_s_memtime() - t_page0));
    a.dbg[(size_t)page * 4 + 2] = (uint64_t)expect;
    a.dbg[(size_t)page * 4 + 3] = (uint64_t)slen;
  }
#endif
}

// ---------------------------------------------------------------------------
// k_snappy_walk: wave per page longer than SNAP_SEG.  Checks the preamble,
// detects a single-literal page (aliased in place, as k_snappy does), and
// finds the stream offset of the token that starts at each SNAP_SEG-th output
// byte.  seg_flag: 0 = segments found, 1 = serial fallback (no token at a
// boundary, a decoded length that differs from the page header, a stream
// that ends early), 2 = nothing to decode.
//
// The token chain is walked lane-parallel, WALK_CHUNK compressed bytes at a
// time, staged in LDS by LDS-DMA.  Lane l owns region [R l, R l + R) (WALK_R) and
// walks WALK_K chains from its first WALK_K bytes, which gives the exact exit
// and output count for every entry a stream of short tokens can have (a
// single speculative start phase-locks on periodic data such as a dictionary
// of increasing integers); pass 1 also marks every token its chains visit
// (merge table).  The regions the true chain visits are found by pointer
// jumping over states (region, entry offset 0 / 1 / later) — a scalar hop
// loop cost ~400 cycles a hop; a lane entered further in (a literal spanning
// its region start) walks from its true entry until it meets a marked token,
// and if its exit differs from the guess the path is found again.  Output positions are an exclusive scan; a lane holding a
// boundary walks its region once more to find the token that starts there.
// ---------------------------------------------------------------------------
// region bytes per lane (speculative chains converge well inside); 65 dwords,
// not 64: the lanes' reads start in 32 different LDS banks (a 256-byte stride
// put all 32 lanes of a group on one bank: 32-way conflicts on every read)
constexpr int WALK_R = 260;
constexpr int WALK_K = 2;                    // exact chains per region (entry offsets 0 .. WALK_K - 1)
static_assert(WALK_K == 2 && 64 * WALK_R * 2 % 16 == 0, "merge table: one chain bit, uint4 fill");
constexpr int WALK_CHUNK = 64 * WALK_R;      // compressed bytes per step
// staged by LDS-DMA in 1 KiB pieces: alignment skew, the chunk, token lookahead
constexpr int WALK_STAGE = (WALK_CHUNK + 32 + 1023) / 1024 * 1024;

// size in the stream and output length of the token at LDS byte p of the
// (16-byte aligned) staging buffer w, branch-free: three dword reads and
// selects, no exec-mask changes, so the walks of several chains interleave
__device__ __forceinline__ void walk_token(const uint32_t *w, int p, int32_t &adv, int32_t &len) {
  const int q = p >> 2, sb = p & 3;
  const uint32_t d0 = w[q], d1 = w[q + 1], d2 = w[q + 2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(d1, d0, sb);  // bytes p .. p + 3
  const uint32_t hi = __builtin_amdgcn_alignbyte(d2, d1, sb);  // bytes p + 4 .. p + 7
  const uint32_t tag = lo & 0xff, t = tag & 3, x = tag >> 2;
  // short literal x + 1 bytes; copy-1 4 + (x & 7) from 2 bytes; copy-2 / -4: x + 1 from 3 / 5
  int32_t l = (int32_t)(t == 1 ? 4 + (x & 7) : x + 1);
  int32_t z = (int32_t)(t == 0 ? x + 2 : t == 1 ? 2 : t == 2 ? 3 : 5);
  // long literal: 1 .. 4 little-endian length bytes follow the tag; lengths
  // past 2^30 do not fit a page (page sizes are int32): clamp, the walk then
  // leaves the page and the segments report it
  const int extra = (int)x - 59;
  const uint32_t lb = (lo >> 8) | (hi << 24);
  const uint32_t v = extra >= 4 ? lb : lb & ((1u << (8 * (extra & 3))) - 1u);
  const int32_t ll = v >= 0x3fffffffu ? 0x3fffffff : (int32_t)v + 1;
  const bool lng = t == 0 && x >= 60;
  len = lng ? ll : l;
  adv = lng ? 1 + extra + ll : z;
}

// the state after exit position x: region x / WALK_R entered at offset 0, 1
// or later (2); 192 past the chunk
__device__ __forceinline__ int walk_state(int32_t x, int cend) {
  if (x >= cend) return 192;
  const int n = x / WALK_R;
  return 3 * n + min(x - WALK_R * n, 2);
}

__global__ __launch_bounds__(64) void k_snappy_walk(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t wbuf[WALK_STAGE];
  // merge table, per region position: 0xffff, or the pass-1 chain k that
  // visits the token starting there (bit 14) and its output before it
  __shared__ __attribute__((aligned(16))) uint16_t wtab[64 * WALK_R];
  __shared__ uint8_t pjt[2][256];  // pass 2: state graph levels (ping-pong)
  __shared__ int32_t xtab[192];    // exit position per state
  __shared__ int32_t etab[64];     // entry position per region (-1: not on the chain)
  // a few serial waves sharing the GPU with k_snappy's whole pages (side
  // stream): their segments wait on them, so they win issue arbitration
  __builtin_amdgcn_s_setprio(3);
  const int lane = lane_id();
  const int wi = blockIdx.x;
  if (wi >= a.nwalk) return;
#ifdef PQ_SNAP_STAMPS
  // diagnostic build: per page, cycles of the whole walk, 100 MHz ticks, staging +
  // pass 1, pass 3, boundaries, path rounds, pass-1 steps, path hops
  uint64_t wst[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t wt0 = __builtin_amdgcn_s_memtime(), wrt0 = __builtin_amdgcn_s_memrealtime();
  uint64_t wtp = wt0;
#define WALK_T(i)                                     \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    wst[i] += t_ - wtp;                               \
    wtp = t_;                                         \
  } while (0)
#define WALK_N(i, v) (wst[i] += (v))
#else
#define WALK_T(i) \
  do {            \
  } while (0)
#define WALK_N(i, v) ((void)0)
#endif
  const int gi = ufirst(a.walk[wi]);
  const int page = ufirst(a.list[gi]);
  const PageDesc d = a.pages[page];
  const int32_t sb = a.seg_base[gi], nseg = a.seg_base[gi + 1] - sb;
  if (a.max_jobs > 0 && lane == 0) a.njobs[gi] = 0u;  // the fallback writes its own
  uint32_t flag = 1;
  if (page_status(a.status, page) < make_status(ST_DECOMPRESS, 0)) {
    flag = 2;
  } else {
    const int64_t lsize = d.kind == PAGE_V2 ? (int64_t)d.v2_rep_len + d.v2_def_len : 0;
    const uint8_t *src = a.in + d.src + lsize;
    const int64_t slen = d.comp_len, expect = d.body_len;
    Win W;
    W.reset();
    int64_t s = 0;
    uint64_t dlen = 0;
    bool ok = false;
    for (int i = 0, sh = 0; s < slen; i++, sh += 7) {
      const uint32_t b = W.byte_at(src + s);
      s++;
      if (b < 0x80) {
        ok = !(i > 9 || (i == 9 && b > 1));
        dlen |= (uint64_t)b << (sh & 63);
        break;
      }
      if (sh < 64) dlen |= (uint64_t)(b & 0x7f) << sh;
    }
    if (lane == 0) a.info[page].alias1 = 0;
    if (ok && dlen == (uint64_t)expect && s < slen) {
      // one literal covering the page: k_snappy's alias (no copy)
      const uint32_t tag = W.byte_at(src + s);
      if ((tag & 3) == 0) {
        uint32_t x = tag >> 2;
        int64_t hs = 1;
        bool lok = true;
        if (x >= 60) {
          const int extra = (int)x - 59;
          hs = 1 + extra;
          if (s + hs > slen) lok = false;
          else {
            x = 0;
            for (int k = 0; k < extra; k++) x |= W.byte_at(src + s + 1 + k) << (8 * k);
          }
        }
        if (lok && (int64_t)x + 1 == expect && s + hs + expect == slen && !d.srec &&
            (d.kind != PAGE_DICT || d.alias_any || ((d.src + lsize + s + hs) & 7) == 0)) {
          if (lane == 0) a.info[page].alias1 = 1 + (int64_t)(d.src + lsize + s + hs);
          flag = 2;
        }
      }
      if (flag != 2) {
        if (lane == 0) a.segs[sb] = s;
        int64_t out = 0, nb = SNAP_SEG;  // output before s; next boundary
        int32_t kb = 1;
        bool fail = false;

        while (kb < nseg && !fail) {
          if (s >= slen) {  // the stream ended before the last boundary
            fail = true;
            break;
          }
          if (out == nb) {  // a boundary exactly at the chunk base
            if (lane == 0) a.segs[sb + kb] = s;
            kb++;
            nb += SNAP_SEG;
            continue;
          }
          {
            // a long literal at s: stepped over from its header, no staging
            // (an incompressible block is one literal); one that spans a
            // boundary means no segments
            const uint32_t tag = W.byte_at(src + s);
            if ((tag & 3) == 0 && (tag >> 2) >= 60) {
              const int extra = (int)(tag >> 2) - 59;
              if (s + 1 + extra > slen) {
                fail = true;
                break;
              }
              uint32_t v = 0;
              for (int k = 0; k < extra; k++) v |= W.byte_at(src + s + 1 + k) << (8 * k);
              const int64_t len = (int64_t)v + 1;
              if (len >= 1024) {
                if (out + len > nb || s + 1 + extra + len > slen) {
                  fail = true;
                  break;
                }
                out += len;
                s += 1 + extra + len;
                continue;
              }
            }
          }
          // stage [s, s + WALK_CHUNK + lookahead) by LDS-DMA, 1 KiB a piece (lane
          // l's 16 bytes at +16 l); readable slack follows every chunk (kPad)
          const uintptr_t A = (uintptr_t)(src + s) & ~(uintptr_t)15;
          const uintptr_t lim = (uintptr_t)a.in_end;  // never past the input allocation (its pad included)
#pragma unroll
          for (int off = 0; off < WALK_STAGE; off += 1024)
            if (A + off + 16 * (uintptr_t)lane + 16 <= lim)
              __builtin_amdgcn_global_load_lds((const void *)(A + off + 16 * (uintptr_t)lane),
                                               (__attribute__((address_space(3))) void *)(wbuf + off), 16, 0, 0);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          wave_lds_sync();
          const uint32_t *wb = (const uint32_t *)wbuf;
          const int boff = (int)((uintptr_t)(src + s) - A);  // LDS byte of stream position s
          // positions relative to s; the chunk holds regions of lanes below
          // nreg (its end is the page end when that comes first)
          const int64_t rest = slen - s;
          const int cend = (int)min<int64_t>(rest, (int64_t)WALK_CHUNK);
          const int r0 = WALK_R * lane, r1 = min(r0 + WALK_R, cend);
          // pass 1: WALK_K chains per lane, from each of the first WALK_K bytes
          // of my region, walked together (independent LDS reads in flight):
          // exact exits and output counts for entries that close to the region
          // start — every entry of a stream of short tokens (copies, literals
          // under WALK_K bytes), where speculation could phase-lock on
          // periodic data (e.g. a dictionary of increasing integers)
          int32_t yk[WALK_K], ok[WALK_K];
#pragma unroll
          for (int k = 0; k < WALK_K; k++) {
            yk[k] = r0 + k;
            ok[k] = 0;
          }
          uint16_t *tab = wtab + WALK_R * lane - r0;  // tab[r], r0 <= r < r1
          for (int i = lane; i < 64 * WALK_R * 2 / 16; i += 64) ((uint4 *)wtab)[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
          wave_lds_sync();
          if (r0 < cend) {
            for (;;) {
              bool more = false;
#pragma unroll
              for (int k = 0; k < WALK_K; k++) {
                // predicated, not branched: finished chains re-read their exit
                const bool act = yk[k] < r1;
                int32_t adv, len;
                if (act) tab[yk[k]] = (uint16_t)((k << 14) | ok[k]);
                walk_token(wb, boff + min(yk[k], cend), adv, len);
                yk[k] = act ? yk[k] + adv : yk[k];
                ok[k] += act ? len : 0;
                more |= yk[k] < r1;
              }
              WALK_N(6, 1);
              if (!ballot(more)) break;
            }
          }
          WALK_T(2);
          // a later entry (inside a literal that spans the region start) uses
          // the last chain as a guess, checked below
          int32_t xg = yk[WALK_K - 1];
          int32_t entry = -1, tx = 0, tout = 0;  // my true entry, exit, output bytes
          int32_t guard = 0;
          for (;;) {
            // pass 2: the true chain's regions.  State 3 l + c = region l
            // entered at offset c (0, 1: exact chains; 2: any later entry, the
            // guess), 192 = past the chunk.  Pointer jumping over the state
            // graph: lane m lands on the m-th state of the chain from state 0
            // (levels 2^j applied for the bits of m, as computed; they commute)
            xtab[3 * lane + 0] = yk[0];
            xtab[3 * lane + 1] = yk[1];
            xtab[3 * lane + 2] = xg;
            pjt[0][3 * lane + 0] = walk_state(yk[0], cend);
            pjt[0][3 * lane + 1] = walk_state(yk[1], cend);
            pjt[0][3 * lane + 2] = walk_state(xg, cend);
            pjt[0][192 + lane] = 192;
            pjt[1][192 + lane] = 192;
            etab[lane] = -1;
            wave_lds_sync();
            int sm = 0;
#pragma unroll
            for (int j = 0; j < 6; j++) {
              const uint8_t *P = pjt[j & 1];
              if ((lane >> j) & 1) sm = P[sm];
              if (j < 5) {
                uint8_t *Q = pjt[(j + 1) & 1];
                const int a0 = P[3 * lane], a1 = P[3 * lane + 1], a2 = P[3 * lane + 2];
                Q[3 * lane] = P[a0];
                Q[3 * lane + 1] = P[a1];
                Q[3 * lane + 2] = P[a2];
              }
              wave_lds_sync();
            }
            // the entry of the m-th state is the exit of the (m - 1)-th: give
            // it to the region's lane
            const int sp = __shfl_up(sm, 1);
            if (sm != 192) etab[sm / 3] = lane == 0 ? 0 : xtab[sp];
            wave_lds_sync();
            entry = etab[lane];
            const int c = entry < 0 ? 0 : min(entry - r0, 2);
            const bool exact = entry >= 0 && c < 2;
            if (exact) {
              tx = c ? yk[1] : yk[0];
              tout = c ? ok[1] : ok[0];
            }
            WALK_T(7);
            // pass 3: path lanes with a guessed exit walk from their true entry
            // until they meet a pass-1 chain (merge table)
            bool bad = false;
            if (entry >= 0 && !exact) {
              int32_t adv, len;
              tout = 0;
              tx = entry;
              while (tx < r1) {
                const uint32_t m = tab[tx];
                if (m != 0xffffu) {
                  const bool k1 = (m >> 14) & 1;
                  tout += (k1 ? ok[WALK_K - 1] : ok[0]) - (int32_t)(m & 0x3fff);
                  tx = k1 ? yk[WALK_K - 1] : yk[0];
                  break;
                }
                walk_token(wb, boff + tx, adv, len);
                tx += adv;
                tout += len;
              }
              bad = tx != xg;
            }
            const uint64_t badm = ballot(bad);
            WALK_N(5, 1);
            if (!badm || ++guard > 64) {
              if (badm) fail = true;
              break;
            }
            if (bad) xg = tx;  // correct the exits and retrace the path
            wave_lds_sync();   // the tables are rewritten
          }
          // the chain leaves the chunk from the one path lane whose exit is past it
          const uint64_t lastm = ballot(entry >= 0 && tx >= cend);
          const int last = lastm ? (int)__builtin_ctzll(lastm) : 0;
          if (!lastm) fail = true;
          WALK_T(3);
          if (fail) break;
          // output positions of the path lanes' first tokens
          int32_t ctot;
          const int32_t ex = wave_excl_scan32(entry >= 0 ? tout : 0, &ctot);
          const int64_t o0 = out + ex;
          // lanes holding boundaries find the token that starts there
          bool bfail = false;
          if (entry >= 0 && o0 + tout > nb) {
            int64_t bnext = nb;
            while (bnext < o0) bnext += SNAP_SEG;  // the first boundary at or after my first token
            int64_t o = o0;
            int32_t r = entry, adv, len;
            while (r < r1 && bnext < o0 + tout) {
              walk_token(wb, boff + r, adv, len);
              if (o == bnext) {
                const int64_t k = bnext / SNAP_SEG;
                if (k < nseg) a.segs[sb + k] = s + r;
                bnext += SNAP_SEG;
              } else if (o < bnext && o + len > bnext) {
                bfail = true;  // a token spans the boundary
                break;
              }
              o += len;
              r += adv;
            }
          }
          WALK_T(4);
          if (ballot(bfail)) {
            fail = true;
            break;
          }
          out += ctot;
          while (nb < out) {  // boundaries passed inside this chunk
            nb += SNAP_SEG;
            kb++;
          }
          s += __builtin_amdgcn_readlane(tx, last);
          wave_lds_sync();
        }
        flag = (!fail && kb >= nseg) ? 0u : 1u;
      }
    }
  }
  if (lane == 0) a.seg_flag[gi] = flag;
#ifdef PQ_SNAP_STAMPS
  wst[0] = __builtin_amdgcn_s_memtime() - wt0;
  wst[1] = __builtin_amdgcn_s_memrealtime() - wrt0;
  if (a.dbg3 && lane == 0)  // after the 256 run-walk stamps
    for (int i = 0; i < 8; i++) a.dbg3[256 + (size_t)page * 8 + i] = wst[i];
#endif
#undef WALK_T
#undef WALK_N
}

// ===========================================================================
// K1b: long literals deferred by k_snappy, copied by every workgroup
// ===========================================================================
constexpr int COPY_TILE = 4096;   // bytes per workgroup instruction (256 lanes x 16 B)
constexpr int COPY_CHUNK = 4;     // tiles per work item (16 KiB)
constexpr int COPY_ITEMS = 4;     // work items per job slot and pass (64 KiB: a google/Go snappy literal)

// Work item i = (job slot i / COPY_ITEMS, chunk i % COPY_ITEMS), grid-strided;
// a job longer than COPY_ITEMS chunks is covered in passes.  Every load of a
// chunk is issued before its stores.
__device__ __forceinline__ void copy_items(const KArgs &a, uint32_t blk, uint32_t nblk) {
  // the count, index and job records were written by k_snappy in the previous
  // launch: read them with vector loads at device scope (a uniform plain load
  // becomes a scalar-cache load, which can return lines of an earlier decode
  // that used the same addresses)
  // the host plan's literal copies (literal-train pages) first, then the
  // deferred literals k_snappy registered
  const uint32_t nh = (uint32_t)a.nhjobs;
  const uint32_t items =
      (nh + __hip_atomic_load(&a.copy_cnt[a.epoch & 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) * COPY_ITEMS;
  for (uint32_t it = blk; it < items; it += nblk) {
    const uint32_t c = it % COPY_ITEMS;
    const uint32_t jn = it / COPY_ITEMS;
    CopyJob job;
    if (jn < nh) {
      const uint64_t *hw = (const uint64_t *)&a.hjobs[4 * (size_t)jn];
      job.src = a.in + __hip_atomic_load(&hw[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      job.dst = a.stage + __hip_atomic_load(&hw[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      job.len = (int64_t)__hip_atomic_load(&hw[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const uint32_t ji =
          (uint32_t)__hip_atomic_load(&a.copy_idx[jn - nh], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint64_t *jw = (const uint64_t *)&a.jobs[ji];
      job.src = (const uint8_t *)(uintptr_t)__hip_atomic_load(&jw[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      job.dst = (uint8_t *)(uintptr_t)__hip_atomic_load(&jw[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      job.len = (int64_t)__hip_atomic_load(&jw[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    PQ_CHK(a.in_end && (job.src < a.in || job.src + job.len > a.in_end || job.dst < a.stage ||
                        job.dst + job.len > a.stage_end || job.len < 0),
           20, (uintptr_t)job.src, job.len, return);
    const int t = threadIdx.x;
    const uintptr_t d0 = (uintptr_t)job.dst, d1 = d0 + (uintptr_t)job.len;
    const uintptr_t A = d0 & ~(uintptr_t)15;
    for (uintptr_t base = A + (uintptr_t)c * COPY_CHUNK * COPY_TILE; base < d1;
         base += (uintptr_t)COPY_ITEMS * COPY_CHUNK * COPY_TILE) {
      uint4 x[COPY_CHUNK];
      uint32_t x4[COPY_CHUNK];
#pragma unroll
      for (int k = 0; k < COPY_CHUNK; k++) {
        const uintptr_t u = base + (uintptr_t)k * COPY_TILE + (uintptr_t)t * 16;
        const bool whole = u >= d0 && u + 16 <= d1;
        const uintptr_t sp = (uintptr_t)job.src + (whole ? u - d0 : 0);
        const uintptr_t sa = sp & ~(uintptr_t)3;
        x[k] = make_uint4(gld32(sa), gld32(sa + 4), gld32(sa + 8), gld32(sa + 12));
        x4[k] = gld32(sa + 16);
      }
#pragma unroll
      for (int k = 0; k < COPY_CHUNK; k++) {
        const uintptr_t u = base + (uintptr_t)k * COPY_TILE + (uintptr_t)t * 16;
        if (u >= d1) continue;
        if (u >= d0 && u + 16 <= d1) {
          const uint32_t skew = (uint32_t)(((uintptr_t)job.src + (u - d0)) & 3);
          uint4 o;
          o.x = __builtin_amdgcn_alignbyte(x[k].y, x[k].x, skew);
          o.y = __builtin_amdgcn_alignbyte(x[k].z, x[k].y, skew);
          o.z = __builtin_amdgcn_alignbyte(x[k].w, x[k].z, skew);
          o.w = __builtin_amdgcn_alignbyte(x4[k], x[k].w, skew);
          gst128(u, o);
        } else {
          for (int b = 0; b < 16; b++) {
            const uintptr_t y = u + b;
            if (y >= d0 && y < d1) *(uint8_t *)y = job.src[y - d0];
          }
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_copy(KArgs a) { copy_items(a, blockIdx.x, gridDim.x); }

// ===========================================================================
// K1w: k_snappy_wg — Snappy (decode_other.go:14-101) by one 512-thread
// workgroup per work item (a whole page, or a 64 KiB segment of a long one),
// with the whole Snappy block window (64 KiB: the encoders' block size, so the
// reach of every copy they write) as history in LDS.  A copy never reads HBM:
// the decode reads the compressed bytes and writes the uncompressed ones
// once.  ~77 KiB of LDS, two workgroups per CU.  Per batch (at most UZ_POS
// compressed bytes, UZ_TOK tokens, UZ_OUT output bytes):
//  1. the batch's compressed bytes in LDS (loaded into registers while the
//     previous batch resolved);
//  2. the token chain by pointer jumping: J_0(p) = p + size of the token at
//     window position p, J_b+1 = J_b o J_b; thread t applies J_b for the set
//     bits b of t (and of t + UZ_T), so it lands on tokens t and t + UZ_T;
//  3. each thread decodes and checks its two tokens (the reference's checks:
//     header inside src, length <= remaining dst, 0 < offset <= d); workgroup
//     scans give their output offsets, cut the batch, and find each copy's
//     chain head: the first of the consecutive copies with its offset before
//     it (a run of overlapping copies — a repeated pattern — all read the
//     bytes just before the run's first copy: byte q of the run is byte
//     head - o + (q - head) mod o);
//  4. token table + output-start bitmap with per-word token counts (token m
//     writes count m + 1 into the words starting inside it);
//  5. every output byte resolved by a thread, one aligned history dword a
//     thread per pass of UZ_PASS bytes: a literal byte from the window, a
//     copy byte from the history, chased to its source when that is a byte of
//     the same pass;
//  6. whole 16-byte chunks from the history to HBM.
// Long literals (tag >= 60 << 2) are copied by the workgroup straight to HBM,
// their last 64 KiB into the history.  A source the pass may overwrite (an
// offset within UZ_PASS of 64 KiB) or older than the history is read back
// from the staged output.
// ===========================================================================
constexpr int UZ_T = 512;                         // threads
constexpr int UZ_W = UZ_T / 64;                   // waves
constexpr int UZ_HIST = 65536;                    // history (ring) bytes
constexpr uint32_t UZ_HMASK = UZ_HIST - 1;
constexpr int UZ_POS = 2048;                      // window positions parsed per batch
constexpr int UZ_STOP = UZ_POS;                   // the chain's end in the jump tables
constexpr int UZ_WIN_DW = (UZ_POS + 64 + 8) / 4;  // staged dwords: skew, positions, a short literal's payload
constexpr int UZ_TOK = 2 * UZ_T;                  // tokens per batch (two per thread)
constexpr int UZ_OUT = 8192;                      // output bytes per batch
constexpr int UZ_PASS = 2 * UZ_T;                 // output bytes resolved per pass (two a thread)
constexpr int UZ_ROUNDS = 10;                     // 2^10 = UZ_TOK
static_assert((1 << UZ_ROUNDS) == UZ_TOK && UZ_WIN_DW > UZ_T && UZ_WIN_DW <= 2 * UZ_T, "k_snappy_wg shapes");

struct UzLds {
  uint8_t hist[UZ_HIST];
  uint32_t win[UZ_WIN_DW + 2];
  union {
    uint16_t jt[2][UZ_POS + 8];  // J_b ping-pong; entry UZ_STOP = UZ_STOP
    uint2 tok[UZ_TOK];           // {out_rel | (len - 1) << 13 | head << 19 | literal << 31,
                                 //  literal: window position of its bytes / copy: offset}
  };
  uint2 bmc[UZ_OUT / 32];        // output-start bits, tokens starting before the word
  int32_t red[2 * UZ_W];         // per wave and token half: output bytes
  __attribute__((aligned(16))) int32_t last[2 * UZ_W][4];  // per wave and half: {last accepted token + 1, its end,
                                                          //  stream bytes after it}
  __attribute__((aligned(16))) uint32_t chn[2 * UZ_W][4];  // per wave and half: first / last token's copy offset
                                                          // (0: not a copy), the scan (lane 0 left out) at lane 63
  uint16_t src[UZ_PASS];         // per byte of the pass: 0x8000 | value, or the pass offset of its source
  uint32_t rflag[3];             // pointer-jumping rounds: any byte left (a slot per round mod 3)
  uint32_t flags;                // 1: a bad token, 2: a source the history may not hold
  uint32_t go;
};

// Output byte q of the batch: its value (0x8000 | value) when its source is
// a literal byte, a byte older than the pass (`base`: the pass's first batch
// offset; earlier bytes of the batch are in the history) or older than the
// batch; else the pass offset of its source byte (a byte of the same pass,
// resolved by pointer jumping).  A copy byte's source is found through its
// run's head: byte q of a run of copies of offset o starting at h is byte
// h - o + (q - h) mod o.  `safe_lo`: older positions the pass may overwrite,
// read back from the staged output.
__device__ __forceinline__ uint32_t uz_direct(const UzLds &U, const uint8_t *wb, int q, int base, int64_t dpos,
                                              int64_t safe_lo, const uint8_t *dst) {
  const uint2 e = U.bmc[q >> 5];
  const int kk = (int)e.y + __builtin_popcount(e.x & (0xffffffffu >> (31 - (q & 31)))) - 1;
  const uint2 t = U.tok[kk];
  const int o = (int)(t.x & 0x1fff);
  if (t.x >> 31) return 0x8000u | wb[t.y + (uint32_t)(q - o)];  // literal
  const int h = (int)((t.x >> 19) & 1023);
  const int oh = h == kk ? o : (int)(U.tok[h].x & 0x1fff);  // the run head's start
  const uint32_t off = t.y, r = (uint32_t)(q - oh);
  const int64_t q2 = (int64_t)oh - (int64_t)off + (int64_t)(r < off ? r : r % off);
  if (q2 >= base) return (uint32_t)(q2 - base);
  const int64_t p = dpos + q2;
  if (q2 >= 0 || p >= safe_lo) return 0x8000u | U.hist[(uint32_t)p & UZ_HMASK];
  const uintptr_t from = (uintptr_t)(dst + p);  // the staged output (flushed by earlier batches)
  const uint32_t w = __hip_atomic_load((const uint32_t *)(from & ~(uintptr_t)3), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return 0x8000u | ((w >> ((from & 3) * 8)) & 0xffu);
}

// Decode the short token at window position pos (its tag is not a long
// literal): output length, literal payload position or copy offset, bytes in
// the stream, and whether its header / payload lies past the block end.
__device__ __forceinline__ void uz_token(const UzLds &U, int sh, int pos, int64_t sabs, int64_t slen, uint32_t &len,
                                         uint32_t &x, bool &lit, bool &bad, int &adv) {
  const int b = sh + pos;
  const uint32_t w0 = U.win[b >> 2], w1 = U.win[(b >> 2) + 1], w2 = U.win[(b >> 2) + 2];
  const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, (uint32_t)b & 3);
  const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, (uint32_t)b & 3);
  const uint32_t tag = lo & 0xff;
  if ((tag & 3) == 0) {
    lit = true;
    len = (tag >> 2) + 1;
    x = (uint32_t)pos + 1;
    adv = 1 + (int)len;
    bad = sabs + 1 + (int64_t)len > slen;
    return;
  }
  lit = false;
  if ((tag & 3) == 1) {
    adv = 2;
    len = 4 + ((tag >> 2) & 7);
    x = ((tag & 0xe0) << 3) | ((lo >> 8) & 0xff);
  } else if ((tag & 3) == 2) {
    adv = 3;
    len = 1 + (tag >> 2);
    x = (lo >> 8) & 0xffff;
  } else {
    adv = 5;
    len = 1 + (tag >> 2);
    x = (lo >> 8) | (hi << 24);
  }
  bad = sabs + adv > slen;
}

// diagnostic build (-DPQ_SNAP_STAMPS, tools/diag_snappy.py): thread 0's
// shader cycles per step of a batch — 0 window, 1 chain, 2 decode + scans,
// 3 table, 4 long literals, 5 byte passes, 6 flush; 7 batches — per page
#ifdef PQ_SNAP_STAMPS
#define UZ_TS(i)                                                    \
  do {                                                              \
    if (tid == 0) {                                                 \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();             \
      if ((i) >= 0) uz_acc[(i) < 0 ? 0 : (i)] += t_ - uz_prev;      \
      uz_prev = t_;                                                 \
    }                                                               \
  } while (0)
#else
#define UZ_TS(i) \
  do {           \
  } while (0)
#endif

template <int MODE>
__global__ __launch_bounds__(UZ_T) __attribute__((amdgpu_waves_per_eu(4))) void k_snappy_wg(KArgs a) {
  __shared__ __attribute__((aligned(16))) UzLds U;
#ifdef PQ_SNAP_STAMPS
  uint64_t uz_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t uz_prev = __builtin_amdgcn_s_memtime();
  const uint64_t uz_t0 = uz_prev;
#endif
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int wv = (int)ufirst((uint32_t)tid >> 6);
  const int wi = blockIdx.x;
  if (MODE == SNAP_ITEMS && wi == 0 && tid == 0) a.copy_cnt[(a.epoch + 1) & 1] = 0;  // the next decode's list
  int gi, seg_k = 0;
  bool seg = false;
  if (MODE == SNAP_FALLBACK) {
    if (wi >= a.nwalk) return;
    gi = a.walk[wi];
  } else {
    if (wi >= a.nitems) return;
    const int2 it = a.sitems[wi];
    gi = it.x;
    seg_k = it.y;
    seg = a.seg_base[gi + 1] - a.seg_base[gi] > 1;
  }
  const int page = a.list[gi];
  // words that other launches write are read by one thread (block-uniform decision)
  if (tid == 0) {
    bool go = page_status(a.status, page) >= make_status(ST_DECOMPRESS, 0);
    if (MODE == SNAP_FALLBACK)
      go = go && __hip_atomic_load(&a.seg_flag[gi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u;
    else if (seg)
      go = go && __hip_atomic_load(&a.seg_flag[gi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
    U.go = go ? 1u : 0u;
    U.rflag[0] = U.rflag[1] = U.rflag[2] = 0u;
    if (!seg && a.max_jobs > 0) a.njobs[gi] = 0u;  // nothing deferred to k_copy
  }
  __syncthreads();
  if (!U.go) return;
  const PageDesc d = a.pages[page];
  const int64_t lsize = d.kind == PAGE_V2 ? (int64_t)d.v2_rep_len + d.v2_def_len : 0;
  const uint8_t *src = a.in + d.src + lsize;
  const int64_t slen = d.comp_len;
  uint8_t *dst = a.stage + d.body;
  const int64_t expect = d.body_len;
  PQ_CHK(a.in_end && (src < a.in || src + slen > a.in_end), 13, (uintptr_t)src, slen, return);
  PQ_CHK(a.stage_end && (dst < a.stage || dst + expect > a.stage_end), 14, (uintptr_t)dst, expect, return);

  int64_t s = 0, seg_lo = 0, dl;
  bool write;
  if (seg) {
    // k_snappy_walk checked the preamble and found the segment's first token
    s = (int64_t)__hip_atomic_load(&a.segs[a.seg_base[gi] + seg_k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s = ufirst64(s);
    seg_lo = (int64_t)seg_k * SNAP_SEG;
    dl = min(seg_lo + SNAP_SEG, expect);
    write = true;
  } else {
    // decodedLen: binary.Uvarint (n <= 0 or > 0xffffffff -> ErrCorrupt)
    uint64_t dlen = 0;
    bool ok = false;
    for (int i = 0, sh = 0; s < slen; i++, sh += 7) {
      const uint32_t b = src[s];
      s++;
      if (b < 0x80) {
        ok = !(i > 9 || (i == 9 && b > 1));
        dlen |= (uint64_t)b << (sh & 63);
        break;
      }
      if (sh < 64) dlen |= (uint64_t)(b & 0x7f) << sh;
    }
    if (!ok || dlen > 0xffffffffull) {
      if (tid == 0) atomicMin(&a.status[page], make_status(ST_DECOMPRESS, E_SNAPPY));
      return;
    }
    write = dlen == (uint64_t)expect;
    dl = (int64_t)dlen;
    if (write && tid == 0) a.info[page].alias1 = 0;
    // a block that is exactly one literal is its own content: left in place (a
    // dictionary page only when 8-byte aligned, as k_snappy; never a page whose
    // k_expand records the host wrote)
    if (write && dl > 0 && s < slen) {
      const uint32_t tag = src[s];
      if ((tag & 3) == 0) {
        uint32_t x = tag >> 2;
        int64_t hs = 1;
        bool ok1 = true;
        if (x >= 60) {
          const int extra = (int)x - 59;
          hs = 1 + extra;
          if (s + hs > slen) ok1 = false;
          else {
            x = 0;
            for (int k = 0; k < extra; k++) x |= (uint32_t)src[s + 1 + k] << (8 * k);
          }
        }
        if (ok1 && (int64_t)x + 1 == dl && s + hs + dl == slen && !d.srec &&
            (d.kind != PAGE_DICT || d.alias_any || ((d.src + lsize + s + hs) & 7) == 0)) {
          if (tid == 0) a.info[page].alias1 = 1 + (int64_t)(d.src + lsize + s + hs);
          return;
        }
      }
    }
  }

  int64_t dpos = seg_lo;
  int64_t F = seg_lo;  // output below F is in HBM; [F, dpos) only in the history
  uint32_t err = E_OK;
  int64_t pf_s = -1;   // stream position of the window prefetched into pw0 / pw1
  uint32_t pw0 = 0, pw1 = 0;
  uint32_t uz_round = 0;  // pointer-jumping rounds so far (rflag slot = round mod 3)
  while (s < slen && (!seg || dpos < dl)) {
    // ---- 1. the window: stream bytes [s, s + UZ_POS + 64) at win byte sh
    const uintptr_t abase = (uintptr_t)(src + s) & ~(uintptr_t)3;
    const int sh = (int)((uintptr_t)(src + s) & 3);
    PQ_CHK(a.in_end && abase + 4 * UZ_WIN_DW > (uintptr_t)a.in_end, 10, abase, a.in_end, err = E_SNAPPY; break);
    if (pf_s != s) {
      pw0 = gld32(abase + 4 * (uintptr_t)tid);
      pw1 = tid < UZ_WIN_DW - UZ_T ? gld32(abase + 4 * (uintptr_t)(UZ_T + tid)) : 0u;
    }
    U.win[tid] = pw0;
    if (tid < UZ_WIN_DW - UZ_T) U.win[UZ_T + tid] = pw1;
    if (tid < UZ_OUT / 32) U.bmc[tid] = make_uint2(0u, 0u);
    if (tid == 0) U.flags = 0u;
    UZ_TS(-1);
    __syncthreads();
    UZ_TS(0);
    const uint8_t *wb = (const uint8_t *)U.win + sh;  // wb[p]: stream byte s + p
    const int64_t lim64 = slen - s - 1;               // the last position inside the block
    const int lim = lim64 < UZ_POS - 1 ? (int)lim64 : UZ_POS - 1;
    const uint32_t tag0 = wb[0];
    if ((tag0 & 3) == 0 && (tag0 >> 2) >= 60) {
      // ---- a long literal: the workgroup copies it
      const int extra = (int)(tag0 >> 2) - 59;
      if (s + 1 + extra > slen) {
        err = E_SNAPPY;
        break;
      }
      uint64_t x = 0;
      for (int k = 0; k < extra; k++) x |= (uint64_t)wb[1 + k] << (8 * k);
      const int64_t len = (int64_t)x + 1;
      const int64_t hs = 1 + extra;
      if (len > dl - dpos || len > slen - s - hs) {
        err = E_SNAPPY;
        break;
      }
      if (write) {
        // the history's pending bytes, then the literal to HBM; its last
        // UZ_HIST bytes also into the history
        if (tid < dpos - F) dst[F + tid] = U.hist[(uint32_t)(F + tid) & UZ_HMASK];
        const uint8_t *ls = src + s + hs;
        uint8_t *D = dst + dpos;
        const int64_t hist_from = len - UZ_HIST;  // literal offsets >= this enter the history
        int64_t head = (int64_t)((16 - ((uintptr_t)D & 15)) & 15);
        if (head > len) head = len;
        if (tid < head) {
          const uint8_t b = ls[tid];
          D[tid] = b;
          if (tid >= hist_from) U.hist[(uint32_t)(dpos + tid) & UZ_HMASK] = b;
        }
        const int64_t nch = (len - head) >> 4;
        const uint8_t *S = ls + head;
        const uint32_t skew = (uint32_t)((uintptr_t)S & 3);
        const uintptr_t SA = (uintptr_t)S & ~(uintptr_t)3;
        for (int64_t c = tid; c < nch; c += UZ_T) {
          const uintptr_t sp = SA + 16 * (uintptr_t)c;
          const uint32_t x0 = gld32(sp), x1 = gld32(sp + 4), x2 = gld32(sp + 8), x3 = gld32(sp + 12), x4 = gld32(sp + 16);
          uint4 o;
          o.x = __builtin_amdgcn_alignbyte(x1, x0, skew);
          o.y = __builtin_amdgcn_alignbyte(x2, x1, skew);
          o.z = __builtin_amdgcn_alignbyte(x3, x2, skew);
          o.w = __builtin_amdgcn_alignbyte(x4, x3, skew);
          gst128((uintptr_t)(D + head + 16 * c), o);
          if (head + 16 * c >= hist_from) *(uint4 *)(U.hist + ((uint32_t)(dpos + head + 16 * c) & UZ_HMASK)) = o;
        }
        const int64_t done = head + nch * 16;
        if (tid < len - done) {
          const uint8_t b = ls[done + tid];
          D[done + tid] = b;
          if (done + tid >= hist_from) U.hist[(uint32_t)(dpos + done + tid) & UZ_HMASK] = b;
        }
        F = dpos + len;
      }
      dpos += len;
      s += hs + len;
      __syncthreads();  // the history's new bytes; the window's last readers
      UZ_TS(4);
      continue;
    }
    // ---- 2. J_0 for positions 4 tid .. 4 tid + 3, then the chain by pointer jumping
    uint16_t *ja = U.jt[0], *jb = U.jt[1];
    {
      uint32_t j4[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int p = 4 * tid + k;
        const uint32_t cls = snappy_tok_class(wb[p]);
        const int nx = p + (int)(cls & 0xff);
        j4[k] = (cls == 0 || p > lim || nx > UZ_POS) ? (uint32_t)UZ_STOP : (uint32_t)nx;
      }
      *(uint2 *)(ja + 4 * tid) = make_uint2(j4[0] | (j4[1] << 16), j4[2] | (j4[3] << 16));
      if (tid == 0) {
        ja[UZ_STOP] = UZ_STOP;
        jb[UZ_STOP] = UZ_STOP;
      }
    }
    __syncthreads();
    int pa = 0, pb = 0;  // the positions of tokens tid (A) and UZ_T + tid (B)
#pragma unroll 1
    for (int b = 0; b < UZ_ROUNDS; b++) {
      const int ha = ja[pa], hb = ja[pb];
      if (b < UZ_ROUNDS - 1) {
        const uint2 q = *(const uint2 *)(ja + 4 * tid);
        const uint32_t n0 = ja[q.x & 0xffff], n1 = ja[q.x >> 16], n2 = ja[q.y & 0xffff], n3 = ja[q.y >> 16];
        *(uint2 *)(jb + 4 * tid) = make_uint2(n0 | (n1 << 16), n2 | (n3 << 16));
      }
      if ((tid >> b) & 1) pa = ha;
      if (((tid + UZ_T) >> b) & 1) pb = hb;
      if (b < UZ_ROUNDS - 1) {
        __syncthreads();
        uint16_t *t = ja;
        ja = jb;
        jb = t;
        // the chain ends within 2^(b+1) tokens: the later tokens do not exist
        // and the earlier ones have taken every jump they need
        if (ja[0] == UZ_STOP) {
          if ((tid >> (b + 1)) != 0) pa = UZ_STOP;
          pb = UZ_STOP;
          break;
        }
      }
    }
    UZ_TS(1);
    // ---- 3. decode + check tokens A and B; output offsets and chain heads by workgroup scans
    const bool vA = pa <= lim && snappy_tok_class(wb[pa]) != 0;
    const bool vB = pb <= lim && snappy_tok_class(wb[pb]) != 0;
    uint32_t lenA = 0, xA = 0, lenB = 0, xB = 0;
    bool litA = false, litB = false, badA = false, badB = false;
    int advA = 0, advB = 0;
    if (vA) uz_token(U, sh, pa, s + pa, slen, lenA, xA, litA, badA, advA);
    if (vB) uz_token(U, sh, pb, s + pb, slen, lenB, xB, litB, badB, advB);
    const int32_t iA = (int32_t)wave_incl_dpp<false>(lenA), iB = (int32_t)wave_incl_dpp<false>(lenB);
    // chain heads: token m continues the copy run of m - 1 when both are copies
    // of one offset; the head of m is the last token <= m that does not, so
    // head + 1 is a max-scan of (head ? m + 1 : 0) over the token order.  In a
    // wave the scan leaves lane 0 out (whether it continues the previous wave's
    // last token is known after the barrier)
    const uint32_t keyA = vA && !litA ? xA : 0u, keyB = vB && !litB ? xB : 0u;
    const uint32_t kpA = dpp_mov<0x138>(keyA), kpB = dpp_mov<0x138>(keyB);  // wave_shr:1 (lane - 1)
    const int mA = tid, mB = UZ_T + tid;
    const uint32_t hA = wave_incl_dpp<true>(lane == 0 || (keyA != 0 && keyA == kpA) ? 0u : (uint32_t)mA + 1);
    const uint32_t hB = wave_incl_dpp<true>(lane == 0 || (keyB != 0 && keyB == kpB) ? 0u : (uint32_t)mB + 1);
    if (lane == 63) {
      U.red[wv] = iA;
      U.red[UZ_W + wv] = iB;
      U.chn[wv][1] = keyA;
      U.chn[wv][2] = hA;
      U.chn[UZ_W + wv][1] = keyB;
      U.chn[UZ_W + wv][2] = hB;
    }
    if (lane == 0) {
      U.chn[wv][0] = keyA;
      U.chn[UZ_W + wv][0] = keyB;
    }
    __syncthreads();  // (also: every jump-table read is done; the table below reuses the space)
    int32_t preA = 0, totA = 0, preB = 0;
#pragma unroll
    for (int w = 0; w < UZ_W; w++) {
      const int32_t ra = U.red[w], rb = U.red[UZ_W + w];
      totA += ra;
      preA += w < wv ? ra : 0;
      preB += w < wv ? rb : 0;
    }
    // heads across waves: the slots (waves) in token order, A then B; a slot's
    // first token is a head unless it continues the previous slot's last one;
    // the max over the earlier slots and the slot's own first token complete
    // the scan
    uint32_t headA = hA, headB = hB;
    {
      uint32_t pre = 0, prev_last = 0;
#pragma unroll 4
      for (int i = 0; i < 2 * UZ_W; i++) {
        const uint4 c = *(const uint4 *)U.chn[i];  // {first key, last key, scan without lane 0 at lane 63}
        const uint32_t mfirst = (uint32_t)((i >= UZ_W ? UZ_T : 0) + (i % UZ_W) * 64);
        const uint32_t h0 = i == 0 || c.x == 0 || c.x != prev_last ? mfirst + 1 : 0u;
        if (i == wv) headA = max(max(headA, pre), h0);
        if (i == UZ_W + wv) headB = max(max(headB, pre), h0);
        pre = max(pre, max(h0, c.z));
        prev_last = c.y;
      }
    }
    const int32_t endA = preA + iA, endB = totA + preB + iB;  // output offsets after each token
    const int64_t room = dl - dpos;
    // a prefix of the tokens: those that fit the batch and start before the end
    // of the output (of the segment: a later token belongs to the next one)
    const bool accA = vA && endA <= UZ_OUT && (int64_t)endA - (int64_t)lenA < room;
    const bool accB = vB && endB <= UZ_OUT && (int64_t)endB - (int64_t)lenB < room;
    const int32_t oA = endA - (int32_t)lenA, oB = endB - (int32_t)lenB;
    // a copy whose source a pass may overwrite (an offset within UZ_PASS + 64 of
    // the history) reads it back from the staged output: flag it
    constexpr int64_t risky_off = UZ_HIST - UZ_PASS - 64;
    uint32_t fl = 0;
    if (accA) {
      const int64_t dd = dpos + oA;
      badA |= (int64_t)lenA > dl - dd;
      if (!litA) {
        badA |= xA == 0 || (int64_t)xA > dd - seg_lo;
        fl |= (int64_t)xA > risky_off ? 2u : 0u;
      }
      fl |= badA ? 1u : 0u;
    }
    if (accB) {
      const int64_t dd = dpos + oB;
      badB |= (int64_t)lenB > dl - dd;
      if (!litB) {
        badB |= xB == 0 || (int64_t)xB > dd - seg_lo;
        fl |= (int64_t)xB > risky_off ? 2u : 0u;
      }
      fl |= badB ? 1u : 0u;
    }
    UZ_TS(2);
    // ---- 4. token table, start bits, per-word counts; the batch's extent
    if (accA) {
      U.tok[mA] = make_uint2((uint32_t)oA | ((lenA - 1) << 13) | ((headA - 1) << 19) | (litA ? 0x80000000u : 0u), xA);
      __hip_atomic_fetch_or(&U.bmc[oA >> 5].x, 1u << (oA & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      for (int32_t w = (oA >> 5) + 1; w <= (endA >> 5) && w < UZ_OUT / 32; w++) U.bmc[w].y = (uint32_t)(mA + 1);
    }
    if (accB) {
      U.tok[mB] = make_uint2((uint32_t)oB | ((lenB - 1) << 13) | ((headB - 1) << 19) | (litB ? 0x80000000u : 0u), xB);
      __hip_atomic_fetch_or(&U.bmc[oB >> 5].x, 1u << (oB & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      for (int32_t w = (oB >> 5) + 1; w <= (endB >> 5) && w < UZ_OUT / 32; w++) U.bmc[w].y = (uint32_t)(mB + 1);
    }
    {
      const uint64_t bA = ballot(accA), bB = ballot(accB);
      const uint32_t fw = (ballot(fl & 1u) ? 1u : 0u) | (ballot(fl & 2u) ? 2u : 0u);
      const int LA = bA ? 63 - __builtin_clzll(bA) : -1, LB = bB ? 63 - __builtin_clzll(bB) : -1;
      if (lane == (LA < 0 ? 0 : LA)) {
        U.last[wv][0] = LA < 0 ? 0 : mA + 1;
        U.last[wv][1] = endA;
        U.last[wv][2] = pa + advA;
      }
      if (lane == (LB < 0 ? 0 : LB)) {
        U.last[UZ_W + wv][0] = LB < 0 ? 0 : mB + 1;
        U.last[UZ_W + wv][1] = endB;
        U.last[UZ_W + wv][2] = pb + advB;
      }
      if (lane == 0 && fw) __hip_atomic_fetch_or(&U.flags, fw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    int ntok = 0, T = 0, cur = 0;
#pragma unroll 4
    for (int q = 0; q < 2 * UZ_W; q++) {
      const int4 l = *(const int4 *)U.last[q];
      if (l.x > ntok) {
        ntok = l.x;
        T = l.y;
        cur = l.z;
      }
    }
    const uint32_t flags = U.flags;
    UZ_TS(3);
    if (ntok == 0 || (flags & 1u)) {  // output complete with tokens left, or a corrupt token
      err = E_SNAPPY;
      break;
    }
    // prefetch the next window (its loads overlap this batch's byte passes)
    const int64_t sn = s + cur;
    if (sn < slen) {
      const uintptr_t an = (uintptr_t)(src + sn) & ~(uintptr_t)3;
      pw0 = gld32(an + 4 * (uintptr_t)tid);
      pw1 = tid < UZ_WIN_DW - UZ_T ? gld32(an + 4 * (uintptr_t)(UZ_T + tid)) : 0u;
      pf_s = sn;
    }
    if (write) {
      if (flags & 2u) {  // a slow-path source: every earlier flush store of the workgroup done
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __syncthreads();
      }
      // ---- 5. every output byte: passes of UZ_PASS bytes, two a thread (an
      // aligned 16-bit history word); the first pass starts at a0 <= 0, its
      // bytes before the batch are the history's
      const int a0 = -(int)((uint32_t)dpos & 3);
      for (int base = a0; base < T; base += UZ_PASS) {
        const int j0 = base + 2 * tid;
        const uint32_t P = (uint32_t)(dpos + j0) & UZ_HMASK;  // even
        const int64_t safe_lo = dpos + base + UZ_PASS - UZ_HIST;
        const uint32_t old = *(const uint16_t *)(U.hist + P);
        uint32_t s0 = j0 >= 0 && j0 < T ? uz_direct(U, wb, j0, base, dpos, safe_lo, dst) : 0x8000u | (old & 0xffu);
        uint32_t s1 = j0 + 1 >= 0 && j0 + 1 < T ? uz_direct(U, wb, j0 + 1, base, dpos, safe_lo, dst) : 0x8000u | (old >> 8);
        *(uint32_t *)(U.src + 2 * tid) = s0 | (s1 << 16);
        // pointer jumping over the pass: a byte's source pointer becomes its
        // source's (a value once that is resolved); in place — a read sees the
        // old or the new pointer, both on the byte's chain
        for (;;) {
          const bool left = !(s0 & 0x8000u) || !(s1 & 0x8000u);
          if (ballot(left) && lane == 0)
            __hip_atomic_fetch_or(&U.rflag[uz_round % 3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          if (tid == 0) U.rflag[(uz_round + 1) % 3] = 0u;
          __syncthreads();
          const bool any = U.rflag[uz_round % 3] != 0u;
          uz_round++;
          if (!any) break;
          if (!(s0 & 0x8000u)) s0 = U.src[s0];
          if (!(s1 & 0x8000u)) s1 = U.src[s1];
          *(uint32_t *)(U.src + 2 * tid) = s0 | (s1 << 16);
        }
        if (j0 + 1 >= 0 && j0 < T) *(uint16_t *)(U.hist + P) = (uint16_t)((s0 & 0xffu) | ((s1 & 0xffu) << 8));
        __syncthreads();
      }
      UZ_TS(5);
      // ---- 6. to HBM: bytes up to the next 16-byte boundary (F is unaligned
      // after a long literal), then whole 16-byte chunks up to floor16(dpos + T)
      const int64_t end = dpos + T;
      int64_t a16 = (F + 15) & ~(int64_t)15;
      if (a16 > end) a16 = end;
      if (tid < a16 - F) dst[F + tid] = U.hist[(uint32_t)(F + tid) & UZ_HMASK];
      F = a16;
      const int64_t e16 = end & ~(int64_t)15;
      if ((F & 15) == 0)
        for (int64_t c = F + 16 * (int64_t)tid; c < e16; c += 16 * UZ_T)
          gst128((uintptr_t)(dst + c), *(const uint4 *)(U.hist + ((uint32_t)c & UZ_HMASK)));
      if (e16 > F) F = e16;
      UZ_TS(6);
    } else {
      __syncthreads();  // the window's and the batch words' readers (the next batch rewrites them)
    }
#ifdef PQ_SNAP_STAMPS
    if (tid == 0) uz_acc[7] += 1;
#endif
    dpos += T;
    s += cur;
  }
  if (err == E_OK && dpos != dl) err = E_SNAPPY;
  if (err == E_OK && write)
    for (int64_t p = F + tid; p < dl; p += UZ_T) dst[p] = U.hist[(uint32_t)p & UZ_HMASK];
  if (err == E_OK && !write) err = E_SIZE;  // compress.go:117-119
  if (seg) {
    // the last segment must end the stream exactly; a segment that does not
    // decode on its own sends the page to the serial decode
    if (err == E_OK && seg_k == a.seg_base[gi + 1] - a.seg_base[gi] - 1 && s != slen) err = E_SNAPPY;
    if (err && tid == 0) atomicMax(&a.seg_flag[gi], 1u);
    err = E_OK;
  }
  if (err && tid == 0) atomicMin(&a.status[page], make_status(ST_DECOMPRESS, err));
#ifdef PQ_SNAP_STAMPS
  if (tid == 0 && a.dbg2)
    for (int q = 0; q < 8; q++) atomicAdd((unsigned long long *)&a.dbg2[(size_t)page * 8 + q], (unsigned long long)uz_acc[q]);
  if (tid == 0 && a.dbg) {
    const uint64_t tt = __builtin_amdgcn_s_memtime() - uz_t0;
    atomicAdd((unsigned long long *)&a.dbg[(size_t)page * 4 + 0], (unsigned long long)tt);
    atomicMax((unsigned long long *)&a.dbg[(size_t)page * 4 + 1], (unsigned long long)tt);
    a.dbg[(size_t)page * 4 + 2] = (uint64_t)expect;
    a.dbg[(size_t)page * 4 + 3] = (uint64_t)slen;
  }
#endif
}

// ===========================================================================
// K0: start of a decode — every page's status back to its host-planned value
// (blockIdx.y == 0) and the validity bitmaps zeroed (blockIdx.y == 1 + range),
// one launch instead of a status upload and a memset per bitmap
// ===========================================================================
__global__ __launch_bounds__(256) void k_reset(KArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x, stride = (uint64_t)gridDim.x * 256;
  if (blockIdx.y == 0) {
    for (uint64_t i = t; i < (uint64_t)a.npages; i += stride) a.status[i] = a.status0[i];
    return;
  }
  const ZeroRange z = a.zr[blockIdx.y - 1];
  for (uint64_t i = t; i < z.words; i += stride) z.ptr[i] = 0u;
}

// ===========================================================================
// K2: dictionary pages (page_dict.go:30-64)
// ===========================================================================
// ===========================================================================
// PLAIN BYTE_ARRAY length prefixes (type_bytearray.go:24-45): [u32 len][bytes]
// ... for n entries.  The chain of entry positions is found 64 entries at a
// time by pointer jumping over a 1 KiB window staged in LDS (J_0(i) = i + 4 +
// len(i), 1024 = stop; lane m lands on entry m after 6 rounds), instead of a
// serial walk.  emit(first entry, entry lane, value offset, length) is called
// by every lane with the batch's entries in lanes < cnt.  Returns the first
// error in entry order: E_EOF (header or bytes past the stream), E_BYTE_ARRAY
// (negative length), or E_OK.
// ===========================================================================
constexpr int BA_WIN = 1024;       // k_decode's window (k_prepare: 960, in its run-walk LDS)
constexpr int BA_WIN_DICT = 2048;  // k_dict_prepare: ~64 entries a batch for ~27-byte strings
template <int W>
struct BaLdsT {
  uint32_t win[W / 4 + 8];
  uint16_t jt[2][W + 8];
};
using BaLds = BaLdsT<BA_WIN>;

template <int WINB, class Emit>
__device__ __forceinline__ uint32_t ba_walk(const uint8_t *vp, int64_t vlen, int64_t n, uint32_t *win, uint16_t *ja0,
                                            uint16_t *jb0, Emit emit) {
  static_assert(WINB % 64 == 0, "window: whole lanes");
  const int lane = lane_id();
  int64_t P = 0, done = 0;
  while (done < n) {
    const int64_t avail = vlen - P;
    const uintptr_t ab = (uintptr_t)(vp + P) & ~(uintptr_t)3;
    const int sh = (int)((uintptr_t)(vp + P) & 3);
    // global (not generic) loads, all issued before the LDS stores: generic
    // loads may alias LDS, and were each waited for before their store
    const __attribute__((address_space(1))) uint32_t *ga = (const __attribute__((address_space(1))) uint32_t *)ab;
    constexpr int NQ = (WINB / 4 + 8 + 63) / 64;
    uint32_t gq[NQ];
#pragma unroll
    for (int q = 0; q < NQ; q++) gq[q] = lane + 64 * q < WINB / 4 + 8 ? ga[lane + 64 * q] : 0u;
#pragma unroll
    for (int q = 0; q < NQ; q++)
      if (lane + 64 * q < WINB / 4 + 8) win[lane + 64 * q] = gq[q];
    wave_lds_sync();
    uint16_t *ja = ja0, *jb = jb0;
    // reads of a group of positions issued before its writes (window and
    // tables are all LDS: a read cannot pass a write that may alias it, and
    // each read / write pair cost an LDS round trip)
    constexpr int NP = WINB / 64;
    constexpr int G = NP % 8 == 0 ? 8 : NP % 5 == 0 ? 5 : NP % 4 == 0 ? 4 : NP % 3 == 0 ? 3 : 1;
#pragma unroll
    for (int g0 = 0; g0 < NP; g0 += G) {
      uint32_t wl[G], wh[G];
#pragma unroll
      for (int q = 0; q < G; q++) {
        const int b = sh + lane + 64 * (g0 + q);
        wl[q] = win[b >> 2];
        wh[q] = win[(b >> 2) + 1];
      }
#pragma unroll
      for (int q = 0; q < G; q++) {
        const int i = lane + 64 * (g0 + q);
        const int b = sh + i;
        const int32_t l = (int32_t)__builtin_amdgcn_alignbyte(wh[q], wl[q], b & 3);
        const bool ok = (int64_t)i + 4 <= avail && l >= 0 && (int64_t)i + 4 + l <= avail;
        const int64_t nx = (int64_t)i + 4 + (int64_t)l;
        ja[i] = (uint16_t)((ok && nx < WINB) ? nx : WINB);
      }
    }
    if (lane == 0) {
      ja[WINB] = WINB;
      jb[WINB] = WINB;
    }
    wave_lds_sync();
    int pos = 0;
#pragma unroll
    for (int bt = 0; bt < 6; bt++) {
      const int hop = ja[pos];
      if (bt < 5) {
#pragma unroll
        for (int g0 = 0; g0 < NP; g0 += G) {
          uint32_t t1[G], t2[G];
#pragma unroll
          for (int q = 0; q < G; q++) t1[q] = ja[lane + 64 * (g0 + q)];
#pragma unroll
          for (int q = 0; q < G; q++) t2[q] = ja[t1[q]];
#pragma unroll
          for (int q = 0; q < G; q++) jb[lane + 64 * (g0 + q)] = (uint16_t)t2[q];
        }
      }
      if ((lane >> bt) & 1) pos = hop;
      if (bt < 5) {
        wave_lds_sync();
        uint16_t *t = ja;
        ja = jb;
        jb = t;
      }
    }
    // this lane's entry
    const bool real = pos < WINB;
    int32_t l = 0;
    uint32_t code = E_OK;
    if (real) {
      const int b = sh + pos;
      const uint64_t w2 = (uint64_t)win[b >> 2] | ((uint64_t)win[(b >> 2) + 1] << 32);
      l = (int32_t)(uint32_t)(w2 >> ((b & 3) * 8));
      if ((int64_t)pos + 4 > avail) code = E_EOF;
      else if (l < 0) code = E_BYTE_ARRAY;
      else if ((int64_t)pos + 4 + l > avail) code = E_EOF;
    }
    wave_lds_sync();
    const int64_t left = n - done;
    const bool mine = lane < left;
    const uint64_t okm = ballot(mine && real && code == E_OK);
    const int cnt = ~okm ? (int)__builtin_ctzll(~okm) : 64;  // leading valid entries
    if (cnt < 64 && cnt < left && ballot(lane == cnt && real && code != E_OK)) {
      return (uint32_t)__builtin_amdgcn_readlane(code, cnt);  // the first failing entry, in order
    }
    if (cnt == 0) return E_EOF;  // nothing readable (cannot happen for avail >= 4)
    emit(done, lane, P + pos + 4, l, cnt);
    const int lp = (int)__builtin_amdgcn_readlane(pos, cnt - 1), ll = (int)__builtin_amdgcn_readlane(l, cnt - 1);
    P += (int64_t)lp + 4 + ll;
    done += cnt;
  }
  return E_OK;
}

__global__ __launch_bounds__(256) void k_dict_prepare(KArgs a) {
  const int gi = blockIdx.x * 4 + (int)ufirst(threadIdx.x >> 6);
  if (gi >= a.nlist) return;
  const int page = ufirst(a.list[gi]);
  const PageDesc d = a.pages[page];
  if (page_status(a.status, page) != STATUS_OK) return;
  const ColDesc c = a.cols[d.col];
  const uint8_t *body = body_ptr(a, d, page);
  const int64_t n = d.num_values, len = d.body_len;
  if (c.ptype != T_BYTE_ARRAY) {
    if (n * (int64_t)c.width > len) set_status(a.status, page, ST_DICT_VALUES, E_EOF);
    return;
  }
  // length-prefix walk (type_bytearray.go:24-45): entry table (offset << 32 | length)
  if (d.swalk >= 0) {  // a long page: walked region-parallel by the k_sw_* launches before this one
    const uint32_t e = __hip_atomic_load(&a.sw_res[d.swalk].err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (e) set_status(a.status, page, ST_DICT_VALUES, e);
    return;
  }
  __shared__ __attribute__((aligned(16))) BaLdsT<BA_WIN_DICT> ba_all[4];
  BaLdsT<BA_WIN_DICT> &bl = ba_all[threadIdx.x >> 6];
  auto put = [&](int64_t first, int ln, int64_t voff, int32_t l, int cnt) {
    if (ln < cnt) a.dict_ent[d.dict_base + first + ln] = ((uint64_t)voff << 32) | (uint32_t)l;
  };
  const uint32_t e = ba_walk<BA_WIN_DICT>(body, len, n, bl.win, bl.jt[0], bl.jt[1], put);
  if (e) set_status(a.status, page, ST_DICT_VALUES, e);
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
__device__ uint32_t layout(const KArgs &a, const PageDesc &d, int page, const ColDesc &c, PageStreams &ps,
                       uint32_t &stage) {
  ps.body = body_ptr(a, d, page);
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
// Region-parallel length-prefix walk of long PLAIN BYTE_ARRAY pages
// (type_bytearray.go:24-45: [u32 len][bytes] ... for the page's non-null
// values; a negative length is an error, a header or bytes past the stream
// io.EOF).  ba_walk finds a page's chain 64 entries at a time in one wave,
// which leaves a 1 MiB page of short strings with ~1,000 dependent steps.
// Here every SW_R-byte region of the values section is walked by its own lane:
//   k_sw_regions  lane = region: the first candidate entry whose chain stays
//                 well-formed for SW_K hops (or to the region end), then the
//                 chain from it through the region: entries, string bytes,
//                 exit, first error;
//   k_sw_link     wave per page, 64 regions a step: a region is on the true
//                 chain when its candidate is the exit of the previous region
//                 on it (a region the chain jumps over has no candidate);
//                 the first region that is not is walked again from the true
//                 entry (global loads).  Exclusive counts give every region's
//                 first value index; the walk ends at the page's n-th value
//                 or at the first error before it (ba_walk's result);
//   k_sw_emit     lane = region on the chain: (offset, length) per value.
// Wrong candidates only cost a re-walk of their region: the result is the
// serial walk's, whatever the bytes.
// ===========================================================================
constexpr int SW_K = 4;                              // hops a candidate must survive
constexpr int SW_MAX_REWALK = 16;                    // k_sw_link: then ba_walk for the rest of the page
constexpr int SW_STAGE_W = (64 * SW_R + 64) / 4;     // staged dwords: 64 regions + header lookahead + skew

// the page's values section (data page: after the V1 level streams)
__device__ __forceinline__ bool sw_values(const KArgs &a, const SwPage &sp, const uint8_t *&vp, int64_t &vlen) {
  const PageDesc d = a.pages[sp.page];
  if (sp.kind == 1) {
    vp = body_ptr(a, d, sp.page);
    vlen = d.body_len;
    return true;
  }
  const ColDesc c = a.cols[d.col];
  PageStreams ps;
  uint32_t stage = 0;
  if (layout(a, d, sp.page, c, ps, stage)) return false;  // k_prepare reports it
  vp = ps.body + ps.val_off;
  vlen = ps.val_len;
  return true;
}

// values bytes [lo, lo + 64 SW_R + 4) into LDS (dword aligned: byte p at
// p - lo + sh); nothing at or past the section end is loaded
__device__ __forceinline__ int sw_stage(uint32_t *st, const uint8_t *vp, int64_t vlen, int64_t lo) {
  const uintptr_t a0 = (uintptr_t)(vp + lo), ab = a0 & ~(uintptr_t)3, lim = (uintptr_t)(vp + vlen);
  const __attribute__((address_space(1))) uint32_t *g = (const __attribute__((address_space(1))) uint32_t *)ab;
  const int lane = lane_id();
  constexpr int NQ = (SW_STAGE_W + 63) / 64;
  constexpr int G = 13;
  static_assert(NQ % G == 0, "groups of loads");
#pragma unroll
  for (int q0 = 0; q0 < NQ; q0 += G) {
    uint32_t v[G];
#pragma unroll
    for (int q = 0; q < G; q++) {
      const int i = lane + 64 * (q0 + q);
      v[q] = (i < SW_STAGE_W && ab + 4 * (uintptr_t)i < lim) ? g[i] : 0u;
    }
#pragma unroll
    for (int q = 0; q < G; q++) {
      const int i = lane + 64 * (q0 + q);
      if (i < SW_STAGE_W) st[i] = v[q];
    }
  }
  return (int)(a0 & 3);
}

__device__ __forceinline__ int32_t sw_rd(const uint32_t *st, int64_t p, int64_t lo, int sh) {
  const int q = (int)(p - lo) + sh;
  return (int32_t)__builtin_amdgcn_alignbyte(st[(q >> 2) + 1], st[q >> 2], q & 3);
}

__global__ __launch_bounds__(64) void k_sw_regions(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t st[SW_STAGE_W];
  const int2 it = a.sw_items[blockIdx.x];
  const int spi = ufirst(it.x), chunk = ufirst(it.y);
  const SwPage sp = a.sw_pages[spi];
  if (page_status(a.status, sp.page) != STATUS_OK) return;
  const uint8_t *vp;
  int64_t vlen;
  if (!sw_values(a, sp, vp, vlen)) return;
  const int lane = lane_id();
  const int64_t lo = (int64_t)chunk * 64 * SW_R;
  const int32_t r = chunk * 64 + lane;
  const int64_t rs = lo + (int64_t)lane * SW_R;
  SwReg out;
  out.c = -1;
  out.x = (int32_t)rs;
  out.cnt = 0;
  out.err = 0;
  out.lsum = 0;
  out.base = -1;
  out.pad = 0;
  // (regions past the values section — body_len counted the V1 levels too —
  // keep an empty record: k_sw_emit never takes them)
  const int sh = lo < vlen ? sw_stage(st, vp, vlen, lo) : 0;
  wave_lds_sync();
  if (rs < vlen) {
    const int64_t re = min(rs + (int64_t)SW_R, vlen);
    // a strong candidate makes at least two hops inside the region (or ends
    // the section): a stray small "length" — the last byte of a string and
    // the low bytes of the next header, ~7 KB for text — jumps out in one.
    // The first weak one is taken only when the region has no strong one
    // (an entry spanning the region end)
    int64_t cand = -1, weak = -1;
    for (int64_t s0 = rs; s0 < re && cand < 0; s0++) {
      int64_t p = s0;
      bool ok = true;
      int h = 0;
      for (; h < SW_K && p < re; h++) {
        const int32_t l = p + 4 <= vlen ? sw_rd(st, p, lo, sh) : -1;
        if (l < 0 || p + 4 + (int64_t)l > vlen) {
          ok = false;
          break;
        }
        p += 4 + (int64_t)l;
      }
      if (!ok) continue;
      if (h >= 2 || p == vlen) cand = s0;
      else if (weak < 0) weak = s0;
    }
    if (cand < 0) cand = weak;
    if (cand >= 0) {
      int64_t p = cand, ls = 0;
      int32_t cnt = 0;
      uint32_t err = E_OK;
      while (p < re) {
        if (p + 4 > vlen) {
          err = E_EOF;
          break;
        }
        const int32_t l = sw_rd(st, p, lo, sh);
        if (l < 0) {
          err = E_BYTE_ARRAY;
          break;
        }
        if (p + 4 + (int64_t)l > vlen) {
          err = E_EOF;
          break;
        }
        cnt++;
        ls += l;
        p += 4 + (int64_t)l;
      }
      out.c = (int32_t)cand;
      out.x = (int32_t)p;
      out.cnt = cnt;
      out.err = err;
      out.lsum = ls;
    }
  }
  if (r < sp.nreg) a.sw_regs[sp.reg0 + r] = out;
}

// the values the length walk reads: the page's non-null values (k_levels'
// count, read at device scope) or the dictionary's entries
__device__ __forceinline__ int64_t sw_count(const KArgs &a, const SwPage &sp) {
  const PageDesc d = a.pages[sp.page];
  if (sp.kind == 0 && d.lvl_base >= 0)
    return __hip_atomic_load(&a.info[sp.page].non_null, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return max(d.num_values, 0);
}

__global__ __launch_bounds__(256) void k_sw_link(KArgs a) {
  const int wl = blockIdx.x * 4 + (int)ufirst(threadIdx.x >> 6);
  if (wl >= a.n_sw_pages) return;
  const int wi = a.sw_page0 + wl;
  const SwPage sp = a.sw_pages[wi];
  const int lane = lane_id();
  if (page_status(a.status, sp.page) != STATUS_OK) return;
  const uint8_t *vp;
  int64_t vlen;
  if (!sw_values(a, sp, vp, vlen)) return;
  const int64_t n = sw_count(a, sp);
  const int64_t nregs = (vlen + SW_R - 1) / SW_R;
  int64_t E = 0;     // the true chain's next entry (values offset)
  int64_t done = 0;  // values before it
  int64_t sb = 0;    // their string bytes
  uint32_t err = E_OK;
  int32_t treg = -1;  // the region holding the n-th value (k_sw_emit adds its bytes)
  bool fin = done >= n;
  int rewalks = 0;
  // one region of the true chain walked again from its entry (global loads):
  // up to the region end, the n-th value or an error
  auto rewalk = [&](int64_t p, int64_t re, int64_t want, int32_t &cnt, int64_t &ls, uint32_t &e) {
    cnt = 0;
    ls = 0;
    e = E_OK;
    while (p < re && cnt < want) {
      if (p + 4 > vlen) {
        e = E_EOF;
        break;
      }
      const int32_t l = (int32_t)load_u32_unaligned(vp + p);
      if (l < 0) {
        e = E_BYTE_ARRAY;
        break;
      }
      if (p + 4 + (int64_t)l > vlen) {
        e = E_EOF;
        break;
      }
      cnt++;
      ls += l;
      p += 4 + (int64_t)l;
    }
    return p;
  };
  for (int64_t c0 = 0; c0 < nregs && !fin; c0 += 64) {
    const int64_t r = c0 + lane;
    SwReg g;
    g.c = -1;
    g.x = 0;
    g.cnt = 0;
    g.err = 0;
    g.lsum = 0;
    if (r < nregs) g = a.sw_regs[sp.reg0 + r];
    const int64_t re = min((r + 1) * (int64_t)SW_R, vlen);
    int32_t my_base = -1, my_c = -1;
    int l0 = 0;
    while (l0 < 64 && !fin) {
      const bool in = lane >= l0 && r < nregs;
      if (!ballot(in)) break;
      const bool has = in && g.c >= 0;
      // entry into this lane's region if every region in [l0, lane) is on the
      // chain: the exit of the last of them with an entry, else E
      const uint64_t below = ballot(has) & ((1ull << lane) - 1ull);
      const int src = below ? 63 - __clzll(below) : -1;
      const int32_t xs = (int32_t)shfl32((uint32_t)g.x, src < 0 ? 0 : src);
      const int64_t entry = src < 0 ? E : (int64_t)xs;
      const bool cons = !in || (has ? entry == (int64_t)g.c : entry >= re);
      const uint64_t badm = ballot(!cons);
      const int m = badm ? (int)__builtin_ctzll(badm) : 64;
      const bool conf = in && has && lane < m;  // on the chain, with entries
      int32_t tot = 0;
      const int32_t ex = wave_excl_scan32(conf ? g.cnt : 0, &tot);
      const int64_t b = done + ex;
      const bool term = conf && (b + g.cnt >= n || (g.err != E_OK && b + g.cnt < n));
      const uint64_t tm = ballot(term);
      const int t = tm ? (int)__builtin_ctzll(tm) : 64;
      const int64_t lsx = wave_incl_scan64(conf && lane < t ? g.lsum : 0);
      const int64_t ls_before = (int64_t)ufirst64((int64_t)shfl64((uint64_t)lsx, 63));
      if (conf && lane <= t) {
        my_base = (int32_t)b;
        my_c = g.c;
      }
      if (tm) {
        const uint32_t te = (uint32_t)__builtin_amdgcn_readlane((int)g.err, t);
        const int64_t tb = (int64_t)ufirst64((int64_t)shfl64((uint64_t)b, t));
        const int32_t tc = (int32_t)__builtin_amdgcn_readlane(g.cnt, t);
        if (te != E_OK && tb + tc < n) {
          err = te;  // ba_walk: the first failing entry in order
        } else {
          treg = (int32_t)(c0 + t);
          done = n;
        }
        sb += ls_before;
        fin = true;
        break;
      }
      done += tot;
      sb += ls_before;
      const uint64_t cm = ballot(conf);
      if (cm) E = (int64_t)(int32_t)shfl32((uint32_t)g.x, 63 - __clzll(cm));
      if (m == 64) break;
      // region c0 + m is not entered where its walk started: walk it from E
      const int64_t rm = c0 + m, rem = min((rm + 1) * (int64_t)SW_R, vlen);
      if (E < rem && ++rewalks > SW_MAX_REWALK) {
        // values that hold well-formed length prefixes themselves mislead the
        // candidates region after region: the rest of the page by ba_walk
        // (regions from here on emit nothing)
        __shared__ __attribute__((aligned(16))) BaLds swb_all[4];
        BaLds &bl = swb_all[threadIdx.x >> 6];
        const PageDesc d = a.pages[sp.page];
        const int32_t nvp = max(d.num_values, 0);
        int32_t *SO = sp.kind == 0 ? a.lens + d.lens_base : nullptr;
        const int64_t d0 = done, E0 = E;
        int64_t acc = 0;
        auto put = [&](int64_t first, int ln, int64_t voff, int32_t l, int cnt) {
          const int64_t t2 = wave_incl_scan64(ln < cnt ? (int64_t)l : 0);
          acc += (int64_t)ufirst64((int64_t)shfl64((uint64_t)t2, 63));
          const int64_t idx = d0 + first + ln;
          if (ln < cnt) {
            if (SO) {
              if (idx < nvp) {
                SO[idx] = (int32_t)(E0 + voff);
                SO[nvp + idx] = l;
              }
            } else {
              a.dict_ent[d.dict_base + idx] = ((uint64_t)(E0 + voff) << 32) | (uint32_t)l;
            }
          }
        };
        err = ba_walk<BA_WIN>(vp + E0, vlen - E0, n - d0, bl.win, bl.jt[0], bl.jt[1], put);
        if (err == E_OK) {
          done = n;
          sb += acc;
        }
        fin = true;
        break;
      }
      if (E < rem) {
        int32_t cnt;
        int64_t ls;
        uint32_t e;
        const int64_t x = rewalk(E, rem, n - done, cnt, ls, e);
        if (lane == m) {
          my_base = (int32_t)done;
          my_c = (int32_t)E;
        }
        if (e != E_OK && done + cnt < n) {
          err = e;
          fin = true;
          break;
        }
        if (done + cnt >= n) {
          treg = (int32_t)rm;  // k_sw_emit adds the bytes of its values before the n-th
          done = n;
          fin = true;
          break;
        }
        done += cnt;
        sb += ls;
        E = x;
      }
      l0 = m + 1;
    }
    if (r < nregs) {
      a.sw_regs[sp.reg0 + r].base = my_base;
      a.sw_regs[sp.reg0 + r].c = my_c;
    }
  }
  // the chain ended (at the section end) before n values: the next header is past it
  if (err == E_OK && done < n) err = E_EOF;
  if (lane == 0) {
    SwRes res;
    res.err = err;
    res.n = (int32_t)n;
    res.sbytes = err == E_OK ? sb : 0;
    res.treg = treg;
    res.pad = 0;
    a.sw_res[wi] = res;
  }
}

__global__ __launch_bounds__(64) void k_sw_emit(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t st[SW_STAGE_W];
  const int2 it = a.sw_items[blockIdx.x];
  const int spi = ufirst(it.x), chunk = ufirst(it.y);
  const SwPage sp = a.sw_pages[spi];
  if (page_status(a.status, sp.page) != STATUS_OK) return;
  // written by k_sw_link in the previous launch: device scope
  const uint32_t rerr = __hip_atomic_load(&a.sw_res[spi].err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int64_t n = __hip_atomic_load(&a.sw_res[spi].n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int32_t treg = __hip_atomic_load(&a.sw_res[spi].treg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (rerr != E_OK || n <= 0) return;
  const int lane = lane_id();
  const int32_t r = chunk * 64 + lane;
  const uint8_t *vp;
  int64_t vlen;
  if (!sw_values(a, sp, vp, vlen)) return;
  const int64_t lo = (int64_t)chunk * 64 * SW_R;
  SwReg g;
  g.base = -1;
  g.c = -1;
  if (r < sp.nreg && lo + (int64_t)lane * SW_R < vlen) g = a.sw_regs[sp.reg0 + r];
  if (!ballot(g.base >= 0)) return;
  const int sh = sw_stage(st, vp, vlen, lo);
  wave_lds_sync();
  if (g.base < 0) return;
  const PageDesc d = a.pages[sp.page];
  const int64_t re = min(lo + (int64_t)(lane + 1) * SW_R, vlen);
  const int32_t nvp = max(d.num_values, 0);
  int32_t *SO = sp.kind == 0 ? a.lens + d.lens_base : nullptr;
  int64_t p = g.c, idx = g.base, ls = 0;
  while (p < re && idx < n) {
    const int32_t l = sw_rd(st, p, lo, sh);
    if (sp.kind == 0) {
      if (idx < nvp) {
        SO[idx] = (int32_t)(p + 4);
        SO[nvp + idx] = l;
      }
    } else {
      a.dict_ent[d.dict_base + idx] = ((uint64_t)(p + 4) << 32) | (uint32_t)l;
    }
    ls += l;
    idx++;
    p += 4 + (int64_t)l;
  }
  if (r == treg) atomicAdd((unsigned long long *)&a.sw_res[spi].sbytes, (unsigned long long)ls);
}

// ===========================================================================
// Run walk for the tiled decode of flat, required, fixed-width RLE_DICTIONARY
// pages (called by k_prepare, consumed by k_expand).
//
// One wave walks the key stream's run headers (hybrid_decoder.go:82-166) into
// a run table in HBM and records, for every RUN_TILE values, the run
// holding the tile's first value.  Trains of identical bit-packed headers
// (what an encoder writes for high-entropy keys) are accepted 64 candidates
// at a time; the train check is only tried when the next header repeats the
// current one, so alternating RLE / bit-packed streams stay a cheap serial
// walk over a register window.
// ===========================================================================

// 1 KiB register window over a byte stream: lane l holds bytes [16l, 16l + 16)
// of the 16-byte aligned window base.  Reads are uniform (v_readlane).
struct Win1K {
  const uint8_t *ab;
  uint4 w;
  __device__ __forceinline__ void reset() { ab = nullptr; }
  __device__ __forceinline__ void fill(const uint8_t *a) {  // window starting at a (aligned down)
    ab = (const uint8_t *)((uintptr_t)a & ~(uintptr_t)15);
    const u32x4 x = *(const __attribute__((address_space(1))) u32x4 *)(ab + 16 * lane_id());
    w = make_uint4(x.x, x.y, x.z, x.w);
  }
  __device__ __forceinline__ void at(const uint8_t *a) {  // make [a, a + 8) resident
    if (!ab || (uint64_t)(a - ab) >= 1024 - 8) fill(a);
  }
  __device__ __forceinline__ uint32_t dw(uint32_t i) {  // dword i of the window
    const int l = (int)(i >> 2);
    const uint32_t c = i & 3;
    const uint32_t x = __builtin_amdgcn_readlane(w.x, l), y = __builtin_amdgcn_readlane(w.y, l),
                   z = __builtin_amdgcn_readlane(w.z, l), q = __builtin_amdgcn_readlane(w.w, l);
    return c == 0 ? x : c == 1 ? y : c == 2 ? z : q;
  }
  __device__ __forceinline__ uint32_t byte_at(const uint8_t *a) {
    at(a);
    const uint32_t off = (uint32_t)(a - ab);
    return (dw(off >> 2) >> ((off & 3) * 8)) & 0xffu;
  }
};

// byte q of the hl-byte uvarint encoding of h
__device__ __forceinline__ uint32_t hdr_byte(uint64_t h, int hl, int q) {
  return (uint32_t)((h >> (7 * q)) & 0x7f) | (q < hl - 1 ? 0x80u : 0u);
}

// record run r = [s, e) as the first run of every tile whose first value it
// holds, with the byte of that value's key: bit-packed data at byte `prm`
// (bw bits a value), or for an RLE run (bw < 0) the byte after it
__device__ __forceinline__ void tiles_of_run(int2 *tf, int64_t s, int64_t e, int32_t r, int64_t prm, int bw) {
  for (int64_t t = (s + RUN_TILE - 1) / RUN_TILE; t * RUN_TILE < e; t++)
    tf[t] = make_int2(r, (int32_t)(bw < 0 ? prm : prm + (((t * RUN_TILE - s) * bw) >> 3)));
}

// ks / slen: the key stream after the bit-width byte; n values; bw bit width
// Run entries are collected one per lane (64 at a time) and written out in
// one lane-parallel burst with their tiles: no store sits in the walk's
// dependency chain (stores and loads share vmcnt on gfx950, so a store in the
// loop would make every window read wait for it).
struct RunBuf {
  uint2 *runs;
  int2 *tf;
  int32_t base, cnt;  // entries written / buffered
  uint2 ent;          // lane k: entry base + k
  int32_t es, ee;     // its values [es, ee)
  int32_t tb, tbw;    // tile key bytes: data byte and bit width (-1: RLE, tb = byte after it)
  __device__ __forceinline__ void emit(int64_t s, int64_t e, uint32_t x, uint32_t y, int64_t b, int w) {
    if (lane_id() == cnt) {
      ent = make_uint2(x, y);
      es = (int32_t)s;
      ee = (int32_t)e;
      tb = (int32_t)b;
      tbw = w;
    }
    if (++cnt == 64) flush();
  }
  __device__ __forceinline__ void flush() {
    if (lane_id() < cnt) {
      runs[base + lane_id()] = ent;
      tiles_of_run(tf, es, ee, base + lane_id(), tb, tbw);
    }
    base += cnt;
    cnt = 0;
  }
  // lanes 0..m-1 hold m new runs: buffer them after the ones already held
  __device__ __forceinline__ void append(int m, uint2 x, int32_t s, int32_t e, int32_t b, int32_t w) {
    if (cnt + m > 64) flush();
    const int l = lane_id(), src = (l - cnt) & 63;
    const bool mine = l >= cnt && l < cnt + m;
    const uint32_t xx = shfl32(x.x, src), xy = shfl32(x.y, src);
    const int32_t ss = (int32_t)shfl32((uint32_t)s, src), ee2 = (int32_t)shfl32((uint32_t)e, src);
    const int32_t bb = (int32_t)shfl32((uint32_t)b, src), ww = (int32_t)shfl32((uint32_t)w, src);
    if (mine) {
      ent = make_uint2(xx, xy);
      es = ss;
      ee = ee2;
      tb = bb;
      tbw = ww;
    }
    cnt += m;
    if (cnt == 64) flush();
  }
};

// Chain mode (streams of short runs, e.g. a bit width 1 key stream that
// alternates RLE and short bit-packed runs): for the 1 KiB register window,
// every byte position p gets, in parallel, the position of the header that
// would follow a one-byte header at p (LDS table).  One lane then hops the
// chain (one LDS read a header), collecting up to 64 header positions, and
// the collected runs are decoded and emitted lane-parallel with a wave prefix
// sum of their lengths.  Anything unusual (multi-byte header, an error, the
// end of the stream) is left to the exact serial step below.
constexpr uint32_t NX_STOP = 0xFFFFu;
#ifndef PQ_CHAIN_WIN
#define PQ_CHAIN_WIN 2048  // run walk chain window (bytes, a multiple of 1 KiB; lbytes / lnx hold it)
#endif
constexpr int CW = PQ_CHAIN_WIN;
static_assert(CW % 1024 == 0 && CW <= 2048, "chain window: lnx holds 2,048 positions");
#ifndef PQ_DEC_DICT_LDS
#define PQ_DEC_DICT_LDS 8192  // k_decode<3> / <2>: dictionaries (<2>: entry tables) up to this many bytes gathered from LDS (0: off)
#endif
#ifndef PQ_LV_AHEAD
#define PQ_LV_AHEAD 1  // k_decode: a step's level scratch loaded one step ahead (0: when the step starts)
#endif

__device__ void walk_runs(const KArgs &a, const PageDesc &d, PageInfo *pi, const uint8_t *ks, int64_t slen,
                          int32_t n, int bw, uint8_t *lbytes, uint16_t *lnx, const uint8_t *dict, uint32_t dict_n) {
  const int lane = lane_id();
  RunBuf R;
  R.runs = a.runs + d.run_base;
  R.tf = a.tile_info + d.tile_base;
  R.base = R.cnt = 0;
  R.ent = make_uint2(0u, 0u);
  R.es = R.ee = R.tb = R.tbw = 0;
  const int32_t cap = d.run_cap - 1;  // entries before the sentinel

  int64_t v = 0;     // values covered
  int64_t hpos = 0;  // next header (stream offset)
  uint32_t err = E_OK;
  Win1K W;
  W.reset();
  int iters = 0;
  if (bw == 0) {  // hybrid_decoder.go:84-86: all zeros, nothing read
    R.emit(0, n, RUN_RLE, 0u, 0, 0);
    v = n;
  }
  const int sz = (bw + 7) >> 3;  // RLE value bytes
  const uint8_t *nx_ab = nullptr;  // window the chain table was built for
  // bit width 1 streams alternate short RLE and bit-packed runs from the
  // start (pyarrow: ~70 runs a 20k-value page): chain mode at once, no exact
  // step (and its register-window load) first
#ifdef PQ_CHAIN_OFF
  bool chain = false;  // (analysis build: the exact serial step only)
#else
  bool chain = bw == 1;  // short runs seen lately: try chain mode
#endif
  // the chain window's bytes (lane l: 16 bytes at 1024 h + 16 l) and the
  // 1 KiB after it, loaded with it: a window that moves on by half its size
  // takes its second half and the prefetched 1 KiB, no load in the chain
  u32x4 cwv[CW / 1024], cpf = u32x4{0, 0, 0, 0};
  while (v < n) {
    // ---- chain mode ----
    if (chain) {
#ifdef PQ_STAMPS
      if (a.dbg3 && (int)(pi - a.info) == 1 && lane == 0 && iters < 60) {
        a.dbg3[iters * 4 + 0] = __builtin_amdgcn_s_memrealtime();
        a.dbg3[iters * 4 + 1] = (uint64_t)hpos | (1ull << 40);
        a.dbg3[iters * 4 + 2] = (uint64_t)v;
        a.dbg3[iters * 4 + 3] = (uint64_t)(R.base + R.cnt);
      }
#endif
      // the chain window: CW bytes of the stream in LDS (lbytes), 16 bytes a
      // lane a load, re-anchored at the next header once it is past the
      // window's first half (bit width 1 pages: 5 window steps with 1 KiB, 2
      // with 2 KiB)
      if (!nx_ab || ks + hpos < nx_ab || (ks + hpos) - nx_ab > CW / 2) {
        const uint8_t *want = (const uint8_t *)((uintptr_t)(ks + hpos) & ~(uintptr_t)15);
        u32x4 *wv = cwv;
        if (CW == 2048 && nx_ab && want >= nx_ab + 1024 && want < nx_ab + 2048) {
          nx_ab += 1024;  // slide: [old + 1 KiB, old + 3 KiB) holds hpos in its first half
          cwv[0] = cwv[CW / 1024 - 1];
          cwv[CW / 1024 - 1] = cpf;
        } else {
          nx_ab = want;
#pragma unroll
          for (int h = 0; h < CW / 1024; h++)
            wv[h] = *(const __attribute__((address_space(1))) u32x4 *)(nx_ab + 1024 * h + 16 * lane);
        }
        if (CW == 2048)  // the next 1 KiB, in flight while this window is walked
          cpf = *(const __attribute__((address_space(1))) u32x4 *)(nx_ab + CW + 16 * lane);
#pragma unroll
        for (int h = 0; h < CW / 1024; h++) {
          *(u32x4 *)(lbytes + 1024 * h + 16 * lane) = wv[h];
          const uint32_t wd[4] = {wv[h].x, wv[h].y, wv[h].z, wv[h].w};
#pragma unroll
          for (int i = 0; i < 16; i += 2) {
            uint32_t two = 0;
#pragma unroll
            for (int k = 0; k < 2; k++) {
              const uint32_t b = (wd[(i + k) >> 2] >> (8 * ((i + k) & 3))) & 0xffu;
              const uint32_t r = 1024 * h + 16 * lane + i + k, g = b >> 1;
              uint32_t nx = NX_STOP;
              if (b < 0x80 && g != 0) nx = min(r + 1 + ((b & 1) ? g * (uint32_t)bw : (uint32_t)sz), NX_STOP - 1);
              two |= nx << (16 * k);
            }
            *(uint32_t *)(lnx + 1024 * h + 16 * lane + i) = two;
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      const int64_t wbo = nx_ab - ks;  // stream offset of window byte 0
      int32_t r = (int32_t)(hpos - wbo), cnt = 0;
      uint32_t myr = 0;
      while (cnt < 64 && r <= CW - 8 - sz && wbo + r < slen) {
        const uint32_t nx = ufirst((uint32_t)lnx[r]);
        if (nx == NX_STOP) break;
        if (lane == cnt) myr = (uint32_t)r;
        cnt++;
        r = (int32_t)nx;
      }
      if (cnt >= 2) {
        const int32_t nr0 = R.base + R.cnt;  // index of the first chained run
        const bool in = lane < cnt;
        const uint32_t b = in ? lbytes[myr] : 0u;
        const bool bp = (b & 1) != 0;
        const uint32_t g = b >> 1;
        const int32_t len = in ? (int32_t)(bp ? g * 8 : g) : 0;
        uint32_t val = 0;
        if (in && !bp)
          for (int k = 0; k < sz; k++) val |= (uint32_t)lbytes[myr + 1 + k] << (8 * k);
        const int32_t incl = wave_incl_scan32(len);
        const int64_t st = v + incl - len;
        const int64_t data = wbo + myr + 1;  // packed data / RLE value
        bool ok = in && st < n && nr0 + lane < cap;
        bool bad = false;
        if (ok) {
          if (bp) {
            const int64_t ng = (min<int64_t>((int64_t)len, (int64_t)n - st) + 7) >> 3;
            bad = data + (ng - 1) * bw >= slen;
          } else {
            bad = data + sz > slen || (bw < 32 && (val >> bw) != 0);
          }
        }
        const uint64_t okm = ballot(ok), badm = ballot(ok && bad);
        const int m = min((int)__popcll(okm), badm ? (int)__builtin_ctzll(badm) : 64);
        if (m > 0) {
          // buffered in lanes with the serial step's runs: no stores before the next window load
          const int64_t e = min<int64_t>(st + len, (int64_t)n);
          R.append(m, make_uint2((uint32_t)st | (bp ? 0u : RUN_RLE), bp ? (uint32_t)data : val), (int32_t)st,
                   (int32_t)e, (int32_t)(bp ? data : data + sz), bp ? bw : -1);
          const int32_t last = m - 1;
          const uint32_t lr = __builtin_amdgcn_readlane(myr, last);
          const uint32_t lb = __builtin_amdgcn_readlane(b, last);
          v = min<int64_t>(v + (int64_t)__builtin_amdgcn_readlane((uint32_t)incl, last), (int64_t)n);
          const int64_t hnext = wbo + lr + 1 + ((lb & 1) ? (int64_t)(lb >> 1) * bw : (int64_t)sz);
          chain = hnext - hpos < 48 * (int64_t)m;  // still short runs on average
          hpos = hnext;
          iters++;
          continue;
        }
      }
      chain = false;  // nothing to chain here: long runs (or an exact step is due)
    }
    // ---- exact serial step ----
#ifdef PQ_STAMPS
    if (a.dbg3 && (int)(pi - a.info) == 1 && lane == 0 && iters < 60) {
      a.dbg3[iters * 4 + 0] = __builtin_amdgcn_s_memrealtime();
      a.dbg3[iters * 4 + 1] = (uint64_t)hpos;
      a.dbg3[iters * 4 + 2] = (uint64_t)v;
      a.dbg3[iters * 4 + 3] = (uint64_t)(R.base + R.cnt);
    }
#endif
    iters++;
    if (R.base + R.cnt >= cap) {  // cannot happen: runs <= min(n, len / 2 + 1) (host sizing)
      err = E_UNSUPPORTED;
      break;
    }
    // readRunHeader :143-166 (readUVariant32, helpers.go:149-165)
    const int64_t h0 = hpos;
    uint64_t h = 0;
    uint32_t sh = 0;
    for (int i = 0;; i++) {
      if (hpos >= slen) {
        err = E_EOF;
        break;
      }
      const uint32_t b = W.byte_at(ks + hpos);
      hpos++;
      if (b < 0x80) {
        if (i > 9 || (i == 9 && b > 1)) err = E_RLE;
        h |= (uint64_t)b << (sh & 63);
        break;
      }
      if (sh < 64) h |= (uint64_t)(b & 0x7f) << sh;
      sh += 7;
    }
    if (err) break;
    if (h > 0x7fffffffull) {  // "int32 out of range"
      err = E_RLE;
      break;
    }
    const int32_t hl = (int32_t)(hpos - h0);
    if (h & 1) {  // bit-packed run of g groups (readBitPackedRun :133-141)
      const int64_t g = (int64_t)(h >> 1);
      if (g == 0) {
        err = E_RLE;
        break;
      }
      // groups the page needs; each must start inside the stream (a short
      // last group is zero-filled, a group starting at the end is io.EOF)
      const int64_t ng = (min<int64_t>(g * 8, (int64_t)n - v) + 7) >> 3;
      if (hpos + (ng - 1) * bw >= slen) {
        const int64_t have = hpos < slen ? (slen - hpos + bw - 1) / bw : 0;
        if (have > 0) R.emit(v, v + have * 8, (uint32_t)v, (uint32_t)hpos, hpos, bw);
        v += have * 8;
        err = E_EOF;
        break;
      }
      const int64_t e = min<int64_t>(v + g * 8, (int64_t)n);
      R.emit(v, e, (uint32_t)v, (uint32_t)hpos, hpos, bw);
      v = e;
      hpos += g * (int64_t)bw;
      if (v >= n) break;
#ifndef PQ_CHAIN_OFF
      chain = hpos - h0 < 48;  // a short run: the next ones may chain
#endif
      // a train?  only if the next header repeats this one (a uvarint's bytes
      // are fixed by its value and length)
      const int64_t stride = hl + g * (int64_t)bw;
      bool same = hpos + hl <= slen;
      for (int q = 0; q < hl && same; q++) same = W.byte_at(ks + hpos + q) == hdr_byte(h, hl, q);
      if (!same) continue;
      R.flush();
      const int32_t nr = R.base;
      // lane k checks for the same header again k strides ahead
      const int64_t cand = hpos + (int64_t)lane * stride;  // candidate header of run nr + lane
      const int64_t cstart = v + (int64_t)lane * g * 8;
      bool ok = cstart < n && nr + lane < cap && cand + hl <= slen;
      if (ok) {
        for (int q = 0; q < hl; q++) ok &= ks[cand + q] == hdr_byte(h, hl, q);
        const int64_t cng = (min<int64_t>(g * 8, (int64_t)n - cstart) + 7) >> 3;
        ok &= cand + hl + (cng - 1) * bw < slen;
      }
      const uint64_t okm = ballot(ok);
      const int m = ~okm ? (int)__builtin_ctzll(~okm) : 64;  // leading accepted candidates (lanes 0..m-1)
      if (m > 0) {
        if (lane < m) {
          R.runs[nr + lane] = make_uint2((uint32_t)cstart, (uint32_t)(cand + hl));
          tiles_of_run(R.tf, cstart, min<int64_t>(cstart + g * 8, (int64_t)n), nr + lane, cand + hl, bw);
        }
        v = min<int64_t>(v + (int64_t)m * g * 8, (int64_t)n);
        hpos += (int64_t)m * stride;
        R.base += m;
      }
    } else {  // RLE run (readRLERunValue :116-131)
      const int64_t cr = (int64_t)(h >> 1);
      if (cr == 0) {
        err = E_RLE;
        break;
      }
      if (hpos >= slen || hpos + sz > slen) {
        err = E_EOF;
        break;
      }
      uint32_t val = 0;
      for (int k = 0; k < sz; k++) val |= W.byte_at(ks + hpos + k) << (8 * k);
      hpos += sz;
      if (bw < 32 && (val >> bw) != 0) {  // "RLE run value is too large"
        err = E_RLE;
        break;
      }
      const int64_t e = min<int64_t>(v + cr, (int64_t)n);
      R.emit(v, e, (uint32_t)v | RUN_RLE, val, hpos, -1);
      v = e;
#ifndef PQ_CHAIN_OFF
      chain = true;
#endif
    }
  }
  R.flush();
  const int32_t nr = R.base;
  const int32_t cover = (int32_t)min<int64_t>(v, (int64_t)n);
  // sentinel, and tiles past the coverage point at it
  const int64_t ntiles = ((int64_t)n + RUN_TILE - 1) / RUN_TILE;
  for (int64_t t = (cover + RUN_TILE - 1) / RUN_TILE + lane; t < ntiles; t += 64) R.tf[t] = make_int2(nr, (int32_t)slen);
  if (lane == 0) {
    R.runs[nr] = make_uint2((uint32_t)cover, 0u);
    pi->cover = cover;
    pi->walk_err = err;
    pi->pad = nr;
  }
  if (err) set_status(a.status, (int)(pi - a.info), ST_VALUES, err | E_LATE);
  // k_expand records, lane k = job k (read back this wave's own tile stores)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int32_t njobs = (n + EX_WAVE_VALUES - 1) / EX_WAVE_VALUES;
  for (int32_t k = lane; k < njobs; k += 64) {
    const int32_t v0 = k * EX_WAVE_VALUES, v1 = min(v0 + EX_WAVE_VALUES, n);
    const int2 t0 = R.tf[v0 / RUN_TILE];
    ExRec rc;
    rc.vals = ks - 1;
    rc.dict = dict;
    rc.runs = R.runs;
    rc.v0 = v0;
    rc.lim = min(v1, cover);
    rc.bw = bw;
    rc.nr = nr;
    rc.first_run = t0.x;
    rc.byte_lo = t0.y;
    rc.byte_hi = v1 >= n ? (int32_t)slen : R.tf[v1 / RUN_TILE].y;
    rc.dict_n = dict_n;
    rc.epoch = a.epoch;
    rc.val_len = (int32_t)slen + 1;
    a.recs[a.page_jobs[d.job_base + k]] = rc;
  }
  PSTAMP((int)(pi - a.info), 3, (uint64_t)nr);
  PSTAMP((int)(pi - a.info), 5, (uint64_t)iters);
  (void)iters;
}


// ===========================================================================
// K3: data page prepare
// ===========================================================================
// Page gi of the list.  mode -1: every page; 0: pages whose body does not
// wait on k_copy (run beside it, k_prepare_copy); 1: only the pages that do.
__device__ __forceinline__ void prepare_page(const KArgs &a, int gi, uint8_t *lbytes, uint16_t *lnx, int mode) {
  if (gi >= a.nlist) return;
  const int lane = lane_id();
  const int page = ufirst(a.list[gi]);
  PSTAMP(page, 0, __builtin_amdgcn_s_memrealtime());
  const PageDesc d = a.pages[page];
  if (d.srec) return;  // tiled PLAIN page: its k_expand records were written by the host
  PageInfo *pi = &a.info[page];
  if (mode >= 0) {
    // deferred literals of this body, or a length walk done by the k_sw_* launches between
    const bool waits = d.train || (d.sidx >= 0 && a.njobs[d.sidx] > 0) || d.swalk >= 0;
    if (waits != (mode == 1)) return;
  }
  if (page_status(a.status, page) != STATUS_OK) return;
  if (d.dict >= 0 && page_status(a.status, d.dict) != STATUS_OK) return;  // reported first anyway
  const ColDesc c = a.cols[d.col];
  PageStreams ps;
  uint32_t stage = ST_REP_INIT;
  uint32_t e = layout(a, d, page, c, ps, stage);
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
  } else if (d.enc == ENC_RLE && c.ptype == T_BOOLEAN) {  // hybridDecoder(1).initSize: the u32 size
    if (ps.val_len < 4) {
      set_status(a.status, page, ST_VAL_INIT, E_EOF);
      return;
    }
  }
  // DELTA_(LENGTH_)BYTE_ARRAY: every length stream is decoded at init
  // (type_bytearray.go:98-108, :186-209); lengths go to the page's scratch
  int32_t dstr_data = 0, dstr_cnt = 0;
  const bool dstr = ((c.ptype == T_BYTE_ARRAY && (d.enc == ENC_DELTA_LBA || d.enc == ENC_DELTA_BA)) ||
                     (c.ptype == T_FLBA && d.enc == ENC_DELTA_BA)) &&
                    d.lens_base >= 0;
  if (dstr) {
    const int32_t nvp = max(d.num_values, 0);
    int32_t *S = a.lens + d.lens_base, *P = S + nvp;
    const uint8_t *vp = ps.body + ps.val_off;
    int64_t pos = 0;
    int32_t cp = 0, cs = 0;
    if (d.enc == ENC_DELTA_BA) {
      e = delta_len_stream(vp, ps.val_len, pos, P, nvp, cp);  // prefix lengths
      if (e) {
        set_status(a.status, page, ST_VAL_INIT, e);
        return;
      }
    }
    e = delta_len_stream(vp, ps.val_len, pos, S, nvp, cs);  // suffix (value) lengths
    if (e) {
      set_status(a.status, page, ST_VAL_INIT, e);
      return;
    }
    if (d.enc == ENC_DELTA_BA && cp != cs) {  // "different number of suffixes and prefixes"
      set_status(a.status, page, ST_VAL_INIT, E_BYTE_ARRAY);
      return;
    }
    dstr_data = (int32_t)pos;
    dstr_cnt = cs;
    if (lane == 0) {
      pi->str_data = dstr_data;
      pi->str_cnt = dstr_cnt;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the counts below read the lengths back
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
  if (d.run_cap > 0) {  // tiled RLE_DICTIONARY page: its run table for k_expand
    if (d.num_values <= 0) return;
    if (d.dict < 0) {  // dictDecoder without a dictionary (type_dict.go:40-42)
      set_status(a.status, page, ST_VALUES, E_DICT);
      return;
    }
    PSTAMP(page, 1, __builtin_amdgcn_s_memrealtime());
    const PageDesc dp = a.pages[d.dict];
    walk_runs(a, d, pi, ps.body + ps.val_off + 1, ps.val_len - 1, d.num_values, idx_bw, lbytes, lnx,
              body_ptr(a, dp, d.dict), (uint32_t)dp.num_values);
    PSTAMP(page, 2, __builtin_amdgcn_s_memrealtime());
    PSTAMP(page, 4, (uint64_t)idx_bw);
    return;
  }
  if (d.job_base >= 0 && d.enc == ENC_PLAIN) {  // tiled PLAIN page: k_expand records
    const int32_t n = d.num_values;
    if ((int64_t)n * c.width > ps.val_len) {  // binary.Read past the values section
      set_status(a.status, page, ST_VALUES, E_EOF);
      return;
    }
    const int32_t njobs = (n + EX_WAVE_VALUES - 1) / EX_WAVE_VALUES;
    for (int32_t k = lane; k < njobs; k += 64) {
      ExRec rc;
      rc.vals = ps.body + ps.val_off;
      rc.dict = nullptr;
      rc.runs = nullptr;
      rc.v0 = k * EX_WAVE_VALUES;
      rc.lim = min(rc.v0 + EX_WAVE_VALUES, n);
      rc.bw = -1;
      rc.nr = rc.first_run = rc.byte_lo = rc.byte_hi = 0;
      rc.dict_n = 0;
      rc.epoch = a.epoch;
      rc.val_len = (int32_t)ps.val_len;
      a.recs[a.page_jobs[d.job_base + k]] = rc;
    }
    return;
  }
  if (!(c.flags & COL_NEEDS_COUNT)) return;

  // counts for lists / strings: decode the level streams (phase 2 stages)
  const int n = d.num_values;
  using Lv = HybS;
  // diagnostic build: count-path stamps (1 levels start, 2 rep done, 6 def
  // done, 7 strings done; 3 values, 4 = 100 + encoding)
  PSTAMP(page, 1, __builtin_amdgcn_s_memrealtime());
  PSTAMP(page, 3, (uint64_t)n);
  PSTAMP(page, 4, (uint64_t)(100 + d.enc));
  int64_t rows = 0, slots = 0, nn = 0;
  if (d.lvl_base >= 0) {
    // k_levels decoded the level streams (and checked them) in the previous
    // launch: its counts, read at device scope
    rows = __hip_atomic_load(&pi->rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    slots = __hip_atomic_load(&pi->slots, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    nn = __hip_atomic_load(&pi->non_null, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    // rows = rep levels 0; non-null = def levels max_def; slots = def levels >= rep_def
    HybS rep, def;
    rep.init(ps.lvl + ps.rep_off, ps.rep_len, bits_len(c.max_rep));
    def.init(ps.lvl + ps.def_off, ps.def_len, bits_len(c.max_def));
    if (c.max_rep > 0) {
      int64_t unused = 0;
      e = rep.count2(n, 0u, 0xffffffffu, rows, unused);
      if (e) {
        set_status(a.status, page, ST_REP, e);
        return;
      }
    }
    if (c.max_def > 0) {
      e = def.count2(n, (uint32_t)c.max_def, c.max_rep > 0 ? (uint32_t)c.rep_def : 0u, nn, slots);
      if (e) {
        set_status(a.status, page, ST_DEF, e);
        return;
      }
    } else {
      nn = slots = n;  // no def levels: every value is defined
    }
  }
  if (c.max_rep == 0) rows = n;
  PSTAMP(page, 6, __builtin_amdgcn_s_memrealtime());
  // string bytes of the non-null values
  int64_t sbytes = 0;
  if ((c.ptype == T_BYTE_ARRAY || dstr) && nn > 0) {
    if (d.enc == ENC_PLAIN) {
      // length prefixes by pointer jumping (ba_walk), in the run walk's LDS
      // each value's (offset, length) goes to the page's scratch for k_decode
      int64_t acc = 0;
      int32_t *SO = d.lens_base >= 0 ? a.lens + d.lens_base : nullptr;
      const int32_t nvp = max(d.num_values, 0);
      auto put = [&](int64_t first, int ln, int64_t voff, int32_t l, int cnt) {
        const int64_t t = wave_incl_scan64(ln < cnt ? (int64_t)l : 0);
        acc += (int64_t)ufirst64((int64_t)shfl64((uint64_t)t, 63));
        if (SO && ln < cnt && first + ln < nvp) {
          SO[first + ln] = (int32_t)voff;
          SO[nvp + first + ln] = l;
        }
      };
      uint32_t e2;
      if (d.swalk >= 0) {  // walked region-parallel by k_sw_regions / _link / _emit (previous launches)
        e2 = __hip_atomic_load(&a.sw_res[d.swalk].err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        acc = __hip_atomic_load(&a.sw_res[d.swalk].sbytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        e2 = ba_walk<960>(ps.body + ps.val_off, ps.val_len, nn, (uint32_t *)lbytes, lnx, lnx + 968, put);
      }
      if (e2) {
        set_status(a.status, page, ST_VALUES, e2);
        return;
      }
      sbytes = acc;
    } else if (d.enc == ENC_RLE_DICT) {
      if (d.dict < 0) {
        // dictDecoder with no dictionary: the first key is out of range
        Lv keys;
        keys.init(ps.body + ps.val_off + 1, ps.val_len - 1, idx_bw);
        uint32_t k;
        e = keys.next(1, k);
        set_status(a.status, page, ST_VALUES, e ? e : E_DICT);
        return;
      }
      const PageDesc dd = a.pages[d.dict];
      const int64_t dn = dd.num_values;
      Lv keys;
      keys.init(ps.body + ps.val_off + 1, ps.val_len - 1, idx_bw);
      // a small dictionary's entry lengths in the wave's LDS (the run walk's
      // buffers are free on this path): 256 keys a step, no global round trip
      // a step (C5's ~9,000 dictionary-string pages: 313 steps a page of a
      // key walk then a dependent entry load, 64 keys each)
      uint32_t *elen = (uint32_t *)lnx;
      const bool elds = dn <= 1024;
      if (elds) {
        for (int64_t i = lane; i < dn; i += 64) elen[i] = (uint32_t)(a.dict_ent[dd.dict_base + i] & 0xffffffffu);
        wave_lds_sync();
      }
      int64_t acc = 0;
      // a page split into k_decode<2> parts: the string bytes before every 256
      // values, where a part's count starts (entry q: values [0, 256 q))
      int64_t *spre = d.sp_base >= 0 && a.str_pre ? a.str_pre + d.sp_base : nullptr;
      for (int64_t k0 = 0; k0 < nn; k0 += 256) {
        const int cnt = (int)min<int64_t>(256, nn - k0);
        if (spre && lane == 0) spre[k0 >> 8] = acc;
        uint32_t k4[4];
        e = keys.next4(cnt, k4);
        if (e) {
          // keys read before the stream error are range-checked first (type_dict.go:44-53)
          bool oob = false;
#pragma unroll
          for (int j = 0; j < 4; j++) oob |= 4 * lane + j < keys.got && (int64_t)k4[j] >= dn;
          set_status(a.status, page, ST_VALUES, ballot(oob) ? E_DICT : e);
          return;
        }
        bool oob = false;
#pragma unroll
        for (int j = 0; j < 4; j++) oob |= 4 * lane + j < cnt && (int64_t)k4[j] >= dn;
        if (ballot(oob)) {
          set_status(a.status, page, ST_VALUES, E_DICT);
          return;
        }
        int64_t l = 0;
#pragma unroll
        for (int j = 0; j < 4; j++)
          if (4 * lane + j < cnt) l += elds ? (int64_t)elen[k4[j]] : (int64_t)(a.dict_ent[dd.dict_base + k4[j]] & 0xffffffffu);
        acc += (int64_t)ufirst64((int64_t)shfl64((uint64_t)wave_incl_scan64(l), 63));
      }
      if (spre && lane == 0) spre[(nn + 255) >> 8] = acc;
      sbytes = acc;
    } else if (dstr) {
      // byteArrayDeltaLengthDecoder.next (:111-123) and, for DELTA_BYTE_ARRAY,
      // the prefix checks of decodeValues (:211-240), in value order
      const int32_t nvp = max(d.num_values, 0);
      const int32_t *S = a.lens + d.lens_base, *P = S + nvp;
      const int64_t vlen = ps.val_len;
      int64_t acc_s = 0, acc_v = 0;
      int64_t prevlen = 0;  // the previous value's length (the first value follows an empty one)
      for (int64_t k0 = 0; k0 < nn; k0 += 64) {
        const int cnt = (int)min<int64_t>(64, nn - k0);
        const int64_t i = k0 + lane;
        const bool act = lane < cnt;
        uint32_t code = 0;
        int64_t s = 0, pl = 0;
        if (act) {
          if (i >= dstr_cnt) code = E_EOF;  // position >= len(lens)
          else {
            s = S[i];
            if (s < 0) code = E_BYTE_ARRAY;  // make([]byte, size) panics in the reference
            if (d.enc == ENC_DELTA_BA) pl = P[i];
          }
        }
        const int64_t s_ok = act && !code ? s : 0;
        const int64_t sincl = wave_incl_scan64(s_ok);
        if (act && !code && dstr_data + acc_s + sincl > vlen) code = E_EOF;  // io.ReadFull
        int64_t vl = s;  // value length
        if (d.enc == ENC_DELTA_BA) {
          vl = (pl > 0 ? pl : 0) + s;
          const int64_t pv = (int64_t)shfl64((uint64_t)vl, lane > 0 ? lane - 1 : 0);
          const int64_t plen_prev = lane == 0 ? prevlen : pv;
          if (act && !code && (pl + s < 0 || plen_prev < pl)) code = E_BYTE_ARRAY;  // "invalid prefix len"
          // FIXED_LEN_BYTE_ARRAY: a value must fill its type_length slot (the
          // reference would keep an odd-length []byte: a documented deviation)
          if (act && !code && c.ptype == T_FLBA && vl != c.width) code = E_BYTE_ARRAY;
        }
        const uint64_t bad = ballot(act && code != 0);
        if (bad) {
          set_status(a.status, page, ST_VALUES, __builtin_amdgcn_readlane(code, __builtin_ctzll(bad)));
          return;
        }
        acc_s += (int64_t)shfl64((uint64_t)sincl, 63);
        acc_v += (int64_t)shfl64((uint64_t)wave_incl_scan64(act ? vl : 0), 63);
        prevlen = (int64_t)shfl64((uint64_t)vl, cnt - 1);
      }
      sbytes = c.ptype == T_FLBA ? 0 : acc_v;  // FIXED_LEN_BYTE_ARRAY: fixed-width slots, no string bytes
    } else {
      set_status(a.status, page, ST_VALUES, E_UNSUPPORTED);
      return;
    }
  }
  PSTAMP(page, 7, __builtin_amdgcn_s_memrealtime());
  if (lane == 0) {
    pi->rows = rows;
    pi->slots = slots;
    pi->non_null = nn;
    pi->str_bytes = sbytes;
  }
}

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_prepare(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t wl_bytes[4][CW];  // run walk: chain window bytes
  __shared__ __attribute__((aligned(16))) uint16_t wl_nx[4][2048];    // run walk: chain table (BYTE_ARRAY walk: two)
  const int wv = (int)ufirst(threadIdx.x >> 6);
  prepare_page(a, (int)blockIdx.x * 4 + wv, wl_bytes[wv], wl_nx[wv], MODE);
}

// k_levels: the level streams of every page with a level scratch
// (PageDesc::lvl_base), one wave a page: run tables (HybT<true>) decoded into
// a byte a level, with the counts k_prepare needs (rows: rep levels 0,
// non-null: def levels max_def, slots: def levels >= rep_def).  Errors in the
// streams are the page's (ST_REP / ST_DEF, the reference's readLevels order);
// k_prepare and k_decode then read the counts and levels instead of the
// streams.  MODE as k_prepare (-1 every page, 0 / 1 pages that do not / do
// wait on k_copy).
template <int MODE>
__device__ __forceinline__ void levels_page(const KArgs &a, int gi, int part) {
  const int lane = lane_id();
  const int page = ufirst(a.list[gi]);
  const PageDesc d = a.pages[page];
  if (d.lvl_base < 0) return;
  if (MODE >= 0) {
    const bool waits = d.train || (d.sidx >= 0 && a.njobs[d.sidx] > 0);
    if (waits != (MODE == 1)) return;
  }
  if (page_status(a.status, page) != STATUS_OK) return;
  if (d.dict >= 0 && page_status(a.status, d.dict) != STATUS_OK) return;
  const ColDesc c = a.cols[d.col];
  PageStreams ps;
  uint32_t stage = ST_REP_INIT;
  uint32_t e = layout(a, d, page, c, ps, stage);
  if (e) {
    set_status(a.status, page, stage, e);
    return;
  }
  const int n = d.num_values;
  uint8_t *lv = a.lvl + d.lvl_base;
  // a list page split into k_decode<3> parts: the streams are counted part by
  // part and the counts before each part kept for it (no rescan of the levels)
  const bool pre = d.part0 >= 0 && a.part_pre != nullptr;
  if (part != 1 && c.max_rep > 0) {
    Hyb rep;
    rep.init(ps.lvl + ps.rep_off, ps.rep_len, bits_len(c.max_rep));
    int64_t rows = 0, unused = 0;
    if (pre) {
      e = E_OK;
      for (int k = d.part0, done = 0; done < n && !e; k++) {
        if (lane == 0) a.part_pre[4 * k] = (int32_t)rows;
        const int hi = ufirst(a.part_tab[3 * k + 2]);
        e = rep.count2(hi - done, 0u, 0xffffffffu, rows, unused, lv);
        done = hi;
      }
    } else {
      e = rep.count2(n, 0u, 0xffffffffu, rows, unused, lv);
    }
    if (e) {
      set_status(a.status, page, ST_REP, e);
      return;
    }
    if (lane == 0) a.info[page].rows = rows;
  }
  if (part == 0) return;
  Hyb def;
  def.init(ps.lvl + ps.def_off, ps.def_len, bits_len(c.max_def));
  int64_t slots = 0, nn = 0;
  if (c.max_rep > 0) lv += n;
  if (d.lvl_bits) {
    // flat page without level output: bit i = (def level i == max_def), all
    // k_decode reads — an eighth of the byte scratch, each word written once
    // (BitOut; k_decode's two-word loads mask what lies past the page)
    BitOut bo;
    bo.g = (uint32_t *)lv;
    bo.pos = 0;
    bo.carry = 0;
    e = def.template count2<true>(n, (uint32_t)c.max_def, 0u, nn, slots, nullptr, &bo);
    bo.finish();
  } else if (pre) {
    e = E_OK;
    for (int k = d.part0, done = 0; done < n && !e; k++) {
      if (lane == 0) {
        a.part_pre[4 * k + 1] = (int32_t)slots;
        a.part_pre[4 * k + 2] = (int32_t)nn;
      }
      const int hi = ufirst(a.part_tab[3 * k + 2]);
      e = def.count2(hi - done, (uint32_t)c.max_def, c.max_rep > 0 ? (uint32_t)c.rep_def : 0u, nn, slots, lv);
      done = hi;
    }
  } else {
    e = def.count2(n, (uint32_t)c.max_def, c.max_rep > 0 ? (uint32_t)c.rep_def : 0u, nn, slots, lv);
  }
  if (e) {
    set_status(a.status, page, ST_DEF, e);
    return;
  }
  if (lane == 0) {
    if (c.max_rep == 0) a.info[page].rows = n;
    a.info[page].slots = slots;
    a.info[page].non_null = nn;
  }
}

// SPLIT (batches with repeated columns): two waves per page — the repetition
// and the definition streams are independent (each its own run chain) and are
// decoded side by side; errors meet in the page status (atomicMin: ST_REP
// before ST_DEF, the reference's order).  Otherwise one wave per page decodes
// both in turn.  Workgroups loop over the pages with a grid stride
// (PQG_LEVELS_CAP: a capped grid for the launch beside the Snappy phase;
// measured slower, so the full grid is the default)
#ifndef PQ_LEVELS_WPE
#define PQ_LEVELS_WPE 4  // k_levels: registers capped for 4 waves a SIMD (the bitmap path took it to 141 VGPRs)
#endif
template <int MODE, bool SPLIT>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PQ_LEVELS_WPE))) void k_levels(KArgs a) {
  const int wv = (int)ufirst(threadIdx.x >> 6);
  const int part = SPLIT ? (wv & 1) : 2;  // 0: repetition levels, 1: definition levels, 2: both
  for (uint32_t b = blockIdx.x;; b += gridDim.x) {
    const int gi = SPLIT ? (int)b * 2 + (wv >> 1) : (int)b * 4 + wv;
    if (gi >= a.nlist) break;
    levels_page<MODE>(a, gi, part);
  }
}


// k_prepare beside k_copy in one launch (batches without BYTE_ARRAY
// dictionaries): the first blocks prepare every page whose body does not wait
// on a deferred literal, the rest copy the deferred literals (mostly large
// dictionaries, which k_prepare only points at).  Neither waits on the other;
// pages that do wait are prepared by k_prepare<1> after this launch.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6))) void k_prepare_copy(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t wl_bytes[4][CW];
  __shared__ __attribute__((aligned(16))) uint16_t wl_nx[4][2048];
  const uint32_t pb = ((uint32_t)a.nlist + 3) / 4;
  if (blockIdx.x < pb) {
    const int wv = (int)ufirst(threadIdx.x >> 6);
    prepare_page(a, (int)blockIdx.x * 4 + wv, wl_bytes[wv], wl_nx[wv], 0);
    return;
  }
  copy_items(a, blockIdx.x - pb, gridDim.x - pb);
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

// gather element j (0..255, four per lane) of a 4-per-lane vector
__device__ __forceinline__ uint32_t pick4(const uint32_t (&v)[4], int j) {
  uint32_t x0 = shfl32(v[0], j >> 2), x1 = shfl32(v[1], j >> 2), x2 = shfl32(v[2], j >> 2), x3 = shfl32(v[3], j >> 2);
  int k = j & 3;
  return k == 0 ? x0 : k == 1 ? x1 : k == 2 ? x2 : x3;
}
__device__ __forceinline__ uint64_t pick4_64(const uint64_t (&v)[4], int j) {
  uint32_t lo[4] = {(uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]};
  uint32_t hi[4] = {(uint32_t)(v[0] >> 32), (uint32_t)(v[1] >> 32), (uint32_t)(v[2] >> 32), (uint32_t)(v[3] >> 32)};
  return ((uint64_t)pick4(hi, j) << 32) | pick4(lo, j);
}

// Bits of one step of a nested column (≤ 256 positions starting at global bit
// b0): the produced entries (prod) hold the positions [0, total) in entry
// order (rel[k]: entry k's position, an exclusive scan), each with bit on[k].
// Every produced entry writes its bit as a byte of an LDS array (distinct
// addresses: no atomics, no bank serialisation), then lane w packs the 32
// bytes of word w (byte * 0x01020408 gathers a dword's four 0/1 bytes into
// bits 24..27) and stores it: plain stores for the words the step covers
// whole, atomicOr for the partial first/last word (shared with the
// neighbouring step or page).  Replaces one global atomic per set bit and the
// former LDS ds_or (up to 32 lanes on one word).
__device__ __forceinline__ uint32_t pack_bytes16(const u32x4 &x) {
  // (bytes outside the step hold stale LDS: each byte's low bit only, so no
  // stale byte carries into a neighbour's bit)
  const uint32_t m = 0x01020408u, b = 0x01010101u;
  return (((x.x & b) * m) >> 24 & 15u) | ((((x.y & b) * m) >> 24 & 15u) << 4) |
         ((((x.z & b) * m) >> 24 & 15u) << 8) | ((((x.w & b) * m) >> 24 & 15u) << 12);
}
__device__ __forceinline__ void wave_bitmap(uint8_t *lb, uint32_t *gbm, int64_t b0, int total, const int (&rel)[4],
                                            const bool (&prod)[4], const bool (&on)[4]) {
  const int lane = lane_id();
  const int sh = (int)(b0 & 31);
  const int nw = (sh + total + 31) >> 5;  // <= 9
#pragma unroll
  for (int k = 0; k < 4; k++)
    if (prod[k]) lb[sh + rel[k]] = on[k] ? 1 : 0;
  wave_lds_sync();
  if (lane < nw) {
    const u32x4 x0 = *(const u32x4 *)(lb + 32 * lane), x1 = *(const u32x4 *)(lb + 32 * lane + 16);
    uint32_t wv = pack_bytes16(x0) | (pack_bytes16(x1) << 16);
    // only positions [sh, sh + total) of the step are its bits
    const int lo = max(sh - 32 * lane, 0), hi = min(sh + total - 32 * lane, 32);
    wv &= (hi >= 32 ? 0xffffffffu : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
    uint32_t *g = gbm + (b0 >> 5) + lane;
    const bool edge = (lane == 0 && sh != 0) || (lane == nw - 1 && ((sh + total) & 31) != 0);
    if (!edge) *g = wv;
    else if (wv) atomicOr(g, wv);
  }
  wave_lds_sync();
}

// One lane's string bytes [sp, sp + len) -> [op, op + len), a range no other
// lane writes: byte head up to a dword-aligned destination, then 16 bytes a
// pass from five dword loads issued together (v_alignbyte by the source skew),
// whole dwords stored, the last partial dword bytewise.  Source reads run up
// to 20 bytes past the string (device buffers carry kPad readable slack).
__device__ __forceinline__ void copy_str(const uint8_t *sp, uint8_t *op, int64_t len) {
  int64_t h = (int64_t)((4 - ((uintptr_t)op & 3)) & 3);
  if (h > len) h = len;
  for (int64_t b = 0; b < h; b++) op[b] = sp[b];
  const uintptr_t sa = (uintptr_t)(sp + h);
  const uint32_t *q = (const uint32_t *)(sa & ~(uintptr_t)3);
  const uint32_t sk = (uint32_t)(sa & 3);
  uint32_t *o = (uint32_t *)(op + h);
  int64_t rem = len - h;
  while (rem > 0) {
    uint32_t w[5];
#pragma unroll
    for (int i = 0; i < 5; i++) w[i] = q[i];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t x = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sk);
      const int64_t r = rem - 4 * i;
      if (r >= 4) o[i] = x;
      else if (r > 0) {
        uint8_t *ob = (uint8_t *)(o + i);
        for (int j = 0; j < (int)r; j++) ob[j] = (uint8_t)(x >> (8 * j));
      }
    }
    q += 4;
    o += 4;
    rem -= 16;
  }
}

// L bytes LDS -> LDS (byte addresses; the ranges of different lanes are
// disjoint): head bytes up to a dword-aligned destination, whole dwords from
// two aligned source dwords each (v_alignbyte), the tail a byte at a time.
__device__ __forceinline__ void lds_copy_bytes(uint32_t src, uint32_t dst, int L) {
  const int h = min((int)((4u - (dst & 3u)) & 3u), L);
#pragma unroll
  for (int b = 0; b < 3; b++)
    if (b < h) lds_st8(dst + b, lds_u8(src + b));
  int pos = h;
  for (; pos + 4 <= L; pos += 4) {
    const uint32_t q = (src + pos) & ~3u;
    lds_st32(dst + pos, __builtin_amdgcn_alignbyte(lds_u32(q + 4), lds_u32(q), (src + pos) & 3u));
  }
#pragma unroll
  for (int b = 0; b < 3; b++)
    if (pos + b < L) lds_st8(dst + pos + b, lds_u8(src + pos + b));
}

// A lane's four strings (device memory) -> an LDS stage (byte addresses
// dst[k]; disjoint ranges): the short ones (<= 16 bytes) from six aligned
// dwords each (global loads cannot alias the LDS stores, so the compiler
// may hoist them); longer ones a dword at a time.  Head bytes to an aligned LDS dword, whole dwords, tail bytes.
#define PQ_GLB1 __attribute__((address_space(1)))
__device__ __forceinline__ void copy_str4_to_lds(const uint8_t *const (&sp)[4], const uint32_t (&dst)[4],
                                                 const int (&ln)[4]) {
  // the loads of a pair of strings go out together, before either one's
  // stores (a wave per page has no other wave to hide their latency)
  uint32_t w2[2][6];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if ((k & 1) == 0) {
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const PQ_GLB1 uint32_t *q = (const PQ_GLB1 uint32_t *)((uintptr_t)sp[k + j] & ~(uintptr_t)3);
        const bool sh = ln[k + j] > 0 && ln[k + j] <= 16;
#pragma unroll
        for (int i = 0; i < 6; i++) w2[j][i] = sh ? q[i] : 0u;
      }
    }
    const int L = ln[k];
    if (L <= 0) continue;
    const uint32_t d = dst[k];
    const int h = min((int)((4u - (d & 3u)) & 3u), L);
    if (L <= 16) {
      uint32_t w[6];
#pragma unroll
      for (int i = 0; i < 6; i++) w[i] = w2[k & 1][i];
      const uint32_t sk = (uint32_t)((uintptr_t)sp[k] & 3);
      uint32_t r[5];
#pragma unroll
      for (int i = 0; i < 5; i++) r[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sk);  // string bytes 4 i ..
#pragma unroll
      for (int b = 0; b < 3; b++)
        if (b < h) lds_st8(d + b, r[0] >> (8 * b));
#pragma unroll
      for (int t = 0; t < 4; t++) {
        const int pos = h + 4 * t;
        const uint32_t u = __builtin_amdgcn_alignbyte(r[t + 1], r[t], (uint32_t)h);
        if (pos + 4 <= L) {
          lds_st32(d + pos, u);
        } else if (pos < L) {
#pragma unroll
          for (int b = 0; b < 3; b++)
            if (pos + b < L) lds_st8(d + pos + b, u >> (8 * b));
        }
      }
    } else {
      const PQ_GLB1 uint8_t *sb = (const PQ_GLB1 uint8_t *)(uintptr_t)sp[k];
      for (int b = 0; b < h; b++) lds_st8(d + b, sb[b]);
      int pos = h;
      for (; pos + 4 <= L; pos += 4) {
        const uintptr_t a = (uintptr_t)(sp[k] + pos);
        const PQ_GLB1 uint32_t *q = (const PQ_GLB1 uint32_t *)(a & ~(uintptr_t)3);
        lds_st32(d + pos, __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3)));
      }
      for (; pos < L; pos++) lds_st8(d + pos, sb[pos]);
    }
  }
}

// ===========================================================================
// k_plain_str: flat required PLAIN BYTE_ARRAY pages (type_bytearray.go:13-55)
// in items of PS_ITEM values, several waves per page.  k_prepare's length walk
// validated the page's chain and left each value's (offset, length) in the
// page's scratch; the chain is contiguous ([u32 len][bytes] per value), so the
// output position of value i inside the page is offset_i - 4 (i + 1) and any
// item can start on its own (k_decode<2> walks a page with one wave).  Item
// list: (page, first value) pairs.
// ===========================================================================
constexpr int PS_ITEM = PLAIN_STR_ITEM;
constexpr int PS_STAGE = 8192;  // staged source bytes per wave and step (longer steps: per-lane copies)
__global__ __launch_bounds__(256) void k_plain_str(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t st_all[4][PS_STAGE / 4 + 8];
  __shared__ int32_t ob_all[4][257];
  const int wv = (int)ufirst(threadIdx.x >> 6);
  const int gi = blockIdx.x * 4 + wv;
  if (gi >= a.nlist) return;
  const int lane = lane_id();
  const int page = ufirst(a.list[2 * gi]);
  const int32_t v0 = ufirst(a.list[2 * gi + 1]);
  if (page_status(a.status, page) != STATUS_OK) return;
  const PageDesc d = a.pages[page];
  const ColDesc c = a.cols[d.col];
  const PageInfo pi = a.info[page];
  const int32_t n = max(d.num_values, 0);
  const int32_t v1 = min(v0 + PS_ITEM, n);
  const uint8_t *vals = body_ptr(a, d, page) + pi.val_off;
  const int64_t vlen = pi.val_len, sb = pi.str_base;
  const int32_t *SO = a.lens + d.lens_base, *SL = SO + n;
  const int64_t slot0 = d.level_base;
  uint32_t *st = st_all[wv];
  int32_t *ob = ob_all[wv];
  const uint8_t *stb = (const uint8_t *)st;
  for (int32_t r = v0; r < v1; r += 256) {
    // value r + 64 k + lane: page-relative output offset out = offset - 4 (i + 1)
    const int32_t ns = min(256, v1 - r);
    int64_t o[4], l[4], out[4];
    bool oob = false;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int32_t i = r + 64 * k + lane;
      o[k] = l[k] = out[k] = 0;
      if (i < v1) {
        o[k] = (uint32_t)SO[i];
        l[k] = (uint32_t)SL[i];
        out[k] = o[k] - 4 * (int64_t)(i + 1);
        // the walk validated the chain: a pair outside the values section or
        // the page's output is stale scratch (never trusted for the copies)
        oob |= out[k] < 0 || o[k] + l[k] > vlen || out[k] + l[k] > pi.str_bytes;
      }
    }
    if (ballot(oob)) {
      set_status(a.status, page, ST_VALUES, E_EOF);
      return;
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int32_t i = r + 64 * k + lane;
      if (i < v1) c.str_offsets[slot0 + i + 1] = sb + out[k] + l[k];
    }
    // the step's output range from its first and last values (wave-uniform loads)
    const int32_t last = r + ns - 1;
    const int64_t P0 = (int64_t)(uint32_t)SO[r] - 4 * (int64_t)(r + 1);
    const int64_t P1 = (int64_t)(uint32_t)SO[last] + (int64_t)(uint32_t)SL[last] - 4 * (int64_t)(last + 1);
    const int64_t span = P1 - P0 + 4 * (int64_t)ns;  // source bytes: lengths + strings
    const uintptr_t src0 = (uintptr_t)(vals + (P0 + 4 * (int64_t)r));  // value r's length prefix
    const uintptr_t A = src0 & ~(uintptr_t)15;
    const int sh = (int)(src0 - A);
    if (span + sh + 16 <= PS_STAGE) {
      // 1. the step's source bytes into LDS (16-byte loads; the readable pad
      //    covers the last chunk) and the values' output starts
      for (int64_t off = 16 * (int64_t)lane; off < span + sh; off += 1024)
        *(uint4 *)(st + off / 4) = *(const uint4 *)(A + off);
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (64 * k + lane < ns) ob[64 * k + lane] = (int32_t)(out[k] - P0);
      if (lane == 0) ob[ns] = 0x7fffffff;
      wave_lds_sync();
      // 2. output dwords by their own lanes, 16 bytes a lane a pass, aligned to
      //    the output buffer: byte p (step-relative) of value v is staged byte
      //    p + 4 (v + 1) + sh.  Value of a byte: the last value starting at or
      //    before it (empty values share their successor's start)
      uint8_t *obase = c.values + sb;
      const int64_t q0 = (int64_t)(((uintptr_t)(obase + P0)) & ~(uintptr_t)15) - (int64_t)(uintptr_t)obase;  // page-relative
      const int32_t len = (int32_t)(P1 - P0);
      for (int64_t q = q0 + 16 * (int64_t)lane; q < P1; q += 1024) {
        const int32_t pr0 = (int32_t)(q - P0);  // step-relative start of this chunk (may be < 0)
        // binary search: last v with ob[v] <= max(pr0, 0)
        const int32_t key = max(pr0, 0);
        int lo = 0, hi = ns;  // ob[lo] <= key < ob[hi]
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (ob[mid] <= key) lo = mid;
          else hi = mid;
        }
        int v = lo;
        int32_t nxt = ob[v + 1];
        uint32_t w4[4];
        bool full = pr0 >= 0 && pr0 + 16 <= len;
#pragma unroll
        for (int dw = 0; dw < 4; dw++) {
          const int32_t p = pr0 + 4 * dw;
          uint32_t x = 0;
          if (p >= 0 && p + 3 < len) {
            while (nxt <= p) nxt = ob[++v + 1];
            if (nxt > p + 3) {  // four bytes of one value: an unaligned staged dword
              const int32_t idx = p + 4 * (v + 1) + sh;
              x = __builtin_amdgcn_alignbyte(st[(idx >> 2) + 1], st[idx >> 2], (uint32_t)(idx & 3));
            } else {
              for (int b = 0; b < 4; b++) {
                while (nxt <= p + b) nxt = ob[++v + 1];
                x |= (uint32_t)stb[p + b + 4 * (v + 1) + sh] << (8 * b);
              }
            }
          } else {
            for (int b = 0; b < 4; b++) {
              const int32_t pb = p + b;
              if (pb < 0 || pb >= len) continue;
              while (nxt <= pb) nxt = ob[++v + 1];
              x |= (uint32_t)stb[pb + 4 * (v + 1) + sh] << (8 * b);
            }
          }
          w4[dw] = x;
        }
        if (full) {
          *(uint4 *)(obase + q) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        } else {  // a step's edge chunk: only its own bytes (the neighbours' are another step's)
          for (int b = 0; b < 16; b++) {
            const int32_t pb = pr0 + b;
            if (pb >= 0 && pb < len) obase[q + b] = (uint8_t)(w4[b >> 2] >> (8 * (b & 3)));
          }
        }
      }
      wave_lds_sync();
    } else {
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int32_t i = r + 64 * k + lane;
        if (i < v1) copy_str(vals + o[k], c.values + sb + out[k], l[k]);
      }
    }
  }
}

// Decode one data page with one wavefront, 256 level entries per step, four
// consecutive entries per lane (page_v1.go:27-55 readValues + data_store.go
// semantics for validity / list offsets).  For flat columns the steps are
// aligned to 256 output slots so each lane owns a 16-byte-aligned slice of
// the values and whole validity words.
template <int KIND>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KIND == 1 ? 5 : KIND == 2 ? 3 : KIND == 3 ? 2 : KIND == 4 ? PQ_K4_WPE : KIND == 5 ? PQ_K5_WPE : 1))) void k_decode(KArgs a) {
  const int gi = blockIdx.x * 4 + (int)ufirst(threadIdx.x >> 6);
  if (gi >= a.nlist) return;
  const int lane = lane_id();
  // KIND 3 with a.parts: this wave decodes level entries [e_lo, e_hi) of its
  // page (a list page has ~80k entries: one wave per page left most of the
  // GPU idle, C4).  Rows, slots and values before e_lo are counted from
  // k_levels' level bytes, the key stream is skipped to the part's first
  // value.  A part after the first that meets an error marks the page
  // ST_REDO, and the redo launch decodes it whole for the reference's status.
  // KIND 2 with a.parts: entries [e_lo, e_hi) of a flat dictionary-string
  // page; the values before e_lo are counted from k_levels' level scratch,
  // their string bytes taken from k_prepare's prefix table (PageDesc::sp_base)
  // KIND 4 with a.parts: as KIND 2's, for a required column (the values
  // before e_lo are e_lo; the walked columns' dictionary pages, C5)
  const bool part = ((KIND == 3 || KIND == 2 || KIND == 4) && a.parts != nullptr) || KIND == 5;
  int page;
  int64_t e_lo = 0, e_hi = 0x7fffffffffffll;
  if (part) {
    page = ufirst(a.parts[3 * gi]);
    e_lo = ufirst(a.parts[3 * gi + 1]);
    e_hi = ufirst(a.parts[3 * gi + 2]);
  } else {
    page = ufirst(a.list[gi]);
  }
  if ((KIND == 3 || KIND == 2 || KIND == 4) && a.redo) {
    if (page_status(a.status, page) != make_status(ST_REDO, 0)) return;
    if (lane == 0) __hip_atomic_store(&a.status[page], STATUS_OK, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else if (page_status(a.status, page) != STATUS_OK) {
    return;
  }
  const PageDesc d = a.pages[page];
  if (d.dict >= 0 && page_status(a.status, d.dict) != STATUS_OK) return;
  if (KIND == 5 && (d.lvl_base < 0 || (d.enc != ENC_RLE_DICT && d.enc != ENC_PLAIN))) {
    // a page the host left whole (no level scratch, or DELTA values) rides in
    // the part list of a batch where other list pages were split: <5> has
    // neither the serial level walk nor the DELTA path, so the redo launch
    // (k_decode<3>, whole pages) decodes it
    set_status(a.status, page, ST_REDO, 0);
    return;
  }
  const ColDesc c = a.cols[d.col];
  const PageInfo pi = a.info[page];
  const int n = d.num_values;
  if (n == 0) return;

  const uint8_t *lvl = d.kind == PAGE_V1 ? body_ptr(a, d, page) : a.in + d.src;
  const uint8_t *vals = body_ptr(a, d, page) + pi.val_off;
  const int64_t vlen = pi.val_len;
  const int w = c.width;
  // KIND (the host routes pages by column class, none with level output but
  // KIND 0): 1 flat fixed-width (4/8-byte, non-BOOLEAN), 2 flat BYTE_ARRAY,
  // 3 nested (lists) of fixed-width values (5: the parts of such pages, whose
  // levels are always in k_levels' scratch and whose values are PLAIN or
  // dictionary: no serial level walk, no DELTA), 4 flat REQUIRED RLE_DICTIONARY
  // BYTE_ARRAY (<2>'s dictionary path alone: a fraction of its registers, so
  // more of these one-wave pages in flight), 0 everything else.  The other
  // paths drop out of each instance and its register budget.
  const bool flat = KIND == 1 || KIND == 2 || KIND == 4 || (KIND == 0 && c.max_rep == 0);
  const bool is_ba = KIND == 2 || KIND == 4 || (KIND == 0 && c.ptype == T_BYTE_ARRAY);
  const bool is_bool = KIND == 0 && c.ptype == T_BOOLEAN;
  const bool emit_lv = KIND == 0 && (c.flags & COL_EMIT_LEVELS);

  HybS rep, def;
  rep.init(lvl + pi.rep_off, pi.rep_len, bits_len(c.max_rep));
  def.init(lvl + pi.def_off, pi.def_len, bits_len(c.max_def));

  HybS keys;
  Delta dz;
  const PageDesc *dp = d.dict >= 0 ? &a.pages[d.dict] : nullptr;
  const uint8_t *dict_vals = nullptr;
  int64_t dict_n = 0, dict_base = 0;
  uint64_t delta_prev = 0;
  if (d.enc == ENC_RLE_DICT) {
    keys.init(vals + 1, vlen - 1, pi.idx_bw);
    if (dp) {
      dict_vals = body_ptr(a, *dp, d.dict);
      dict_n = dp->num_values;
      dict_base = dp->dict_base;
    }
  } else if (KIND != 2 && KIND != 4 && KIND != 5 && d.enc == ENC_DELTA_BP) {
    dz.init(vals, vlen, c.ptype == T_INT32);
    delta_prev = (uint64_t)dz.first;
  } else if (d.enc == ENC_RLE && is_bool) {
    // booleanRLEDecoder (type_boolean.go:97-117): u32 size, then a bit width 1
    // hybrid stream limited to it (checked >= 4 bytes in k_prepare)
    const uint32_t sz = load_u32_unaligned(vals);
    keys.init(vals + 4, min<int64_t>((int64_t)sz, vlen - 4), 1);
  }
  __shared__ BaLds ba_all[4];  // PLAIN BYTE_ARRAY length walk, one per wave
  BaLds &bl = ba_all[threadIdx.x >> 6];
  __shared__ __attribute__((aligned(16))) uint8_t bmw_all[4][320];  // nested-column bitmap bytes of a step
  uint8_t *bmw = bmw_all[threadIdx.x >> 6];
  // lists of 4/8-byte dictionary values (KIND 3): a dictionary of up to
  // DEC_DICT_LDS bytes is copied into the wave's LDS once, and the step's
  // gathers read it there instead of from L2 (one dependent global round trip
  // less a step; C4's 2,001-entry INT32 dictionaries)
  // (KIND 2, dictionary strings: the entries' (offset, length) pairs)
  constexpr int DLW = (KIND == 3 || KIND == 2 || KIND == 4 || KIND == 5) && PQ_DEC_DICT_LDS >= 8 ? PQ_DEC_DICT_LDS / 4 : 1;
  __shared__ uint32_t dlds_all[4][DLW];
  uint32_t *dlds = dlds_all[threadIdx.x >> 6];
  const int64_t dlb = KIND == 2 || KIND == 4 ? dict_n * 8 : dict_n * (int64_t)w;  // bytes staged
  const bool dict_lds = (KIND == 3 || KIND == 2 || KIND == 4 || KIND == 5) && DLW > 1 && dp && d.enc == ENC_RLE_DICT &&
                        (KIND == 2 || KIND == 4 || w == 4 || w == 8) && dlb <= (int64_t)DLW * 4;
  // (<4>: when the dictionary page's values fit beside the entry table they
  // are staged too, and a step's string bytes are assembled in the rest of
  // the area and stored as whole 16-byte chunks; see the outputs)
  const int64_t sb_off = (dlb + 15) & ~(int64_t)15;  // staged values' byte offset in dlds
  const int64_t dvb = KIND == 4 && dp ? (int64_t)dp->body_len : 0;
  const int64_t stg_off = (sb_off + dvb + 32 + 15) & ~(int64_t)15;  // the step's output bytes
  const bool str_lds = KIND == 4 && dict_lds && dvb > 0 && stg_off + 1024 <= (int64_t)DLW * 4;
  const uint32_t str_lb = lds_addr(dlds) + (uint32_t)sb_off, stg_lb = lds_addr(dlds) + (uint32_t)stg_off;
  const int64_t stg_cap = (int64_t)DLW * 4 - stg_off - 32;
  if (dict_lds) {
    const int nw = (int)((dlb + 3) >> 2);
    if (KIND == 2 || KIND == 4) {
      const uint32_t *ent = (const uint32_t *)(a.dict_ent + dict_base);
      for (int i = lane; i < nw; i += 64) dlds[i] = ent[i];
      if (str_lds)
        for (int i = lane; i < (int)((dvb + 3) >> 2) + 2; i += 64)
          dlds[sb_off / 4 + i] = load_u32_unaligned(dict_vals + 4 * (int64_t)i);
    } else {
      for (int i = lane; i < nw; i += 64) dlds[i] = load_u32_unaligned(dict_vals + 4 * (int64_t)i);
    }
    wave_lds_sync();
  }
  int64_t spos = 0;
  // DELTA strings: lengths decoded and validated by k_prepare (scratch); suffix
  // bytes start at str_data.  DELTA_BYTE_ARRAY bytes are written by k_dba.
  // FIXED_LEN_BYTE_ARRAY DELTA_BYTE_ARRAY (KIND 0 only): slots zeroed here,
  // the values written by k_dba
  const bool fl_dba = KIND == 0 && c.ptype == T_FLBA && d.enc == ENC_DELTA_BA && d.lens_base >= 0;
  const bool dstr = (KIND != 4 && is_ba && (d.enc == ENC_DELTA_LBA || d.enc == ENC_DELTA_BA) && d.lens_base >= 0) || fl_dba;
  const bool defer_bytes = dstr && d.enc == ENC_DELTA_BA;
  int64_t dpos = pi.str_data;

  const int64_t slot_base = flat ? d.level_base : pi.slot_base;
  int64_t e0 = 0, slot_run = 0, row_run = 0, nn_run = 0, str_run = pi.str_base;
  uint32_t err = E_OK, err_stage = 0;
  const int64_t e_end = part ? min<int64_t>(e_hi, (int64_t)n) : (int64_t)n;
  if ((KIND == 2 || KIND == 4) && part && e_lo > 0) {
    // (only dictionary pages with a prefix table and, nullable, a level
    // scratch are split)
    if (d.sp_base < 0 || d.enc != ENC_RLE_DICT || (KIND == 2 && !(d.lvl_bits || d.lvl_base >= 0)) ||
        (KIND == 4 && c.max_def != 0)) {
      set_status(a.status, page, ST_REDO, 0);
      return;
    }
    int64_t cn = 0;  // values (def == max_def) among entries [0, e_lo)
    if (KIND == 4) {
      cn = lane == 0 ? e_lo : 0;  // required: every entry is a value
    } else if (d.lvl_bits) {
      const uint32_t *lw = (const uint32_t *)(a.lvl + d.lvl_base);
      const int64_t nw = e_lo >> 5;
      for (int64_t w = lane; w < nw; w += 64) cn += __popc(lw[w]);
      if (lane == 0 && (e_lo & 31)) cn += __popc(lw[nw] & ((1u << (e_lo & 31)) - 1u));
    } else {
      const uint8_t *ld = a.lvl + d.lvl_base;
      for (int64_t b = lane; b < e_lo; b += 64) cn += (int)ld[b] == c.max_def;
    }
    nn_run = wave_sum32((int32_t)cn);
    row_run = e_lo;
    slot_run = e_lo;
    e0 = e_lo;
    // the string bytes of values [0, nn_run): the table's entry at the 256-value
    // step below, then the keys of the step's first nn_run & 255 values
    const int64_t q = nn_run & ~(int64_t)255;
    if (keys.skip(q) != E_OK) {
      set_status(a.status, page, ST_REDO, 0);
      return;
    }
    int64_t sb = a.str_pre[d.sp_base + (q >> 8)];
    const int rem = (int)(nn_run - q);
    if (rem > 0) {
      uint32_t k4[4];
      if (keys.next4(rem, k4) != E_OK) {
        set_status(a.status, page, ST_REDO, 0);
        return;
      }
      int64_t l = 0;
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (4 * lane + j < rem && (int64_t)k4[j] < dict_n)
          l += (int64_t)(uint32_t)(a.dict_ent[dict_base + k4[j]] & 0xffffffffu);
      sb += wave_sum64(l);
    }
    str_run = pi.str_base + sb;
  } else if (part && e_lo > 0 && d.part0 >= 0) {
    // rows (rep 0), slots (def >= rep_def) and values (def == max_def) before
    // the part: counted by k_levels
    row_run = ufirst(a.part_pre[4 * gi]);
    slot_run = ufirst(a.part_pre[4 * gi + 1]);
    nn_run = ufirst(a.part_pre[4 * gi + 2]);
    e0 = e_lo;
    if (d.enc == ENC_RLE_DICT && keys.skip(nn_run) != E_OK) {
      set_status(a.status, page, ST_REDO, 0);
      return;
    }
  } else if (part && e_lo > 0) {
    // rows (rep 0), slots (def >= rep_def) and values (def == max_def) of the
    // entries before the part: 16 level bytes of each stream a lane a pass
    const uint8_t *lr = a.lvl + d.lvl_base, *ld = lr + n;
    const uint32_t dsh = (uint32_t)((uintptr_t)ld & 3);
    const uint32_t *la = (const uint32_t *)lr, *da = (const uint32_t *)((uintptr_t)ld & ~(uintptr_t)3);
    int32_t cr = 0, cs = 0, cn = 0;
    for (int64_t b = 16 * (int64_t)lane; b < e_lo; b += 1024) {
      uint32_t rw[4], dw[5];
#pragma unroll
      for (int q = 0; q < 4; q++) rw[q] = la[(b >> 2) + q];
#pragma unroll
      for (int q = 0; q < 5; q++) dw[q] = da[(b >> 2) + q];
#pragma unroll
      for (int q = 0; q < 16; q++) {
        const bool in = b + q < e_lo;
        const uint32_t rv = __builtin_amdgcn_ubfe(rw[q >> 2], 8 * (q & 3), 8);
        const uint32_t dx = __builtin_amdgcn_alignbyte(dw[(q >> 2) + 1], dw[q >> 2], dsh);
        const uint32_t dv = __builtin_amdgcn_ubfe(dx, 8 * (q & 3), 8);
        cr += in && rv == 0;
        cs += in && (int)dv >= c.rep_def;
        cn += in && (int)dv == c.max_def;
      }
    }
    row_run = wave_sum32(cr);
    slot_run = wave_sum32(cs);
    nn_run = wave_sum32(cn);
    e0 = e_lo;
    if (d.enc == ENC_RLE_DICT && keys.skip(nn_run) != E_OK) {
      set_status(a.status, page, ST_REDO, 0);
      return;
    }
  }

  // the level scratch of the step at e: its 4 entries of this lane, packed —
  // bitmap: the def == max_def bits; bytes: rep bytes (low word), def bytes.
  // Loaded a step ahead (PQ_LV_AHEAD): the next step's level loads are in
  // flight beside this step's key / dictionary / value loads, so a step waits
  // on one round trip instead of two
  auto step_cnt = [&](int64_t e) { return (int)min<int64_t>(n - e, flat ? 256 - ((slot_base + e) & 255) : 256); };
  auto lv_load = [&](int64_t e) -> uint64_t {
    if (e >= e_end) return 0;
    const int ce = step_cnt(e);
    if (d.lvl_bits) {
      const uint32_t *lw = (const uint32_t *)(a.lvl + d.lvl_base);
      const int64_t b = e + 4 * lane;
      const uint64_t two = 4 * lane < ce ? (uint64_t)lw[b >> 5] | ((uint64_t)lw[(b >> 5) + 1] << 32) : 0ull;
      return (two >> (b & 31)) & 15u;
    }
    if (d.lvl_base < 0) return 0;
    const uint8_t *lr = a.lvl + d.lvl_base + e, *ld = lr + (c.max_rep > 0 ? (int64_t)n : 0);
    uint32_t pr = 0, pd = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int j = 4 * lane + k;
      if (j < ce) {
        if (!flat) pr |= (uint32_t)lr[j] << (8 * k);
        pd |= (uint32_t)ld[j] << (8 * k);
      }
    }
    return (uint64_t)pr | ((uint64_t)pd << 32);
  };
  uint64_t lv_next = PQ_LV_AHEAD ? lv_load(e0) : 0;
#ifdef PQ_DEC_STAMPS
  uint64_t dacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t dprev = __builtin_amdgcn_s_memtime();
  const uint64_t dt0 = dprev;
#endif
  while (e0 < e_end) {
    DEC_T(-1);
    const int cnt = step_cnt(e0);
    uint32_t r[4] = {0, 0, 0, 0}, dl[4] = {0, 0, 0, 0};
    const uint64_t lv = PQ_LV_AHEAD ? lv_next : lv_load(e0);
    if (PQ_LV_AHEAD) lv_next = lv_load(e0 + cnt);
    if (d.lvl_bits) {  // k_levels' bitmap (flat): def == max_def or not
#pragma unroll
      for (int k = 0; k < 4; k++) dl[k] = 4 * lane + k < cnt && ((lv >> k) & 1u) ? (uint32_t)c.max_def : 0u;
    } else if (d.lvl_base >= 0) {  // decoded (and checked) by k_levels
#pragma unroll
      for (int k = 0; k < 4; k++) {
        r[k] = (uint32_t)(lv >> (8 * k)) & 0xffu;
        dl[k] = (uint32_t)(lv >> (32 + 8 * k)) & 0xffu;
      }
    } else if (KIND != 4 && KIND != 5) {  // (<4>: required, no levels; <5>: level scratch always)
      if (!flat) {
        err = rep.next4(cnt, r);
        if (err) {
          err_stage = ST_REP;
          break;
        }
      }
      if (c.max_def > 0) {
        err = def.next4(cnt, dl);
        if (err) {
          err_stage = ST_DEF;
          break;
        }
      }
    }
    bool act[4], valid[4], slot[4];
    int nv = 0, ns = 0, nr = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      act[k] = 4 * lane + k < cnt;
      valid[k] = act[k] && (int)dl[k] == c.max_def;
      slot[k] = act[k] && (flat || (int)dl[k] >= c.rep_def);
      nv += valid[k];
      ns += slot[k];
      nr += act[k] && r[k] == 0;
    }
    int32_t m, mslots, mrows;
    const int32_t vbase = wave_excl_scan32(nv, &m);       // dense rank of my first valid entry
    const int32_t sbase = flat ? 4 * lane : wave_excl_scan32(ns, &mslots);
    if (flat) mslots = cnt;
    const bool dense = m == cnt;  // no nulls in this step: entry j is dense value j

    if (emit_lv) {
#pragma unroll
      for (int k = 0; k < 4; k++)
        if (act[k]) {
          c.def_out[d.level_base + e0 + 4 * lane + k] = (uint8_t)dl[k];
          c.rep_out[d.level_base + e0 + 4 * lane + k] = (uint8_t)r[k];
        }
    }
    if (!flat) {  // rows start where rep == 0 (data_store.go:188-202)
      const int32_t rbase = wave_excl_scan32(nr, &mrows);
      int ri = 0, si = 0;
      int rrel[4];
      bool lv[4], rp[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        rrel[k] = rbase + ri;
        rp[k] = act[k] && r[k] == 0;
        lv[k] = act[k] && r[k] == 0 && (int)dl[k] >= c.rep_def - 1;
        if (act[k] && r[k] == 0) {
          int64_t row = pi.row_base + row_run + rbase + ri;
          if (c.list_offsets) c.list_offsets[row] = (int32_t)(slot_base + slot_run + sbase + si);
          ri++;
        }
        si += slot[k];
      }
      if (c.list_validity) wave_bitmap(bmw, c.list_validity, pi.row_base + row_run, mrows, rrel, rp, lv);
      row_run += mrows;
    }

    DEC_T(0);  // levels, counts, scans
    // ---- the m dense values of this step, in dense order (value j: lane j>>2, element j&3) ----
    uint64_t v[4] = {0, 0, 0, 0};
    int64_t soff[4] = {0, 0, 0, 0}, slen[4] = {0, 0, 0, 0};
    const uint8_t *sbase_ptr = nullptr;
    if (m > 0) {
      if (is_bool) {
        uint32_t bv[4] = {0, 0, 0, 0};
        if (d.enc == ENC_RLE) {  // type_boolean.go:106-117
          uint32_t kk[4];
          err = keys.next4(m, kk);
          if (err) {
            err_stage = ST_VALUES;
            break;
          }
          int vi = 0;
#pragma unroll
          for (int k = 0; k < 4; k++) {
            bv[k] = dense ? kk[k] : pick4(kk, valid[k] ? vbase + vi : 0);
            vi += valid[k];
          }
        } else {  // PLAIN, type_boolean.go:43-68: a byte per 8 values, LSB first
          if ((nn_run + m + 7) >> 3 > vlen) {
            err = E_EOF;
            err_stage = ST_VALUES;
            break;
          }
          int vi = 0;
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (valid[k]) {
              const int64_t jv = nn_run + vbase + vi;
              bv[k] = (vals[jv >> 3] >> (jv & 7)) & 1u;
              vi++;
            }
        }
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = bv[k] == 1;
      } else if (d.enc == ENC_PLAIN && !is_ba) {
        if ((nn_run + m) * (int64_t)w > vlen) {
          err = E_EOF;
          err_stage = ST_VALUES;
          break;
        }
        if (w == 4 || w == 8) {
          int vi = 0;
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (valid[k]) {
              const uint8_t *vp = vals + (nn_run + vbase + vi) * (int64_t)w;
              v[k] = w == 4 ? (uint64_t)load_u32_unaligned(vp) : load_u64_unaligned(vp);
              vi++;
            }
        }
      } else if (d.enc == ENC_RLE_DICT) {
        if (!dp) {
          err = E_DICT;
          err_stage = ST_VALUES;
          break;
        }
        uint32_t kk[4];
        err = keys.next4(m, kk);
        DEC_T(1);  // the key stream
        if (err) {
          // decodeValues checks each key as it reads it (type_dict.go:44-53): an
          // out-of-range key among those read before the stream error comes first
          bool oob = false;
#pragma unroll
          for (int k = 0; k < 4; k++) oob |= 4 * lane + k < keys.got && (int64_t)kk[k] >= dict_n;
          if (ballot(oob)) err = E_DICT;
          err_stage = ST_VALUES;
          break;
        }
        uint32_t key[4];
        if (dense) {
#pragma unroll
          for (int k = 0; k < 4; k++) key[k] = kk[k];
        } else {
          int vi = 0;
#pragma unroll
          for (int k = 0; k < 4; k++) {
            key[k] = pick4(kk, valid[k] ? vbase + vi : 0);
            vi += valid[k];
          }
        }
        bool bad = false;
#pragma unroll
        for (int k = 0; k < 4; k++) bad |= valid[k] && (int64_t)key[k] >= dict_n;
        if (ballot(bad)) {
          err = E_DICT;
          err_stage = ST_VALUES;
          break;
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (valid[k]) {
            if (is_ba) {
              const uint64_t ent = dict_lds ? ((uint64_t)dlds[2 * key[k]] | ((uint64_t)dlds[2 * key[k] + 1] << 32))
                                            : a.dict_ent[dict_base + key[k]];
              soff[k] = (int64_t)(ent >> 32);
              slen[k] = (int64_t)(ent & 0xffffffffu);
            } else if (w == 4) {
              v[k] = dict_lds ? dlds[key[k]] : load_u32_unaligned(dict_vals + (int64_t)key[k] * 4);
            } else if (w == 8) {
              v[k] = dict_lds ? ((uint64_t)dlds[2 * key[k]] | ((uint64_t)dlds[2 * key[k] + 1] << 32))
                              : load_u64_unaligned(dict_vals + (int64_t)key[k] * 8);
            } else {
              soff[k] = (int64_t)key[k] * w;
            }
          }
        sbase_ptr = dict_vals;
      } else if (KIND != 2 && KIND != 4 && KIND != 5 && d.enc == ENC_DELTA_BP) {
        uint64_t dv[4];
        err = dz.template next4<KIND != 3>(m, dv);  // <3> is register-bound
        if (err) {
          err_stage = ST_VALUES;
          break;
        }
        // v[j] = prev + sum of the deltas before j (wrapping, deltabp_decoder.go:327-333)
        uint64_t loc = dv[0] + dv[1] + dv[2] + dv[3];
        uint64_t incl = wave_incl_scan_u64(loc);
        uint64_t base = delta_prev + (incl - loc);
        uint64_t val[4];
        val[0] = base;
        val[1] = base + dv[0];
        val[2] = val[1] + dv[1];
        val[3] = val[2] + dv[2];
        delta_prev += shfl64(incl, 63);
        if (dense) {
#pragma unroll
          for (int k = 0; k < 4; k++) v[k] = val[k];
        } else {
          int vi = 0;
#pragma unroll
          for (int k = 0; k < 4; k++) {
            v[k] = pick4_64(val, valid[k] ? vbase + vi : 0);
            vi += valid[k];
          }
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (c.ptype == T_INT32) v[k] &= 0xffffffffull;
      } else if (dstr) {
        // value j -> lane j>>2, element j&3: suffix lengths S, prefix lengths P
        const int32_t nvp = max(n, 0);
        const int32_t *S = a.lens + d.lens_base, *P = S + nvp;
        uint32_t eo[4] = {0, 0, 0, 0}, el[4] = {0, 0, 0, 0};
        int64_t sl4[4];
        int64_t loc = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int t = 4 * lane + k;
          const int64_t i = nn_run + t;
          sl4[k] = t < m ? (int64_t)S[i] : 0;
          int64_t vl = sl4[k];
          if (d.enc == ENC_DELTA_BA && t < m) {
            const int32_t pl = P[i];
            vl += pl > 0 ? pl : 0;
          }
          el[k] = (uint32_t)vl;
          loc += sl4[k];
        }
        const int64_t incl = wave_incl_scan64(loc);
        int64_t o = dpos + (incl - loc);
#pragma unroll
        for (int k = 0; k < 4; k++) {
          eo[k] = (uint32_t)o;
          o += sl4[k];
        }
        dpos += (int64_t)shfl64((uint64_t)incl, 63);
        int vi = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          int j = valid[k] ? vbase + vi : 0;
          uint32_t oo = dense ? eo[k] : pick4(eo, j), ll = dense ? el[k] : pick4(el, j);
          if (valid[k]) {
            soff[k] = oo;
            slen[k] = ll;
          }
          vi += valid[k];
        }
        sbase_ptr = vals;
      } else if (KIND != 4 && d.enc == ENC_PLAIN && is_ba && d.lens_base >= 0) {
        // offsets and lengths left by k_prepare's walk (which validated the
        // whole chain); dense value nn_run + j -> lane j>>2, element j&3
        const int32_t nvp = max(n, 0);
        const int32_t *SO = a.lens + d.lens_base, *SL = SO + nvp;
        uint32_t eo[4] = {0, 0, 0, 0}, el[4] = {0, 0, 0, 0};
        bool oob = false;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int t = 4 * lane + k;
          if (t < m) {
            eo[k] = (uint32_t)SO[nn_run + t];
            el[k] = (uint32_t)SL[nn_run + t];
            oob |= (int64_t)eo[k] + (int64_t)el[k] > vlen;
          }
        }
        // the walk validated the chain: a pair outside the values section is
        // stale scratch (never trusted for the copies below)
        if (ballot(oob)) {
          err = E_EOF;
          err_stage = ST_VALUES;
          break;
        }
        int vi = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          int j = valid[k] ? vbase + vi : 0;
          uint32_t o = dense ? eo[k] : pick4(eo, j), l = dense ? el[k] : pick4(el, j);
          if (valid[k]) {
            soff[k] = o;
            slen[k] = l;
          }
          vi += valid[k];
        }
        sbase_ptr = vals;
      } else if (KIND != 4 && d.enc == ENC_PLAIN && is_ba) {
        // length chain (type_bytearray.go:24-45) by pointer jumping, 64 entries a
        // batch; entry j of the step goes to lane j>>2, element j&3
        uint32_t eo[4] = {0, 0, 0, 0}, el[4] = {0, 0, 0, 0};
        int64_t adv = 0;
        err = ba_walk<BA_WIN>(vals + spos, vlen - spos, m, bl.win, bl.jt[0], bl.jt[1],
                              [&](int64_t first, int ln, int64_t voff, int32_t l, int cnt) {
                                const uint32_t vo = (uint32_t)(spos + voff);
#pragma unroll
                                for (int k = 0; k < 4; k++) {
                                  const int src = 4 * lane + k - (int)first;
                                  const uint32_t o2 = (uint32_t)__shfl((int)vo, src & 63);
                                  const uint32_t l2 = (uint32_t)__shfl((int)l, src & 63);
                                  if (src >= 0 && src < cnt) {
                                    eo[k] = o2;
                                    el[k] = l2;
                                  }
                                }
                                adv = (int64_t)shfl64((uint64_t)(voff + l), cnt - 1);
                              });
        if (err) {
          err_stage = ST_VALUES;
          break;
        }
        spos += adv;
        int vi = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          int j = valid[k] ? vbase + vi : 0;
          uint32_t o = dense ? eo[k] : pick4(eo, j), l = dense ? el[k] : pick4(el, j);
          if (valid[k]) {
            soff[k] = o;
            slen[k] = l;
          }
          vi += valid[k];
        }
        sbase_ptr = vals;
      } else {
        err = E_UNSUPPORTED;
        err_stage = ST_VALUES;
        break;
      }
    }

    DEC_T(2);  // key checks, dictionary entries
    // ---- outputs ----
    if (is_ba) {
      int64_t ll[4], tot = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        ll[k] = valid[k] ? slen[k] : 0;
        tot += ll[k];
      }
      int64_t incl = wave_incl_scan64(tot);
      int64_t start = str_run + incl - tot;
      int si = 0;
      const int64_t T = (int64_t)shfl64((uint64_t)incl, 63);  // the step's string bytes
      // <2>'s stage: the PLAIN walk's LDS, free on this path, from 16 bytes in
      // (a chunk's first read reaches up to 15 bytes before the step's bytes)
      constexpr int64_t BA_STG = (int64_t)sizeof(BaLds) - 48;
      if (KIND == 2 && d.enc == ENC_RLE_DICT && !defer_bytes && T <= BA_STG) {
        // Dictionary strings (any dictionary size, nulls allowed): each lane
        // copies its values' bytes from the dictionary into an LDS stage,
        // then the step's output is stored as whole 16-byte chunks (C4's
        // 1,000-word dictionary column: its per-string byte / dword stores
        // were 54 % of a step, tools/diag_decode.py)
        const int64_t P0 = str_run;
        const uint32_t stg = lds_addr(&bl) + 16u;
        const uint8_t *cs[4];
        uint32_t cd[4];
        int cl[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          cs[k] = sbase_ptr + (valid[k] ? soff[k] : 0);
          cd[k] = stg + (uint32_t)(start - P0);
          cl[k] = slot[k] && valid[k] ? (int)ll[k] : 0;
          if (slot[k]) {
            start += ll[k];
            c.str_offsets[slot_base + slot_run + sbase + si + 1] = start;
            si++;
          }
        }
        copy_str4_to_lds(cs, cd, cl);
        wave_lds_sync();
        uint8_t *ov = c.values;
        const int64_t P1 = P0 + T;
        const int64_t q0 = (int64_t)(((uintptr_t)(ov + P0)) & ~(uintptr_t)15) - (int64_t)(uintptr_t)ov;
        for (int64_t q = q0 + 16 * (int64_t)lane; q < P1; q += 1024) {
          const int32_t pr0 = (int32_t)(q - P0);
          const uint32_t sa = stg + (uint32_t)(pr0 + 16) - 16u;
          const uint32_t s4 = sa & ~3u;
          uint32_t w[5];
#pragma unroll
          for (int i = 0; i < 5; i++) w[i] = lds_u32(s4 + 4 * i);
          uint32_t x[4];
#pragma unroll
          for (int i = 0; i < 4; i++) x[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sa & 3u);
          if (pr0 >= 0 && pr0 + 16 <= (int32_t)T) {
            *(uint4 *)(ov + q) = make_uint4(x[0], x[1], x[2], x[3]);
          } else {
            for (int b = 0; b < 16; b++) {
              const int32_t pb = pr0 + b;
              if (pb >= 0 && pb < (int32_t)T) ov[q + b] = (uint8_t)(x[b >> 2] >> (8 * (b & 3)));
            }
          }
        }
        wave_lds_sync();
      } else if (KIND == 4 && str_lds && T <= stg_cap) {
        // Small dictionary staged in LDS: each lane assembles its values'
        // bytes in the LDS stage (LDS to LDS), then the step's output goes
        // out as whole 16-byte chunks, a chunk a lane.  Storing each string
        // a byte / dword at a time from its lane took ~10 scattered store
        // requests a value, which bounded C5's dictionary-string pages.
        const int64_t P0 = str_run;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          if (slot[k]) {
            if (valid[k] && ll[k] > 0) lds_copy_bytes(str_lb + (uint32_t)soff[k], stg_lb + (uint32_t)(start - P0), (int)ll[k]);
            start += ll[k];
            c.str_offsets[slot_base + slot_run + sbase + si + 1] = start;
            si++;
          }
        }
        wave_lds_sync();
        uint8_t *ov = c.values;
        const int64_t P1 = P0 + T;
        const int64_t q0 = (int64_t)(((uintptr_t)(ov + P0)) & ~(uintptr_t)15) - (int64_t)(uintptr_t)ov;
        for (int64_t q = q0 + 16 * (int64_t)lane; q < P1; q += 1024) {
          const int32_t pr0 = (int32_t)(q - P0);  // step-relative start of this chunk (> -16)
          const uint32_t sa = stg_lb + (uint32_t)(pr0 + 16) - 16u;  // (the stage has 16 bytes before it)
          const uint32_t s4 = sa & ~3u;
          uint32_t w[5];
#pragma unroll
          for (int i = 0; i < 5; i++) w[i] = lds_u32(s4 + 4 * i);
          uint32_t x[4];
#pragma unroll
          for (int i = 0; i < 4; i++) x[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sa & 3u);
          if (pr0 >= 0 && pr0 + 16 <= (int32_t)T) {
            *(uint4 *)(ov + q) = make_uint4(x[0], x[1], x[2], x[3]);
          } else {  // an edge chunk: only the step's own bytes
            for (int b = 0; b < 16; b++) {
              const int32_t pb = pr0 + b;
              if (pb >= 0 && pb < (int32_t)T) ov[q + b] = (uint8_t)(x[b >> 2] >> (8 * (b & 3)));
            }
          }
        }
        wave_lds_sync();
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++) {
          if (slot[k]) {
            start += ll[k];
            c.str_offsets[slot_base + slot_run + sbase + si + 1] = start;
            if (valid[k] && !defer_bytes) copy_str(sbase_ptr + soff[k], c.values + start - ll[k], ll[k]);
            si++;
          }
        }
      }
      str_run += T;
    } else if (flat && (w == 4 || w == 8)) {
      const int64_t s0 = slot_base + slot_run + 4 * lane;  // my four slots
      uint64_t o[4];
#pragma unroll
      for (int k = 0; k < 4; k++) o[k] = valid[k] ? v[k] : 0;
      if (act[3] && (s0 & 3) == 0) {
        if (w == 4) {
          *(uint4 *)(c.values + s0 * 4) = make_uint4((uint32_t)o[0], (uint32_t)o[1], (uint32_t)o[2], (uint32_t)o[3]);
        } else {
          *(uint4 *)(c.values + s0 * 8) = make_uint4((uint32_t)o[0], (uint32_t)(o[0] >> 32), (uint32_t)o[1], (uint32_t)(o[1] >> 32));
          *(uint4 *)(c.values + s0 * 8 + 16) = make_uint4((uint32_t)o[2], (uint32_t)(o[2] >> 32), (uint32_t)o[3], (uint32_t)(o[3] >> 32));
        }
      } else {
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (act[k]) {
            if (w == 4) *(uint32_t *)(c.values + (s0 + k) * 4) = (uint32_t)o[k];
            else *(uint64_t *)(c.values + (s0 + k) * 8) = o[k];
          }
      }
    } else {
      int si = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (slot[k]) {
          int64_t sl = slot_base + slot_run + sbase + si;
          if (is_bool) c.values[sl] = valid[k] ? (uint8_t)v[k] : (uint8_t)0;
          else if (w == 4) *(uint32_t *)(c.values + sl * 4) = valid[k] ? (uint32_t)v[k] : 0u;
          else if (w == 8) *(uint64_t *)(c.values + sl * 8) = valid[k] ? v[k] : 0ull;
          else {
            uint8_t *op = c.values + sl * (int64_t)w;
            const uint8_t *sp = d.enc == ENC_PLAIN ? vals + (nn_run + vbase) * (int64_t)w : sbase_ptr + soff[k];
            if (valid[k] && d.enc == ENC_PLAIN) {
              int vi = 0;
              for (int q = 0; q < k; q++) vi += valid[q];
              sp = vals + (nn_run + vbase + vi) * (int64_t)w;
            }
            for (int b = 0; b < w; b++) op[b] = valid[k] && !fl_dba ? sp[b] : 0;
          }
          si++;
        }
      }
    }
    DEC_T(3);  // string / value outputs
    if (KIND != 4 && c.max_def > 0) {
      if (flat) {
        // 4 bits per lane -> 32-bit words owned by lanes 8q (this step covers 256 aligned slots
        // except a page's first/last step, which share words with neighbouring pages)
        uint32_t nib = (valid[0] ? 1u : 0u) | (valid[1] ? 2u : 0u) | (valid[2] ? 4u : 0u) | (valid[3] ? 8u : 0u);
        uint32_t word = nib << (4 * (lane & 7));
        word |= __shfl_xor(word, 1);
        word |= __shfl_xor(word, 2);
        word |= __shfl_xor(word, 4);
        const int64_t sbit = slot_base + slot_run;  // first slot of this step
        if ((lane & 7) == 0 && 4 * lane < cnt) {
          const int64_t b0 = sbit + 4 * lane;  // first bit of my word
          const bool whole = (b0 & 31) == 0 && 4 * lane + 32 <= cnt;
          if (whole) c.validity[b0 >> 5] = word;
          else {
            int sh = (int)(b0 & 31);
            uint64_t wv = (uint64_t)word << sh;
            if ((uint32_t)wv) atomicOr(&c.validity[b0 >> 5], (uint32_t)wv);
            if ((uint32_t)(wv >> 32)) atomicOr(&c.validity[(b0 >> 5) + 1], (uint32_t)(wv >> 32));
          }
        }
      } else {
        int si = 0, srel[4];
        bool sv[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          srel[k] = sbase + si;
          sv[k] = slot[k] && valid[k];
          si += slot[k];
        }
        wave_bitmap(bmw, c.validity, slot_base + slot_run, mslots, srel, slot, sv);
      }
    }
    slot_run += mslots;
    nn_run += m;
    DEC_T(4);  // validity bitmaps, counters
    e0 += cnt;
  }
#ifdef PQ_DEC_STAMPS
  if ((KIND == 1 || KIND == 2 || KIND == 4 || KIND == 5) && a.dbg2 && lane < 8) {
    const uint64_t mine = lane == 0 ? dacc[0] : lane == 1 ? dacc[1] : lane == 2 ? dacc[2] : lane == 3 ? dacc[3]
                                                                      : lane == 4 ? dacc[4] : 0ull;
    atomicAdd((unsigned long long *)&a.dbg2[(size_t)page * 8 + lane], (unsigned long long)mine);
  }
  if ((KIND == 1 || KIND == 2 || KIND == 4 || KIND == 5) && a.dbg2 && lane == 0) atomicAdd((unsigned long long *)&a.dbg2[(size_t)page * 8 + 7], 1ull);
  if ((KIND == 1 || KIND == 2 || KIND == 4 || KIND == 5) && a.dbg && lane == 0) {
    atomicAdd((unsigned long long *)&a.dbg[(size_t)page * 4 + 0], (unsigned long long)(__builtin_amdgcn_s_memtime() - dt0));
    atomicMax((unsigned long long *)&a.dbg[(size_t)page * 4 + 1], (unsigned long long)(__builtin_amdgcn_s_memtime() - dt0));
    a.dbg[(size_t)page * 4 + 2] = (uint64_t)n;
    a.dbg[(size_t)page * 4 + 3] = (uint64_t)e0;
  }
#endif
  // a later-found level error can outrank this one: k_level_check re-walks
  // the earlier level streams (the reference decodes all rep levels, then all
  // def levels, then the values, page_v1.go:37-52)
  if (err) {
    if (part && e_lo > 0) set_status(a.status, page, ST_REDO, 0);  // the redo launch finds the first error
    else set_status(a.status, page, err_stage, err);
  }
}

// Wave copy of up to MAXC KiB, in passes of 4 KiB with every load of a pass
// issued before its stores (16-byte aligned stores after a short head,
// funnel-shifted dword loads).
template <int MAXC>
__device__ __forceinline__ void copy_tile(const uint8_t *s, uint8_t *D, int64_t len, int lane) {
  constexpr int PASS = 4;
  int64_t head = (int64_t)((16 - ((uintptr_t)D & 15)) & 15);
  if (head > len) head = len;
  if (lane < head) D[lane] = s[lane];
  const int64_t body = (len - head) >> 4;
  const uintptr_t S = (uintptr_t)(s + head);
  const uintptr_t D16 = (uintptr_t)(D + head);
  const uint32_t skew = (uint32_t)(S & 3);
  const uintptr_t SA = S & ~(uintptr_t)3;
  for (int i0 = 0; i0 < MAXC && 64 * i0 < body; i0 += PASS) {
    uint4 x[PASS];
    uint32_t x4[PASS];
#pragma unroll
    for (int i = 0; i < PASS; i++) {
      const int64_t c = lane + 64 * (i0 + i);
      const uintptr_t src = SA + 16 * (uintptr_t)(c < body ? c : 0);
      x[i] = make_uint4(gld32(src), gld32(src + 4), gld32(src + 8), gld32(src + 12));
      x4[i] = gld32(src + 16);
    }
#pragma unroll
    for (int i = 0; i < PASS; i++) {
      const int64_t c = lane + 64 * (i0 + i);
      if (c < body) {
        uint4 o;
        o.x = __builtin_amdgcn_alignbyte(x[i].y, x[i].x, skew);
        o.y = __builtin_amdgcn_alignbyte(x[i].z, x[i].y, skew);
        o.z = __builtin_amdgcn_alignbyte(x[i].w, x[i].z, skew);
        o.w = __builtin_amdgcn_alignbyte(x4[i], x[i].w, skew);
        gst128(D16 + 16 * (uintptr_t)c, o);
      }
    }
  }
  const int64_t done = head + body * 16;
  if (lane < len - done) D[done + lane] = s[done + lane];
}

__device__ __forceinline__ const uint8_t *body_of(const KArgs &a, uint8_t src, uint64_t body, int64_t alias1) {
  if (src == BODY_RAW) return a.in + body;
  if (src == BODY_SNAPPY && alias1) return a.in + (alias1 - 1);
  return a.stage + body;
}

// Everything k_expand needs about its page, loaded in one round trip.
struct ExPage {
  int32_t n, cover, nr, bw, val_len;
  uint32_t dict_n;
  const uint8_t *vals;  // values section
  const uint8_t *dict;  // dictionary values
  const uint2 *runs;    // run table
  bool ok;              // page and dictionary clean so far
  bool plain;
};

// Run-table window in registers: lane i holds entry wb + i; the sentinel and
// everything after it read as start = INT32_MAX, so "start <= j" ballots are
// lane prefixes.
struct RunWin {
  int32_t wb, start;
  uint32_t prm, rle;
  __device__ __forceinline__ void load(const uint2 *runs, int32_t nr, int32_t base) {
    wb = base;
    const int32_t ei = wb + lane_id();
    const uint2 e = ei < nr ? runs[ei] : make_uint2(0x7fffffffu, 0u);
    start = ei < nr ? (int32_t)(e.x & ~RUN_RLE) : 0x7fffffff;
    rle = e.x & RUN_RLE;
    prm = e.y;
  }
};

// Keys of [v0, lim) (at most 512 values) read straight from HBM/L2 at their
// own bit offsets — the path for key ranges whose runs or bytes exceed the
// staged form below (very short runs).  Value j = v0 + 64 k + lane.
__device__ void expand_direct(const KArgs &a, const ExPage &P, int page, int w, uint8_t *out, int32_t v0,
                              int32_t lim, int32_t tfi) {
  constexpr int R = 8;
  const int lane = lane_id();
  const uint8_t *ks = P.vals + 1;
  const uintptr_t ks_al = (uintptr_t)ks & ~(uintptr_t)3;
  const uint32_t ks_sh = (uint32_t)((uintptr_t)ks & 3) * 8;
  const int32_t end_bit = (P.val_len - 1) * 8;
  const int bw = P.bw;
  const uint32_t mask = bw >= 32 ? 0xffffffffu : ((1u << bw) - 1);
  RunWin W;
  W.load(P.runs, P.nr, tfi);
  uint32_t ko[R];
  uint32_t rle_bits = 0;
#pragma unroll
  for (int k = 0; k < R; k++) {
    ko[k] = 0;
    const int32_t rl = v0 + 64 * k;
    if (rl >= lim) continue;
    const int32_t rh = min(rl + 64, lim);
    uint64_t m = ballot(W.start <= rl);
    while (m == ~0ull) {  // every window entry starts at or before the row: slide forward
      W.load(P.runs, P.nr, W.wb + 63);
      m = ballot(W.start <= rl);
    }
    int32_t ri = max((int32_t)__popcll(m) - 1, 0);
    int32_t ns = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, ri + 1);
    if (ns < rh && ri > 0) {  // runs start inside the row: put the row's first run at lane 0
      W.load(P.runs, P.nr, W.wb + ri);
      ri = 0;
      ns = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, 1);
    }
    const int32_t j = rl + lane;
    int32_t s0 = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, ri);
    uint32_t p0 = __builtin_amdgcn_readlane(W.prm, ri), f0 = __builtin_amdgcn_readlane(W.rle, ri);
    for (int32_t q = ri + 1; q < 64 && ns < rh;) {  // runs that start inside this row
      const bool mine = j >= ns;
      const uint32_t pq = __builtin_amdgcn_readlane(W.prm, q), fq = __builtin_amdgcn_readlane(W.rle, q);
      s0 = mine ? ns : s0;
      p0 = mine ? pq : p0;
      f0 = mine ? fq : f0;
      q++;
      ns = q < 64 ? (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, q) : 0x7fffffff;
    }
    ko[k] = f0 ? p0 : p0 * 8 + (uint32_t)(j - s0) * (uint32_t)bw;
    rle_bits |= (f0 ? 1u : 0u) << k;
  }
  uint64_t raw[R];
#pragma unroll
  for (int k = 0; k < R; k++) {
    const uint32_t t = ks_sh + (((rle_bits >> k) & 1) ? 0u : ko[k]);
    raw[k] = gld64(ks_al + ((t >> 5) << 2));
  }
  uint32_t key[R];
  bool bad = false;
#pragma unroll
  for (int k = 0; k < R; k++) {
    const bool act = v0 + 64 * k + lane < lim;
    const uint32_t t = ks_sh + ko[k];
    uint32_t kv = (uint32_t)(raw[k] >> (t & 31)) & mask;
    const int32_t avail = end_bit - (int32_t)ko[k];
    kv &= avail >= bw ? 0xffffffffu : avail <= 0 ? 0u : ((1u << avail) - 1);
    kv = ((rle_bits >> k) & 1) ? ko[k] : kv;
    bad |= act && kv >= P.dict_n;
    key[k] = act && kv < P.dict_n ? kv : 0u;
  }
  if (ballot(bad)) {
    set_status(a.status, page, ST_VALUES, E_DICT);
    return;
  }
  const uintptr_t dict_al = (uintptr_t)P.dict & ~(uintptr_t)3;
  const uint32_t dsh = (uint32_t)((uintptr_t)P.dict & 3);
#pragma unroll
  for (int k = 0; k < R; k++) {
    const int32_t j = v0 + 64 * k + lane;
    if (j >= lim) continue;
    const uintptr_t q = dict_al + (size_t)key[k] * w;
    const uint32_t x0 = gld32(q), x1 = gld32(q + 4);
    if (w == 4) {
      gst32((uintptr_t)out + 4 * (uintptr_t)j, __builtin_amdgcn_alignbyte(x1, x0, dsh));
    } else {
      const uint32_t x2 = gld32(q + 8);
      gst64((uintptr_t)out + 8 * (uintptr_t)j,
            ((uint64_t)__builtin_amdgcn_alignbyte(x2, x1, dsh) << 32) | __builtin_amdgcn_alignbyte(x1, x0, dsh));
    }
  }
}

// ===========================================================================
// K5t: k_expand — tiled decode of flat, required, fixed-width (4 / 8 byte)
// PLAIN and RLE_DICTIONARY pages (the hot shape of C1 / C2 / C5).
//
// One wave per TileJob (EX_WAVE consecutive values of one page), four jobs per
// 256-thread workgroup.  RLE_DICTIONARY (type_dict.go:39-59):
//   1. one round trip for the job's descriptors and its tile_info (first run
//      and first key byte of its first tile and of the next job's);
//   2. one round trip for the run-table window (lane i = run i) and, in
//      parallel, the job's key bytes staged into LDS with 16-byte loads;
//   3. rows of 256 values, four consecutive values per lane: each key is two
//      LDS dwords and a funnel shift (or its run's RLE value), range-checked;
//      then every dictionary gather of the job is issued back to back and
//      each lane stores 16 / 32 contiguous bytes per row.
// Jobs whose values span more runs or key bytes than the staged form holds
// fall back to expand_direct.  PLAIN (type_int32.go:23-37,
// type_int64.go:23-37) is a 16-byte copy of the job's bytes.  The grid is
// dealt so that the jobs of one column chunk (one dictionary) share an XCD's
// L2 (host side).
// ===========================================================================
#ifndef PQ_NO_WINDOWED
#define PQ_NO_WINDOWED 0  // 1 (analysis variant): jobs past the run window go to expand_direct as before
#endif
constexpr int EX_WAVE = EX_WAVE_VALUES;       // values per wave
constexpr int EX_ROW = 256;                   // values per row (4 per lane)
constexpr int EX_ROWS = EX_WAVE / EX_ROW;     // rows per wave
static_assert(EX_WAVE % RUN_TILE == 0, "tile_info granularity");

// The four keys of a lane whose first key sits at staged bit lb0, all in one
// bit-packed run: CLS 0 (bw <= 8) one 32-bit window, 1 (bw <= 16) one 64-bit
// window, 2 a dword pair per key.
template <int CLS>
__device__ __forceinline__ void row_keys(const uint32_t *kspan, uint32_t lb0, int bw, uint32_t mask, uint32_t (&k)[4]) {
  const uint32_t *dw = kspan + (lb0 >> 5);
  const uint32_t sh = lb0 & 31;
  if (CLS == 0) {
    const uint32_t x = __builtin_amdgcn_alignbit(dw[1], dw[0], sh);
#pragma unroll
    for (int q = 0; q < 4; q++) k[q] = __builtin_amdgcn_ubfe(x, (uint32_t)(q * bw), (uint32_t)bw);
  } else if (CLS == 1) {
    const uint32_t d1 = dw[1];
    const uint64_t x = ((uint64_t)__builtin_amdgcn_alignbit(dw[2], d1, sh) << 32) | __builtin_amdgcn_alignbit(d1, dw[0], sh);
#pragma unroll
    for (int q = 0; q < 4; q++) k[q] = (uint32_t)(x >> (q * bw)) & mask;
  } else {
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t lb = lb0 + (uint32_t)(q * bw);
      const uint32_t *dq = kspan + (lb >> 5);
      k[q] = __builtin_amdgcn_alignbit(dq[1], dq[0], lb & 31) & mask;
    }
  }
}

// A wave-uniform load through the scalar cache (constant address space): for
// data written by an earlier launch and read-only in this one (job records,
// tile jobs, groups), so the compiler never falls back to vector loads.
template <class T>
__device__ __forceinline__ T sload(const T *p) {
  static_assert(sizeof(T) % 16 == 0, "whole 16-byte pieces");
  union {
    T t;
    u32x4 v[sizeof(T) / 16];
  } u;
  const __attribute__((address_space(4))) u32x4 *q = (const __attribute__((address_space(4))) u32x4 *)p;
#pragma unroll
  for (int i = 0; i < (int)(sizeof(T) / 16); i++) u.v[i] = q[i];
  return u.t;
}

// A staged job whose runs do not fit the 64-lane window (run-heavy key
// streams: SURVEY.md §8(d) C2's run-heavy variant, ~128 runs a job), row by
// row: before each row of EX_ROW values the window is moved so that the row's
// first run is lane 0 (one load, only when the row's runs leave the window),
// then each value takes its run among the runs starting inside the row
// (wave-uniform, as the general rows of expand_job), its key from the staged
// bytes or the run's RLE value, a range check, the gather and the store.  A
// row holding more run starts than the window (runs of one or two values)
// goes to expand_direct.  (Inlined: as a call its frame took k_expand_mix<4>
// from 73 VGPRs to 101 and 544 bytes of scratch a lane.)
template <int WIDTH, bool LD>
__device__ __forceinline__ void expand_windowed(const KArgs &a, const TileJob &tj, const ExRec &rc,
                                             const PQ_LDS uint32_t *kspan, int64_t lbase, const PQ_LDS uint32_t *sdict) {
  const int lane = lane_id();
  const int32_t v0 = rc.v0, lim = rc.lim;
  const int bw = rc.bw;
  const uint32_t mask = bw >= 32 ? 0xffffffffu : ((1u << bw) - 1);
  const int32_t end_bit32 = (int32_t)(((int64_t)rc.val_len - 1) * 8);
  const uint32_t dsh = (uint32_t)((uintptr_t)rc.dict & 3);
  const __amdgpu_buffer_rsrc_t dra = __builtin_amdgcn_make_buffer_rsrc(
      (void *)((uintptr_t)rc.dict & ~(uintptr_t)3), (short)0, (int)(rc.dict_n * (uint32_t)WIDTH + 12), 0x00020000);
  const __amdgpu_buffer_rsrc_t ors =
      __builtin_amdgcn_make_buffer_rsrc((void *)tj.out, (short)0, (int)((uint32_t)lim * (uint32_t)WIDTH), 0x00020000);
  const bool out_al = ((uintptr_t)tj.out & 15) == 0;
  RunWin W;
  W.load(rc.runs, rc.nr, rc.first_run);
  for (int32_t rl = v0; rl < lim; rl += EX_ROW) {
    const int32_t rh = min(rl + EX_ROW, lim);
    int32_t ri = max((int32_t)__popcll(ballot(W.start <= rl)) - 1, 0);
    if ((int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, 63) < rh) {  // the row's runs leave the window
      W.load(rc.runs, rc.nr, W.wb + ri);
      ri = 0;
    }
    if ((int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, 63) < rh) {  // > 62 run starts in the row
      ExPage P;
      P.nr = rc.nr;
      P.bw = rc.bw;
      P.val_len = rc.val_len;
      P.dict_n = rc.dict_n;
      P.vals = rc.vals;
      P.dict = rc.dict;
      P.runs = rc.runs;
      expand_direct(a, P, tj.page, WIDTH, tj.out, rl, rh, W.wb + ri);
      continue;
    }
    const int32_t j0 = rl + 4 * lane;
    int32_t sq[4];
    uint32_t pq[4], fq[4];
    {
      const int32_t s0 = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, ri);
      const uint32_t p0 = __builtin_amdgcn_readlane(W.prm, ri), f0 = __builtin_amdgcn_readlane(W.rle, ri);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        sq[q] = s0;
        pq[q] = p0;
        fq[q] = f0;
      }
      for (int x = ri + 1; x < 64; x++) {
        const int32_t ns = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, x);
        if (ns >= rh) break;
        const uint32_t px = __builtin_amdgcn_readlane(W.prm, x), fx = __builtin_amdgcn_readlane(W.rle, x);
#pragma unroll
        for (int q = 0; q < 4; q++)
          if (j0 + q >= ns) {
            sq[q] = ns;
            pq[q] = px;
            fq[q] = fx;
          }
      }
    }
    uint32_t key[4];
    bool bad = false;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int32_t j = j0 + q;
      const bool act = j < lim;
      const uint32_t pr = pq[q], fr = fq[q];
      const int32_t bb = (int32_t)pr * 8 + (j - sq[q]) * bw;  // stream bit of the key (pages < 256 MiB)
      const uint32_t lb = (fr || !act) ? 0u : (uint32_t)(bb - (int32_t)lbase);
      const PQ_LDS uint32_t *dw = kspan + (lb >> 5);
      uint32_t kv = __builtin_amdgcn_alignbit(dw[1], dw[0], lb & 31) & mask;
      const int32_t avail = end_bit32 - bb;  // zero-fill past the stream end (hybrid_decoder.go:133-141)
      kv &= avail >= bw ? 0xffffffffu : avail <= 0 ? 0u : ((1u << avail) - 1);
      kv = fr ? pr : kv;
      bad |= act && kv >= rc.dict_n;
      key[q] = act && kv < rc.dict_n ? kv : 0u;
    }
    if (ballot(bad)) {
      set_status(a.status, tj.page, ST_VALUES, E_DICT);  // type_dict.go:51-53
      return;
    }
    typedef typename std::conditional<WIDTH == 4, uint32_t, uint64_t>::type VT;
    VT val[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      if (LD) {
        val[q] = WIDTH == 4 ? (VT)sdict[key[q]] : (VT)((const PQ_LDS uint64_t *)sdict)[key[q]];
      } else if (WIDTH == 4) {
        const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(dra, key[q] * 4, 0, 0);
        val[q] = (VT)__builtin_amdgcn_alignbyte(x.y, x.x, dsh);
      } else {
        const u32x3 x = __builtin_amdgcn_raw_buffer_load_b96(dra, key[q] * 8, 0, 0);
        val[q] = (VT)(((uint64_t)__builtin_amdgcn_alignbyte(x.z, x.y, dsh) << 32) | __builtin_amdgcn_alignbyte(x.y, x.x, dsh));
      }
    }
    const uint32_t off = (uint32_t)j0 * (uint32_t)WIDTH;
    if (j0 + 4 <= lim && out_al) {
      if (WIDTH == 4) {
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{(uint32_t)val[0], (uint32_t)val[1], (uint32_t)val[2], (uint32_t)val[3]}, ors, off, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{(uint32_t)val[0], (uint32_t)((uint64_t)val[0] >> 32), (uint32_t)val[1],
                                                     (uint32_t)((uint64_t)val[1] >> 32)},
                                               ors, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{(uint32_t)val[2], (uint32_t)((uint64_t)val[2] >> 32), (uint32_t)val[3],
                                                     (uint32_t)((uint64_t)val[3] >> 32)},
                                               ors, off + 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (j0 + q >= lim) continue;
        if (WIDTH == 4) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)val[q], ors, off + 4 * q, 0, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)val[q], (uint32_t)((uint64_t)val[q] >> 32)}, ors,
                                                off + 8 * q, 0, 0);
      }
    }
  }
}

// One job (EX_WAVE values of one page) by one wave.  kspan: this wave's
// staging area (ex_lds bytes); sdict: the dictionary resident in LDS, or null.
template <int WIDTH, bool LD>
__device__ __forceinline__ void expand_job(const KArgs &a, const TileJob &tj, const ExRec &rc, uint32_t *kspan,
                                           int ex_lds, const uint32_t *sdict) {
  const int lane = lane_id();
  const int page = tj.page;
  STAMP(1);
  const int32_t v0 = rc.v0, lim = rc.lim;
  if (v0 >= lim) return;
  constexpr int w = WIDTH;
  if (rc.bw < 0) {  // PLAIN (type_int32.go:23-37, type_int64.go:23-37): a copy of the job's bytes
    copy_tile<EX_WAVE * 8 / 1024>(rc.vals + (int64_t)v0 * w, tj.out + (int64_t)v0 * w, (int64_t)(lim - v0) * w, lane);
    return;
  }
  // ---- RLE_DICTIONARY ----
  ExPage P;
  P.nr = rc.nr;
  P.bw = rc.bw;
  P.val_len = rc.val_len;
  P.dict_n = rc.dict_n;
  P.vals = rc.vals;
  P.dict = rc.dict;
  P.runs = rc.runs;
  const int bw = P.bw;
  const uint8_t *ks = P.vals + 1;
  const int64_t slen = (int64_t)P.val_len - 1;
  // 2. window and staged key bytes, in parallel
  RunWin W;
  W.load(P.runs, P.nr, rc.first_run);
  const int64_t byte_lo = rc.byte_lo, byte_hi = (int64_t)rc.byte_hi + 16;
  const uintptr_t A = ((uintptr_t)ks + (uintptr_t)byte_lo) & ~(uintptr_t)15;
  const int64_t nb = (int64_t)((uintptr_t)ks + (uintptr_t)byte_hi - A);
  const bool staged = nb <= ex_lds;
  if (staged) {
    // LDS-DMA: lane l's 16 bytes of chunk i land at kspan + 1024 i + 16 l (the
    // last chunk only as far as the span: kspan is sized in 256-byte steps).
    // Bytes past the stream end are never used as key bits (fast rows stay
    // inside it, the general path masks them), so they are staged as they are.
    const uintptr_t src = A + 16 * (uintptr_t)lane;
    for (int32_t off = 0; off < nb; off += 1024)
      if (off + 16 * lane < nb)
        __builtin_amdgcn_global_load_lds((const void *)(src + off),
                                         (__attribute__((address_space(3))) void *)(kspan + off / 4), 16, 0, 0);
  }
  // every run meeting [v0, lim) must sit in lanes 0..62 (its end is the next
  // lane's start); rows meeting more than two runs (short RLE runs among
  // bit-packed ones: bit width 1) take the general row path
  const bool fits = staged && (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, 63) >= lim;
  STAMP(2);
  if (!fits) {
    if (staged && !PQ_NO_WINDOWED) {  // more runs than the window holds: row by row, the window moved along
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the staged bytes (LDS-DMA)
      expand_windowed<WIDTH, LD>(a, tj, rc, (const PQ_LDS uint32_t *)kspan, (int64_t)(A - (uintptr_t)ks) * 8,
                                 (const PQ_LDS uint32_t *)sdict);
      return;
    }
    for (int32_t c = v0; c < lim; c += 512)
      expand_direct(a, P, page, w, tj.out, c, min(c + 512, lim), a.tile_info[tj.tf + (c - v0) / RUN_TILE].x);
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the staged bytes (LDS-DMA) and the window
  STAMP(3);
  const int64_t lbase = (int64_t)(A - (uintptr_t)ks) * 8;  // stream bit of kspan bit 0
  const int64_t end_bit = slen * 8;
  const uint32_t mask = bw >= 32 ? 0xffffffffu : ((1u << bw) - 1);
  const uint32_t dsh = (uint32_t)((uintptr_t)P.dict & 3);
  // per window lane (run): the staged bit of its key j is c + j * bw, and okm
  // marks bit-packed runs whose keys all lie inside the stream (the fast rows)
  const int32_t w_end = (int32_t)shfl32((uint32_t)W.start, min(lane + 1, 63));
  const int32_t w_c = (int32_t)(W.prm * 8) - W.start * bw - (int32_t)lbase;
  const uint64_t okm = ballot(!W.rle && W.start != 0x7fffffff &&
                              (int64_t)W.prm * 8 + (int64_t)(min(w_end, lim) - W.start) * bw <= end_bit);
  // 3. per half (four rows, value j = row start + 4 lane + q): keys from LDS,
  //    range check, then the half's gathers back to back; stores trail.
  //    Dictionary reads and output writes go through buffer resources
  //    (32-bit offsets; a read past the dictionary returns zero).
  const __amdgpu_buffer_rsrc_t drs =
      __builtin_amdgcn_make_buffer_rsrc((void *)P.dict, (short)0, (int)(P.dict_n * (uint32_t)w + 8), 0x00020000);
  const __amdgpu_buffer_rsrc_t ors =
      __builtin_amdgcn_make_buffer_rsrc((void *)tj.out, (short)0, (int)((uint32_t)lim * (uint32_t)w), 0x00020000);
  constexpr int HR = EX_ROWS / 2;
  const int32_t end_bit32 = (int32_t)end_bit;
#ifdef PQ_ONECLS
  const int cls = 2;
#else
  const int cls = bw <= 8 ? 0 : bw <= 16 ? 1 : 2;
#endif
  typedef typename std::conditional<WIDTH == 4, uint32_t, uint64_t>::type VT;
  VT val[2][HR][4];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint32_t key[HR][4];
    bool bad = false;
    uint32_t kmax = 0;  // largest key of the fast rows
    // scalar plan of the half's rows: the run of the row start (ri), the next
    // run's start (s1) and the staged-bit constants of both; `fast` rows are
    // full, bit-packed only and inside the stream
    int32_t rs1[HR], rc0[HR], rc1[HR];
    bool all_fast = true;
#pragma unroll
    for (int r = 0; r < HR; r++) {
      const int32_t rl = v0 + (h * HR + r) * EX_ROW;
      const int32_t rh = min(rl + EX_ROW, lim);
      const uint64_t m = ballot(W.start <= rl);
      const int32_t ri = max((int32_t)__popcll(m) - 1, 0);
      rs1[r] = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, ri + 1);
      rc0[r] = (int32_t)__builtin_amdgcn_readlane((uint32_t)w_c, ri);
      rc1[r] = (int32_t)__builtin_amdgcn_readlane((uint32_t)w_c, ri + 1);
      const int32_t rs2 = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, min(ri + 2, 63));
      all_fast &= rl < lim && rh - rl == EX_ROW && ((okm >> ri) & 1) &&
                  (rs1[r] >= rh || (((okm >> (ri + 1)) & 1) && rs2 >= rh));
    }
    if (all_fast) {
      // straight-line: every row's LDS reads go out together.  The four keys of
      // a lane are taken from the run of its first key; the one lane per row
      // where a run starts among them is fixed up below.
      uint32_t lb0[HR];
#pragma unroll
      for (int r = 0; r < HR; r++) {
        const int32_t j0 = v0 + (h * HR + r) * EX_ROW + 4 * lane;
        lb0[r] = (uint32_t)(j0 >= rs1[r] ? rc1[r] : rc0[r]) + __umul24((uint32_t)j0, (uint32_t)bw);
      }
      switch (cls) {
        case 0:
#pragma unroll
          for (int r = 0; r < HR; r++) row_keys<0>(kspan, lb0[r], bw, mask, key[r]);
          break;
        case 1:
#pragma unroll
          for (int r = 0; r < HR; r++) row_keys<1>(kspan, lb0[r], bw, mask, key[r]);
          break;
        default:
#pragma unroll
          for (int r = 0; r < HR; r++) row_keys<2>(kspan, lb0[r], bw, mask, key[r]);
          break;
      }
#pragma unroll
      for (int r = 0; r < HR; r++) {
        const int32_t j0 = v0 + (h * HR + r) * EX_ROW + 4 * lane;
        if (j0 < rs1[r] && j0 + 3 >= rs1[r]) {
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int32_t j = j0 + q;
            const uint32_t lb = (uint32_t)((j >= rs1[r] ? rc1[r] : rc0[r]) + j * bw);
            const uint32_t *dq = kspan + (lb >> 5);
            key[r][q] = __builtin_amdgcn_alignbit(dq[1], dq[0], lb & 31) & mask;
          }
        }
        kmax = max(kmax, max(max(key[r][0], key[r][1]), max(key[r][2], key[r][3])));
      }
    } else {
#pragma unroll
    for (int r = 0; r < HR; r++) {
      const int32_t rl = v0 + (h * HR + r) * EX_ROW;
      const int32_t j0 = rl + 4 * lane;
#pragma unroll
      for (int q = 0; q < 4; q++) key[r][q] = 0;
      if (rl >= lim) continue;
      const int32_t rh = min(rl + EX_ROW, lim);
      const uint64_t m = ballot(W.start <= rl);
      const int32_t ri = max((int32_t)__popcll(m) - 1, 0);
      // at most two runs meet a row (checked per wave above): the row's run and the next
      const int32_t s1 = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, ri + 1);
      const int32_t c0 = (int32_t)__builtin_amdgcn_readlane((uint32_t)w_c, ri);
      const bool one = s1 >= rh;  // the whole row inside run ri
      const bool two = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, min(ri + 2, 63)) >= rh;
      const bool fast = ((okm >> ri) & 1) && (one || (((okm >> (ri + 1)) & 1) && two)) && rh - rl == EX_ROW;
      if (fast) {  // full row, bit-packed runs only, nothing past the stream end
        uint32_t lb0;
        if (one) {
          lb0 = (uint32_t)(c0 + j0 * bw);
        } else {
          const int32_t c1 = (int32_t)__builtin_amdgcn_readlane((uint32_t)w_c, ri + 1);
          lb0 = (uint32_t)((j0 >= s1 ? c1 : c0) + j0 * bw);
        }
        switch (cls) {
          case 0: row_keys<0>(kspan, lb0, bw, mask, key[r]); break;
          case 1: row_keys<1>(kspan, lb0, bw, mask, key[r]); break;
          default: row_keys<2>(kspan, lb0, bw, mask, key[r]); break;
        }
        if (!one && j0 < s1 && j0 + 3 >= s1) {  // the one lane of the row where a run starts
          const int32_t c1 = (int32_t)__builtin_amdgcn_readlane((uint32_t)w_c, ri + 1);
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int32_t j = j0 + q;
            const uint32_t lb = (uint32_t)((j >= s1 ? c1 : c0) + j * bw);
            const uint32_t *dq = kspan + (lb >> 5);
            key[r][q] = __builtin_amdgcn_alignbit(dq[1], dq[0], lb & 31) & mask;
          }
        }
        kmax = max(kmax, max(max(key[r][0], key[r][1]), max(key[r][2], key[r][3])));
        continue;
      }
      // general row: each value's run among every run meeting the row (the
      // row's first run, then each run starting inside it, wave-uniform)
      int32_t sq[4];
      uint32_t pq[4], fq[4];
      {
        const int32_t s0 = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, ri);
        const uint32_t p0 = __builtin_amdgcn_readlane(W.prm, ri), f0 = __builtin_amdgcn_readlane(W.rle, ri);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          sq[q] = s0;
          pq[q] = p0;
          fq[q] = f0;
        }
        for (int x = ri + 1; x < 64; x++) {
          const int32_t ns = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, x);
          if (ns >= rh) break;
          const uint32_t px = __builtin_amdgcn_readlane(W.prm, x), fx = __builtin_amdgcn_readlane(W.rle, x);
#pragma unroll
          for (int q = 0; q < 4; q++)
            if (j0 + q >= ns) {
              sq[q] = ns;
              pq[q] = px;
              fq[q] = fx;
            }
        }
      }
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int32_t j = j0 + q;
        const bool act = j < lim;
        const uint32_t pr = pq[q], fr = fq[q];
        const int32_t sr = sq[q];
        const int32_t bb = (int32_t)pr * 8 + (j - sr) * bw;  // stream bit of the key (pages < 256 MiB)
        const uint32_t lb = (fr || !act) ? 0u : (uint32_t)(bb - (int32_t)lbase);
        const uint32_t *dw = kspan + (lb >> 5);
        uint32_t kv = __builtin_amdgcn_alignbit(dw[1], dw[0], lb & 31) & mask;
        const int32_t avail = end_bit32 - bb;  // zero-fill past the stream end (hybrid_decoder.go:133-141)
        kv &= avail >= bw ? 0xffffffffu : avail <= 0 ? 0u : ((1u << avail) - 1);
        kv = fr ? pr : kv;
        bad |= act && kv >= P.dict_n;
        key[r][q] = act ? kv : 0u;
      }
    }
    }
    if (ballot(bad || kmax >= P.dict_n)) {
      // dictionary index out of range (type_dict.go:51-53); it precedes any later header error
      set_status(a.status, page, ST_VALUES, E_DICT);
      return;
    }
    // gathers (an unaligned dictionary is read as aligned dwords + a funnel shift)
    if (LD) {  // ds_read: the dictionary is resident in this workgroup's LDS
#pragma unroll
      for (int r = 0; r < HR; r++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
          if (WIDTH == 4) val[h][r][q] = sdict[key[r][q]];
          else val[h][r][q] = ((const uint64_t *)sdict)[key[r][q]];
        }
    } else if (dsh == 0) {
#pragma unroll
      for (int r = 0; r < HR; r++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
          if (WIDTH == 4) {
            val[h][r][q] = __builtin_amdgcn_raw_buffer_load_b32(drs, key[r][q] * 4, 0, 0);
          } else {
            const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(drs, key[r][q] * 8, 0, 0);
            val[h][r][q] = ((uint64_t)x.y << 32) | x.x;
          }
        }
    } else {
      const __amdgpu_buffer_rsrc_t dra = __builtin_amdgcn_make_buffer_rsrc(
          (void *)((uintptr_t)P.dict & ~(uintptr_t)3), (short)0, (int)(P.dict_n * (uint32_t)w + 12), 0x00020000);
#pragma unroll
      for (int r = 0; r < HR; r++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
          if (WIDTH == 4) {
            const u32x2 x = __builtin_amdgcn_raw_buffer_load_b64(dra, key[r][q] * 4, 0, 0);
            val[h][r][q] = __builtin_amdgcn_alignbyte(x.y, x.x, dsh);
          } else {
            const u32x3 x = __builtin_amdgcn_raw_buffer_load_b96(dra, key[r][q] * 8, 0, 0);
            val[h][r][q] = ((uint64_t)__builtin_amdgcn_alignbyte(x.z, x.y, dsh) << 32) |
                           __builtin_amdgcn_alignbyte(x.y, x.x, dsh);
          }
        }
    }
  }
  STAMP(4);
  // 4. stores: 16 / 32 contiguous bytes per lane per row
  const bool out_al = ((uintptr_t)tj.out & 15) == 0;
#pragma unroll
  for (int h = 0; h < 2; h++)
#pragma unroll
    for (int r = 0; r < HR; r++) {
      const int32_t j0 = v0 + (h * HR + r) * EX_ROW + 4 * lane;
      const uint32_t off = (uint32_t)j0 * (uint32_t)w;
      if (j0 + 4 <= lim && out_al) {
        if (WIDTH == 4) {
          __builtin_amdgcn_raw_buffer_store_b128(
              u32x4{(uint32_t)val[h][r][0], (uint32_t)val[h][r][1], (uint32_t)val[h][r][2], (uint32_t)val[h][r][3]},
              ors, off, 0, 0);
        } else {
          __builtin_amdgcn_raw_buffer_store_b128(
              u32x4{(uint32_t)val[h][r][0], (uint32_t)((uint64_t)val[h][r][0] >> 32), (uint32_t)val[h][r][1],
                    (uint32_t)((uint64_t)val[h][r][1] >> 32)},
              ors, off, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(
              u32x4{(uint32_t)val[h][r][2], (uint32_t)((uint64_t)val[h][r][2] >> 32), (uint32_t)val[h][r][3],
                    (uint32_t)((uint64_t)val[h][r][3] >> 32)},
              ors, off + 16, 0, 0);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
          if (j0 + q >= lim) continue;
          if (WIDTH == 4) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)val[h][r][q], ors, off + 4 * q, 0, 0);
          else
            __builtin_amdgcn_raw_buffer_store_b64(
                u32x2{(uint32_t)val[h][r][q], (uint32_t)((uint64_t)val[h][r][q] >> 32)}, ors, off + 8 * q, 0, 0);
        }
      }
    }
  STAMP(5);
}



// ===========================================================================
// K5w: k_expand_wg — RLE_DICTIONARY chunks whose dictionary is past the mixed
// launch's LDS groups (C2's bit widths 13-17: 32 KiB .. 640 KiB).  Gathering
// those through L1/L2 is bound by the L2's request rate (one 128-byte line a
// value: ~250-300 Gvalues/s for the whole chip, tools/gather_bench2.hip,
// whatever the load's cache policy); from LDS the same gathers run at ~1,150.
// One 1,024-thread workgroup a CU (sixteen waves) owns the CU's whole LDS:
//  * the dictionary fits (<= WG_SLICE bytes): copied once, then the waves take
//    the group's jobs in turn and gather with ds_read;
//  * otherwise (at most WG_SLICES slices): the group's jobs go in rounds of
//    sixteen, one a wave; a round's keys are extracted into registers, then
//    the dictionary streams through the LDS slice by slice and every key
//    inside a slice gathers from it (the L2 serves whole lines of the
//    dictionary instead of one line a value).
// Keys are read straight from the key stream into registers (no LDS staging:
// the LDS is the dictionary's): per row of 256 values a lane loads the 16
// bytes holding its four keys; a lane where a run starts among them loads the
// next run's first bytes too; rows the fast form does not cover (RLE runs,
// the stream's end, a page's last partial row) load each key's 8 bytes.
// ===========================================================================

// bits [o, o + 32) of the 128-bit little-endian value d, o < 96
__device__ __forceinline__ uint32_t bits_at(const u32x4 &d, uint32_t o) {
  const uint32_t s = o & 31, i = o >> 5;
  const uint32_t x0 = __builtin_amdgcn_alignbit(d.y, d.x, s);
  const uint32_t x1 = __builtin_amdgcn_alignbit(d.z, d.y, s);
  const uint32_t x2 = __builtin_amdgcn_alignbit(d.w, d.z, s);
  return i == 0 ? x0 : i == 1 ? x1 : x2;
}

// A job's ExRec and TileJob as ONE lane-distributed vector load (lane l < 16:
// dword l of the record, lanes 16..23: dword l - 16 of the tile entry), so a
// wave loads its next jobs' descriptors ahead under vmcnt: a scalar load in
// flight would be waited for by the first LDS read of the job in between.
__device__ __forceinline__ uint32_t job_load(const KArgs &a, int j) {
  const int lane = lane_id();
  const uint32_t *p = lane < 16 ? (const uint32_t *)(a.recs + j) + lane : (const uint32_t *)(a.tiles + j) + (lane & 7);
  return *p;
}
__device__ __forceinline__ void job_unpack(uint32_t v, TileJob &tj, ExRec &rc) {
  union {
    ExRec r;
    uint32_t d[16];
  } ur;
  union {
    TileJob t;
    uint32_t d[8];
  } ut;
#pragma unroll
  for (int i = 0; i < 16; i++) ur.d[i] = __builtin_amdgcn_readlane(v, i);
#pragma unroll
  for (int i = 0; i < 8; i++) ut.d[i] = __builtin_amdgcn_readlane(v, 16 + i);
  rc = ur.r;
  tj = ut.t;
}

// a vector-held descriptor's job is a live RLE_DICTIONARY job (record of
// this decode, values to decode, not PLAIN); its run window
__device__ __forceinline__ bool job_dict_live(const KArgs &a, uint32_t v) {
  const uint32_t ep = __builtin_amdgcn_readlane(v, 14);
  const int32_t v0 = (int32_t)__builtin_amdgcn_readlane(v, 6), lim = (int32_t)__builtin_amdgcn_readlane(v, 7);
  const int32_t bw = (int32_t)__builtin_amdgcn_readlane(v, 8);
  return rec_live(ep, a.epoch) && v0 < lim && bw >= 0;
}
__device__ __forceinline__ void job_window(RunWin &W, uint32_t v) {
  const uint64_t rp = readlane_u64(v, 4, 5);
  W.load((const uint2 *)rp, (int32_t)__builtin_amdgcn_readlane(v, 9), (int32_t)__builtin_amdgcn_readlane(v, 10));
}

// The keys of job tj (values [v0, lim) of its page) into key[r][q] (value
// v0 + 256 r + 4 lane + q), read from the key stream without staging; W: the
// job's run window (RunWin::load(rc.runs, rc.nr, rc.first_run), loaded ahead).
// Returns 0 (keys valid, each < dict_n), 1 (the job is outside this form:
// more runs than the window holds, two run starts in one row, a lane where
// runs start in two rows, or a bit width past 20 — the caller uses
// expand_direct) or 2 (a dictionary index out of range: status set,
// type_dict.go:51-53).
__device__ __forceinline__ int keys_direct(const KArgs &a, const TileJob &tj, const ExRec &rc, const RunWin &W,
                                           uint32_t (&key)[EX_ROWS][4]) {
  const int lane = lane_id();
  const int32_t v0 = rc.v0, lim = rc.lim;
  const int bw = rc.bw;
  if (bw > 20) return 1;
  const uint8_t *ks = rc.vals + 1;
  const int32_t slen = rc.val_len - 1;
  // every run meeting [v0, lim) must sit in lanes 0..62 (its end is the next lane's start),
  // and no row of EX_ROW values may hold two run starts (rows meet at most two runs)
  const int32_t rs = W.start > v0 && W.start < lim && ((W.start - v0) & (EX_ROW - 1)) ? (W.start - v0) / EX_ROW : -1 - lane;
  const int32_t rs_next = (int32_t)shfl32((uint32_t)rs, min(lane + 1, 63));
  if ((int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, 63) < lim || ballot(lane < 63 && rs >= 0 && rs == rs_next))
    return 1;
  // the key stream as a buffer from its first aligned dword, 20 bytes past its
  // end readable (a page's body is followed by >= 16 bytes of the batch's
  // buffers: the next 16-byte aligned body or the input's pad), so a 16-byte
  // load holding a stream's last keys is never cut by the range check; bits
  // past the end are masked off below (general rows) or never used (fast rows)
  const uintptr_t kb = (uintptr_t)ks & ~(uintptr_t)3;
  const int32_t ksh = (int32_t)((uintptr_t)ks & 3) * 8;
  const __amdgpu_buffer_rsrc_t krs =
      __builtin_amdgcn_make_buffer_rsrc((void *)kb, (short)0, (int)((uint32_t)slen + 20u), 0x00020000);
  const uint32_t mask = (1u << bw) - 1;
  const int32_t w_end = (int32_t)shfl32((uint32_t)W.start, min(lane + 1, 63));
  // per window lane (run): the buffer bit of its key j is w_c + j * bw; okm marks
  // bit-packed runs whose keys all lie inside the stream (the fast rows)
  const int32_t w_c = (int32_t)(W.prm * 8) + ksh - W.start * bw;
  const uint64_t okm = ballot(!W.rle && W.start != 0x7fffffff &&
                              (int64_t)W.prm * 8 + (int64_t)(min(w_end, lim) - W.start) * bw <= (int64_t)slen * 8);
  // the rows' plan (wave-uniform): the run of the row start, the next run's
  // start, fast = full, bit-packed only, inside the stream; and the one row
  // where this lane's four keys meet a run start (a lane meeting two: outside)
  int32_t ri[EX_ROWS], s1[EX_ROWS];
  uint32_t fastm = 0;
  int strow = -1, nst = 0;
#pragma unroll
  for (int r = 0; r < EX_ROWS; r++) {
    const int32_t rl = v0 + r * EX_ROW, j0 = rl + 4 * lane;
    const int32_t rh = min(rl + EX_ROW, lim);
    ri[r] = max((int32_t)__popcll(ballot(W.start <= rl)) - 1, 0);
    s1[r] = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, ri[r] + 1);
    const bool one = s1[r] >= rh;
    if (rl < lim && ((okm >> ri[r]) & 1) && (one || ((okm >> (ri[r] + 1)) & 1)) && rh - rl == EX_ROW) {
      fastm |= 1u << r;
      if (!one && j0 < s1[r] && j0 + 3 >= s1[r]) {
        strow = r;
        nst++;
      }
    }
  }
  if (ballot(nst > 1)) return 1;
  // 1. the fast rows' loads, all in flight together: 16 bytes from the lane's
  //    first key, and at the straddling lane the next run's first bytes
  u32x4 d[EX_ROWS], e = u32x4{0, 0, 0, 0};
  uint32_t lbs = 0;
#pragma unroll
  for (int r = 0; r < EX_ROWS; r++) {
    d[r] = u32x4{0, 0, 0, 0};
    if (!((fastm >> r) & 1)) continue;
    const int32_t j0 = v0 + r * EX_ROW + 4 * lane;
    const int32_t c0 = (int32_t)__builtin_amdgcn_readlane((uint32_t)w_c, ri[r]);
    const int32_t c1 = (int32_t)__builtin_amdgcn_readlane((uint32_t)w_c, ri[r] + 1);
    const uint32_t lb0 = (uint32_t)((j0 >= s1[r] ? c1 : c0) + j0 * bw);
    d[r] = __builtin_amdgcn_raw_buffer_load_b128(krs, (lb0 >> 5) * 4, 0, 0);
    if (strow == r) {
      lbs = (uint32_t)(c1 + s1[r] * bw);
      e = __builtin_amdgcn_raw_buffer_load_b128(krs, (lbs >> 5) * 4, 0, 0);
    }
  }
  bool bad = false;
  uint32_t kmax = 0;
  // 2. general rows (RLE runs, the stream's end, a page's last partial row):
  //    each key's 8 bytes, a row at a time (rare)
#pragma unroll
  for (int r = 0; r < EX_ROWS; r++) {
#pragma unroll
    for (int q = 0; q < 4; q++) key[r][q] = 0;
    const int32_t rl = v0 + r * EX_ROW, j0 = rl + 4 * lane;
    if (rl >= lim || ((fastm >> r) & 1)) continue;
    const int32_t s0 = (int32_t)__builtin_amdgcn_readlane((uint32_t)W.start, ri[r]);
    const uint32_t p0 = __builtin_amdgcn_readlane(W.prm, ri[r]), f0 = __builtin_amdgcn_readlane(W.rle, ri[r]);
    const uint32_t p1 = __builtin_amdgcn_readlane(W.prm, ri[r] + 1), f1 = __builtin_amdgcn_readlane(W.rle, ri[r] + 1);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int32_t j = j0 + q;
      const bool act = j < lim;
      const bool sel = j >= s1[r];
      const uint32_t pr = sel ? p1 : p0, fr = sel ? f1 : f0;
      const int32_t sr = sel ? s1[r] : s0;
      const int32_t bb = (int32_t)pr * 8 + (j - sr) * bw;  // stream bit of the key (pages < 256 MiB)
      const u32x2 y = (fr || !act) ? u32x2{0, 0}
                                   : __builtin_amdgcn_raw_buffer_load_b64(krs, ((uint32_t)(bb + ksh) >> 5) * 4, 0, 0);
      uint32_t kv = __builtin_amdgcn_alignbit(y.y, y.x, (uint32_t)(bb + ksh) & 31) & mask;
      const int32_t avail = slen * 8 - bb;  // zero-fill past the stream end (hybrid_decoder.go:133-141)
      kv &= avail >= bw ? 0xffffffffu : avail <= 0 ? 0u : ((1u << avail) - 1);
      kv = fr ? pr : kv;
      bad |= act && kv >= rc.dict_n;
      key[r][q] = act ? kv : 0u;
    }
  }
  // 3. the fast rows' keys
#pragma unroll
  for (int r = 0; r < EX_ROWS; r++) {
    if (!((fastm >> r) & 1)) continue;
    const int32_t j0 = v0 + r * EX_ROW + 4 * lane;
    const int32_t c0 = (int32_t)__builtin_amdgcn_readlane((uint32_t)w_c, ri[r]);
    const int32_t c1 = (int32_t)__builtin_amdgcn_readlane((uint32_t)w_c, ri[r] + 1);
    const uint32_t sh = (uint32_t)((j0 >= s1[r] ? c1 : c0) + j0 * bw) & 31;
    if (bw <= 8) {
      const uint32_t x = __builtin_amdgcn_alignbit(d[r].y, d[r].x, sh);
#pragma unroll
      for (int q = 0; q < 4; q++) key[r][q] = __builtin_amdgcn_ubfe(x, (uint32_t)(q * bw), (uint32_t)bw);
    } else if (bw <= 16) {
      const uint64_t x = ((uint64_t)__builtin_amdgcn_alignbit(d[r].z, d[r].y, sh) << 32) |
                         __builtin_amdgcn_alignbit(d[r].y, d[r].x, sh);
#pragma unroll
      for (int q = 0; q < 4; q++) key[r][q] = (uint32_t)(x >> (q * bw)) & mask;
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) key[r][q] = bits_at(d[r], sh + (uint32_t)(q * bw)) & mask;
    }
    if (strow == r) {  // keys from the run starting at s1: bits of e
#pragma unroll
      for (int q = 0; q < 4; q++)
        if (j0 + q >= s1[r]) key[r][q] = bits_at(e, (lbs & 31) + (uint32_t)((j0 + q - s1[r]) * bw)) & mask;
    }
    kmax = max(kmax, max(max(key[r][0], key[r][1]), max(key[r][2], key[r][3])));
  }
  if (ballot(bad || kmax >= rc.dict_n)) {
    set_status(a.status, tj.page, ST_VALUES, E_DICT);  // type_dict.go:51-53
    return 2;
  }
  return 0;
}

// the job's values, 16 / 32 contiguous bytes per lane per row (as expand_job)
template <int WIDTH, class VT>
__device__ __forceinline__ void store_rows(const TileJob &tj, int32_t v0, int32_t lim, const VT (&val)[EX_ROWS][4]) {
  const int lane = lane_id();
  const __amdgpu_buffer_rsrc_t ors =
      __builtin_amdgcn_make_buffer_rsrc((void *)tj.out, (short)0, (int)((uint32_t)lim * (uint32_t)WIDTH), 0x00020000);
  const bool out_al = ((uintptr_t)tj.out & 15) == 0;
#pragma unroll
  for (int r = 0; r < EX_ROWS; r++) {
    const int32_t j0 = v0 + r * EX_ROW + 4 * lane;
    const uint32_t off = (uint32_t)j0 * (uint32_t)WIDTH;
    if (j0 + 4 <= lim && out_al) {
      if (WIDTH == 4) {
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{(uint32_t)val[r][0], (uint32_t)val[r][1], (uint32_t)val[r][2], (uint32_t)val[r][3]}, ors, off, 0, 0);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{(uint32_t)val[r][0], (uint32_t)((uint64_t)val[r][0] >> 32), (uint32_t)val[r][1],
                  (uint32_t)((uint64_t)val[r][1] >> 32)},
            ors, off, 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{(uint32_t)val[r][2], (uint32_t)((uint64_t)val[r][2] >> 32), (uint32_t)val[r][3],
                  (uint32_t)((uint64_t)val[r][3] >> 32)},
            ors, off + 16, 0, 0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 4; q++) {
        if (j0 + q >= lim) continue;
        if (WIDTH == 4) __builtin_amdgcn_raw_buffer_store_b32((uint32_t)val[r][q], ors, off + 4 * q, 0, 0);
        else
          __builtin_amdgcn_raw_buffer_store_b64(u32x2{(uint32_t)val[r][q], (uint32_t)((uint64_t)val[r][q] >> 32)}, ors,
                                                off + 8 * q, 0, 0);
      }
    }
  }
}

// a job outside the register form: keys and gathers straight from HBM / L2
// (not inlined: rare, and its registers stay out of the kernel's allocation)
__device__ __noinline__ void wg_direct(const KArgs &a, int page, uint8_t *out, int32_t tf, int32_t v0, int32_t lim,
                                       const uint8_t *vals, const uint8_t *dict, const uint2 *runs, int32_t nr,
                                       int32_t bw, int32_t val_len, uint32_t dict_n, int width) {
  ExPage P;
  P.nr = nr;
  P.bw = bw;
  P.val_len = val_len;
  P.dict_n = dict_n;
  P.vals = vals;
  P.dict = dict;
  P.runs = runs;
  for (int32_t c = v0; c < lim; c += 512)
    expand_direct(a, P, page, width, out, c, min(c + 512, lim), a.tile_info[tf + (c - v0) / RUN_TILE].x);
}
#define WG_DIRECT(tj, rc, W) \
  wg_direct(a, (tj).page, (tj).out, (tj).tf, (rc).v0, (rc).lim, (rc).vals, (rc).dict, (rc).runs, (rc).nr, (rc).bw, \
            (rc).val_len, (rc).dict_n, (W))

// LDS <- dictionary bytes [b0, b0 + nbytes) (aligned dwords; an unaligned
// dictionary is funnel-shifted), PF 16-byte pieces a thread in flight
template <int NT, int PF>
__device__ __forceinline__ void dict_to_lds(uint32_t *lds, const __amdgpu_buffer_rsrc_t rs, uint32_t dsh, uint32_t b0,
                                            uint32_t nbytes) {
  const uint32_t n16 = (nbytes + 15) / 16;
  for (uint32_t i0 = threadIdx.x; i0 < n16; i0 += PF * NT) {
    u32x4 x[PF];
    uint32_t y[PF];
#pragma unroll
    for (int q = 0; q < PF; q++) {
      const uint32_t i = i0 + q * NT;
      x[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, b0 + 16 * i, 0, 0);  // out of range: zeros
      y[q] = dsh ? __builtin_amdgcn_raw_buffer_load_b32(rs, b0 + 16 * i + 16, 0, 0) : 0u;
    }
#pragma unroll
    for (int q = 0; q < PF; q++) {
      const uint32_t i = i0 + q * NT;
      if (i < n16)
        *(u32x4 *)(lds + 4 * i) =
            u32x4{__builtin_amdgcn_alignbyte(x[q].y, x[q].x, dsh), __builtin_amdgcn_alignbyte(x[q].z, x[q].y, dsh),
                  __builtin_amdgcn_alignbyte(x[q].w, x[q].z, dsh), __builtin_amdgcn_alignbyte(y[q], x[q].w, dsh)};
    }
  }
}

// LDS <- dictionary bytes [0, nbytes) of a 16-byte aligned source by LDS-DMA
// (1 KiB a wave instruction, every piece of the workgroup in flight at once);
// the caller waits (vmcnt) and syncs
__device__ __forceinline__ void dict_dma(uint32_t *lds, const uint8_t *src, uint32_t nbytes) {
  const int lane = lane_id();
  const uint32_t wv = ufirst(threadIdx.x >> 6);
  for (uint32_t c = wv; c * 1024 < nbytes; c += WG_WAVES)
    if (c * 1024 + 16 * lane < nbytes)
      __builtin_amdgcn_global_load_lds((const void *)(src + c * 1024 + 16 * lane),
                                       (__attribute__((address_space(3))) void *)(lds + c * 256), 16, 0, 0);
}

template <int WIDTH>
__global__ __launch_bounds__(WG_WAVES * 64) void k_expand_wg(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_dyn[];
  typedef typename std::conditional<WIDTH == 4, uint32_t, uint64_t>::type VT;
  const LdsGroup g = sload(a.lgroups + blockIdx.x);
  if (g.njobs <= 0) return;  // an empty slot of the XCD dealing (block-uniform)
  WSTAMP(0);
  const int wv = (int)ufirst(threadIdx.x >> 6);
  const int jend = g.job0 + g.njobs;
  // this wave's first two jobs' descriptors, in flight during the dictionary copy
  int j = g.job0 + wv;
  uint32_t vcur = j < jend ? job_load(a, j) : 0u;
  uint32_t vnext = j + WG_WAVES < jend ? job_load(a, j + WG_WAVES) : 0u;
  // the chunk's dictionary: the group's first record (written by this decode's
  // k_prepare), or the dictionary page itself when that job failed or is PLAIN
  const ExRec r0 = sload(a.recs + g.job0);
  const uint8_t *dict;
  uint32_t dn;
  if (rec_live(r0.epoch, a.epoch) && r0.dict) {
    dict = r0.dict;
    dn = r0.dict_n;
  } else {
    if (page_status(a.status, g.dpage) != STATUS_OK) return;  // no record of the chunk was written
    const PageDesc dp = a.pages[g.dpage];
    dict = body_ptr(a, dp, g.dpage);
    dn = (uint32_t)max(dp.num_values, 0);
  }
  const uint32_t dsh = (uint32_t)((uintptr_t)dict & 3);
#if defined(PQ_WG_CHECK) || defined(PQ_WG_SIMPLE)
  const bool dma = false;  // (analysis build: the register copy)
#else
  const bool dma = ((uintptr_t)dict & 15) == 0;
#endif
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)((uintptr_t)dict & ~(uintptr_t)3), (short)0, (int)((dn * (uint32_t)WIDTH + dsh + 3) & ~3u), 0x00020000);
  constexpr uint32_t SE = WG_SLICE / WIDTH;  // entries a slice
  constexpr int NT = WG_WAVES * 64;
  // (8-byte values: the host sends only dictionaries of one slice — a sliced
  // round's 64 value registers a lane would not fit beside its keys)
  const bool sliced = WIDTH == 4 && dn > SE;
  if (!sliced) {  // resident: the whole dictionary, once
    if (dma) {
      dict_dma(lds_dyn, dict, min(dn, SE) * (uint32_t)WIDTH);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      dict_to_lds<NT, 4>(lds_dyn, rs, dsh, 0, min(dn, SE) * (uint32_t)WIDTH);
    }
    __syncthreads();
  }
  RunWin W;
  if (j < jend && job_dict_live(a, vcur)) job_window(W, vcur);
  WSTAMP(1);
  // rounds of WG_WAVES jobs, one a wave (resident: each wave runs on through
  // its jobs without waiting for the others; sliced: the dictionary streams
  // through the LDS once a round).  Software-pipelined: while job j's keys load
  // and gather, job j + WG_WAVES's run window and job j + 2 WG_WAVES's
  // descriptors are in flight.
  for (int j0 = g.job0; j0 < jend; j0 += WG_WAVES, j += WG_WAVES) {
    const uint32_t vfar = j + 2 * WG_WAVES < jend ? job_load(a, j + 2 * WG_WAVES) : 0u;
    RunWin Wn;
    if (j + WG_WAVES < jend && job_dict_live(a, vnext)) job_window(Wn, vnext);
    TileJob tj;
    ExRec rc;
    job_unpack(vcur, tj, rc);
#ifdef PQ_WG_SIMPLE
    // analysis build: plain scalar descriptor loads and the window loaded here
    if (j < jend) {
      tj = sload(a.tiles + j);
      rc = sload(a.recs + j);
      if (rec_live(rc.epoch, a.epoch) && rc.v0 < rc.lim && rc.bw >= 0) W.load(rc.runs, rc.nr, rc.first_run);
    }
#endif
#ifdef PQ_WG_CHECK
    // analysis build: the pipelined descriptors and window against the plain loads
    if (j < jend) {
      const TileJob tj2 = sload(a.tiles + j);
      const ExRec rc2 = sload(a.recs + j);
      const bool bad_t = tj2.out != tj.out || tj2.page != tj.page || tj2.tf != tj.tf;
      const bool bad_r = rc2.vals != rc.vals || rc2.dict != rc.dict || rc2.runs != rc.runs || rc2.v0 != rc.v0 ||
                         rc2.lim != rc.lim || rc2.bw != rc.bw || rc2.nr != rc.nr || rc2.first_run != rc.first_run ||
                         rc2.epoch != rc.epoch || rc2.val_len != rc.val_len || rc2.dict_n != rc.dict_n;
      bool bad_w = false;
      if (rec_live(rc2.epoch, a.epoch) && rc2.v0 < rc2.lim && rc2.bw >= 0) {
        RunWin W2;
        W2.load(rc2.runs, rc2.nr, rc2.first_run);
        bad_w = ballot(W2.start != W.start || W2.prm != W.prm || W2.rle != W.rle) != 0;
      }
      if (bad_t || bad_r || bad_w) {
        if (lane_id() == 0)
          printf("k_expand_wg check: block %d wave %d job %d: tile %d rec %d window %d (out %p/%p vals %p/%p runs %p/%p "
                 "v0 %d/%d lim %d/%d bw %d/%d)\n",
                 (int)blockIdx.x, wv, j, (int)bad_t, (int)bad_r, (int)bad_w, (void *)tj.out, (void *)tj2.out,
                 (const void *)rc.vals, (const void *)rc2.vals, (const void *)rc.runs, (const void *)rc2.runs, rc.v0,
                 rc2.v0, rc.lim, rc2.lim, rc.bw, rc2.bw);
        tj = tj2;
        rc = rc2;
        rc.epoch = ~a.epoch & 0x7fffffffu;  // skipped
      }
    }
#endif
    int k = 3;  // 0 keys ready, 1 outside the register form, 2 failed, 3 nothing to do
    uint32_t key[EX_ROWS][4];
    WSTAMP(2);
    if (j < jend && rec_live(rc.epoch, a.epoch) && rc.v0 < rc.lim) {  // (else: the page failed before k_prepare finished it)
      if (rc.bw < 0)  // PLAIN (a dictionary chunk's fallback page): a copy of the job's bytes
        copy_tile<EX_WAVE * 8 / 1024>(rc.vals + (int64_t)rc.v0 * WIDTH, tj.out + (int64_t)rc.v0 * WIDTH,
                                      (int64_t)(rc.lim - rc.v0) * WIDTH, lane_id());
      else
        k = keys_direct(a, tj, rc, W, key);
      if (k == 0 && !sliced && dn > SE) k = 1;  // (not sent by the host: a dictionary past the LDS)
    }
    WSTAMP(3);
    VT val[EX_ROWS][4];
    if (!sliced) {
      if (k == 0) {
#pragma unroll
        for (int r = 0; r < EX_ROWS; r++)
#pragma unroll
          for (int q = 0; q < 4; q++) {
            if (WIDTH == 4) val[r][q] = lds_dyn[key[r][q]];
            else val[r][q] = ((const uint64_t *)lds_dyn)[key[r][q]];
          }
      }
    } else {
#pragma unroll
      for (int r = 0; r < EX_ROWS; r++)
#pragma unroll
        for (int q = 0; q < 4; q++) val[r][q] = 0;
      for (uint32_t base = 0; base < dn; base += SE) {
        __syncthreads();  // the previous slice's gathers are done
        if (dma) {
          dict_dma(lds_dyn, dict + (size_t)base * WIDTH, min(dn - base, SE) * (uint32_t)WIDTH);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
          dict_to_lds<NT, 2>(lds_dyn, rs, dsh, base * (uint32_t)WIDTH, min(dn - base, SE) * (uint32_t)WIDTH);
        }
        __syncthreads();
        if (k == 0) {
#pragma unroll
          for (int r = 0; r < EX_ROWS; r++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
              const uint32_t rel = key[r][q] - base;
              if (rel < SE) val[r][q] = lds_dyn[rel];
            }
        }
      }
    }
    WSTAMP(4);
    if (k == 0) store_rows<WIDTH>(tj, rc.v0, rc.lim, val);
    if (k == 1) WG_DIRECT(tj, rc, WIDTH);  // after the round: nothing of it live across the call
    WSTAMP(5);
    W = Wn;
    vcur = vnext;
    vnext = vfar;
  }
}

// ===========================================================================
// K5m: k_expand_mix — the tiled decode in 256-thread workgroups, one per
// LdsGroup (host-built, see the planner in pq_host.cpp):
//  * dpage >= 0: consecutive jobs of one column chunk whose dictionary fits in
//    LDS.  The dictionary is copied into LDS once (aligned dwords; an
//    unaligned page is funnel-shifted), then the four waves take the jobs in
//    turn and gather with ds_read instead of L1/L2 requests, which bound the
//    random gathers of dictionaries past the L1 (tools/gather_bench.hip);
//  * dpage < 0: one job per wave, gathers through L1/L2 (dictionaries too
//    large for LDS, PLAIN pages).
// Both kinds share one launch, so L2-bound and LDS-bound blocks overlap.
// ===========================================================================
constexpr int LD_WAVES = LD_WAVES_H;

// the two block kinds as separate (non-inlined) functions: each keeps the
// register allocation and schedule it gets on its own
template <int WIDTH>
__device__ __forceinline__ void mix_global(const KArgs &a, const LdsGroup &g, uint32_t *lds_dyn) {
  const int wv = (int)ufirst(threadIdx.x >> 6);
  const int j = (int)blockIdx.x * LD_WAVES + wv;
  const TileJob tj = sload(a.tiles + j);
  const ExRec rc = sload(a.recs + j);
  if (!rec_live(rc.epoch, a.epoch)) return;  // an unused slot, or the page failed before k_prepare finished it
  expand_job<WIDTH, false>(a, tj, rc, lds_dyn + wv * (g.kspan / 4), g.kspan, nullptr);
}

template <int WIDTH, int NW = LD_WAVES>
__device__ __forceinline__ void mix_lds(const KArgs &a, const LdsGroup &g, uint32_t *lds_dyn) {
  const int wv = (int)ufirst(threadIdx.x >> 6);
  const int jend = g.job0 + g.njobs;
  // the group's first record (its dictionary: pointer and size, written by this
  // decode's k_prepare) and this wave's first job, loaded together
  const ExRec r0 = sload(a.recs + g.job0);
  int j = g.job0 + wv;
  TileJob tj = {};
  ExRec rc = {};
  if (j < jend) {
    tj = sload(a.tiles + j);
    rc = sload(a.recs + j);
  }
  const uint8_t *dict;
  uint32_t dn;
  if (rec_live(r0.epoch, a.epoch) && r0.dict) {
    dict = r0.dict;
    dn = r0.dict_n;
  } else {  // a failed or PLAIN first page: the dictionary page itself
    if (page_status(a.status, g.dpage) != STATUS_OK) return;  // no record of the chunk was written
    const PageDesc dp = a.pages[g.dpage];
    dict = body_ptr(a, dp, g.dpage);
    dn = (uint32_t)max(dp.num_values, 0);
  }
  const uint32_t nbytes = min(dn * (uint32_t)WIDTH, (uint32_t)g.dict_bytes);
  const uint32_t dsh = (uint32_t)((uintptr_t)dict & 3);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void *)((uintptr_t)dict & ~(uintptr_t)3), (short)0, (int)((nbytes + dsh + 3) & ~3u), 0x00020000);
  const uint32_t n16 = (nbytes + 15) / 16;
  // the copy: four 16-byte pieces per thread in flight at a time
  constexpr uint32_t T = NW * 64;
  for (uint32_t i0 = threadIdx.x; i0 < n16; i0 += 4 * T) {
    u32x4 x[4];
    uint32_t y[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t i = i0 + q * T;
      x[q] = __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * i, 0, 0);  // out of range: zeros
      y[q] = dsh ? __builtin_amdgcn_raw_buffer_load_b32(rs, 16 * i + 16, 0, 0) : 0u;
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint32_t i = i0 + q * T;
      if (i < n16)
        *(u32x4 *)(lds_dyn + 4 * i) =
            u32x4{__builtin_amdgcn_alignbyte(x[q].y, x[q].x, dsh), __builtin_amdgcn_alignbyte(x[q].z, x[q].y, dsh),
                  __builtin_amdgcn_alignbyte(x[q].w, x[q].z, dsh), __builtin_amdgcn_alignbyte(y[q], x[q].w, dsh)};
    }
  }
  __syncthreads();
  uint32_t *kspan = lds_dyn + g.dict_bytes / 4 + wv * (g.kspan / 4);
  for (; j < jend; j += NW) {
    if (j != g.job0 + wv) {
      tj = sload(a.tiles + j);
      rc = sload(a.recs + j);
    }
    if (!rec_live(rc.epoch, a.epoch)) continue;  // the page failed before k_prepare finished it
    expand_job<WIDTH, true>(a, tj, rc, kspan, g.kspan, lds_dyn);
  }
}

template <int WIDTH>
__global__ __launch_bounds__(LD_WAVES_H * 64) void k_expand_mix(KArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_dyn[];
  STAMP(0);
  // (batches without k_level_check: the next decode's statuses, as it would)
  if (a.status_next)
    for (int i = blockIdx.x * (LD_WAVES_H * 64) + threadIdx.x; i < a.npages; i += gridDim.x * (LD_WAVES_H * 64))
      a.status_next[i] = a.status0[i];
  const LdsGroup g = sload(a.lgroups + blockIdx.x);
  if (g.dpage < 0) mix_global<WIDTH>(a, g, lds_dyn);
  else mix_lds<WIDTH>(a, g, lds_dyn);
#ifdef PQ_STAMPS
  if (a.dbg && lane_id() == 0)  // the wave's end
    a.dbg[((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 8 + 6] = __builtin_amdgcn_s_memrealtime();
#endif
}

// ===========================================================================
// K5b: k_dba — DELTA_BYTE_ARRAY value bytes (type_bytearray.go:211-240): value
// i = previous value[:prefix_i] + suffix_i, rebuilt in value order by one wave
// per page.  The first DBA_PREV bytes of the previous value are kept in LDS
// (updated in place: only the suffix is written); a prefix reaching past them
// is read back from the previous value in the output (every value is written
// there), so values of any length decode.  Lengths were decoded and validated
// by k_prepare, and the string offsets / validity written by k_decode; a
// batch's suffix bytes are contiguous in the page and staged in LDS when they
// fit.  FIXED_LEN_BYTE_ARRAY pages (getFixedLenByteArrayValuesDecoder,
// chunk_reader.go:86-96) write value i to the slot of the i-th defined level.
// ===========================================================================
constexpr int DBA_PREV = 16384, DBA_STAGE = 8192;  // per wave: 96 KiB of LDS per workgroup

// One value: out[0, plen + s) = prev value[0, plen) + suffix[0, s), where the
// previous value starts at `pv` in the output and its first DBA_PREV bytes
// are in `prev` (LDS), which then holds the new value's.
__device__ __forceinline__ void dba_value(uint8_t *prev, const uint8_t *suffix, int32_t plen, int32_t s, uint8_t *out,
                                          const uint8_t *pv, int lane) {
  const int32_t vl = plen + s;
  if (vl <= DBA_PREV) {
    for (int32_t b = lane; b < s; b += 64) prev[plen + b] = suffix[b];
    for (int32_t b = lane; b < vl; b += 64) out[b] = prev[b];
    return;
  }
  if (plen > DBA_PREV) {
    // the previous value's bytes past the LDS copy, from the output this wave
    // wrote: its stores retired, then read at device scope (past a stale L1 line)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    for (int32_t b = DBA_PREV + lane; b < plen; b += 64)
      out[b] = (uint8_t)__hip_atomic_load(pv + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  for (int32_t b = lane; b < min(plen, DBA_PREV); b += 64) out[b] = prev[b];
  for (int32_t b = lane; b < s; b += 64) {
    const uint8_t x = suffix[b];
    out[plen + b] = x;
    if (plen + b < DBA_PREV) prev[plen + b] = x;
  }
}

__global__ __launch_bounds__(256) void k_dba(KArgs a) {
  __shared__ uint8_t prev_all[4][DBA_PREV];
  __shared__ uint8_t stage_all[4][DBA_STAGE];
  const int wv = (int)ufirst(threadIdx.x >> 6);
  const int gi = blockIdx.x * 4 + wv;
  if (gi >= a.nlist) return;
  const int lane = lane_id();
  const int page = ufirst(a.list[gi]);
  if (page_status(a.status, page) != STATUS_OK) return;
  const PageDesc d = a.pages[page];
  const ColDesc c = a.cols[d.col];
  const PageInfo pi = a.info[page];
  const int64_t nn = pi.non_null;
  const uint8_t *data = body_ptr(a, d, page) + pi.val_off + pi.str_data;
  const int32_t nvp = max(d.num_values, 0);
  const int32_t *S = a.lens + d.lens_base, *P = S + nvp;
  uint8_t *prev = prev_all[wv], *stage = stage_all[wv];
  if (c.ptype == T_FLBA) {
    // every value is c.width bytes (k_prepare checked prefix + suffix ==
    // width); value i goes to the slot of the i-th level with def == max_def,
    // found 64 levels at a time from k_levels' bytes
    const int w = c.width;
    const bool flat = c.max_rep == 0;
    uint8_t *vout = c.values + (flat ? d.level_base : pi.slot_base) * (int64_t)w;
    const uint8_t *ld = c.max_def > 0 ? a.lvl + d.lvl_base + (c.max_rep > 0 ? (int64_t)nvp : 0) : nullptr;
    int64_t i = 0, slot_run = 0, soff = 0;
    const uint8_t *pv = vout;
    for (int64_t e0 = 0; e0 < nvp && i < nn; e0 += 64) {
      const int cnt = (int)min<int64_t>(64, nvp - e0);
      const int dl = lane >= cnt ? -1
                     : d.lvl_bits ? ((((const uint32_t *)ld)[(e0 + lane) >> 5] >> ((e0 + lane) & 31)) & 1u ? c.max_def : 0)
                     : ld ? (int)ld[e0 + lane]
                          : c.max_def;
      const uint64_t vm = ballot(lane < cnt && dl == c.max_def);
      const uint64_t sm = ballot(lane < cnt && (flat || dl >= c.rep_def));
      const uint32_t my_slot = (uint32_t)__builtin_popcountll(sm & ((1ull << lane) - 1));  // within the 64
      uint64_t rem = vm;
      while (rem && i < nn) {
        const int t = (int)__builtin_ctzll(rem);
        rem &= rem - 1;
        const int64_t slot = slot_run + (int64_t)__builtin_amdgcn_readlane(my_slot, t);
        const int32_t pl = P[i], plen = pl > 0 ? pl : 0;
        uint8_t *op = vout + slot * (int64_t)w;
        dba_value(prev, data + soff, plen, w - plen, op, pv, lane);
        pv = op;
        soff += w - plen;
        i++;
      }
      slot_run += __builtin_popcountll(sm);
    }
    return;
  }
  uint8_t *out = c.values + pi.str_base;
  int64_t soff = 0, ooff = 0, poff = 0;
  for (int64_t i0 = 0; i0 < nn; i0 += 64) {
    const int cnt = (int)min<int64_t>(64, nn - i0);
    const int32_t s_l = lane < cnt ? S[i0 + lane] : 0;
    const int32_t p_l = lane < cnt ? P[i0 + lane] : 0;
    int32_t stot;
    const int32_t sexcl = wave_excl_scan32(s_l, &stot);
    const bool staged = stot <= DBA_STAGE;
    if (staged)
      for (int32_t b = lane; b < stot; b += 64) stage[b] = data[soff + b];
    for (int t = 0; t < cnt; t++) {
      const int32_t s = (int32_t)__builtin_amdgcn_readlane((uint32_t)s_l, t);
      const int32_t pl = (int32_t)__builtin_amdgcn_readlane((uint32_t)p_l, t);
      const int32_t so = (int32_t)__builtin_amdgcn_readlane((uint32_t)sexcl, t);
      const int32_t plen = pl > 0 ? pl : 0;
      dba_value(prev, staged ? stage + so : data + soff + so, plen, s, out + ooff, out + poff, lane);
      poff = ooff;
      ooff += plen + s;
    }
    soff += stot;
  }
}

// level-error precedence pass: for pages that failed in k_decode at the
// values or def stage, finish decoding the earlier level streams to see if
// the reference would have failed there first.
__global__ __launch_bounds__(256) void k_level_check(KArgs a) {
  if (a.status_next)
    for (int i = blockIdx.x * 256 + threadIdx.x; i < a.npages; i += gridDim.x * 256) a.status_next[i] = a.status0[i];
  const int gi = blockIdx.x * 4 + (int)ufirst(threadIdx.x >> 6);
  if (gi >= a.nlist) return;
  const int page = ufirst(a.list[gi]);
  uint32_t st = page_status(a.status, page);
  if (st == STATUS_OK) {
    // a key-stream header error found by k_runs, unless a dictionary error
    // among the values before it was reported by k_expand
    const uint32_t we = ufirst(a.info[page].walk_err);
    if (we) set_status(a.status, page, ST_VALUES, we);
    return;
  }
  if ((st >> 16) <= ST_REP) return;
  const PageDesc d = a.pages[page];
  const ColDesc c = a.cols[d.col];
  const PageInfo pi = a.info[page];
  const int n = d.num_values;
  const uint8_t *lvl = d.kind == PAGE_V1 ? body_ptr(a, d, page) : a.in + d.src;
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
  void *jobs;
  uint32_t *njobs;
  uint32_t max_jobs;
  const int32_t *job_base;
  const int32_t *job_owner;
  uint64_t *dbg;
  uint64_t *dbg2;
  int32_t npages_dbg;
  uint32_t *copy_cnt;
  int32_t *copy_idx;
  int32_t *lens;
  uint8_t *lvl;
  void *runs;
  void *tile_info;
  const void *tiles;
  int32_t ex_lds;
  void *recs;
  const int32_t *page_jobs;
  uint32_t epoch;
  const void *lgroups;
  int32_t ldn[6];   // k_expand_mix blocks of 4-byte, 8-byte columns ([0], [1])
  int32_t ldl[6];   // their dynamic LDS bytes
  const uint32_t *status0;
  const void *zr;
  int32_t nzr, npages;
  const uint8_t *in_end, *stage_end;
  const void *sitems;
  int32_t nitems, nwalk;
  const int32_t *walk, *seg_base;
  int64_t *segs;
  uint32_t *seg_flag;
  const int32_t *parts;  // k_decode<3> / <2>: (page, first level, end level) triplets instead of `list`
  int32_t redo;          // k_decode<3> / <2>: decode again (whole) the pages whose parts failed
  int64_t *str_pre;      // k_prepare -> k_decode<2> parts: string bytes before every 256 values of a page
  const int64_t *hjobs;
  int32_t nhjobs;
  int32_t grid_cap;  // k_levels<-1>: at most this many workgroups (grid-stride loop)
  int32_t snappy_wg;  // Snappy items by k_snappy_wg (workgroup per page, 64 KiB LDS history) instead of k_snappy
  const int32_t *part_tab;  // the list-page parts (page, first level, end level), for k_levels
  int32_t *part_pre;        // per part: rows, slots, values before its first level (k_levels -> k_decode<3>)
  uint32_t *status_next;
  const void *sw_pages;
  void *sw_regs;
  void *sw_res;
  const void *sw_items;
  int32_t n_sw_items, n_sw_pages, sw_page0;
};

static pq::KArgs to_k(const pq_launch_args *p) {
  pq::KArgs k;
  k.sitems = (const int2 *)p->sitems;
  k.nitems = p->nitems;
  k.nwalk = p->nwalk;
  k.walk = p->walk;
  k.seg_base = p->seg_base;
  k.segs = p->segs;
  k.seg_flag = p->seg_flag;
  k.in_end = p->in_end;
  k.stage_end = p->stage_end;
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
  k.jobs = (pq::CopyJob *)p->jobs;
  k.njobs = p->njobs;
  k.max_jobs = p->max_jobs;
  k.job_base = p->job_base;
  k.job_owner = p->job_owner;
  k.copy_cnt = p->copy_cnt;
  k.copy_idx = p->copy_idx;
  k.lens = p->lens;
  k.lvl = p->lvl;
  k.status0 = p->status0;
  k.zr = (const pq::ZeroRange *)p->zr;
  k.nzr = p->nzr;
  k.npages = p->npages;
  k.dbg = p->dbg;
  k.dbg2 = p->dbg2;
  k.dbg3 = p->dbg2 ? p->dbg2 + 8 * (size_t)p->npages_dbg : nullptr;
  k.runs = (uint2 *)p->runs;
  k.tile_info = (int2 *)p->tile_info;
  k.ex_lds = p->ex_lds;
  k.recs = (pq::ExRec *)p->recs;
  k.page_jobs = p->page_jobs;
  k.epoch = p->epoch;
  k.tiles = (const pq::TileJob *)p->tiles;
  k.lgroups = (const pq::LdsGroup *)p->lgroups;
  k.parts = p->parts;
  k.redo = p->redo;
  k.str_pre = p->str_pre;
  k.part_tab = p->part_tab;
  k.part_pre = p->part_pre;
  k.hjobs = p->hjobs;
  k.status_next = p->status_next;
  k.sw_pages = (const pq::SwPage *)p->sw_pages;
  k.sw_regs = (pq::SwReg *)p->sw_regs;
  k.sw_res = (pq::SwRes *)p->sw_res;
  k.sw_items = (const int2 *)p->sw_items;
  k.n_sw_items = p->n_sw_items;
  k.n_sw_pages = p->n_sw_pages;
  k.sw_page0 = p->sw_page0;
  k.nhjobs = p->nhjobs;
  return k;
}

// the last failed launch (kernel id, HIP error), for the host's error text
int pq_launch_fail_which = -1;
int pq_launch_fail_err = 0;
static int launch_status(int which) {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  pq_launch_fail_which = which;
  pq_launch_fail_err = (int)e;
  return 17;
}

int pq_launch(int which, const pq_launch_args *p, hipStream_t s) {
  pq::KArgs k = to_k(p);
  if (which == 4) {
    if (k.ncols <= 0) return 0;
    hipLaunchKernelGGL(pq::k_scan, dim3(k.ncols), dim3(256), 0, s, k);
    return launch_status(which);
  }
  if (which == 13) {  // k_reset
    hipLaunchKernelGGL(pq::k_reset, dim3(64, 1 + (k.nzr > 0 ? k.nzr : 0)), dim3(256), 0, s, k);
    return launch_status(which);
  }
  if (which == 12) {  // k_prepare_copy: the prepare blocks, then the copy grid
    const uint32_t items = (k.max_jobs + (uint32_t)k.nhjobs) * pq::COPY_ITEMS;
#ifdef PQ_ANALYSIS
    // PQG_COPY_BLOCKS: the copy grid's cap (analysis build only)
    static const uint32_t cap = getenv("PQG_COPY_BLOCKS") ? (uint32_t)atoi(getenv("PQG_COPY_BLOCKS")) : 1024u;
#else
    constexpr uint32_t cap = 1024u;
#endif
    const uint32_t cb = items < cap ? items : cap;
    const uint32_t pb = ((uint32_t)(k.nlist > 0 ? k.nlist : 0) + 3) / 4;
    if (pb + cb == 0) return 0;
    hipLaunchKernelGGL(pq::k_prepare_copy, dim3(pb + (cb ? cb : 1)), dim3(256), 0, s, k);
    return launch_status(which);
  }
  if (which == 6) {  // deferred literal copies: fixed grid, the job count lives on the device
    if (k.max_jobs == 0 && k.nhjobs == 0) return 0;
    const uint32_t items = (k.max_jobs + (uint32_t)k.nhjobs) * pq::COPY_ITEMS;
    hipLaunchKernelGGL(pq::k_copy, dim3(items < 4096 ? items : 4096), dim3(256), 0, s, k);
    return launch_status(which);
  }
  if (which == 9 || which == 22) {  // k_expand_mix (9) / k_expand_wg (22): one workgroup per LdsGroup
    static bool attr = false;
    if (!attr) {
      hipFuncSetAttribute((const void *)pq::k_expand_mix<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      hipFuncSetAttribute((const void *)pq::k_expand_mix<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      hipFuncSetAttribute((const void *)pq::k_expand_wg<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      hipFuncSetAttribute((const void *)pq::k_expand_wg<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
      attr = true;
    }
    if (which == 22) {
      // k_expand_wg: its groups after the mixed ones, absolute job indices
      const pq::LdsGroup *bg = (const pq::LdsGroup *)p->lgroups + p->ldn[0] + p->ldn[1];
      for (int w = 0; w < 2; w++) {
        if (p->ldn[2 + w] <= 0) continue;
        pq::KArgs kb = k;
        kb.lgroups = bg + (w ? p->ldn[2] : 0);
        const dim3 grid(p->ldn[2 + w]), blk(pq::WG_WAVES * 64);
        if (w == 0) hipLaunchKernelGGL(pq::k_expand_wg<4>, grid, blk, (size_t)pq::WG_SLICE, s, kb);
        else hipLaunchKernelGGL(pq::k_expand_wg<8>, grid, blk, (size_t)pq::WG_SLICE, s, kb);
      }
      return launch_status(which);
    }
    const dim3 blk(pq::LD_WAVES_H * 64);
    if (p->ldn[0] > 0) hipLaunchKernelGGL(pq::k_expand_mix<4>, dim3(p->ldn[0]), blk, (size_t)p->ldl[0], s, k);
    if (p->ldn[1] > 0) {
      k.lgroups = (const pq::LdsGroup *)p->lgroups + p->ldn[0];
      k.tiles = (const pq::TileJob *)p->tiles + (size_t)p->ldn[0] * pq::LD_WAVES_H;  // slots and job indices
      k.recs = (pq::ExRec *)p->recs + (size_t)p->ldn[0] * pq::LD_WAVES_H;           // are launch-relative
      hipLaunchKernelGGL(pq::k_expand_mix<8>, dim3(p->ldn[1]), blk, (size_t)p->ldl[1], s, k);
    }
    return launch_status(which);
  }
  if (which == 28 || which == 30) {  // k_sw_regions / k_sw_emit: one wave per 64 regions
    if (k.n_sw_items <= 0) return 0;
    if (which == 28) hipLaunchKernelGGL(pq::k_sw_regions, dim3(k.n_sw_items), dim3(64), 0, s, k);
    else hipLaunchKernelGGL(pq::k_sw_emit, dim3(k.n_sw_items), dim3(64), 0, s, k);
    return launch_status(which);
  }
  if (which == 29) {  // k_sw_link: one wave per page
    if (k.n_sw_pages <= 0) return 0;
    hipLaunchKernelGGL(pq::k_sw_link, dim3((k.n_sw_pages + 3) / 4), dim3(256), 0, s, k);
    return launch_status(which);
  }
  // k_snappy (wave per page) by default; k_snappy_wg (workgroup per page,
  // the whole 64 KiB history in LDS) when the batch asks for it (PQG_SNAPPY_WG=1)
  const bool snappy_v1 = p->snappy_wg == 0;
  if (which == 0) {  // Snappy over work items (pages, or segments of long pages)
    if (k.nitems <= 0) return 0;
    if (snappy_v1) hipLaunchKernelGGL(pq::k_snappy<pq::SNAP_ITEMS>, dim3((k.nitems + 3) / 4), dim3(256), 0, s, k);
    else hipLaunchKernelGGL(pq::k_snappy_wg<pq::SNAP_ITEMS>, dim3(k.nitems), dim3(pq::UZ_T), 0, s, k);
    return launch_status(which);
  }
  if (which == 17 || which == 18) {  // k_snappy_walk / serial fallback over the segmented pages
    if (k.nwalk <= 0) return 0;
    if (which == 17) hipLaunchKernelGGL(pq::k_snappy_walk, dim3(k.nwalk), dim3(64), 0, s, k);
    else if (snappy_v1) hipLaunchKernelGGL(pq::k_snappy<pq::SNAP_FALLBACK>, dim3((k.nwalk + 3) / 4), dim3(256), 0, s, k);
    else hipLaunchKernelGGL(pq::k_snappy_wg<pq::SNAP_FALLBACK>, dim3(k.nwalk), dim3(pq::UZ_T), 0, s, k);
    return launch_status(which);
  }
  if (k.nlist <= 0) return 0;
  dim3 grid((k.nlist + 3) / 4), block(256);
  switch (which) {
    case 1: hipLaunchKernelGGL(pq::k_dict_prepare, grid, block, 0, s, k); break;
    case 2: hipLaunchKernelGGL(pq::k_prepare<-1>, grid, block, 0, s, k); break;
    case 11: hipLaunchKernelGGL(pq::k_prepare<1>, grid, block, 0, s, k); break;
    case 19: hipLaunchKernelGGL((pq::k_levels<-1, false>), p->grid_cap > 0 && (int)grid.x > p->grid_cap ? dim3(p->grid_cap) : grid, block, 0, s, k); break;
    case 20: hipLaunchKernelGGL((pq::k_levels<0, false>), grid, block, 0, s, k); break;
    case 21: hipLaunchKernelGGL((pq::k_levels<1, false>), grid, block, 0, s, k); break;
    // two waves a page (batches with repeated columns)
    case 24: {
      const int g24 = (k.nlist + 1) / 2;
      hipLaunchKernelGGL((pq::k_levels<-1, true>), dim3(p->grid_cap > 0 && g24 > p->grid_cap ? p->grid_cap : g24), block, 0, s, k);
      break;
    }
    case 25: hipLaunchKernelGGL((pq::k_levels<0, true>), dim3((k.nlist + 1) / 2), block, 0, s, k); break;
    case 26: hipLaunchKernelGGL((pq::k_levels<1, true>), dim3((k.nlist + 1) / 2), block, 0, s, k); break;
    case 3: hipLaunchKernelGGL(pq::k_decode<0>, grid, block, 0, s, k); break;
    case 14: hipLaunchKernelGGL(pq::k_decode<1>, grid, block, 0, s, k); break;
    case 15: hipLaunchKernelGGL(pq::k_decode<2>, grid, block, 0, s, k); break;
    case 31: hipLaunchKernelGGL(pq::k_decode<4>, grid, block, 0, s, k); break;
    case 32: hipLaunchKernelGGL(pq::k_decode<5>, grid, block, 0, s, k); break;
    case 16: hipLaunchKernelGGL(pq::k_decode<3>, grid, block, 0, s, k); break;
    case 5: hipLaunchKernelGGL(pq::k_level_check, grid, block, 0, s, k); break;
    case 10: hipLaunchKernelGGL(pq::k_dba, grid, block, 0, s, k); break;
    case 23: hipLaunchKernelGGL(pq::k_plain_str, grid, block, 0, s, k); break;
    default:
      pq_launch_fail_which = which;
      return 1;
  }
  return launch_status(which);
}

}  // extern "C"
