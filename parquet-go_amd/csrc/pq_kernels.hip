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
  uint64_t *dbg;          // diagnostic build only (-DPQ_STAMPS): per-workgroup s_memtime stamps
};

#ifdef PQ_STAMPS
#define STAMP(i)                                                                              \
  do {                                                                                        \
    if (a.dbg && threadIdx.x == 0) a.dbg[(size_t)blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
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
constexpr int RING = 8192;  // per-wave LDS history (bytes)
constexpr int RING_MASK = RING - 1;
constexpr int SNAPPY_WAVES = 4;

// Literal run: dst[dpos, dpos+len) = s[0, len).  The staging page base is
// 16-byte aligned, so after a <16-byte head every lane stores whole 16-byte
// chunks (1 KiB per wave instruction); the source is read as aligned dwords
// and funnel-shifted (v_alignbyte) by the uniform source/destination skew.
// Only the last RING bytes also enter the LDS history.
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

__global__ __launch_bounds__(256) void k_snappy(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t ring_all[SNAPPY_WAVES][RING];
  const int lane = lane_id();
  const int wv = (int)ufirst(threadIdx.x >> 6);  // wave-uniform (keeps per-wave state in SGPRs)
  const int gi = blockIdx.x * SNAPPY_WAVES + wv;
  if (gi >= a.nlist) return;
  const int page = ufirst(a.list[gi]);
  const PageDesc d = a.pages[page];
  if (a.max_jobs > 0 && lane == 0) a.njobs[gi] = 0u;  // no deferred jobs unless written below
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
  // a block that is exactly one literal is its own content: leave it in place
  if (write && lane == 0) a.info[page].alias1 = 0;
  // (data pages only: dictionaries stay in 16-byte aligned staging for aligned gathers)
  if (write && dl > 0 && s < slen && d.kind != PAGE_DICT) {
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
      if (ok && (int64_t)x + 1 == dl && s + hs + dl == slen) {
        if (lane == 0) a.info[page].alias1 = 1 + (int64_t)(d.src + lsize + s + hs);
        return;
      }
    }
  }
  int64_t dpos = 0;
  uint32_t err = E_OK;
  int ndefer = 0;                      // deferred literals: lane k holds entry k
  const uint8_t *pend_src = nullptr;   // last deferred literal whose tail is not yet in the history
  int64_t pend_dpos = 0, pend_len = 0;
  int64_t def_dst = 0, def_len = 0;
  uint64_t def_src = 0;
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
        bool deferred = false;
        if (length >= BIG_LITERAL && ndefer < MAX_DEFER && a.max_jobs > 0) {
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
        const int m = (int)__builtin_ctzll(~okm);
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
      if (pend_len) {
        ring_fill(pend_src, pend_dpos, pend_len, ring, lane);
        pend_len = 0;
      }
      // forward, possibly self-overlapping copy of <= 64 bytes
      uint8_t b = 0;
      bool act = lane < length;
      int64_t from = dpos - offset + (offset >= length ? (int64_t)lane : (int64_t)lane % offset);
      if (offset <= RING) {
        if (act) b = ring[from & RING_MASK];
      } else {
        // far copy: make this wave's earlier stores visible, read through L2
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        const uint8_t *lit = nullptr;  // inside a deferred literal: read the payload instead
        for (int k = 0; k < ndefer; k++) {
          int64_t kd = (int64_t)shfl64((uint64_t)def_dst, k), kl = (int64_t)shfl64((uint64_t)def_len, k);
          uint64_t ks = shfl64(def_src, k);
          if (from >= kd && from < kd + kl) lit = (const uint8_t *)(uintptr_t)ks + (from - kd);
        }
        if (act) {
          if (lit) {
            b = *lit;
          } else {
            const uint32_t *wp = (const uint32_t *)((uintptr_t)(dst + from) & ~(uintptr_t)3);
            uint32_t word = __hip_atomic_load(wp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            b = (uint8_t)(word >> (((uintptr_t)(dst + from) & 3) * 8));
          }
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
  if (a.max_jobs > 0 && lane == 0) a.njobs[gi] = err ? 0u : (uint32_t)ndefer;
  if (err) set_status(a.status, page, ST_DECOMPRESS, err);
}

// ===========================================================================
// K1b: long literals deferred by k_snappy, copied by every workgroup
// ===========================================================================
constexpr int COPY_TILE = 4096;  // bytes per workgroup step (256 lanes x 16 B)

__global__ __launch_bounds__(256) void k_copy(KArgs a) {
  // one workgroup per job (google/Go snappy literals are <= 64 KB; longer ones loop)
  const uint32_t j = blockIdx.x;
  if (j >= a.max_jobs) return;
  const int32_t q = a.job_owner[j];
  if ((uint32_t)(j - a.job_base[q]) >= a.njobs[q]) return;
  const CopyJob job = a.jobs[j];
  const int t = threadIdx.x;
  const uintptr_t d0 = (uintptr_t)job.dst, d1 = d0 + (uintptr_t)job.len;
  const uintptr_t A = d0 & ~(uintptr_t)15;
  for (uintptr_t base = A; base < d1; base += 4 * COPY_TILE) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      uintptr_t u = base + (uintptr_t)k * COPY_TILE + (uintptr_t)t * 16;
      if (u >= d1) continue;
      if (u >= d0 && u + 16 <= d1) {
        const uint8_t *s = job.src + (u - d0);
        const uint32_t skew = (uint32_t)((uintptr_t)s & 3);
        const uint32_t *sa = (const uint32_t *)((uintptr_t)s & ~(uintptr_t)3);
        uint4 x = *(const uint4 *)sa;
        uint32_t x4 = sa[4];
        uint4 o;
        o.x = __builtin_amdgcn_alignbyte(x.y, x.x, skew);
        o.y = __builtin_amdgcn_alignbyte(x.z, x.y, skew);
        o.z = __builtin_amdgcn_alignbyte(x.w, x.z, skew);
        o.w = __builtin_amdgcn_alignbyte(x4, x.w, skew);
        *(uint4 *)u = o;
      } else {
        for (int b = 0; b < 16; b++) {
          uintptr_t x = u + b;
          if (x >= d0 && x < d1) *(uint8_t *)x = job.src[x - d0];
        }
      }
    }
  }
}

// ===========================================================================
// K2: dictionary pages (page_dict.go:30-64)
// ===========================================================================
__global__ __launch_bounds__(256) void k_dict_prepare(KArgs a) {
  const int gi = blockIdx.x * 4 + (int)ufirst(threadIdx.x >> 6);
  if (gi >= a.nlist) return;
  const int lane = lane_id();
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
// K3: data page prepare
// ===========================================================================
__global__ __launch_bounds__(256) void k_prepare(KArgs a) {
  const int gi = blockIdx.x * 4 + (int)ufirst(threadIdx.x >> 6);
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

// Decode one data page with one wavefront, 256 level entries per step, four
// consecutive entries per lane (page_v1.go:27-55 readValues + data_store.go
// semantics for validity / list offsets).  For flat columns the steps are
// aligned to 256 output slots so each lane owns a 16-byte-aligned slice of
// the values and whole validity words.
__global__ __launch_bounds__(256) void k_decode(KArgs a) {
  const int gi = blockIdx.x * 4 + (int)ufirst(threadIdx.x >> 6);
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

  const uint8_t *lvl = d.kind == PAGE_V1 ? body_ptr(a, d, page) : a.in + d.src;
  const uint8_t *vals = body_ptr(a, d, page) + pi.val_off;
  const int64_t vlen = pi.val_len;
  const int w = c.width;
  const bool flat = c.max_rep == 0;
  const bool is_ba = c.ptype == T_BYTE_ARRAY;

  Hyb rep, def;
  rep.init(lvl + pi.rep_off, pi.rep_len, bits_len(c.max_rep));
  def.init(lvl + pi.def_off, pi.def_len, bits_len(c.max_def));

  Hyb keys;
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
  } else if (d.enc == ENC_DELTA_BP) {
    dz.init(vals, vlen, c.ptype == T_INT32);
    delta_prev = (uint64_t)dz.first;
  }
  Win SW;  // string-length window (PLAIN BYTE_ARRAY)
  SW.reset();
  int64_t spos = 0;

  const int64_t slot_base = flat ? d.level_base : pi.slot_base;
  int64_t e0 = 0, slot_run = 0, row_run = 0, nn_run = 0, str_run = pi.str_base;
  uint32_t err = E_OK, err_stage = 0;

  while (e0 < n) {
    const int cnt = (int)min<int64_t>(n - e0, flat ? 256 - ((slot_base + e0) & 255) : 256);
    uint32_t r[4] = {0, 0, 0, 0}, dl[4] = {0, 0, 0, 0};
    if (c.max_rep > 0) {
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

    if (c.flags & COL_EMIT_LEVELS) {
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
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (act[k] && r[k] == 0) {
          int64_t row = pi.row_base + row_run + rbase + ri;
          c.list_offsets[row] = (int32_t)(slot_base + slot_run + sbase + si);
          if ((int)dl[k] >= c.rep_def - 1) atomicOr(&c.list_validity[row >> 5], 1u << (row & 31));
          ri++;
        }
        si += slot[k];
      }
      row_run += mrows;
    }

    // ---- the m dense values of this step, in dense order (value j: lane j>>2, element j&3) ----
    uint64_t v[4] = {0, 0, 0, 0};
    int64_t soff[4] = {0, 0, 0, 0}, slen[4] = {0, 0, 0, 0};
    const uint8_t *sbase_ptr = nullptr;
    if (m > 0) {
      if (d.enc == ENC_PLAIN && !is_ba) {
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
        if (err) {
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
              uint64_t ent = a.dict_ent[dict_base + key[k]];
              soff[k] = (int64_t)(ent >> 32);
              slen[k] = (int64_t)(ent & 0xffffffffu);
            } else if (w == 4) {
              v[k] = load_u32_unaligned(dict_vals + (int64_t)key[k] * 4);
            } else if (w == 8) {
              v[k] = load_u64_unaligned(dict_vals + (int64_t)key[k] * 8);
            } else {
              soff[k] = (int64_t)key[k] * w;
            }
          }
        sbase_ptr = dict_vals;
      } else if (d.enc == ENC_DELTA_BP) {
        uint64_t dv[4];
        err = dz.next4(m, dv);
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
      } else if (d.enc == ENC_PLAIN && is_ba) {
        // serial length walk (type_bytearray.go:24-45); value j -> lane j>>2, element j&3
        uint32_t eo[4] = {0, 0, 0, 0}, el[4] = {0, 0, 0, 0};
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
          if (lane == (j >> 2)) {
            int k = j & 3;
            if (k == 0) { eo[0] = (uint32_t)(spos + 4); el[0] = (uint32_t)l; }
            else if (k == 1) { eo[1] = (uint32_t)(spos + 4); el[1] = (uint32_t)l; }
            else if (k == 2) { eo[2] = (uint32_t)(spos + 4); el[2] = (uint32_t)l; }
            else { eo[3] = (uint32_t)(spos + 4); el[3] = (uint32_t)l; }
          }
          spos += 4 + l;
        }
        if (err) {
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
      } else {
        err = E_UNSUPPORTED;
        err_stage = ST_VALUES;
        break;
      }
    }

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
#pragma unroll
      for (int k = 0; k < 4; k++) {
        if (slot[k]) {
          start += ll[k];
          c.str_offsets[slot_base + slot_run + sbase + si + 1] = start;
          if (valid[k]) {
            const uint8_t *sp = sbase_ptr + soff[k];
            uint8_t *op = c.values + start - ll[k];
            for (int64_t b = 0; b < ll[k]; b++) op[b] = sp[b];
          }
          si++;
        }
      }
      str_run += (int64_t)shfl64((uint64_t)incl, 63);
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
          if (w == 4) *(uint32_t *)(c.values + sl * 4) = valid[k] ? (uint32_t)v[k] : 0u;
          else if (w == 8) *(uint64_t *)(c.values + sl * 8) = valid[k] ? v[k] : 0ull;
          else {
            uint8_t *op = c.values + sl * (int64_t)w;
            const uint8_t *sp = d.enc == ENC_PLAIN ? vals + (nn_run + vbase) * (int64_t)w : sbase_ptr + soff[k];
            if (valid[k] && d.enc == ENC_PLAIN) {
              int vi = 0;
              for (int q = 0; q < k; q++) vi += valid[q];
              sp = vals + (nn_run + vbase + vi) * (int64_t)w;
            }
            for (int b = 0; b < w; b++) op[b] = valid[k] ? sp[b] : 0;
          }
          si++;
        }
      }
    }
    if (c.max_def > 0) {
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
        int si = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          if (slot[k]) {
            int64_t sl = slot_base + slot_run + sbase + si;
            if (valid[k]) atomicOr(&c.validity[sl >> 5], 1u << (sl & 31));
            si++;
          }
        }
      }
    }
    slot_run += mslots;
    nn_run += m;
    e0 += cnt;
  }
  // a later-found level error can outrank this one: k_level_check re-walks
  // the earlier level streams (the reference decodes all rep levels, then all
  // def levels, then the values, page_v1.go:37-52)
  if (err) set_status(a.status, page, err_stage, err);
}

// ===========================================================================
// K5f: flat, required, fixed-width pages (PLAIN / RLE_DICTIONARY) — the hot
// shape of C1/C2/C5.  One wave per page, 1024 values per step, 16
// consecutive values per lane (64-128 output bytes per lane, 16-byte
// stores).  The encoded index stream is read through an 8 KB per-wave LDS
// window (headers and bit-packed data alike), so a step costs one global
// round trip: the dictionary gathers.
// ===========================================================================
constexpr int FW_WIN = 8192;     // LDS window per wave
constexpr int FW_WAVES = 4;
constexpr int FW_STEP = 1024;    // values per step
constexpr int FW_PER_LANE = 16;

struct LdsWin {
  uint8_t *lds;        // this wave's window
  const uint8_t *p;    // stream start
  int64_t len;         // stream length
  int64_t lo, hi;      // stream offsets currently held: [lo, hi)
  const uint8_t *ab;   // absolute address of lds[0]

  // make [a, b) (stream offsets, b - a <= FW_WIN - 32) resident
  __device__ __forceinline__ void ensure(int64_t a, int64_t b) {
    if (a >= lo && b <= hi) return;
    const uintptr_t A = (uintptr_t)(p + a) & ~(uintptr_t)15;
    const uintptr_t E = (uintptr_t)(p + len) + 16;  // never read past the stream end + 16 (buffers are padded)
    const uintptr_t last = (E - 16) & ~(uintptr_t)15;
    const int lane = lane_id();
    uint4 v[FW_WIN / 1024];
#pragma unroll
    for (int k = 0; k < FW_WIN / 1024; k++) {  // all loads first, then all LDS stores
      uintptr_t src = A + (uintptr_t)(k * 1024 + lane * 16);
      v[k] = *(const uint4 *)(src < E ? src : last);
    }
#pragma unroll
    for (int k = 0; k < FW_WIN / 1024; k++) {
      uintptr_t src = A + (uintptr_t)(k * 1024 + lane * 16);
      *(uint4 *)(lds + k * 1024 + lane * 16) = src < E ? v[k] : make_uint4(0, 0, 0, 0);
    }
    ab = (const uint8_t *)A;
    lo = (int64_t)(A - (uintptr_t)p);
    hi = lo + FW_WIN;
  }
  __device__ __forceinline__ uint32_t byte(int64_t off) { return lds[(p + off) - ab]; }
  // bits [bitpos, bitpos + bw) of the stream; bytes at/after len read as zero
  __device__ __forceinline__ uint32_t bits(int64_t bitpos, int bw) {
    int64_t byteoff = bitpos >> 3;
    int sh = (int)(bitpos & 7);
    uintptr_t la = (uintptr_t)((p + byteoff) - ab);
    const uint32_t *q = (const uint32_t *)(lds + (la & ~(uintptr_t)3));
    uint64_t v = ((uint64_t)q[1] << 32) | q[0];
    v >>= (la & 3) * 8 + sh;
    uint32_t val = (uint32_t)v & (bw == 32 ? 0xffffffffu : ((1u << bw) - 1));
    int64_t avail = (len - byteoff) * 8 - sh;
    if (avail < bw) val = avail <= 0 ? 0u : (val & ((1u << avail) - 1));
    return val;
  }
};

__global__ __launch_bounds__(256) void k_decode_flat(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t win_all[FW_WAVES][FW_WIN + 16];
  const int wv = (int)ufirst(threadIdx.x >> 6);  // wave-uniform (keeps per-wave state in SGPRs)
  const int gi = blockIdx.x * FW_WAVES + wv;
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
  const uint8_t *vals = body_ptr(a, d, page) + pi.val_off;
  const int64_t vlen = pi.val_len;
  const int w = c.width;  // 4 or 8
  uint8_t *out = c.values + d.level_base * w;

  if (d.enc == ENC_PLAIN) {
    // a straight copy of n*w bytes (binary.Read per value, type_int32.go:23-37)
    if ((int64_t)n * w > vlen) {
      set_status(a.status, page, ST_VALUES, E_EOF);
      return;
    }
    copy_bytes_wave(vals, out, (int64_t)n * w, lane);
    return;
  }

  // RLE_DICTIONARY (type_dict.go:39-59) over the hybrid key stream
  const PageDesc *dp = d.dict >= 0 ? &a.pages[d.dict] : nullptr;
  if (!dp) {
    set_status(a.status, page, ST_VALUES, E_DICT);
    return;
  }
  const uint8_t *dict = body_ptr(a, *dp, d.dict);
  const int64_t dict_n = dp->num_values;
  const int bw = pi.idx_bw;

  LdsWin L;
  L.lds = win_all[wv];
  L.p = vals + 1;
  L.len = vlen - 1;
  L.lo = 1;
  L.hi = 0;  // empty
  L.ab = nullptr;

  // hybrid run state (hybrid_decoder.go:82-166), wave-uniform
  int64_t pos = 0, rem = 0, data = 0, vi = 0;
  uint32_t rle_val = 0;
  bool rle = false;
  uint32_t err = E_OK;
  const bool aligned_dict = (((uintptr_t)dict) & (w - 1)) == 0;

  for (int64_t e0 = 0; e0 < n && !err; e0 += FW_STEP) {
    const int cnt = (int)min<int64_t>(FW_STEP, n - e0);
    uint32_t key[FW_PER_LANE];
#pragma unroll
    for (int k = 0; k < FW_PER_LANE; k++) key[k] = 0;
    int got = 0;
    if (bw > 0) {
      while (got < cnt) {
        if (rem == 0) {
          // readRunHeader: uvarint from the LDS window
          uint64_t h = 0;
          uint32_t sh = 0;
          for (int i = 0;; i++) {
            if (pos >= L.len) {
              err = E_EOF;
              break;
            }
            L.ensure(pos, pos + 16);
            uint32_t b = ufirst(L.byte(pos));
            pos++;
            if (b < 0x80) {
              if (i > 9 || (i == 9 && b > 1)) err = E_RLE;
              h |= (uint64_t)b << (sh & 63);
              break;
            }
            if (sh < 64) h |= (uint64_t)(b & 0x7f) << sh;
            sh += 7;
          }
          if (err) break;
          if (h > 0x7fffffffull) {
            err = E_RLE;
            break;
          }
          if (h & 1) {
            int64_t g = (int64_t)(h >> 1);
            if (g == 0) {
              err = E_RLE;
              break;
            }
            rle = false;
            rem = g * 8;
            data = pos;
            vi = 0;
            pos = data + g * (int64_t)bw;
          } else {
            int64_t cr = (int64_t)(h >> 1);
            if (cr == 0) {
              err = E_RLE;
              break;
            }
            int sz = (bw + 7) >> 3;
            if (pos >= L.len || pos + sz > L.len) {
              err = E_EOF;
              break;
            }
            L.ensure(pos, pos + 16);
            uint32_t v = 0;
            for (int k = 0; k < sz; k++) v |= ufirst(L.byte(pos + k)) << (8 * k);
            pos += sz;
            if (bw < 32 && (v >> bw) != 0) {
              err = E_RLE;
              break;
            }
            rle = true;
            rem = cr;
            rle_val = v;
          }
        }
        const int take = (int)min<int64_t>(rem, (int64_t)(cnt - got));
        if (rle) {
#pragma unroll
          for (int k = 0; k < FW_PER_LANE; k++) {
            int j = FW_PER_LANE * lane + k;
            key[k] = (j >= got && j < got + take) ? rle_val : key[k];
          }
        } else {
          const int64_t last_group = (vi + take - 1) >> 3;
          if (data + last_group * bw >= L.len) {
            err = E_EOF;
            break;
          }
          const int64_t b_first = data + ((vi * bw) >> 3);
          const int64_t b_last = data + (((vi + take) * (int64_t)bw + 7) >> 3);
          L.ensure(b_first, b_last + 8);
          // bit offset of chunk value 0 relative to lds[0] (fits 32 bits: the window is 8 KB)
          const int32_t rbit0 = (int32_t)(((L.p + data) - L.ab) * 8 + (vi - got) * (int64_t)bw);
          const uint32_t mask = bw == 32 ? 0xffffffffu : ((1u << bw) - 1);
          const bool tail = b_last + 8 > L.len;  // values may touch bytes past the stream end
          const int64_t end_bit = ((L.p + L.len) - L.ab) * 8;
          // issue every LDS read of the lane's 16 values back to back, select afterwards
#pragma unroll
          for (int k = 0; k < FW_PER_LANE; k++) {
            const int j = FW_PER_LANE * lane + k;
            const bool in = j >= got && j < got + take;
            const int32_t rb = in ? rbit0 + j * bw : 0;
            const uint32_t *q = (const uint32_t *)(L.lds + ((rb >> 3) & ~3));
            uint64_t v = ((uint64_t)q[1] << 32) | q[0];
            uint32_t val = (uint32_t)(v >> (rb & 31)) & mask;
            // zero-fill past the stream end (hybrid_decoder.go:133-141), branch-free
            const int32_t avail = tail ? (int32_t)min<int64_t>(end_bit - rb, 64) : 64;
            const uint32_t amask = avail <= 0 ? 0u : (avail >= 32 ? 0xffffffffu : ((1u << avail) - 1));
            val &= amask;
            key[k] = in ? val : key[k];
          }
          vi += take;
        }
        rem -= take;
        got += take;
      }
      if (err) break;
    }
    // gather + store
    bool bad = false;
#pragma unroll
    for (int k = 0; k < FW_PER_LANE; k++) bad |= (FW_PER_LANE * lane + k < cnt) && (int64_t)key[k] >= dict_n;
    if (ballot(bad)) {
      err = E_DICT;
      break;
    }
    const int64_t s0 = e0 + FW_PER_LANE * lane;  // my first entry
    const bool full = FW_PER_LANE * lane + FW_PER_LANE <= cnt;
    if (w == 4) {
      uint32_t v[FW_PER_LANE];
#pragma unroll
      for (int k = 0; k < FW_PER_LANE; k++) {
        const uint8_t *src = dict + (int64_t)key[k] * 4;
        v[k] = aligned_dict ? *(const uint32_t *)src : load_u32_unaligned(src);
      }
      uint32_t *o = (uint32_t *)(out + s0 * 4);
      if (full && (((uintptr_t)o) & 15) == 0) {
#pragma unroll
        for (int k = 0; k < FW_PER_LANE; k += 4) *(uint4 *)(o + k) = make_uint4(v[k], v[k + 1], v[k + 2], v[k + 3]);
      } else {
#pragma unroll
        for (int k = 0; k < FW_PER_LANE; k++)
          if (FW_PER_LANE * lane + k < cnt) o[k] = v[k];
      }
    } else {
      uint64_t v[FW_PER_LANE];
#pragma unroll
      for (int k = 0; k < FW_PER_LANE; k++) {
        const uint8_t *src = dict + (int64_t)key[k] * 8;
        v[k] = aligned_dict ? *(const uint64_t *)src : load_u64_unaligned(src);
      }
      uint64_t *o = (uint64_t *)(out + s0 * 8);
      if (full && (((uintptr_t)o) & 15) == 0) {
#pragma unroll
        for (int k = 0; k < FW_PER_LANE; k += 2)
          *(uint4 *)(o + k) = make_uint4((uint32_t)v[k], (uint32_t)(v[k] >> 32), (uint32_t)v[k + 1], (uint32_t)(v[k + 1] >> 32));
      } else {
#pragma unroll
        for (int k = 0; k < FW_PER_LANE; k++)
          if (FW_PER_LANE * lane + k < cnt) o[k] = v[k];
      }
    }
  }
  if (err) set_status(a.status, page, ST_VALUES, err);
}

// ===========================================================================
// K5d: flat, required, fixed-width RLE_DICTIONARY pages whose key stream fits
// in LDS — one 256-thread workgroup per page.
//   1. the whole key stream is staged into LDS with 16-byte loads;
//   2. wave 0 walks the run headers (hybrid_decoder.go:143-166) into an LDS
//      run table.  The walk is speculative: after a bit-packed header it
//      checks, one candidate per lane, whether the next 63 runs repeat the
//      same header at the same stride (what an encoder writes for
//      high-entropy keys) and accepts the matching prefix in one step;
//   3. all four waves decode 1024-value steps (step s -> wave s % 4) with the
//      run table held in registers (lane i = entry i of a 64-entry window):
//      keys from LDS, dictionary gathers from HBM/L2, 16-byte stores.
// A page with more runs than the table holds is processed in table-sized
// rounds.
// ===========================================================================
constexpr int DW_RUNS = 512;  // run-table entries per round

struct RunEnt {
  int32_t start;    // first value of the run (page-relative)
  int32_t bitpos;   // bit offset of the run's data in the staged stream; -1 for RLE
  uint32_t rle_val;
  int32_t pad;
};

// DW_STREAM: staged key-stream bytes per workgroup.  Three instantiations
// (8 / 31 / 56 KB) so small pages do not pay the LDS (occupancy) of big ones;
// the host routes each page by its body length.
template <int DW_STREAM>
__global__ __launch_bounds__(256) void k_decode_dict_wg(KArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t sstream[DW_STREAM + 32];
  __shared__ __attribute__((aligned(16))) RunEnt runs[DW_RUNS + 1];
  __shared__ int32_t s_nruns, s_cover, s_err, s_dict_err;
  const int wv = (int)ufirst(threadIdx.x >> 6);
  const int lane = lane_id();
  if ((int)blockIdx.x >= a.nlist) return;
  const int page = ufirst(a.list[blockIdx.x]);
  if (page_status(a.status, page) != STATUS_OK) return;
  const PageDesc d = a.pages[page];
  if (d.dict < 0 || page_status(a.status, d.dict) != STATUS_OK) {
    if (d.dict < 0 && threadIdx.x == 0) atomicMin(&a.status[page], make_status(ST_VALUES, E_DICT));
    return;
  }
  const ColDesc c = a.cols[d.col];
  const PageInfo pi = a.info[page];
  const int n = (int)ufirst((uint32_t)d.num_values);
  if (n == 0) return;
  const uint8_t *vals = body_ptr(a, d, page) + pi.val_off;
  const int64_t slen = ufirst64((int64_t)pi.val_len - 1);  // key stream after the bit-width byte
  const uint8_t *ks = vals + 1;
  const int w = (int)ufirst((uint32_t)c.width);
  uint8_t *out = c.values + d.level_base * w;
  const PageDesc dp = a.pages[d.dict];
  const uint8_t *dict = body_ptr(a, dp, d.dict);
  const int64_t dict_n = ufirst64(dp.num_values);
  const int bw = (int)ufirst((uint32_t)pi.idx_bw);
  const bool aligned_dict = (((uintptr_t)dict) & (w - 1)) == 0;

  STAMP(0);
  // 1. stage the key stream: sstream[i] = byte at address A + i, A = ks aligned down to 16
  const uintptr_t A = (uintptr_t)ks & ~(uintptr_t)15;
  const int32_t skew = (int32_t)ufirst((uint32_t)((uintptr_t)ks - A));
  const int64_t nbytes = skew + slen;  // the host routes only pages that fit
  for (int64_t off = (int64_t)threadIdx.x * 16; off < nbytes + 16; off += 256 * 16)
    *(uint4 *)(sstream + off) = off < nbytes ? *(const uint4 *)(A + off) : make_uint4(0, 0, 0, 0);
  if (threadIdx.x == 0) {
    s_err = 0;
    s_dict_err = 0;
  }
  __syncthreads();
  STAMP(1);

  int64_t hpos = 0;        // wave 0: next header (stream offset)
  int32_t covered = 0;     // values covered by completed rounds
  const int64_t end_bit = (int64_t)(skew + slen) * 8;
  const uint32_t mask = bw == 32 ? 0xffffffffu : ((1u << bw) - 1);

  while (covered < n) {
    // 2. wave 0 walks up to DW_RUNS run headers
    if (wv == 0) {
      int32_t nr = 0, v = covered;
      uint32_t err = E_OK;
      if (bw == 0) {  // hybrid_decoder.go:84-86: all zeros, nothing read
        if (lane == 0) runs[0] = RunEnt{v, -1, 0u, 0};
        nr = 1;
        v = n;
      }
      while (v < n && nr < DW_RUNS && !err) {
        hpos = ufirst64(hpos);
        v = (int32_t)ufirst((uint32_t)v);
        nr = (int32_t)ufirst((uint32_t)nr);
        const int64_t h0 = hpos;
        uint64_t h = 0;
        uint32_t sh = 0;
        for (int i = 0;; i++) {
          if (hpos >= slen) {
            err = E_EOF;
            break;
          }
          uint32_t b = ufirst(sstream[skew + hpos]);
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
        if (h > 0x7fffffffull) {
          err = E_RLE;
          break;
        }
        const int32_t hl = (int32_t)(hpos - h0);  // header length in bytes
        if (h & 1) {
          const int64_t g = (int64_t)(h >> 1);
          if (g == 0) {
            err = E_RLE;
            break;
          }
          // every group the page needs must start inside the stream (:133-141)
          int64_t need = min<int64_t>(g * 8, (int64_t)(n - v));
          if (hpos + ((need - 1) >> 3) * bw >= slen) {
            err = E_EOF;
            break;
          }
          if (lane == 0) runs[nr] = RunEnt{v, (int32_t)((skew + hpos) * 8), 0u, 0};
          v = (int32_t)min<int64_t>((int64_t)v + g * 8, (int64_t)n);
          hpos += g * (int64_t)bw;
          nr++;
          // speculate: lane k checks for the same header again k strides ahead
          const int64_t stride = hl + g * (int64_t)bw;
          const int64_t cand = hpos + (int64_t)lane * stride;  // candidate header of run nr + lane
          const int64_t cstart = (int64_t)v + (int64_t)lane * g * 8;
          bool ok = cstart < n && nr + lane < DW_RUNS && cand + hl <= slen;
          if (ok) {
            for (int q = 0; q < hl; q++) ok &= sstream[skew + cand + q] == sstream[skew + h0 + q];
            const int64_t cneed = min<int64_t>(g * 8, (int64_t)n - cstart);
            ok &= cand + hl + ((cneed - 1) >> 3) * bw < slen;
          }
          const uint64_t okm = ballot(ok);
          const int m = (int)__builtin_ctzll(~okm);  // leading accepted candidates (lanes 0..m-1)
          if (m > 0) {
            if (lane < m) runs[nr + lane] = RunEnt{(int32_t)cstart, (int32_t)((skew + cand + hl) * 8), 0u, 0};
            v = (int32_t)min<int64_t>((int64_t)v + (int64_t)m * g * 8, (int64_t)n);
            hpos += (int64_t)m * stride;
            nr += m;
          }
        } else {
          int64_t cr = (int64_t)(h >> 1);
          if (cr == 0) {
            err = E_RLE;
            break;
          }
          int sz = (bw + 7) >> 3;
          if (hpos >= slen || hpos + sz > slen) {
            err = E_EOF;
            break;
          }
          uint32_t val = 0;
          for (int k = 0; k < sz; k++) val |= ufirst(sstream[skew + hpos + k]) << (8 * k);
          hpos += sz;
          if (bw < 32 && (val >> bw) != 0) {
            err = E_RLE;
            break;
          }
          if (lane == 0) runs[nr] = RunEnt{v, -1, val, 0};
          v = (int32_t)min<int64_t>((int64_t)v + cr, (int64_t)n);
          nr++;
        }
      }
      if (lane == 0) {
        runs[nr] = RunEnt{v, 0, 0u, 0};  // sentinel: end of coverage
        s_nruns = nr;
        s_cover = v;
        if (err) s_err = (int32_t)err;
      }
    }
    __syncthreads();
    STAMP(2);
    const int32_t nr = (int32_t)ufirst((uint32_t)s_nruns), cover = (int32_t)ufirst((uint32_t)s_cover);
    // on a header error, the values before it are still decoded: a dictionary
    // index error among them comes first in the reference (type_dict.go:45-53)

    // 3. steps of 1024 values over [covered, cover); step boundaries are page-absolute.
    // Run table window in registers: lane i holds entry wb + i (and the next start).
    int32_t wb = -1;
    int32_t r_start = 0, r_next = 0, r_bit = 0;
    uint32_t r_val = 0;
    for (int32_t e0 = (covered / FW_STEP) * FW_STEP + wv * FW_STEP; e0 < cover; e0 += FW_WAVES * FW_STEP) {
      const int32_t lo = max(e0, covered), hi = min(e0 + FW_STEP, cover);
      // window containing the run of `lo`: first entry with start <= lo < next start
      while (true) {
        if (wb < 0 || !(ufirst(__builtin_amdgcn_readlane(r_start, 0)) <= lo &&
                        lo < (int32_t)__builtin_amdgcn_readlane(r_next, min(63, nr - 1 - wb)))) {
          // (re)load: binary search the LDS table for the run of lo, window starts there
          int32_t l = 0, h2 = nr - 1;
          while (l < h2) {
            int32_t mid = (l + h2 + 1) >> 1;
            if ((int32_t)ufirst((uint32_t)runs[mid].start) <= lo) l = mid;
            else h2 = mid - 1;
          }
          wb = l;
          const int32_t ei = min(wb + lane, nr - 1);
          const RunEnt re = runs[ei];
          r_start = re.start;
          r_bit = re.bitpos;
          r_val = re.rle_val;
          r_next = runs[ei + 1].start;
        }
        break;
      }
      // per-lane: run of my first value j0, found by binary search over the window lanes
      const int32_t j0 = e0 + FW_PER_LANE * lane;
      const int32_t wn = min(64, nr - wb);  // valid window entries
      int32_t ri = 0;
#pragma unroll
      for (int stp = 32; stp >= 1; stp >>= 1) {
        int32_t cand = ri + stp;
        int32_t cs = (int32_t)shfl32((uint32_t)r_start, min(cand, 63));
        if (cand < wn && cs <= j0) ri = cand;
      }
      int32_t my_start = (int32_t)shfl32((uint32_t)r_start, ri);
      int32_t my_next = (int32_t)shfl32((uint32_t)r_next, ri);
      int32_t my_bit = (int32_t)shfl32((uint32_t)r_bit, ri);
      uint32_t my_val = shfl32(r_val, ri);
      uint32_t key[FW_PER_LANE];
#pragma unroll
      for (int k = 0; k < FW_PER_LANE; k++) {
        const int32_t j = j0 + k;
        const bool cross = j >= my_next && ri + 1 < wn;  // crossed into the next run (rare: runs are long)
        if (ballot(cross)) {  // wave-uniform branch: every lane takes part in the shuffles
          ri += cross ? 1 : 0;
          my_start = (int32_t)shfl32((uint32_t)r_start, ri);
          my_next = (int32_t)shfl32((uint32_t)r_next, ri);
          my_bit = (int32_t)shfl32((uint32_t)r_bit, ri);
          my_val = shfl32(r_val, ri);
        }
        const bool in = j >= lo && j < hi;
        const int32_t rb = (in && my_bit >= 0) ? my_bit + (j - my_start) * bw : 0;
        const uint32_t *q = (const uint32_t *)(sstream + ((rb >> 3) & ~3));
        uint64_t vv = ((uint64_t)q[1] << 32) | q[0];
        uint32_t val = (uint32_t)(vv >> (rb & 31)) & mask;
        const int32_t avail = (int32_t)min<int64_t>(end_bit - rb, 64);  // zero past the stream end
        val &= avail <= 0 ? 0u : (avail >= 32 ? 0xffffffffu : ((1u << avail) - 1));
        key[k] = my_bit < 0 ? my_val : val;
      }
      bool bad = false;
#pragma unroll
      for (int k = 0; k < FW_PER_LANE; k++) {
        const int32_t j = j0 + k;
        bad |= j >= lo && j < hi && (int64_t)key[k] >= dict_n;
      }
      if (ballot(bad)) {
        if (lane == 0) {
          atomicMin(&a.status[page], make_status(ST_VALUES, E_DICT));
          s_dict_err = 1;
        }
        continue;
      }
      const bool full = j0 >= lo && j0 + FW_PER_LANE <= hi;
      if (w == 4) {
        uint32_t vv[FW_PER_LANE];
#pragma unroll
        for (int k = 0; k < FW_PER_LANE; k++) {
          const uint8_t *sp = dict + (int64_t)(j0 + k < hi ? key[k] : 0) * 4;
          vv[k] = aligned_dict ? *(const uint32_t *)sp : load_u32_unaligned(sp);
        }
        uint32_t *o = (uint32_t *)(out + (int64_t)j0 * 4);
        if (full && (((uintptr_t)o) & 15) == 0) {
#pragma unroll
          for (int k = 0; k < FW_PER_LANE; k += 4) *(uint4 *)(o + k) = make_uint4(vv[k], vv[k + 1], vv[k + 2], vv[k + 3]);
        } else {
#pragma unroll
          for (int k = 0; k < FW_PER_LANE; k++)
            if (j0 + k >= lo && j0 + k < hi) o[k] = vv[k];
        }
      } else {
        uint64_t vv[FW_PER_LANE];
#pragma unroll
        for (int k = 0; k < FW_PER_LANE; k++) {
          const uint8_t *sp = dict + (int64_t)(j0 + k < hi ? key[k] : 0) * 8;
          vv[k] = aligned_dict ? *(const uint64_t *)sp : load_u64_unaligned(sp);
        }
        uint64_t *o = (uint64_t *)(out + (int64_t)j0 * 8);
        if (full && (((uintptr_t)o) & 15) == 0) {
#pragma unroll
          for (int k = 0; k < FW_PER_LANE; k += 2)
            *(uint4 *)(o + k) = make_uint4((uint32_t)vv[k], (uint32_t)(vv[k] >> 32), (uint32_t)vv[k + 1], (uint32_t)(vv[k + 1] >> 32));
        } else {
#pragma unroll
          for (int k = 0; k < FW_PER_LANE; k++)
            if (j0 + k >= lo && j0 + k < hi) o[k] = vv[k];
        }
      }
    }
    covered = cover;
    __syncthreads();  // the run table is rewritten next round
    STAMP(3);
    if (s_err) {
      if (threadIdx.x == 0 && !s_dict_err) atomicMin(&a.status[page], make_status(ST_VALUES, (uint32_t)s_err));
      return;
    }
    if (s_dict_err) return;
  }
}

// level-error precedence pass: for pages that failed in k_decode at the
// values or def stage, finish decoding the earlier level streams to see if
// the reference would have failed there first.
__global__ __launch_bounds__(256) void k_level_check(KArgs a) {
  const int gi = blockIdx.x * 4 + (int)ufirst(threadIdx.x >> 6);
  if (gi >= a.nlist) return;
  const int page = ufirst(a.list[gi]);
  uint32_t st = page_status(a.status, page);
  if (st == STATUS_OK || (st >> 16) <= ST_REP) return;
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
  k.jobs = (pq::CopyJob *)p->jobs;
  k.njobs = p->njobs;
  k.max_jobs = p->max_jobs;
  k.job_base = p->job_base;
  k.job_owner = p->job_owner;
  k.dbg = p->dbg;
  return k;
}

int pq_launch(int which, const pq_launch_args *p, hipStream_t s) {
  pq::KArgs k = to_k(p);
  if (which == 4) {
    if (k.ncols <= 0) return 0;
    hipLaunchKernelGGL(pq::k_scan, dim3(k.ncols), dim3(256), 0, s, k);
    return hipGetLastError() == hipSuccess ? 0 : 17;
  }
  if (which == 6) {  // deferred literal copies: fixed grid, the job count lives on the device
    if (k.max_jobs == 0) return 0;
    hipLaunchKernelGGL(pq::k_copy, dim3(k.max_jobs), dim3(256), 0, s, k);
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
    case 7: hipLaunchKernelGGL(pq::k_decode_flat, grid, block, 0, s, k); break;
    case 8: hipLaunchKernelGGL(pq::k_decode_dict_wg<8 * 1024>, dim3(k.nlist), block, 0, s, k); break;
    case 9: hipLaunchKernelGGL(pq::k_decode_dict_wg<31 * 1024>, dim3(k.nlist), block, 0, s, k); break;
    case 10: hipLaunchKernelGGL(pq::k_decode_dict_wg<56 * 1024>, dim3(k.nlist), block, 0, s, k); break;
    default: return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 17;
}

}  // extern "C"
