// pq_host.cpp — host side of libpqgpu.so: compact-Thrift footer and page-header
// parsing, schema -> levels, the page walker that builds the batch descriptor
// table, the codec registry, and the C ABI declared in include/pqgpu.h.
//
// Host work is limited to what the reference does before the per-value loops:
// readFileMetaData (file_meta.go:14-62), makeSchema (schema.go:996),
// readChunk/readPages page-header walk (chunk_reader.go:206-378).  Every byte
// of page payload goes to HBM in one hipMemcpyAsync per batch; decompression
// (Snappy) and all decoding run in pq_kernels.hip.
#include <chrono>
#include <ctype.h>
#include <errno.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <pthread.h>
#include <sched.h>
#include <zlib.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pqgpu.h"
#include "pq_common.h"



using namespace pq;

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
  int32_t ldn[6];   // k_expand_ld groups per (width 4, 8) x LDS class, in that order
  int32_t ldl[6];   // dynamic LDS bytes of each
  const uint32_t *status0;
  const void *zr;
  int32_t nzr, npages;
  const uint8_t *in_end, *stage_end;  // allocation ends (incl. pad): bounds of the guarded debug build
  const void *sitems;                 // k_snappy work items {Snappy-list position, segment}
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
int pq_launch(int which, const pq_launch_args *p, hipStream_t s);
int pq_launch_inflate(const pq::InflateArgs *a, hipStream_t s);  // pq_inflate.hip
int pq_launch_nest(const pq::NestArgs *a, hipStream_t s);        // pq_nest.hip
extern int pq_launch_fail_which, pq_launch_fail_err;
static constexpr int64_t kSnapSeg = 65536;  // pq_kernels.hip SNAP_SEG
}

namespace {

thread_local std::string g_err;
void set_err(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}

// ---------------------------------------------------------------------------
// compact Thrift reader (read side only; unknown fields skipped)
// ---------------------------------------------------------------------------
struct TReader {
  const uint8_t *p;
  size_t n, pos = 0;
  bool err = false;
  int depth = 0;
  TReader(const uint8_t *ptr, size_t len) : p(ptr), n(len) {}
  uint8_t byte() {
    if (pos >= n) {
      err = true;
      return 0;
    }
    return p[pos++];
  }
  uint64_t uvar() {
    uint64_t x = 0;
    for (int s = 0; s < 70; s += 7) {
      uint8_t b = byte();
      if (err) return 0;
      x |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return x;
    }
    err = true;
    return 0;
  }
  int64_t zz() {
    uint64_t u = uvar();
    return (int64_t)(u >> 1) ^ -(int64_t)(u & 1);
  }
  // returns field id (>0), 0 at stop/error; -1 for an explicit id of 0
  int field(int16_t &last, int &type) {
    uint8_t h = byte();
    if (err || h == 0) return 0;
    type = h & 0x0f;
    int delta = h >> 4;
    last = delta ? (int16_t)(last + delta) : (int16_t)zz();
    return last == 0 ? -1 : last;
  }
  void list_header(int &etype, int64_t &size) {
    uint8_t h = byte();
    size = h >> 4;
    etype = h & 0x0f;
    if (size == 15) size = (int64_t)uvar();
    if (size < 0 || (uint64_t)size > (n - pos) * 8 + 16) err = true;
  }
  void skip(int type) {
    if (err) return;
    switch (type) {
      case 1: case 2: break;
      case 3: byte(); break;
      case 4: case 5: case 6: uvar(); break;
      case 7:
        if (n - pos < 8) err = true;
        else pos += 8;
        break;
      case 8: {
        uint64_t l = uvar();
        if (err || l > n - pos) err = true;
        else pos += l;
        break;
      }
      case 9: case 10: {
        int et;
        int64_t sz;
        list_header(et, sz);
        for (int64_t i = 0; i < sz && !err; i++) {
          if (et == 1 || et == 2) byte();
          else skip(et);
        }
        break;
      }
      case 11: {
        uint64_t sz = uvar();
        if (sz == 0) break;
        uint8_t kv = byte();
        if (sz > n - pos) {
          err = true;
          break;
        }
        for (uint64_t i = 0; i < sz && !err; i++) {
          skip(kv >> 4);
          skip(kv & 15);
        }
        break;
      }
      case 12: {
        if (++depth > 64) {
          err = true;
          break;
        }
        int16_t last = 0;
        int t;
        while (!err && field(last, t) != 0) skip(t);
        depth--;
        break;
      }
      default: err = true;
    }
  }
  int32_t i32(int type) {
    if (type == 3) return (int8_t)byte();
    if (type != 4 && type != 5) {
      skip(type);
      err = true;
      return 0;
    }
    return (int32_t)zz();
  }
  int64_t i64(int type) {
    if (type != 4 && type != 5 && type != 6) {
      skip(type);
      err = true;
      return 0;
    }
    return zz();
  }
  std::string str(int type) {
    if (type != 8) {
      skip(type);
      err = true;
      return {};
    }
    uint64_t l = uvar();
    if (err || l > n - pos) {
      err = true;
      return {};
    }
    std::string s((const char *)p + pos, l);
    pos += l;
    return s;
  }
};

struct SchemaElem {  // parquet/parquet.go:3381
  bool has_type = false, has_rep = false, has_children = false, int_unsigned = false;
  int32_t type = 0, type_length = 0, repetition = 0, num_children = 0, converted = -1;
  std::string name;
  bool has_name = false;
};
struct ColumnChunkMeta {  // parquet/parquet.go:8042 / :6822
  bool has_meta = false, has_file_path = false, has_dict_off = false;
  int32_t type = 0, codec = 0;
  int64_t num_values = 0, total_uncompressed = 0, total_compressed = 0, data_page_offset = 0, dict_page_offset = 0;
};
struct RowGroupMeta {
  std::vector<ColumnChunkMeta> cols;
  int64_t num_rows = 0, total_byte_size = 0;
};

void read_int_type(TReader &t, bool &uns) {
  int16_t last = 0;
  int ty, f;
  bool bw = false, sg = false, is_signed = true;
  while ((f = t.field(last, ty)) != 0 && !t.err) {
    if (f == 1 && ty == 3) {
      t.byte();
      bw = true;
    } else if (f == 2 && (ty == 1 || ty == 2)) {
      is_signed = ty == 1;
      sg = true;
    } else t.skip(ty);
  }
  if (!bw || !sg) t.err = true;
  uns = !is_signed;
}
void read_schema_elem(TReader &t, SchemaElem &e) {
  int16_t last = 0;
  int ty, f;
  while ((f = t.field(last, ty)) != 0 && !t.err) {
    switch (f) {
      case 1: e.type = t.i32(ty); e.has_type = true; break;
      case 2: e.type_length = t.i32(ty); break;
      case 3: e.repetition = t.i32(ty); e.has_rep = true; break;
      case 4: e.name = t.str(ty); e.has_name = true; break;
      case 5: e.num_children = t.i32(ty); e.has_children = true; break;
      case 6: e.converted = t.i32(ty); break;
      case 10:
        if (ty == 12) {
          int16_t l2 = 0;
          int t2, f2;
          while ((f2 = t.field(l2, t2)) != 0 && !t.err) {
            if (f2 == 10 && t2 == 12) {
              bool u = false;
              read_int_type(t, u);
              e.int_unsigned = u;
            } else t.skip(t2);
          }
        } else t.skip(ty);
        break;
      default: t.skip(ty);
    }
  }
  if (!e.has_name) t.err = true;
}
void read_col_meta(TReader &t, ColumnChunkMeta &c) {
  int16_t last = 0;
  int ty, f;
  unsigned seen = 0;
  while ((f = t.field(last, ty)) != 0 && !t.err) {
    switch (f) {
      case 1: c.type = t.i32(ty); seen |= 1; break;
      case 2: t.skip(ty); seen |= 2; break;
      case 3: t.skip(ty); seen |= 4; break;
      case 4: c.codec = t.i32(ty); seen |= 8; break;
      case 5: c.num_values = t.i64(ty); seen |= 16; break;
      case 6: c.total_uncompressed = t.i64(ty); seen |= 32; break;
      case 7: c.total_compressed = t.i64(ty); seen |= 64; break;
      case 9: c.data_page_offset = t.i64(ty); seen |= 128; break;
      case 11: c.dict_page_offset = t.i64(ty); c.has_dict_off = true; break;
      default: t.skip(ty);
    }
  }
  if (seen != 255) t.err = true;
}
void read_col_chunk(TReader &t, ColumnChunkMeta &c) {
  int16_t last = 0;
  int ty, f;
  bool has_off = false;
  while ((f = t.field(last, ty)) != 0 && !t.err) {
    if (f == 1) {
      t.str(ty);
      c.has_file_path = true;
    } else if (f == 2) {
      t.i64(ty);
      has_off = true;
    } else if (f == 3 && ty == 12) {
      read_col_meta(t, c);
      c.has_meta = true;
    } else t.skip(ty);
  }
  if (!has_off) t.err = true;
}

// PageHeader parquet/parquet.go:5794 (+ :3953, :4303, :4522)
struct PageHeader {
  int32_t type = 0, uncompressed = 0, compressed = 0;
  bool has_dph = false, has_dict = false, has_v2 = false;
  int32_t dp_num_values = 0, dp_encoding = 0, dp_def_enc = 0, dp_rep_enc = 0;
  int32_t dict_num_values = 0, dict_encoding = 0;
  int32_t v2_num_values = 0, v2_encoding = 0, v2_def_len = 0, v2_rep_len = 0;
};
void read_page_header(TReader &t, PageHeader &h) {
  int16_t last = 0;
  int ty, f;
  unsigned seen = 0;
  while ((f = t.field(last, ty)) != 0 && !t.err) {
    if (f == 1) {
      h.type = t.i32(ty);
      seen |= 1;
    } else if (f == 2) {
      h.uncompressed = t.i32(ty);
      seen |= 2;
    } else if (f == 3) {
      h.compressed = t.i32(ty);
      seen |= 4;
    } else if (f == 5 && ty == 12) {
      int16_t l2 = 0;
      int t2, f2;
      unsigned s2 = 0;
      while ((f2 = t.field(l2, t2)) != 0 && !t.err) {
        switch (f2) {
          case 1: h.dp_num_values = t.i32(t2); s2 |= 1; break;
          case 2: h.dp_encoding = t.i32(t2); s2 |= 2; break;
          case 3: h.dp_def_enc = t.i32(t2); s2 |= 4; break;
          case 4: h.dp_rep_enc = t.i32(t2); s2 |= 8; break;
          default: t.skip(t2);
        }
      }
      if (s2 != 15) t.err = true;
      h.has_dph = true;
    } else if (f == 7 && ty == 12) {
      int16_t l2 = 0;
      int t2, f2;
      unsigned s2 = 0;
      while ((f2 = t.field(l2, t2)) != 0 && !t.err) {
        switch (f2) {
          case 1: h.dict_num_values = t.i32(t2); s2 |= 1; break;
          case 2: h.dict_encoding = t.i32(t2); s2 |= 2; break;
          default: t.skip(t2);
        }
      }
      if (s2 != 3) t.err = true;
      h.has_dict = true;
    } else if (f == 8 && ty == 12) {
      int16_t l2 = 0;
      int t2, f2;
      unsigned s2 = 0;
      while ((f2 = t.field(l2, t2)) != 0 && !t.err) {
        switch (f2) {
          case 1: h.v2_num_values = t.i32(t2); s2 |= 1; break;
          case 2: t.i32(t2); s2 |= 2; break;
          case 3: t.i32(t2); s2 |= 4; break;
          case 4: h.v2_encoding = t.i32(t2); s2 |= 8; break;
          case 5: h.v2_def_len = t.i32(t2); s2 |= 16; break;
          case 6: h.v2_rep_len = t.i32(t2); s2 |= 32; break;
          default: t.skip(t2);
        }
      }
      if (s2 != 63) t.err = true;
      h.has_v2 = true;
    } else t.skip(ty);
  }
  if (seen != 7) t.err = true;
}

int value_width(int ptype, int type_length) {
  switch (ptype) {
    case T_INT32: case T_FLOAT: return 4;
    case T_INT64: case T_DOUBLE: return 8;
    case T_INT96: return 12;
    case T_FLBA: return type_length;
    case T_BOOLEAN: return 1;  // one byte (0 / 1) per value
    default: return 0;
  }
}

// ---------------------------------------------------------------------------
// codec registry (compress.go:16-27, :130-156)
// ---------------------------------------------------------------------------
struct Codec {
  pqg_decompress_fn fn = nullptr;  // nullptr: built-in
  void *user = nullptr;
};
std::shared_mutex g_codec_mu;
std::map<int, Codec> &codecs() {
  static std::map<int, Codec> m = {{PQG_CODEC_UNCOMPRESSED, {}}, {PQG_CODEC_SNAPPY, {}}, {PQG_CODEC_GZIP, {}}};
  return m;
}

int gzip_inflate(const uint8_t *src, size_t n, uint8_t *dst, size_t cap, size_t *out_len) {
  z_stream zs;
  memset(&zs, 0, sizeof(zs));
  if (inflateInit2(&zs, 16 + MAX_WBITS) != Z_OK) return PQG_ERR_CODEC;
  zs.next_in = (Bytef *)src;
  zs.avail_in = (uInt)n;
  zs.next_out = dst;
  zs.avail_out = (uInt)cap;
  int rc = inflate(&zs, Z_FINISH);
  *out_len = cap - zs.avail_out;
  inflateEnd(&zs);
  if (rc == Z_STREAM_END) return PQG_OK;
  return rc == Z_BUF_ERROR ? PQG_ERR_SIZE : PQG_ERR_CODEC;
}

// Host decompression for pages whose codec is not run on the GPU.  Returns
// 0, or a status; the size check of newBlockReader is done by the caller.
int host_decompress(int codec, const uint8_t *src, size_t n, uint8_t *dst, size_t cap, size_t *out_len,
                    bool *on_device) {
  std::shared_lock<std::shared_mutex> lk(g_codec_mu);  // held during the call, like compress.go:91-92
  auto it = codecs().find(codec);
  if (it == codecs().end()) return PQG_ERR_CODEC;
  if (it->second.fn) {
    *on_device = false;
    return it->second.fn(it->second.user, src, n, dst, cap, out_len);
  }
  switch (codec) {
    case PQG_CODEC_UNCOMPRESSED:
      *on_device = false;
      if (n > cap) return PQG_ERR_SIZE;
      memcpy(dst, src, n);
      *out_len = n;
      return PQG_OK;
    case PQG_CODEC_SNAPPY:
      *on_device = true;
      return PQG_OK;
    case PQG_CODEC_GZIP:
      *on_device = false;
      return gzip_inflate(src, n, dst, cap, out_len);
  }
  return PQG_ERR_CODEC;
}
bool codec_builtin(int codec, bool *registered) {
  std::shared_lock<std::shared_mutex> lk(g_codec_mu);
  auto it = codecs().find(codec);
  *registered = it != codecs().end();
  return *registered && it->second.fn == nullptr;
}

}  // namespace

// ===========================================================================
// objects
// ===========================================================================
// Host threads that fill the pinned upload ring: each ring buffer's gather
// (memcpy from the file mapping) is split into parts run by the pool and the
// calling thread together, so the copy into pinned memory keeps up with the
// PCIe DMA (one thread copies at about half the DMA rate).
// The GPU's NUMA node (its PCI device's numa_node in sysfs) and the CPUs of
// that node this process may run on: the pinned upload ring is allocated and
// first touched there, and the gather threads run there, so the H2D DMA
// reads memory on the GPU's own socket (the box of round 6: GPU on node 1 of
// 2, the process allowed on all 256 CPUs of both; tools/numa_probe.py).
// PQG_NO_NUMA=1 (analysis) leaves placement to the scheduler.
static bool gpu_node_cpus(int device, cpu_set_t *out) {
  char bdf[64] = {0};
  if (hipDeviceGetPCIBusId(bdf, (int)sizeof(bdf), device) != hipSuccess) return false;
  for (char *q = bdf; *q; q++) *q = (char)tolower((unsigned char)*q);
  char path[256];
  snprintf(path, sizeof(path), "/sys/bus/pci/devices/%s/numa_node", bdf);
  FILE *f = fopen(path, "r");
  int node = -1;
  if (!f) return false;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  if (node < 0) return false;
  snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", node);
  f = fopen(path, "r");
  if (!f) return false;
  char list[4096] = {0};
  const bool ok = fgets(list, sizeof(list), f) != nullptr;
  fclose(f);
  if (!ok) return false;
  cpu_set_t allowed;
  if (sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return false;
  CPU_ZERO(out);
  for (char *tok = strtok(list, ",\n"); tok; tok = strtok(nullptr, ",\n")) {
    int a = -1, b = -1;
    if (sscanf(tok, "%d-%d", &a, &b) < 2) b = a;
    for (int c = a; c >= 0 && c <= b && c < CPU_SETSIZE; c++)
      if (CPU_ISSET(c, &allowed)) CPU_SET(c, out);
  }
  return CPU_COUNT(out) > 0;
}

struct GatherPool {
  std::vector<std::thread> th;
  cpu_set_t cpus;          // where the threads run (when `bind`)
  bool bind = false;
  std::mutex mu;
  std::condition_variable go, done_cv;
  std::function<void(int)> job;
  int nparts = 0, next = 0, done = 0;
  uint64_t gen = 0;
  bool stop = false;
  void start(int n) {
    for (int i = 0; i < n; i++)
      th.emplace_back([this] {
        if (bind) pthread_setaffinity_np(pthread_self(), sizeof(cpus), &cpus);
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
          go.wait(lk, [&] { return stop || gen != seen; });
          if (stop) return;
          seen = gen;
          while (next < nparts) {
            const int p = next++;
            lk.unlock();
            job(p);
            lk.lock();
            if (++done == nparts) done_cv.notify_all();
          }
        }
      });
  }
  // runs f(0 .. parts-1) on the pool and the calling thread; returns when all are done
  void run(int parts, const std::function<void(int)> &f) {
    std::unique_lock<std::mutex> lk(mu);
    job = f;
    nparts = parts;
    next = done = 0;
    gen++;
    go.notify_all();
    while (next < nparts) {
      const int p = next++;
      lk.unlock();
      f(p);
      lk.lock();
      if (++done == nparts) done_cv.notify_all();
    }
    done_cv.wait(lk, [&] { return done == nparts; });
    nparts = 0;
  }
  ~GatherPool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    go.notify_all();
    for (auto &t : th) t.join();
  }
};

struct pqg_ctx {
  int device = 0;
  int cus = 256;  // compute units (k_snappy's segmentation threshold)
  hipStream_t stream = nullptr;
  hipStream_t side[3] = {nullptr, nullptr, nullptr};  // concurrent size-class decode launches
  hipEvent_t fork = nullptr, join[3] = {nullptr, nullptr, nullptr};
  std::mutex launch_mu;  // (lane 0: the fields above)
  // a second decode lane (stream, side streams, fork / join events): a
  // pqg_stream puts consecutive slices on alternate lanes, so the next slice's
  // decode runs beside the tail of the current one
  struct Lane {
    hipStream_t stream = nullptr;
    hipStream_t side[3] = {nullptr, nullptr, nullptr};
    hipEvent_t fork = nullptr, join[3] = {nullptr, nullptr, nullptr};
    std::mutex mu;
  } lane1;
  // batch set-up stream: the H2D copies of chunk bytes run here, and a batch's
  // decodes wait on its `ready` event, so a pqg_stream worker can upload the
  // next slice while the context stream decodes the current one
  hipStream_t upload = nullptr;
  // (launch_mu: launch sequences, which share a lane's fork / join events,
  // from several host threads — a pqg_stream's worker runs counting passes
  // beside the caller's decodes)
  // pinned upload ring (allocated on first use): chunk bytes are copied into
  // one buffer while the DMA of the previous one runs
  static constexpr int kRingBufs = 4;
  static constexpr size_t kRingBytes = 16u << 20;
  void *pin[kRingBufs] = {};
  hipEvent_t pin_ev[kRingBufs] = {};
  bool pin_busy[kRingBufs] = {};  // pin_ev recorded after a DMA that may still read the buffer
  std::chrono::steady_clock::time_point pin_t[kRingBufs];  // when each buffer's last DMA was issued
  int pin_next = 0;
  std::mutex upload_mu;  // one ring_upload at a time per context
  GatherPool pool;       // PQG_UPLOAD_THREADS - 1 helper threads (started on first upload)
  bool pool_started = false;
  std::string err;
};

// host -> device upload of the input layout straight from the file's pages
// through the context's pinned ring (each buffer filled — by the gather pool —
// while the DMA of the previous one runs); alignment gaps are zeroed.  The
// DMAs are queued on `s` and the call returns without waiting for the last
// ones (a later upload waits for a buffer's event before refilling it).
static bool getenv_flag(const char *name);
// Analysis knobs (A/B routes and tuning sweeps of DESIGN.md): read only in
// the analysis build (`make -C parquet-go_amd/csrc analysis` ->
// libpqgpu_analysis.so, -DPQ_ANALYSIS); the shipped library takes every
// default, so each route it can take is one the GPU suite runs.
static const char *knob(const char *name) {
#ifdef PQ_ANALYSIS
  return getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}
static bool knob_flag(const char *name) {
  const char *v = knob(name);
  return v && v[0] == '1';
}
template <class Layout>
static int ring_upload(pqg_ctx *c, uint8_t *dst, const Layout &in, hipStream_t s, double *gather_ms = nullptr,
                       double *wait_ms = nullptr) {
  const size_t n = in.n;
  std::lock_guard<std::mutex> lk(c->upload_mu);
  if (!c->pin[0]) {
    // allocated and first touched by this thread moved to the GPU's node
    static const bool numa_off = knob_flag("PQG_NO_NUMA");
    cpu_set_t old;
    bool moved = false;
    if (!numa_off && gpu_node_cpus(c->device, &c->pool.cpus) &&
        pthread_getaffinity_np(pthread_self(), sizeof(old), &old) == 0) {
      c->pool.bind = true;
      moved = pthread_setaffinity_np(pthread_self(), sizeof(c->pool.cpus), &c->pool.cpus) == 0;
    }
    for (int i = 0; i < pqg_ctx::kRingBufs; i++) {
      if (hipHostMalloc(&c->pin[i], pqg_ctx::kRingBytes, hipHostMallocDefault) != hipSuccess ||
          hipEventCreateWithFlags(&c->pin_ev[i], hipEventDisableTiming) != hipSuccess) {
        c->pin[i] = nullptr;
        if (moved) pthread_setaffinity_np(pthread_self(), sizeof(old), &old);
        for (const auto &r : in.ranges)  // pageable fallback
          if (r.len && hipMemcpy(dst + r.off, r.src, r.len, hipMemcpyHostToDevice) != hipSuccess) return 1;
        return 0;
      }
      memset(c->pin[i], 0, pqg_ctx::kRingBytes);
    }
    if (moved) pthread_setaffinity_np(pthread_self(), sizeof(old), &old);
  }
  if (!c->pool_started) {
    const char *e = getenv("PQG_UPLOAD_THREADS");
    const int nt = std::max(1, std::min(e ? atoi(e) : 6, 32));
    c->pool.start(nt - 1);
    c->pool_started = true;
  }
  const int nthreads = (int)c->pool.th.size() + 1;
  static const bool trace = getenv("PQG_TRACE_CREATE") != nullptr;
  double t_wait = 0, t_gather = 0;
  auto now = [] { return std::chrono::steady_clock::now(); };
  size_t off = 0;
  while (off < n) {
    const int k = c->pin_next;
    const size_t m = std::min(pqg_ctx::kRingBytes, n - off);
    auto t0 = now();
    const bool was_busy = c->pin_busy[k];
    static const bool poll = knob_flag("PQG_RING_POLL");
    if (c->pin_busy[k]) {
      if (poll) {  // (analysis: busy-poll the buffer's event instead of a blocking wait)
        hipError_t q;
        while ((q = hipEventQuery(c->pin_ev[k])) == hipErrorNotReady) std::this_thread::yield();
        if (q != hipSuccess) return 1;
      } else if (hipEventSynchronize(c->pin_ev[k]) != hipSuccess) {
        return 1;
      }
    }
    auto t1 = now();
    const double w_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
    t_wait += w_ms;
    if (trace && was_busy && w_ms > 1.0)  // a long wait for a ring buffer's previous DMA
      fprintf(stderr, "ring_upload: buffer %d (bytes %zu of %zu) waited %.2f ms for its DMA issued %.2f ms earlier\n", k,
              off, n, w_ms, std::chrono::duration<double, std::milli>(t1 - c->pin_t[k]).count());
    c->pin_busy[k] = false;
    // gather [off, off + m) of the layout into the pinned buffer, in parts of >= 1 MiB
    uint8_t *pb = (uint8_t *)c->pin[k];
    const int parts = (int)std::max<size_t>(1, std::min<size_t>((size_t)nthreads, m >> 20));
    auto part = [&](int p) {
      const size_t lo = off + m * (size_t)p / (size_t)parts, hi = off + m * (size_t)(p + 1) / (size_t)parts;
      // first range ending after lo
      size_t ri = (size_t)(std::upper_bound(in.ranges.begin(), in.ranges.end(), lo,
                                            [](size_t v, const decltype(in.ranges[0]) &r) { return v < r.off + r.len; }) -
                           in.ranges.begin());
      size_t at = lo;
      while (at < hi) {
        while (ri < in.ranges.size() && in.ranges[ri].off + in.ranges[ri].len <= at) ri++;
        const size_t next = ri < in.ranges.size() ? in.ranges[ri].off : n;
        if (at < next) {  // alignment gap
          const size_t z = std::min(next, hi) - at;
          memset(pb + (at - off), 0, z);
          at += z;
          continue;
        }
        const auto &r = in.ranges[ri];
        const size_t z = std::min(r.off + r.len, hi) - at;
        memcpy(pb + (at - off), r.src + (at - r.off), z);
        at += z;
      }
    };
    if (parts > 1) c->pool.run(parts, part);
    else part(0);
    t_gather += std::chrono::duration<double, std::milli>(now() - t1).count();
    if (hipMemcpyAsync(dst + off, c->pin[k], m, hipMemcpyHostToDevice, s) != hipSuccess) return 1;
    c->pin_t[k] = now();
    hipEventRecord(c->pin_ev[k], s);
    c->pin_busy[k] = true;
    off += m;
    c->pin_next = (k + 1) % pqg_ctx::kRingBufs;
  }
  if (gather_ms) *gather_ms += t_gather;
  if (wait_ms) *wait_ms += t_wait;
  if (trace)
    fprintf(stderr, "ring_upload %.1f MB: gather %.2f ms (%.1f GB/s, %d threads), ring wait %.2f ms\n", n / 1e6, t_gather,
            t_gather > 0 ? n / t_gather / 1e6 : 0.0, nthreads, t_wait);
  return 0;
}

struct pqg_file {
  const uint8_t *data = nullptr;
  size_t len = 0;
  bool owned = false, mapped = false;
  std::vector<SchemaElem> schema;
  std::vector<RowGroupMeta> rgs;
  std::vector<pqg_column_info> leaves;
  std::vector<std::vector<int>> leaf_rdefs;  // per leaf: def level of each repeated ancestor, outermost first
  int64_t num_rows = 0;
  std::string err;
  ~pqg_file() {
    if (mapped) munmap((void *)data, len);
    else if (owned) free((void *)data);
  }
};

struct ChunkError {  // a host-detected error that ends a chunk's page walk
  int rg, leaf, ord;
  uint32_t stage, code;
};

struct ColumnPlan {
  int leaf;
  pqg_column_info info;
  int flags;
  int32_t page_begin, page_end;
  int64_t levels;
  // device outputs
  void *values = nullptr, *validity = nullptr, *list_offsets = nullptr, *list_validity = nullptr,
       *str_offsets = nullptr, *def_out = nullptr, *rep_out = nullptr;
  size_t values_bytes = 0, validity_bytes = 0, list_off_bytes = 0, list_val_bytes = 0, str_off_bytes = 0;
  int64_t slots = 0, rows = 0, str_bytes = 0;
  // max_rep >= 2: every level's offsets / validity and the leaf slots'
  // validity (k_nest_*, pq_nest.hip), from the emitted levels
  std::vector<int> rdefs;  // def level of each repeated ancestor
  void *nest_off = nullptr, *nest_val = nullptr, *nest_sums = nullptr, *nest_cnt = nullptr;
  int64_t nest_ostride = 0, nest_vstride = 0;
  int32_t nest_nblocks = 0;
};

struct pqg_batch {
  pqg_ctx *ctx = nullptr;
  pqg_file *file = nullptr;
  int rg_begin = 0, rg_end = 0, flags = 0;
  std::vector<ColumnPlan> cols;
  std::vector<int64_t> page_foff;  // per page: payload offset in the file (host)
  std::vector<PageDesc> pages;
  std::vector<uint32_t> status0;  // host-side initial status per page
  std::vector<int32_t> snappy_list, dict_list, data_list;
  std::vector<int32_t> gzip_list;  // gzip pages inflated by k_inflate (BODY_GZIP)
  int32_t gz_off = 0;              // their position in d_lists
  // k_prepare split around the region-parallel length walk: the data pages
  // without a walk (beside it) and those with one (after it), in d_lists
  int32_t prep_a_off = 0, prep_a_n = 0, prep_b_off = 0, prep_b_n = 0;
  int32_t prep_bw = 0;  // the first prep_bw of the after-walk list: walked columns' pages without a walk
  // level / prepare / scan chain split by column kind (round 6): the data
  // pages of repeated columns (all of them k_decode<3> / <5> pages) on side
  // stream 2 up to their decode, the other columns' on the context stream,
  // in d_lists; column runs [c0, c1) of each kind for k_scan
  bool rep_split = false;
  int32_t rep_off = 0, rep_n = 0, flat_off = 0, flat_n = 0;
  std::vector<std::pair<int32_t, int32_t>> rep_cruns, flat_cruns;
  // scan / decode split by length walk (see where it is planned): column runs
  // with (w) and without (o) walked pages, and the walked columns'
  // k_decode<4> pages (the last ngen_str4_w of that launch's list)
  bool sw_split = false;
  int32_t ngen_str4_w = 0;
  std::vector<std::pair<int32_t, int32_t>> w_cruns, o_cruns;
  std::vector<char> w_col;  // per column: it has a walked page
  // Snappy segments: pages longer than kSnapSeg are decoded by one wave per
  // 64 KiB segment (k_snappy_walk finds the segment starts)
  std::vector<int32_t> seg_base;      // per Snappy-list position (+1): first segment
  std::vector<int32_t> snap_items;    // {position, segment} pairs, longest first
  std::vector<int32_t> walk_list;     // positions of the segmented pages
  int32_t n_whole_items = 0;          // snap_items of whole data pages (first), then whole dictionary pages,
  int32_t n_dict_items = 0;           // then segments
  int32_t *d_sitems = nullptr, *d_seg_base = nullptr, *d_walk = nullptr;
  int64_t *d_segs = nullptr;
  uint32_t *d_seg_flag = nullptr;
  std::vector<int32_t> general_list;  // data pages for k_decode (wave per page): k_decode<0> pages, then
  std::vector<int32_t> general_flat;  // k_decode<1> pages (appended to general_list after planning)
  std::vector<int32_t> general_str4;  // k_decode<4> pages (flat required RLE_DICTIONARY BYTE_ARRAY), first of the strings
  std::vector<int32_t> general_str;   // k_decode<2> pages (flat BYTE_ARRAY), appended after those
  std::vector<int32_t> general_nest;  // k_decode<3> pages (lists of fixed-width values), appended last
  int32_t ngen_flat = 0, ngen_str = 0, ngen_str4 = 0, ngen_nest = 0;  // (ngen_str counts <4>'s pages too)
  std::vector<int32_t> dba_list;      // DELTA_BYTE_ARRAY pages: value bytes by k_dba
  std::vector<int32_t> nest_parts;    // k_decode<3> waves: (page, first level, end level) triplets
  std::vector<int32_t> pstr_items;    // k_plain_str: (page, first value) pairs of flat required PLAIN strings
  bool data_may_defer = false;        // some data page's Snappy body may hold a deferred literal
  std::vector<TileJob> tiles;         // k_expand work list (XCD-affine order)
  int64_t run_entries = 0, tile_entries = 0;
  bool any_count = false;
  std::vector<ChunkError> chunk_errors;
  int64_t input_bytes = 0, staged_bytes = 0, h2d_bytes = 0, host_inflated = 0, dict_entries = 0;
  int64_t gzip_in_bytes = 0;  // compressed bytes of the BODY_GZIP pages (k_inflate's input)
  int64_t literal_pages = 0;  // Snappy pages that are one literal, read in place (no k_snappy work)
  // Snappy pages that are only literals (snappy_literal_train): copied by
  // k_copy from the plan, (stream offset in d_in, offset in d_stage, length,
  // 0) per literal; no k_snappy work
  std::vector<int64_t> hjobs;
  int64_t train_pages = 0;
  int64_t *d_hjobs = nullptr;
  // device
  uint8_t *d_in = nullptr, *d_stage = nullptr;
  uint8_t *d_in_alloc = nullptr;  // the allocation d_in lives in (PQG_DEBUG_INPUT_HIGH_WORD shifts d_in inside it)
  size_t in_alloc = 0, stage_alloc = 0;  // bytes incl. pad
  PageDesc *d_pages = nullptr;
  PageInfo *d_info = nullptr;
  uint32_t *d_status = nullptr;  // two arrays of npages (epoch parity)
  bool st_ready[2] = {false, false};  // that array already holds the planned statuses
  uint32_t *d_status0 = nullptr;  // initial statuses (k_reset copies them in every decode)
  void *d_zr = nullptr;           // ZeroRange table of the validity bitmaps
  int32_t nzr = 0;
  ColDesc *d_cols = nullptr;
  uint64_t *d_dict = nullptr;
  int32_t *d_lists = nullptr;
  int32_t *d_parts = nullptr;  // nest_parts on the device
  std::vector<int32_t> str_parts;  // k_decode<2> waves: (page, first level, end level) triplets
  int64_t str_pre_entries = 0;     // prefix-table entries of the split pages (PageDesc::sp_base)
  bool str_split = false;          // some k_decode<2> page is split
  int32_t *d_str_parts = nullptr;
  std::vector<int32_t> str4w_parts;  // walked columns' k_decode<4> waves: (page, first value, end value)
  bool str4w_split = false;          // some of those pages is split
  int32_t *d_str4w_parts = nullptr;
  int64_t *d_str_pre = nullptr;
  int32_t *d_part_pre = nullptr;  // per part: counts before it (k_levels -> k_decode<3>)
  void *d_jobs = nullptr;        // deferred long-literal copy jobs (k_snappy -> k_copy)
  uint32_t *d_njobs = nullptr;   // per Snappy page: jobs written
  int32_t *d_job_base = nullptr, *d_job_owner = nullptr;
  uint32_t max_jobs = 0;
  uint32_t *d_copy_cnt = nullptr;  // deferred literals registered per decode (two, by epoch parity)
  int32_t *d_copy_idx = nullptr;   // their job slots, compact
  int32_t *d_lens = nullptr;       // DELTA string pages: length scratch
  // long PLAIN BYTE_ARRAY pages: region-parallel length walk (k_sw_*)
  std::vector<SwPage> sw_dict, sw_data;  // while planning: dictionary pages, data pages
  std::vector<SwPage> sw_pages;           // dictionary pages first, then data pages
  std::vector<int32_t> sw_items;  // (sw page, chunk of 64 regions) pairs, the dictionary pages' first
  int32_t sw_ndict = 0, sw_dict_items = 0;
  int64_t sw_nreg = 0;
  SwPage *d_sw_pages = nullptr;
  int32_t *d_sw_items = nullptr;
  SwReg *d_sw_regs = nullptr;
  SwRes *d_sw_res = nullptr;
  int64_t lens_entries = 0;
  int64_t lvl_bytes = 0;     // decoded-level scratch (PageDesc::lvl_base)
  // a level page whose streams sit in a compressed V1 body, or whose chunk has
  // a dictionary: k_levels must follow the Snappy phase; otherwise (V2 pages:
  // raw level bytes) it runs beside it (lvl_early)
  bool lvl_late = false;
  uint8_t *d_lvl = nullptr;
  uint64_t *d_dbg = nullptr;     // diagnostic stamps (PQ_STAMPS builds only)
  uint64_t *d_dbg2 = nullptr;
  void *d_runs = nullptr;        // run tables (k_prepare's run walk -> k_expand)
  void *d_runs_alloc = nullptr;  // the allocation d_runs lives in (PQG_DEBUG_INPUT_HIGH_WORD shifts it too)
  void *d_tile_info = nullptr;     // per RUN_TILE values of a tiled page: {first run, first key byte}
  int32_t ex_lds = 0;              // k_expand staged key bytes per wave
  void *d_recs = nullptr;          // k_expand job records (k_prepare writes them every decode)
  int32_t *d_page_jobs = nullptr;  // per tiled page: positions of its jobs in the launch order
  int64_t page_job_entries = 0;
  uint32_t epoch = 0;
  TileJob *d_tiles = nullptr;
  std::vector<LdsGroup> lgroups;     // k_expand_ld groups, 4-byte columns first
  LdsGroup *d_lgroups = nullptr;
  double create_ms[4] = {};          // host time of pqg_batch_create: plan, alloc, upload, outputs + tables
  double upload_gather_ms = 0, upload_wait_ms = 0;  // inside upload: pinned-ring gather, ring-buffer waits
  int32_t ldn[6] = {}, ldl[6] = {};  // groups and LDS bytes: [0], [1] k_expand_mix (width 4, 8),
                                     // [2], [3] k_expand_wg (width 4, 8)
  std::vector<ColDesc> hcols;
  // timing: a ring of event sets, one per decode, harvested by pqg_batch_kernel_times
  static constexpr int kRing = 64;
  hipEvent_t ev[kRing][8] = {};
  int nev = 0;
  bool seg_times = false;  // PQG_SEGMENT_TIMES=1: events between every phase (adds launch gaps)
  int time_every = 1;      // pqg_batch_set_timing: events on every n-th decode (0: none)
  int64_t decodes = 0;
  int ring_head = 0, ring_count = 0;
  double kms_sum[8] = {};
  int kms_n = 0;
  int err_rg = -1, err_leaf = -1, err_page = -1;
  bool decoded = false;
  hipEvent_t ready = nullptr;  // recorded on the context's upload stream after the chunk bytes' H2D
  bool ready_final = false;    // `ready` recorded after every set-up copy (else copies may be in flight)
  bool counted = false;        // the last launch was the counting pass (the next decode resumes from it)
  bool all_srec = false;  // every data page has host-written records: no k_prepare work
  bool no_levels = false;  // no data page has level streams (every selected column required, flat)
  int lane = 0;  // decode lane of the context (pqg_stream: alternate slices)
  std::vector<ExRec> recs_host;  // tiled PLAIN pages' static k_expand records (upload source)
  std::vector<uint8_t> tab_host;  // the small tables (d_pages, d_info, d_lists, ...): host image, uploaded at
                                  // the end of d_in
  std::vector<ColDesc> hcols0;    // column descriptors as first uploaded (before the counting pass)
  std::vector<ZeroRange> zr_host;
};

// timed segments: with PQG_SEGMENT_TIMES every phase, otherwise the decode phase only
static const char *kSegNames[] = {"k_snappy+k_copy", "k_dict_prepare", "k_prepare", "k_scan", "k_decode+k_expand",
                                  "k_level_check"};
static const char *kDecodeName[] = {"k_decode+k_expand"};

#define HIPCHK(x)                                                                 \
  do {                                                                            \
    hipError_t _e = (x);                                                          \
    if (_e != hipSuccess) {                                                       \
      set_err("HIP error %s at %s:%d", hipGetErrorString(_e), __FILE__, __LINE__); \
      return PQG_ERR_DEVICE;                                                      \
    }                                                                             \
  } while (0)

extern "C" {

int pqg_abi_version(void) { return PQGPU_ABI_VERSION; }

int pqg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int pqg_last_error(pqg_ctx *ctx, char *buf, size_t cap) {
  (void)ctx;
  if (buf && cap) snprintf(buf, cap, "%s", g_err.c_str());
  return (int)g_err.size();
}

int pqg_ctx_create(int device, pqg_ctx **out) {
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    set_err("no HIP device available");
    return PQG_ERR_DEVICE;
  }
  if (device < 0 || device >= n) {
    set_err("device %d out of range (%d devices)", device, n);
    return PQG_ERR_ARG;
  }
  HIPCHK(hipSetDevice(device));
  pqg_ctx *c = new pqg_ctx();
  c->device = device;
  hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device);
  if (c->cus <= 0) c->cus = 256;
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    set_err("hipStreamCreate failed");
    return PQG_ERR_DEVICE;
  }
  // PQG_SIDE_PRIO (analysis): three digits, side streams 0..2, '0' default
  // priority, '1' the greatest, '2' the least.  Side stream 0 at the
  // greatest priority gave C5 14.72 / 14.74 -> 14.56 / 14.48 ms but C1 0.0321
  // -> 0.0330 ms (C2, C3, C4 unchanged); a separate greatest-priority stream
  // for the walk-split batches alone cost C4 2.38 -> 2.87 ms and C5 0.7 ms
  // (not understood; probably the streams' hardware-queue mapping, 4 queues
  // a process on the box), so every side stream
  // keeps the default priority (profiles/r06/evidence/side_prio_*.txt)
  int prio_lo = 0, prio_hi = 0;
  hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  const char *sp = knob("PQG_SIDE_PRIO") ? knob("PQG_SIDE_PRIO") : "000";
  for (int i = 0; i < 3; i++) {
    const char m = sp && (int)strlen(sp) > i ? sp[i] : '0';
    const hipError_t se = m == '0' ? hipStreamCreateWithFlags(&c->side[i], hipStreamNonBlocking)
                                   : hipStreamCreateWithPriority(&c->side[i], hipStreamNonBlocking,
                                                                 m == '1' ? prio_hi : prio_lo);
    if (se != hipSuccess || hipEventCreateWithFlags(&c->join[i], hipEventDisableTiming) != hipSuccess) {
      set_err("hipStreamCreate failed");
      return PQG_ERR_DEVICE;
    }
  }
  hipEventCreateWithFlags(&c->fork, hipEventDisableTiming);
  if (hipStreamCreateWithFlags(&c->lane1.stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->lane1.fork, hipEventDisableTiming) != hipSuccess) {
    set_err("hipStreamCreate failed");
    return PQG_ERR_DEVICE;
  }
  for (int i = 0; i < 3; i++) {
    if (hipStreamCreateWithFlags(&c->lane1.side[i], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->lane1.join[i], hipEventDisableTiming) != hipSuccess) {
      set_err("hipStreamCreate failed");
      return PQG_ERR_DEVICE;
    }
  }
  if (hipStreamCreateWithFlags(&c->upload, hipStreamNonBlocking) != hipSuccess) {
    set_err("hipStreamCreate failed");
    return PQG_ERR_DEVICE;
  }
  *out = c;
  return PQG_OK;
}

void pqg_ctx_destroy(pqg_ctx *ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  for (int i = 0; i < 3; i++) {
    if (ctx->side[i]) hipStreamDestroy(ctx->side[i]);
    if (ctx->join[i]) hipEventDestroy(ctx->join[i]);
  }
  if (ctx->fork) hipEventDestroy(ctx->fork);
  if (ctx->lane1.stream) hipStreamDestroy(ctx->lane1.stream);
  for (int i = 0; i < 3; i++) {
    if (ctx->lane1.side[i]) hipStreamDestroy(ctx->lane1.side[i]);
    if (ctx->lane1.join[i]) hipEventDestroy(ctx->lane1.join[i]);
  }
  if (ctx->lane1.fork) hipEventDestroy(ctx->lane1.fork);
  if (ctx->upload) {
    hipStreamSynchronize(ctx->upload);
    hipStreamDestroy(ctx->upload);
  }
  for (int i = 0; i < pqg_ctx::kRingBufs; i++) {
    if (ctx->pin[i]) hipHostFree(ctx->pin[i]);
    if (ctx->pin_ev[i]) hipEventDestroy(ctx->pin_ev[i]);
  }
  pqg_release_cache(ctx->device);  // the device's idle cached buffers
  delete ctx;
}

void *pqg_ctx_stream(pqg_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

// ---------------------------------------------------------------------------
// codec registry API
// ---------------------------------------------------------------------------
int pqg_register_block_compressor(int codec, pqg_decompress_fn fn, void *user) {
  if (codec < 0) {
    set_err("invalid codec %d", codec);
    return PQG_ERR_ARG;
  }
  std::unique_lock<std::shared_mutex> lk(g_codec_mu);
  if (!fn && codec > PQG_CODEC_GZIP) {
    codecs().erase(codec);
    return PQG_OK;
  }
  codecs()[codec] = Codec{fn, user};
  return PQG_OK;
}

int pqg_get_registered_codecs(int *out, int cap) {
  std::unique_lock<std::shared_mutex> lk(g_codec_mu);  // compress.go:142 takes the write lock too
  int i = 0;
  for (auto &kv : codecs()) {
    if (i < cap && out) out[i] = kv.first;
    i++;
  }
  return i;
}

// forward
static int device_snappy_block(pqg_ctx *ctx, const uint8_t *src, size_t n, uint8_t *dst, size_t expect, int *code);

int pqg_decompress_block(pqg_ctx *ctx, int codec, const uint8_t *src, size_t src_len, uint8_t *dst, size_t dst_cap,
                         size_t expect_len, size_t *out_len) {
  if (!src && src_len) return PQG_ERR_ARG;
  bool on_device = false;
  size_t got = 0;
  std::vector<uint8_t> tmp;
  uint8_t *target = dst;
  size_t cap = dst_cap;
  if (dst_cap < expect_len) {
    tmp.resize(expect_len + 1);
    target = tmp.data();
    cap = expect_len;
  }
  int rc = host_decompress(codec, src, src_len, target, cap, &got, &on_device);
  if (rc) {
    set_err("decompression failed (codec %d): status %d", codec, rc);
    return rc;
  }
  if (on_device) {
    if (!ctx) {
      set_err("SNAPPY decompression needs a GPU context");
      return PQG_ERR_ARG;
    }
    int code = 0;
    rc = device_snappy_block(ctx, src, src_len, target, expect_len, &code);
    if (rc) return rc;
    if (code) {
      set_err("snappy: %s", code == PQG_ERR_SIZE ? "decompressed size mismatch" : "corrupt input");
      return code;
    }
    got = expect_len;
  }
  if (got != expect_len) {  // compress.go:117-119
    set_err("decompressed data must be %zu byte but its %zu byte", expect_len, got);
    return PQG_ERR_SIZE;
  }
  if (target != dst) {
    set_err("destination too small");
    return PQG_ERR_ARG;
  }
  if (out_len) *out_len = got;
  return PQG_OK;
}

// ---------------------------------------------------------------------------
// file
// ---------------------------------------------------------------------------
static int walk_schema(pqg_file *f, size_t &idx, const std::string &prefix, int d, int r, int rep_def, int depth,
                       std::vector<int> rdefs = {}) {
  if (depth > 64 || idx >= f->schema.size()) return PQG_ERR_SCHEMA;
  const SchemaElem &e = f->schema[idx];
  if (e.name.empty() || !e.has_rep) return PQG_ERR_SCHEMA;  // schema.go:792-798
  if (e.repetition != 0) d++;                               // :800-802
  if (e.repetition == 2) {                                  // :804-806
    r++;
    rep_def = d;
    rdefs.push_back(d);
  }
  std::string name = prefix.empty() ? e.name : prefix + "." + e.name;
  idx++;
  if (!e.has_children || e.num_children == 0) {
    if (!e.has_type) return PQG_ERR_SCHEMA;
    pqg_column_info L;
    memset(&L, 0, sizeof(L));
    snprintf(L.name, sizeof(L.name), "%s", name.c_str());
    L.physical_type = e.type;
    L.type_length = e.type_length;
    L.max_def = d;
    L.max_rep = r;
    L.rep_def = rep_def;
    L.converted_type = e.converted;
    int uns = 0;
    if (e.type == T_INT32 && (e.converted == 11 || e.converted == 12 || e.converted == 13)) uns = 1;
    if (e.type == T_INT64 && e.converted == 14) uns = 1;
    if (e.int_unsigned) uns = 1;
    L.unsigned_int = uns;
    L.value_width = value_width(e.type, e.type_length);
    f->leaves.push_back(L);
    f->leaf_rdefs.push_back(rdefs);
    return 0;
  }
  for (int c = 0; c < e.num_children; c++) {
    int rc = walk_schema(f, idx, name, d, r, rep_def, depth + 1, rdefs);
    if (rc) return rc;
  }
  return 0;
}

static int parse_file(pqg_file *f) {
  const uint8_t *b = f->data;
  size_t len = f->len;
  if (len < 12 || memcmp(b, "PAR1", 4) != 0) {
    set_err("invalid parquet file header");
    return PQG_ERR_FORMAT;
  }
  if (memcmp(b + len - 4, "PAR1", 4) != 0) {
    set_err("invalid parquet file footer");
    return PQG_ERR_FORMAT;
  }
  int32_t fl;
  memcpy(&fl, b + len - 8, 4);
  if (fl <= 0 || (size_t)fl > len - 8) {
    set_err("invalid footer len %d", fl);
    return PQG_ERR_FORMAT;
  }
  TReader t(b + len - 8 - fl, (size_t)fl);
  int16_t last = 0;
  int ty, fid;
  unsigned seen = 0;
  while ((fid = t.field(last, ty)) != 0 && !t.err) {  // FileMetaData parquet.go:10564
    if (fid == 1) {
      t.i32(ty);
      seen |= 1;
    } else if (fid == 2 && ty == 9) {
      int et;
      int64_t sz;
      t.list_header(et, sz);
      if (t.err || et != 12) {
        t.err = true;
        break;
      }
      f->schema.resize((size_t)sz);
      for (int64_t i = 0; i < sz && !t.err; i++) read_schema_elem(t, f->schema[(size_t)i]);
      seen |= 2;
    } else if (fid == 3) {
      f->num_rows = t.i64(ty);
      seen |= 4;
    } else if (fid == 4 && ty == 9) {
      int et;
      int64_t sz;
      t.list_header(et, sz);
      if (t.err || et != 12) {
        t.err = true;
        break;
      }
      f->rgs.resize((size_t)sz);
      for (int64_t i = 0; i < sz && !t.err; i++) {  // RowGroup parquet.go:8561
        RowGroupMeta &g = f->rgs[(size_t)i];
        int16_t l2 = 0;
        int t2, f2;
        unsigned s2 = 0;
        while ((f2 = t.field(l2, t2)) != 0 && !t.err) {
          if (f2 == 1 && t2 == 9) {
            int e2;
            int64_t n2;
            t.list_header(e2, n2);
            if (t.err || e2 != 12) {
              t.err = true;
              break;
            }
            g.cols.resize((size_t)n2);
            for (int64_t j = 0; j < n2 && !t.err; j++) read_col_chunk(t, g.cols[(size_t)j]);
            s2 |= 1;
          } else if (f2 == 2) {
            g.total_byte_size = t.i64(t2);
            s2 |= 2;
          } else if (f2 == 3) {
            g.num_rows = t.i64(t2);
            s2 |= 4;
          } else t.skip(t2);
        }
        if (s2 != 7) t.err = true;
      }
      seen |= 8;
    } else t.skip(ty);
  }
  if (t.err || seen != 15) {
    set_err("read file meta failed");
    return PQG_ERR_THRIFT;
  }
  if (f->schema.empty()) {
    set_err("empty schema");
    return PQG_ERR_SCHEMA;
  }
  size_t idx = 1;
  for (int c = 0; c < f->schema[0].num_children; c++) {
    int rc = walk_schema(f, idx, "", 0, 0, 0, 0);
    if (rc) {
      set_err("invalid schema");
      return rc;
    }
  }
  return PQG_OK;
}

int pqg_file_open_buffer(const uint8_t *data, size_t len, int copy, pqg_file **out) {
  *out = nullptr;
  if (!data) {
    set_err("null buffer");
    return PQG_ERR_ARG;
  }
  pqg_file *f = new pqg_file();
  if (copy) {
    uint8_t *p = (uint8_t *)malloc(len ? len : 1);
    memcpy(p, data, len);
    f->data = p;
    f->owned = true;
  } else {
    f->data = data;
  }
  f->len = len;
  int rc = parse_file(f);
  if (rc) {
    delete f;
    return rc;
  }
  *out = f;
  return PQG_OK;
}

int pqg_file_open_path(const char *path, pqg_file **out) {
  *out = nullptr;
  int fd = open(path, O_RDONLY);
  if (fd < 0) {
    set_err("open %s: %s", path, strerror(errno));
    return PQG_ERR_FORMAT;
  }
  struct stat st;
  if (fstat(fd, &st) != 0 || st.st_size < 12) {
    close(fd);
    set_err("invalid parquet file header");
    return PQG_ERR_FORMAT;
  }
  void *m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
  close(fd);
  if (m == MAP_FAILED) {
    set_err("mmap failed");
    return PQG_ERR_FORMAT;
  }
  pqg_file *f = new pqg_file();
  f->data = (const uint8_t *)m;
  f->len = (size_t)st.st_size;
  f->mapped = true;
  int rc = parse_file(f);
  if (rc) {
    delete f;
    return rc;
  }
  *out = f;
  return PQG_OK;
}

int pqg_file_open_many(const char *const *paths, int n, int threads, pqg_file **out, int *failed) {
  if (failed) *failed = -1;
  if (n < 0 || (n > 0 && (!paths || !out))) {
    set_err("bad arguments");
    return PQG_ERR_ARG;
  }
  for (int i = 0; i < n; i++) out[i] = nullptr;
  std::vector<int> rcs((size_t)n, PQG_OK);
  std::vector<std::string> errs((size_t)n);
  int nt = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
  nt = std::max(1, std::min(nt, n));
  std::atomic<int> next{0};
  auto work = [&] {
    for (int i; (i = next.fetch_add(1)) < n;) {
      rcs[(size_t)i] = pqg_file_open_path(paths[i], &out[i]);
      if (rcs[(size_t)i]) errs[(size_t)i] = g_err;  // this thread's message
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < nt; t++) th.emplace_back(work);
  work();
  for (auto &t : th) t.join();
  for (int i = 0; i < n; i++)
    if (rcs[(size_t)i]) {
      if (failed) *failed = i;
      set_err("%s: %s", paths[i], errs[(size_t)i].c_str());
      return rcs[(size_t)i];
    }
  return PQG_OK;
}

void pqg_file_close(pqg_file *f) { delete f; }
int64_t pqg_file_num_rows(const pqg_file *f) { return f->num_rows; }
int pqg_file_row_group_count(const pqg_file *f) { return (int)f->rgs.size(); }
int64_t pqg_file_row_group_num_rows(const pqg_file *f, int rg) {
  return rg >= 0 && rg < (int)f->rgs.size() ? f->rgs[(size_t)rg].num_rows : -1;
}
int64_t pqg_file_row_group_byte_size(const pqg_file *f, int rg) {
  if (rg < 0 || rg >= (int)f->rgs.size()) return -1;
  int64_t s = 0;
  for (auto &c : f->rgs[(size_t)rg].cols) s += c.total_uncompressed;
  return s;
}
// Estimated GPU decode cost of row group rg for shard balancing (relative
// units: ~ns on one MI355X), from the footer and the dictionary page headers
// alone (no page walk).  Per chunk: its uncompressed bytes at ~2 TB/s
// (output writes + staged reads), Snappy input at the measured k_snappy rate
// (~0.5 GB/s a page-wave, ~400 GB/s over the chip), and for a dictionary
// chunk its values at the gather rate of the dictionary's index bit width
// (LDS groups ~780 Gvalues/s up to 2^12 entries, L1/L2 ~350 at
// 2^13..2^15 and ~280 past, bit width 1 ~360).  A row group's chunks of one
// bit width decode at about that rate whatever its neighbours are, so byte
// sizes alone (dictionary pages count, keys do not) misjudge C2's row groups
// by up to ~2x.
double pqg_file_row_group_cost(const pqg_file *f, int rg) {
  if (rg < 0 || rg >= (int)f->rgs.size()) return -1.0;
  double ns = 0.0;
  for (size_t li = 0; li < f->rgs[(size_t)rg].cols.size(); li++) {
    const ColumnChunkMeta &c = f->rgs[(size_t)rg].cols[li];
    ns += (double)std::max<int64_t>(c.total_uncompressed, 0) / 2000.0;  // bytes / (2 TB/s) in ns
    if (c.codec == PQG_CODEC_SNAPPY) ns += (double)std::max<int64_t>(c.total_compressed, 0) / 400.0;
    // the dictionary page: at dictionary_page_offset when it is set before the
    // data pages, else (writers that leave it unset) possibly the chunk's
    // first page, at data_page_offset
    const bool at_dict = c.has_dict_off && c.dict_page_offset > 0 && c.dict_page_offset < c.data_page_offset;
    const int64_t off = at_dict ? c.dict_page_offset : c.data_page_offset;
    if (off <= 0 || (uint64_t)off >= f->len) continue;
    TReader t(f->data + off, f->len - (size_t)off);
    PageHeader h;
    read_page_header(t, h);
    if (t.err || h.type != 2 || !h.has_dict || h.dict_num_values <= 0) continue;
    int bw = 0;
    while (bw < 32 && ((int64_t)1 << bw) < (int64_t)h.dict_num_values) bw++;
    const double gvals = bw <= 1 ? 360.0 : bw <= 12 ? 780.0 : bw <= 15 ? 350.0 : 280.0;
    ns += (double)std::max<int64_t>(c.num_values, 0) / gvals;
  }
  return ns;
}
int pqg_file_column_count(const pqg_file *f) { return (int)f->leaves.size(); }
int pqg_file_column_info(const pqg_file *f, int leaf, pqg_column_info *out) {
  if (leaf < 0 || leaf >= (int)f->leaves.size()) return PQG_ERR_ARG;
  *out = f->leaves[(size_t)leaf];
  return PQG_OK;
}
int pqg_file_find_column(const pqg_file *f, const char *name) {
  for (size_t i = 0; i < f->leaves.size(); i++)
    if (strcmp(f->leaves[i].name, name) == 0) return (int)i;
  return -1;
}
int pqg_file_select_columns(const pqg_file *f, const char *const *names, int nnames, int *out, int cap) {
  int k = 0;
  for (size_t i = 0; i < f->leaves.size(); i++) {
    bool sel = nnames == 0;
    for (int j = 0; j < nnames && !sel; j++) {  // schema.go:296-312
      size_t l = strlen(names[j]);
      const char *nm = f->leaves[i].name;
      if (strcmp(nm, names[j]) == 0 || (strncmp(nm, names[j], l) == 0 && nm[l] == '.')) sel = true;
    }
    if (sel) {
      if (k < cap) out[k] = (int)i;
      k++;
    }
  }
  return k;
}
int pqg_file_last_error(const pqg_file *f, char *buf, size_t cap) {
  (void)f;
  if (buf && cap) snprintf(buf, cap, "%s", g_err.c_str());
  return (int)g_err.size();
}

// ---------------------------------------------------------------------------
// batch planning
// ---------------------------------------------------------------------------
// Raw Snappy block (decode.go:32-75) that is exactly one literal holding
// `expect` bytes: the uvarint decoded length equals `expect`, the first tag is
// a literal of that length and the stream ends with it.  *data = offset of
// the literal's bytes.  Anything else (including a corrupt stream) is left to
// k_snappy, which reports the reference's error.
static bool getenv_flag(const char *name) {
  const char *v = getenv(name);
  return v && v[0] == '1';
}

// decodedLen's binary.Uvarint (decode.go:38-46), with k_snappy's rules exactly:
// up to 10 bytes, the 10th at most 1, over-long (non-minimal) encodings
// accepted.  Returns the header length, 0 when the varint is malformed.
static int64_t snappy_uvarint(const uint8_t *p, int64_t n, uint64_t *v) {
  uint64_t x = 0;
  uint32_t sh = 0;
  for (int64_t i = 0; i < n; i++) {
    const uint8_t b = p[i];
    if (b < 0x80) {
      if (i > 9 || (i == 9 && b > 1)) return 0;
      *v = x | ((uint64_t)b << (sh & 63));
      return i + 1;
    }
    if (sh < 64) x |= (uint64_t)(b & 0x7f) << sh;
    sh += 7;
  }
  return 0;
}

static bool snappy_single_literal(const uint8_t *p, int64_t n, int64_t expect, int64_t *data) {
  uint64_t v = 0;
  int64_t i = snappy_uvarint(p, n, &v);
  if (i == 0 || v == 0 || v != (uint64_t)expect || v > 0xffffffffull || i >= n) return false;
  const uint8_t tag = p[i];
  if (tag & 3) return false;
  uint64_t x = tag >> 2;
  int64_t hs = 1;
  if (x >= 60) {
    const int extra = (int)x - 59;
    hs = 1 + extra;
    if (i + hs > n) return false;
    x = 0;
    for (int k = 0; k < extra; k++) x |= (uint64_t)p[i + 1 + k] << (8 * k);
  }
  if (x + 1 != v || i + hs + (int64_t)v != n) return false;
  *data = i + hs;
  return true;
}

// Raw Snappy block that is only literals (an incompressible page longer than
// one 64 KiB encoder block: a train of maximal literals) decoding to exactly
// `expect` bytes and ending with the stream — valid by decode_other.go:16-99
// (every literal inside src and dst, d == len(dst) at the end), and its output
// is the literals' payloads back to back.  Fills `lits` with (stream offset,
// output offset, length) per literal; the page is then copied by k_copy from
// the plan, with no k_snappy work.  Literals must average >= 4 KiB (short
// literal trains are not worth a copy item each); anything else answers false
// and is left to k_snappy, which reports the reference's errors.
static bool snappy_literal_train(const uint8_t *p, int64_t n, int64_t expect, std::vector<int64_t> &lits) {
  lits.clear();
  uint64_t v = 0;
  int64_t i = snappy_uvarint(p, n, &v);
  if (i == 0 || v == 0 || v != (uint64_t)expect || v > 0xffffffffull) return false;
  const int64_t max_lits = expect / 4096 + 1;
  int64_t d = 0;
  while (i < n) {
    const uint8_t tag = p[i];
    if (tag & 3) return false;
    uint64_t x = tag >> 2;
    int64_t hs = 1;
    if (x >= 60) {
      const int extra = (int)x - 59;
      hs = 1 + extra;
      if (i + hs > n) return false;
      x = 0;
      for (int k = 0; k < extra; k++) x |= (uint64_t)p[i + 1 + k] << (8 * k);
    }
    const int64_t len = (int64_t)x + 1;
    if (len > expect - d || len > n - i - hs) return false;
    if ((int64_t)(lits.size() / 3) >= max_lits) return false;
    lits.push_back(i + hs);
    lits.push_back(d);
    lits.push_back(len);
    i += hs + len;
    d += len;
  }
  return d == expect && !lits.empty();
}

static int supported_encoding(int ptype, int enc) {
  if (enc == ENC_PLAIN_DICT) enc = ENC_RLE_DICT;  // chunk_reader.go:145-147
  switch (ptype) {
    case T_BYTE_ARRAY:
      return enc == ENC_PLAIN || enc == ENC_RLE_DICT || enc == ENC_DELTA_LBA || enc == ENC_DELTA_BA ? 0 : PQG_ERR_ENCODING;
    case T_FLBA:  // getFixedLenByteArrayValuesDecoder chunk_reader.go:86-96
      return enc == ENC_PLAIN || enc == ENC_RLE_DICT || enc == ENC_DELTA_BA ? 0 : PQG_ERR_ENCODING;
    case T_FLOAT: case T_DOUBLE: case T_INT96:
      return enc == ENC_PLAIN || enc == ENC_RLE_DICT ? 0 : PQG_ERR_ENCODING;
    case T_INT32: case T_INT64:
      return enc == ENC_PLAIN || enc == ENC_RLE_DICT || enc == ENC_DELTA_BP ? 0 : PQG_ERR_ENCODING;
    case T_BOOLEAN:  // getBooleanValuesDecoder chunk_reader.go:58-69 (boolean dictionaries are not built)
      return enc == ENC_PLAIN || enc == ENC_RLE ? 0 : enc == ENC_RLE_DICT ? PQG_ERR_UNSUPPORTED : PQG_ERR_ENCODING;
  }
  return PQG_ERR_ENCODING;
}

namespace {
struct HostBuf {  // the device input buffer's layout: byte ranges of the (mapped) file, 16-byte aligned
  struct Range {
    const uint8_t *src;
    size_t off, len;
  };
  std::vector<Range> ranges;
  size_t n = 0;
  size_t append(const uint8_t *src, size_t k, size_t align = 16, size_t phase = 0) {
    const size_t off = ((n + align - 1) & ~(align - 1)) + phase;
    ranges.push_back({src, off, k});
    n = off + k;
    return off;
  }
};
constexpr size_t kPad = 4096;  // readable slack after every device buffer (1 KiB register windows)
}  // namespace

// Snappy stream whose first 256 KiB of output (or 4096 tokens) are at least
// 3/4 long literals (>= 1 KiB): an incompressible body, which one k_snappy
// wave hands to k_copy a token at a time — nothing serial to cut into
// segments.  A peek at the host copy; anything malformed answers false.
static bool snappy_long_literals(const uint8_t *p, int64_t n) {
  int64_t i = 0;
  for (int k = 0; k < 10 && i < n; k++)  // preamble
    if (p[i++] < 0x80) break;
  int64_t out = 0, lit = 0;
  for (int t = 0; t < 4096 && i < n && out < (256 << 10); t++) {
    const uint32_t tag = p[i], x = tag >> 2;
    int64_t len, adv;
    if ((tag & 3) == 0) {
      if (x < 60) {
        len = x + 1;
        adv = 1 + len;
      } else {
        const int extra = (int)x - 59;
        if (i + 1 + extra > n) return false;
        uint32_t v = 0;
        for (int q = 0; q < extra; q++) v |= (uint32_t)p[i + 1 + q] << (8 * q);
        len = (int64_t)v + 1;
        adv = 1 + extra + len;
      }
      if (len >= 1024) lit += len;
    } else {
      len = (tag & 3) == 1 ? 4 + (x & 7) : x + 1;
      adv = (tag & 3) == 1 ? 2 : (tag & 3) == 2 ? 3 : 5;
    }
    out += len;
    i += adv;
  }
  return out > 0 && lit * 4 >= out * 3;
}

static int plan_chunk(pqg_batch *B, HostBuf &in, std::vector<std::pair<uint64_t, std::vector<uint8_t>>> &host_bodies,
                      int64_t &stage_off, int ci, int rg) {
  pqg_file *f = B->file;
  ColumnPlan &cp = B->cols[(size_t)ci];
  const pqg_column_info &L = cp.info;
  const RowGroupMeta &G = f->rgs[(size_t)rg];
  const bool bits_off = getenv_flag("PQG_LEVEL_BYTES");  // (per chunk: tests switch it per batch)
  auto chunk_err = [&](int ord, uint32_t stage, int code, const char *msg) {
    B->chunk_errors.push_back({rg, cp.leaf, ord, stage, (uint32_t)code});
    (void)msg;
    return 0;
  };
  if (cp.leaf >= (int)G.cols.size()) return chunk_err(-1, 0, PQG_ERR_PAGE, "column index out of bounds");
  const ColumnChunkMeta &C = G.cols[(size_t)cp.leaf];
  if (C.has_file_path) return chunk_err(-1, 0, PQG_ERR_PAGE, "nyi: data is in another file");
  if (!C.has_meta) return chunk_err(-1, 0, PQG_ERR_PAGE, "missing meta data");
  if (C.type != L.physical_type) return chunk_err(-1, 0, PQG_ERR_PAGE, "wrong type in chunk metadata");
  int64_t offset = C.has_dict_off ? C.dict_page_offset : C.data_page_offset;
  if (offset < 0 || (uint64_t)offset > f->len) return chunk_err(-1, 0, PQG_ERR_SIZE, "seek");

  bool registered = false;
  bool builtin = codec_builtin(C.codec, &registered);
  const bool device_codec = builtin && C.codec == PQG_CODEC_SNAPPY;

  // walk page headers exactly like readPages (chunk_reader.go:206-284)
  struct Walked {
    PageHeader h;
    int64_t payload;  // file offset of the payload
    int ord;
  };
  std::vector<Walked> walked;
  int64_t pos = offset, count = 0;
  int ord = 0;
  bool have_dict = false;
  int64_t chunk_lo = offset, chunk_hi = offset;
  while (C.total_compressed - count > 0) {
    if ((uint64_t)pos >= f->len) return chunk_err(ord, 0, PQG_ERR_THRIFT, "page header past end of file");
    TReader t(f->data + pos, f->len - (size_t)pos);
    PageHeader h;
    read_page_header(t, h);
    if (t.err) {
      chunk_err(ord, 0, PQG_ERR_THRIFT, "page header");
      break;
    }
    pos += (int64_t)t.pos;
    count += (int64_t)t.pos;
    Walked w{h, pos, ord};
    if (h.type == 2) {  // DICTIONARY_PAGE
      if (have_dict) {
        chunk_err(ord, 0, PQG_ERR_PAGE, "there should be only one dictionary");
        break;
      }
      have_dict = true;
      walked.push_back(w);
      int64_t csz = h.compressed > 0 ? h.compressed : 0;
      chunk_hi = std::max(chunk_hi, std::min<int64_t>(pos + csz, (int64_t)f->len));
      pos += csz;
      count += csz;
      if (h.compressed < 0) break;  // page errors at its own stage; the walk cannot continue
      if (C.has_dict_off && C.dict_page_offset != pos) {  // :243-249
        count += C.data_page_offset - pos;
        pos = C.data_page_offset;
        if (pos < 0 || (uint64_t)pos > f->len) {
          chunk_err(ord + 1, 0, PQG_ERR_SIZE, "seek");
          break;
        }
        chunk_lo = std::min(chunk_lo, pos);
      }
      ord++;
      continue;
    }
    if (h.type != 0 && h.type != 3) {
      chunk_err(ord, 0, PQG_ERR_PAGE, "DATA_PAGE or DATA_PAGE_V2 type supported");
      break;
    }
    walked.push_back(w);
    if (h.compressed < 0) break;
    chunk_hi = std::max(chunk_hi, std::min<int64_t>(pos + h.compressed, (int64_t)f->len));
    pos += h.compressed;
    count += h.compressed;
    ord++;
  }
  // upload the chunk bytes once.  A chunk with a dictionary page is placed
  // so that the dictionary's values start 16-byte aligned: uncompressed, its
  // payload; Snappy, the data of its first literal (an incompressible
  // dictionary is one literal, which k_snappy then leaves in place instead of
  // copying it, and L1/L2 gathers read it aligned)
  size_t phase = 0;
  if (!walked.empty() && walked[0].h.type == 2 && (C.codec == PQG_CODEC_UNCOMPRESSED || device_codec)) {
    int64_t h = 0;
    const int64_t p0 = walked[0].payload, pend = std::min<int64_t>(p0 + walked[0].h.compressed, (int64_t)f->len);
    if (device_codec) {  // varint decoded length, then the tag (+ 1..4 length bytes for literals >= 61 bytes)
      int64_t q = p0;
      while (q < pend && (f->data[q] & 0x80)) q++;
      q++;
      if (q < pend && (f->data[q] & 3) == 0) {
        const uint32_t x = f->data[q] >> 2;
        h = (q - p0) + 1 + (x >= 60 ? (int64_t)(x - 59) : 0);
      } else {
        h = -1;  // not a literal first: nothing to align
      }
    }
    if (h >= 0 && p0 >= chunk_lo) phase = (size_t)((16 - ((p0 - chunk_lo + h) & 15)) & 15);
  }
  size_t base = in.append(f->data + chunk_lo, (size_t)(chunk_hi - chunk_lo), 16, phase);
  B->input_bytes += chunk_hi - chunk_lo;

  int32_t dict_idx = -1;
  int64_t level_base = cp.levels;
  for (auto &w : walked) {
    const PageHeader &h = w.h;
    PageDesc d;
    memset(&d, 0, sizeof(d));
    d.job_base = -1;  // not a tiled page
    d.lens_base = -1;
    d.lvl_base = -1;
    d.part0 = -1;
    d.sp_base = -1;
    d.sidx = -1;
    d.swalk = -1;
    d.col = ci;
    d.rg = rg;
    d.ord = w.ord;
    d.dict = dict_idx;
    d.src = base + (uint64_t)(w.payload - chunk_lo);
    B->page_foff.push_back(w.payload);  // host copy of the payload (segment planning peeks at it)
    uint32_t st = STATUS_OK;
    auto fail = [&](uint32_t stage, int code) {
      if (st == STATUS_OK) st = make_status(stage, (uint32_t)code);
    };
    const int64_t avail = (int64_t)f->len - w.payload;
    bool needs_device_codec = false, gz_dev = false;
    std::vector<int64_t> train;
    int64_t comp = 0, body = 0, lsize = 0;
    if (h.type == 2) {
      d.kind = PAGE_DICT;
      d.num_values = h.dict_num_values;
      if (!h.has_dict || h.dict_num_values < 0) fail(ST_HEADER, PQG_ERR_PAGE);
      if (L.physical_type == T_FLBA && L.type_length <= 0) fail(ST_HEADER, PQG_ERR_SCHEMA);
      if (h.dict_encoding != ENC_PLAIN && h.dict_encoding != ENC_PLAIN_DICT) fail(ST_V2_ENC, PQG_ERR_ENCODING);
      comp = h.compressed;
      body = h.uncompressed;
      d.dict_base = B->dict_entries;
      if (L.physical_type == T_BYTE_ARRAY && h.dict_num_values > 0) B->dict_entries += h.dict_num_values;
    } else if (h.type == 0) {
      d.kind = PAGE_V1;
      d.num_values = h.dp_num_values;
      if (!h.has_dph) fail(ST_HEADER, PQG_ERR_PAGE);
      if (L.max_rep > 0 && h.dp_rep_enc != ENC_RLE) fail(ST_HEADER, PQG_ERR_ENCODING);
      if (L.max_def > 0 && h.dp_def_enc != ENC_RLE) fail(ST_HEADER, PQG_ERR_ENCODING);
      if (h.dp_num_values < 0) fail(ST_HEADER, PQG_ERR_PAGE);
      int e = supported_encoding(L.physical_type, h.dp_encoding);
      if (e) fail(ST_V1_ENC, e);
      d.enc = (uint8_t)(h.dp_encoding == ENC_PLAIN_DICT ? ENC_RLE_DICT : h.dp_encoding);
      comp = h.compressed;
      body = h.uncompressed;
    } else {
      d.kind = PAGE_V2;
      d.num_values = h.v2_num_values;
      if (!h.has_v2 || h.v2_num_values < 0 || h.v2_rep_len < 0 || h.v2_def_len < 0) fail(ST_HEADER, PQG_ERR_PAGE);
      int e = supported_encoding(L.physical_type, h.v2_encoding);
      if (e) fail(ST_V2_ENC, e);
      d.enc = (uint8_t)(h.v2_encoding == ENC_PLAIN_DICT ? ENC_RLE_DICT : h.v2_encoding);
      lsize = (int64_t)std::max(h.v2_rep_len, 0) + std::max(h.v2_def_len, 0);
      if (lsize > 0 && lsize > avail) fail(ST_V2_LEVELS, PQG_ERR_EOF);
      d.v2_rep_len = h.v2_rep_len;
      d.v2_def_len = h.v2_def_len;
      comp = (int64_t)h.compressed - lsize;
      body = (int64_t)h.uncompressed - lsize;
      if (comp < 0 || body < 0) fail(ST_V2_SIZE, PQG_ERR_SIZE);
    }
    if (d.num_values < 0) d.num_values = 0;
    d.comp_len = (int32_t)std::max<int64_t>(comp, 0);
    d.body_len = (int32_t)std::max<int64_t>(body, 0);
    d.level_base = level_base;
    // decompression stage (newBlockReader compress.go:102-122)
    if (st == STATUS_OK || (st >> 16) > ST_DECOMPRESS) {
      if (comp < 0 || body < 0) {
        fail(ST_DECOMPRESS, PQG_ERR_SIZE);
      } else if (comp > avail - lsize) {
        fail(ST_DECOMPRESS, PQG_ERR_SIZE);  // short read
      } else if (!registered) {
        fail(ST_DECOMPRESS, PQG_ERR_CODEC);
      } else if (device_codec) {
        // a block that is exactly one literal (an incompressible page: C2's
        // keys, random values) is its own content: the page is read in place
        // as if uncompressed, no k_snappy work (k_snappy's alias1 check,
        // decided here from the payload the host already has)
        int64_t lit = -1;
        if (C.codec == PQG_CODEC_SNAPPY && snappy_single_literal(f->data + w.payload + lsize, comp, body, &lit) &&
            (h.type != 2 || ((d.src + (uint64_t)(lsize + lit)) & 7) == 0)) {
          d.body_src = BODY_RAW;
          d.body = d.src + (uint64_t)(lsize + lit);
          B->literal_pages++;
        } else if (C.codec == PQG_CODEC_SNAPPY && !(h.type == 2 && L.physical_type == T_BYTE_ARRAY) &&
                   !knob_flag("PQG_NO_TRAIN") &&
                   snappy_literal_train(f->data + w.payload + lsize, comp, body, train)) {
          // a train of literals: staged by k_copy from the plan (a BYTE_ARRAY
          // dictionary is read by k_dict_prepare before k_copy runs: k_snappy)
          d.body_src = BODY_SNAPPY;
          d.body = (uint64_t)stage_off;
          d.train = 1;
          for (size_t q = 0; q < train.size(); q += 3) {
            B->hjobs.push_back((int64_t)d.src + lsize + train[q]);
            B->hjobs.push_back((int64_t)stage_off + train[q + 1]);
            B->hjobs.push_back(train[q + 2]);
            B->hjobs.push_back(0);
          }
          stage_off += ((body + 15) & ~15) + 16;
          B->staged_bytes += body;
          B->train_pages++;
          if (h.type != 2) B->data_may_defer = true;
        } else {
          needs_device_codec = true;
        }
      } else if (builtin && C.codec == PQG_CODEC_UNCOMPRESSED) {
        if (comp != body) fail(ST_DECOMPRESS, PQG_ERR_SIZE);
      } else if (builtin && C.codec == PQG_CODEC_GZIP && !(B->flags & PQG_BATCH_HOST_INFLATE)) {
        // gzip on the GPU: the member is uploaded as stored and k_inflate
        // writes the body into staging (zlib's outcome, pq_inflate.hip)
        d.body_src = BODY_GZIP;
        d.body = (uint64_t)stage_off;
        stage_off += ((body + 15) & ~15) + 16;
        B->staged_bytes += body;
        B->gzip_in_bytes += comp;
        gz_dev = true;
      } else {
        // host codec (gzip / user-registered): inflate now, upload into staging
        std::vector<uint8_t> out((size_t)body + 1);
        size_t got = 0;
        bool ondev = false;
        int rc = host_decompress(C.codec, f->data + w.payload + lsize, (size_t)comp, out.data(), (size_t)body, &got,
                                 &ondev);
        if (rc) fail(ST_DECOMPRESS, rc);
        else if (got != (size_t)body) fail(ST_DECOMPRESS, PQG_ERR_SIZE);
        else {
          out.resize((size_t)body);
          d.body_src = BODY_HOST;
          d.body = (uint64_t)stage_off;
          host_bodies.emplace_back((uint64_t)stage_off, std::move(out));
          stage_off += ((body + 15) & ~15) + 16;
          B->host_inflated++;
        }
      }
    }
    if (needs_device_codec) {
      d.body_src = BODY_SNAPPY;
      d.body = (uint64_t)stage_off;
      stage_off += ((body + 15) & ~15) + 16;
      B->staged_bytes += body;
    } else if (d.body_src == BODY_RAW && !d.body) {
      d.body = d.src + (uint64_t)lsize;
    }
    int32_t my_index = (int32_t)B->pages.size();
    B->pages.push_back(d);
    B->status0.push_back(st);
    if (gz_dev) B->gzip_list.push_back(my_index);
    if (d.kind == PAGE_DICT) {
      dict_idx = my_index;
      if (L.physical_type == T_BYTE_ARRAY) {
        B->dict_list.push_back(my_index);  // k_dict_prepare: the length-prefix walk
        static const bool swd_off = knob_flag("PQG_NO_SWALK");
        if (!swd_off && body >= SW_MIN && d.num_values > 0) {  // region-parallel (k_sw_*) before it
          const int32_t nreg = (int32_t)((body + SW_R - 1) / SW_R);
          B->pages.back().swalk = (int32_t)B->sw_dict.size();
          B->sw_dict.push_back(SwPage{my_index, 0, nreg, 1});
        }
      } else if (L.physical_type == T_BOOLEAN) {
        if (B->status0.back() == STATUS_OK) B->status0.back() = make_status(ST_DICT_VALUES, (uint32_t)PQG_ERR_UNSUPPORTED);
      } else if ((int64_t)std::max(d.num_values, 0) * L.value_width > (int64_t)d.body_len &&
                 B->status0.back() == STATUS_OK) {
        // fixed width: the only check is the size (page_dict.go:54-61 reading
        // num_values values), known here from the header
        B->status0.back() = make_status(ST_DICT_VALUES, (uint32_t)PQG_ERR_EOF);
      }
    } else {
      B->data_list.push_back(my_index);
      level_base += d.num_values;
      // pages with levels: k_levels leaves them decoded (a byte each) with the
      // counts k_prepare needs, for k_prepare and k_decode
      if (L.max_def > 0 && L.max_def < 256 && d.num_values > 0) {
        B->pages.back().lvl_base = B->lvl_bytes;
        // flat pages without level output: a bit per level (k_decode needs only
        // def == max_def), an eighth of the scratch traffic (C3's nullable doubles)
        B->pages.back().lvl_bits = (int16_t)(L.max_rep == 0 && !(B->flags & PQG_BATCH_LEVELS) && !bits_off);
        // (bits: the bitmap and one word after it)
        B->lvl_bytes += B->pages.back().lvl_bits
                            ? ((((int64_t)d.num_values + 7) >> 3) + 8 + 15) & ~(int64_t)15
                            : (((int64_t)(L.max_rep > 0 ? 2 : 1) * d.num_values) + 15) & ~(int64_t)15;
        if (d.kind != PAGE_V2 || d.dict >= 0) B->lvl_late = true;
      }
      if ((L.physical_type == T_BYTE_ARRAY && (d.enc == ENC_DELTA_LBA || d.enc == ENC_DELTA_BA)) ||
          (L.physical_type == T_FLBA && d.enc == ENC_DELTA_BA)) {
        B->pages.back().lens_base = B->lens_entries;  // suffix lengths, then prefix lengths
        B->lens_entries += 2 * (int64_t)std::max(d.num_values, 0);
      } else if (L.physical_type == T_BYTE_ARRAY && d.enc == ENC_PLAIN && L.value_width <= 0) {
        // PLAIN strings: k_prepare's length walk leaves each value's offset and
        // length here for k_decode (offsets, then lengths)
        B->pages.back().lens_base = B->lens_entries;
        B->lens_entries += 2 * (int64_t)std::max(d.num_values, 0);
        // a long page: its walk split over SW_R-byte regions (k_sw_*), when
        // its non-null count comes from k_levels (or every value is defined)
        static const bool sw_off = knob_flag("PQG_NO_SWALK");
        if (!sw_off && body >= SW_MIN && d.num_values > 0 && (L.max_def == 0 || B->pages.back().lvl_base >= 0)) {
          const int32_t nreg = (int32_t)((body + SW_R - 1) / SW_R);
          B->pages.back().swalk = (int32_t)B->sw_data.size();
          B->sw_data.push_back(SwPage{my_index, 0, nreg, 0});
          B->data_may_defer = true;  // k_prepare<1> takes them after the walk
        }
      }
    }
    if (needs_device_codec) {
      B->pages.back().sidx = (int32_t)B->snappy_list.size();
      B->snappy_list.push_back(my_index);
      // a data page whose body may wait on k_copy (literals >= 16 KiB are deferred)
      if (d.kind != PAGE_DICT && body >= 16 * 1024) B->data_may_defer = true;
    }
  }
  cp.levels = level_base;
  return 0;
}

// Device memory cache.  Batches come and go (a pqg_stream makes one per
// slice) and hipMalloc / hipFree cost tens of µs each — hipFree also waits for
// the whole device — so released buffers are kept per device in size classes
// (2^k, 1.25, 1.5, 1.75 x 2^k) and handed out again.  A buffer is released
// only after its batch's work has finished (pqg_batch_destroy synchronises).
// Held bytes are capped (PQG_DEV_CACHE_MB, default 32 GiB); a failed
// hipMalloc releases the device's cache and retries.
}  // extern "C" (the cache is C++)
namespace {
struct DevCache {
  std::mutex mu;
  std::multimap<std::pair<int, size_t>, void *> idle;  // (device, class bytes) -> buffer
  std::map<void *, std::pair<int, size_t>> live;
  size_t idle_bytes = 0;
};
DevCache &dev_cache() {
  static DevCache *c = new DevCache();  // never destroyed: buffers outlive static destructors
  return *c;
}
size_t size_class(size_t n) {
  if (n <= 4096) return 4096;
  size_t p = 4096;
  while (p * 2 < n) p *= 2;  // p < n <= 2p
  for (int q = 5; q <= 8; q++)
    if (n <= p * (size_t)q / 4) return p * (size_t)q / 4;
  return 2 * p;
}
void release_idle(DevCache &c, int dev) {  // caller holds c.mu
  for (auto it = c.idle.begin(); it != c.idle.end();) {
    if (dev >= 0 && it->first.first != dev) {
      ++it;
      continue;
    }
    hipFree(it->second);
    c.idle_bytes -= it->first.second;
    it = c.idle.erase(it);
  }
}
}  // namespace
extern "C" {

// Idle bytes the cache may hold: PQG_DEV_CACHE_MB, else an eighth of the
// device's memory capped at 8 GiB (torch's allocator or another process on
// the device cannot reclaim what the cache holds; a failed hipMalloc here
// releases it, pqg_ctx_destroy and pqg_release_cache too).
static size_t dev_cache_cap() {
  if (getenv("PQG_DEV_CACHE_MB")) return (size_t)atoll(getenv("PQG_DEV_CACHE_MB")) << 20;
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess || tot == 0) tot = (size_t)64 << 30;
  return std::min(tot / 8, (size_t)8 << 30);
}

int pqg_release_cache(int device) {
  DevCache &c = dev_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  release_idle(c, device);
  return PQG_OK;
}

static int alloc_dev(void **p, size_t n) {
  int dev = 0;
  hipGetDevice(&dev);
  const size_t cls = size_class(n + kPad);
  DevCache &c = dev_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.idle.find({dev, cls});
  if (it != c.idle.end()) {
    *p = it->second;
    c.idle.erase(it);
    c.idle_bytes -= cls;
    c.live[*p] = {dev, cls};
    return 0;
  }
  hipError_t e = hipMalloc(p, cls);
  if (e != hipSuccess && !c.idle.empty()) {
    release_idle(c, dev);
    e = hipMalloc(p, cls);
  }
  if (e != hipSuccess) {
    *p = nullptr;
    set_err("hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
    return PQG_ERR_DEVICE;
  }
  c.live[*p] = {dev, cls};
  return 0;
}

static void free_dev(void *p) {
  if (!p) return;
  DevCache &c = dev_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  auto it = c.live.find(p);
  if (it == c.live.end()) {
    hipFree(p);
    return;
  }
  static const size_t cap = dev_cache_cap();
  const auto key = it->second;
  c.live.erase(it);
  if (c.idle_bytes + key.second > cap) {
    hipFree(p);
    return;
  }
  c.idle.insert({key, p});
  c.idle_bytes += key.second;
}

static int launch_all(pqg_batch *B, bool upto_scan, bool timed);

struct LaneRef {
  hipStream_t stream;
  hipStream_t *side;
  hipEvent_t fork;
  hipEvent_t *join;
  std::mutex *mu;
};
static LaneRef lane_of(pqg_batch *B);
static hipStream_t bstream(pqg_batch *B);

// Everything after the batch object exists: any failure returns a status and
// pqg_batch_create releases the partial batch (device buffers, pinned status)
static int batch_init(pqg_batch *B, pqg_ctx *ctx, pqg_file *f, int rg_begin, int rg_end, const int *leaves,
                      int nleaves, int flags) {
  {
    const char *st = getenv("PQG_SEGMENT_TIMES");
    B->seg_times = st && st[0] == '1';
  }
  std::vector<int> sel;
  if (nleaves == 0 || !leaves) {
    for (int i = 0; i < (int)f->leaves.size(); i++) sel.push_back(i);
  } else {
    sel.assign(leaves, leaves + nleaves);
  }
  for (int l : sel) {
    if (l < 0 || l >= (int)f->leaves.size()) {
      set_err("leaf %d out of range", l);
      return PQG_ERR_ARG;
    }
    ColumnPlan cp;
    cp.leaf = l;
    cp.info = f->leaves[(size_t)l];
    cp.flags = 0;
    if (cp.info.max_rep > 0 || cp.info.physical_type == T_BYTE_ARRAY) cp.flags |= COL_NEEDS_COUNT;
    if (flags & PQG_BATCH_LEVELS) cp.flags |= COL_EMIT_LEVELS;
    // max_rep >= 2: the levels are kept (the nested offsets are built from them)
    if (cp.info.max_rep >= 2) {
      cp.flags |= COL_EMIT_LEVELS;
      if ((size_t)l < f->leaf_rdefs.size()) cp.rdefs = f->leaf_rdefs[(size_t)l];
    }
    cp.levels = 0;
    B->cols.push_back(cp);
  }
  // host time of each batch-creation phase (pqg_batch_stats::create_*_ms;
  // PQG_TRACE_CREATE=1: also on stderr)
  const bool trace = getenv("PQG_TRACE_CREATE") != nullptr;
  auto t_last = std::chrono::steady_clock::now();
  int nphase = 0;
  auto phase = [&](const char *what) {
    auto t = std::chrono::steady_clock::now();
    const double ms = std::chrono::duration<double, std::milli>(t - t_last).count();
    if (nphase < 4) B->create_ms[nphase++] = ms;
    if (trace) fprintf(stderr, "pqg_batch_create %-14s %8.2f ms\n", what, ms);
    t_last = t;
  };
  HostBuf in;
  std::vector<std::pair<uint64_t, std::vector<uint8_t>>> host_bodies;
  int64_t stage_off = 0;
  for (size_t ci = 0; ci < B->cols.size(); ci++) {
    B->cols[ci].page_begin = (int32_t)B->pages.size();
    for (int rg = rg_begin; rg < rg_end; rg++) plan_chunk(B, in, host_bodies, stage_off, (int)ci, rg);
    B->cols[ci].page_end = (int32_t)B->pages.size();
  }
  const size_t npages = B->pages.size();
  // route data pages: flat required fixed-width PLAIN / RLE_DICTIONARY pages
  // take the tiled path (run walk in k_prepare + k_expand), everything else k_decode
  std::vector<std::vector<TileJob>> chunk_tiles;  // tiles grouped by column chunk (one dictionary)
  std::vector<int32_t> page_need(npages, 0);      // staged key bytes per job of a tiled RLE page
  int32_t last_chunk_key = -1;
  for (int32_t pi : B->data_list) {
    PageDesc &d = B->pages[(size_t)pi];
    const ColumnPlan &cp = B->cols[(size_t)d.col];
    const pqg_column_info &L = cp.info;
    bool tiled = L.max_rep == 0 && L.max_def == 0 && (L.value_width == 4 || L.value_width == 8) &&
                 L.physical_type != T_BYTE_ARRAY && !(cp.flags & COL_EMIT_LEVELS) &&
                 (d.enc == ENC_PLAIN || d.enc == ENC_RLE_DICT);
    if (!tiled) {
      // flat fixed-width pages (DELTA, nullable, PLAIN inside non-tiled
      // columns) go to the k_decode<1> instance, the rest to k_decode<0>
      // (FIXED_LEN_BYTE_ARRAY DELTA_BYTE_ARRAY pages: k_decode<0> + k_dba)
      const bool fl_dba = L.physical_type == T_FLBA && d.enc == ENC_DELTA_BA;
      const bool flat_fw = L.max_rep == 0 && (L.value_width == 4 || L.value_width == 8) &&
                           L.physical_type != T_BYTE_ARRAY && L.physical_type != T_BOOLEAN &&
                           !(cp.flags & COL_EMIT_LEVELS) && !fl_dba;
      const bool flat_ba = L.max_rep == 0 && L.physical_type == T_BYTE_ARRAY && !(cp.flags & COL_EMIT_LEVELS);
      const bool nest_fw = L.max_rep > 0 && (L.value_width == 4 || L.value_width == 8) &&
                           L.physical_type != T_BYTE_ARRAY && L.physical_type != T_BOOLEAN &&
                           !(cp.flags & COL_EMIT_LEVELS) && !fl_dba;
      static const bool pstr_off = knob("PQG_NO_PLAIN_STR") != nullptr;
      if (flat_ba && L.max_def == 0 && d.enc == ENC_PLAIN && d.lens_base >= 0 && !pstr_off) {
        // several waves per page (k_plain_str) over k_prepare's (offset, length) scratch
        for (int32_t v = 0; v < std::max(d.num_values, 0); v += PLAIN_STR_ITEM) {
          B->pstr_items.push_back(pi);
          B->pstr_items.push_back(v);
        }
        continue;
      }
      // flat required dictionary strings: k_decode<4> (the dictionary path of
      // <2> alone, 8 waves a SIMD instead of 3; PQG_NO_DEC4=1, analysis: <2>)
      static const bool dec4_off = knob_flag("PQG_NO_DEC4");
      const bool str4 = flat_ba && L.max_def == 0 && d.enc == ENC_RLE_DICT && !dec4_off;
      (flat_fw   ? B->general_flat
       : str4    ? B->general_str4
       : flat_ba ? B->general_str
       : nest_fw ? B->general_nest
                 : B->general_list)
          .push_back(pi);
      if ((L.physical_type == T_BYTE_ARRAY || fl_dba) && d.enc == ENC_DELTA_BA) B->dba_list.push_back(pi);
      // k_prepare validates DELTA_BYTE_ARRAY lengths on the count path
      if (fl_dba) B->cols[(size_t)d.col].flags |= COL_NEEDS_COUNT;
      continue;
    }
    const int32_t n = std::max(d.num_values, 0);
    const int32_t nt = (n + RUN_TILE - 1) / RUN_TILE;
    // a PLAIN page's k_expand records depend only on its header (flat and
    // required: the values section is the whole body): written by the host
    // once; a page too short for its values is left to k_prepare's check
    static const bool srec_off = knob_flag("PQG_NO_STATIC_RECORDS");
    if (d.enc == ENC_PLAIN && !srec_off && B->status0[(size_t)pi] == STATUS_OK &&
        (int64_t)n * L.value_width <= (int64_t)d.body_len)
      d.srec = 1;
    d.job_base = (int32_t)B->page_job_entries;
    B->page_job_entries += (n + EX_WAVE_VALUES - 1) / EX_WAVE_VALUES;
    d.tile_base = (int32_t)B->tile_entries;
    B->tile_entries += nt;
    if (d.enc == ENC_RLE_DICT) {
      // every run holds >= 1 value and >= 2 key-stream bytes (bit width >= 1), so
      // runs <= min(n, len / 2 + 1); + the sentinel
      d.run_base = B->run_entries;
      d.run_cap = (int32_t)std::min<int64_t>(n, (int64_t)d.body_len / 2 + 1) + 2;
      B->run_entries += d.run_cap;
      // staged key bytes of a wave: the page's bytes per value x EX_WAVE_VALUES (+ slack);
      // denser spots fall back to direct loads
      if (n > 0) {
        const int64_t need = ((int64_t)d.body_len * EX_WAVE_VALUES + n - 1) / n + 96;
        page_need[(size_t)pi] = (int32_t)std::min<int64_t>(need, EX_WAVE_VALUES * 4 + 256);
        B->ex_lds = std::max(B->ex_lds, page_need[(size_t)pi]);
      }
    }
    const int32_t key = d.dict >= 0 ? d.dict : -2 - d.col * 1000003 - d.rg;
    if (chunk_tiles.empty() || key != last_chunk_key) chunk_tiles.emplace_back();
    last_chunk_key = key;
    // output pointer and width are filled in once the outputs exist
    for (int32_t v = 0; v < n; v += EX_WAVE_VALUES)
      chunk_tiles.back().push_back(TileJob{nullptr, pi, d.dict, v, d.tile_base + v / RUN_TILE, 0, 0});
  }
  for (auto &cp : B->cols) B->any_count |= (cp.flags & COL_NEEDS_COUNT) != 0;
  // 4-byte columns' jobs first (k_expand<4>), then 8-byte ones (k_expand<8>).
  // k_expand_mix blocks (512 threads, eight waves), per value width:
  //  * LDS groups: chunks whose dictionary fits in LDS beside four waves'
  //    staged keys (within LD_MIX_MAX) and whose jobs amortise copying it;
  //    groups are small (one job per wave unless the dictionary is large:
  //    output >= 2 x dictionary), measured faster than longer-lived groups
  //    (the copy at most a quarter of the output) -> groups of consecutive jobs;
  //  * global blocks: every other job, one per wave, gathering through L1/L2.
  //    (Workgroups of four waves: a workgroup holds its slot until its last
  //    wave ends, and jobs vary in length.)
  //    XCD affinity (speed only, never correctness): blocks b and b + 8 share
  //    an XCD's L2 under round-robin dispatch, so whole chunks (one dictionary
  //    each) are dealt to the 8 block residues, balanced by job count.
  // Blocks are emitted in rounds of 8 (one per residue), global and LDS rounds
  // interleaved by job count so that L2-bound gathers and LDS-bound ones share
  // the machine for the whole launch.
  B->ex_lds = (B->ex_lds + 255) & ~255;  // LDS-DMA pieces of 16 bytes per lane, the last one partial
  const bool ld_off = knob("PQG_NO_LDS_DICT") != nullptr;
  std::vector<TileJob> slot_tiles, ld_tiles, big_tiles;
  std::vector<LdsGroup> big_groups[2];
  const int64_t ld_max = knob("PQG_LD_MAX_KB") ? 1024 * (int64_t)atoi(knob("PQG_LD_MAX_KB")) : LD_MIX_MAX;
  // which chunks fit the mixed launch's LDS groups (class 1), or k_expand_wg's
  // workgroup-a-CU form (class 2: the dictionary in at most WG_MAX_SLICES
  // slices of a CU's LDS), else the mixed launch's L1/L2 blocks
  bool wg_off = false;
  auto ld_class = [&](const std::vector<TileJob> &ct, int32_t W, int64_t &dbytes, int32_t &ks) {
    dbytes = 0;
    ks = 0;
    if (ld_off || ct.empty() || ct[0].dict < 0) return 0;
    dbytes = ((int64_t)std::max(B->pages[(size_t)ct[0].dict].num_values, 0) * W + 15) & ~15;
    for (const TileJob &tj : ct) ks = std::max(ks, page_need[(size_t)tj.page]);
    ks = (ks + 255) & ~255;
    const int64_t J = (int64_t)ct.size();
    if (dbytes <= 0 || ks <= 0) return 0;
    const bool amortised = dbytes * 4 <= J * EX_WAVE_VALUES * W;
    if (amortised && dbytes + (int64_t)LD_WAVES_H * ks <= ld_max) return 1;
    // (8-byte values: one slice at most — k_expand_wg keeps no sliced form for them)
    static const int64_t wg_slices = knob("PQG_WG_SLICES") ? std::max(1, atoi(knob("PQG_WG_SLICES"))) : WG_MAX_SLICES;
    if (!wg_off && dbytes <= (W == 4 ? wg_slices : 1) * (int64_t)WG_SLICE && dbytes <= J * EX_WAVE_VALUES * W)
      return 2;
    return 0;
  };
  // k_expand_wg is its own launch after the mixed one: it pays when its chunks
  // are a good part of the tiled jobs (single-width files at bit widths 13-17:
  // 1.3-2.4x the L1/L2 rates); in C2, where they are a quarter of the jobs,
  // the mixed launch's L1/L2 blocks run beside its LDS groups while the extra
  // launch runs alone (measured: C2 decode phase 0.193 -> 0.212 ms with it).
  // PQG_BIG=1 / PQG_NO_BIG=1 force it on / off.
  {
    int64_t nwg = 0, nall = 0;
    for (const auto &ct : chunk_tiles) {
      if (ct.empty()) continue;
      const int32_t W = B->cols[(size_t)B->pages[(size_t)ct[0].page].col].info.value_width;
      int64_t db;
      int32_t ks;
      nall += (int64_t)ct.size();
      if (ld_class(ct, W, db, ks) == 2) nwg += (int64_t)ct.size();
    }
    wg_off = getenv("PQG_NO_BIG") != nullptr || (getenv("PQG_BIG") == nullptr && nwg * 3 < nall);
  }
  for (int ws = 0; ws < 2; ws++) {
    const int32_t W = ws == 0 ? 4 : 8;
    struct LdG {
      const std::vector<TileJob> *ct;
      int64_t j0, j1;
      int32_t dict_bytes, kspan;
    };
    std::vector<LdG> ldg;
    std::vector<std::vector<TileJob>> bins(8);
    std::vector<const std::vector<TileJob> *> gchunks;  // chunks gathering through L1/L2
    std::vector<std::pair<const std::vector<TileJob> *, int64_t>> wg_chunks;  // (chunk, dictionary bytes)
    for (const auto &ct : chunk_tiles) {
      if (ct.empty() || B->cols[(size_t)B->pages[(size_t)ct[0].page].col].info.value_width != W) continue;
      bool ld = false;
      int64_t dbytes;
      int32_t ks;
      const int cls = ld_class(ct, W, dbytes, ks);
      if (cls) {
        const int64_t J = (int64_t)ct.size();
        if (cls == 1) {
          const int64_t amort = knob("PQG_LD_AMORT") ? atoi(knob("PQG_LD_AMORT")) : 2;
          int64_t G = (dbytes * amort + (int64_t)EX_WAVE_VALUES * W - 1) / ((int64_t)EX_WAVE_VALUES * W);
          const int64_t gmin = knob("PQG_LD_GMIN") ? atoi(knob("PQG_LD_GMIN")) : LD_WAVES_H;
          G = std::min<int64_t>(std::max<int64_t>((G + LD_WAVES_H - 1) / LD_WAVES_H * LD_WAVES_H, gmin), 128);
          const int64_t ng = (J + G - 1) / G;
          for (int64_t q = 0; q < ng; q++) ldg.push_back({&ct, q * J / ng, (q + 1) * J / ng, (int32_t)dbytes, ks});
          ld = true;
          B->pages[(size_t)ct[0].dict].alias_any = 1;  // copied into LDS with a funnel shift anyway
        } else {
          // k_expand_wg: groups of WG_JOBS jobs (one round of WG_WAVES jobs when
          // the dictionary is sliced: every round streams the whole of it)
          wg_chunks.push_back({&ct, dbytes});
          ld = true;
          B->pages[(size_t)ct[0].dict].alias_any = 1;  // copied into LDS with a funnel shift
        }
      }
      if (!ld) gchunks.push_back(&ct);
    }
    // L1/L2 chunks to the 8 XCD residues.  A chunk whose dictionary is large
    // (> PQG_XCD_SPLIT_KB, default 1 MiB) stays whole on one XCD (two such
    // dictionaries would not share one 4 MiB L2); the others are then poured
    // into the least-loaded residues, split at job boundaries where a residue
    // fills up (their dictionaries are then cached by two L2s), so every XCD
    // gets the same number of L2-bound jobs (PQG_XCD_SPLIT_KB=0: whole chunks
    // only, least loaded first)
    {
      static const int64_t split_max = knob("PQG_XCD_SPLIT_KB") ? 1024 * (int64_t)atoi(knob("PQG_XCD_SPLIT_KB"))
                                                                  : (int64_t)1 << 20;
      auto dict_bytes_of = [&](const std::vector<TileJob> &ct) {
        return ct[0].dict >= 0 ? (int64_t)std::max(B->pages[(size_t)ct[0].dict].num_values, 0) * W : 0;
      };
      std::vector<const std::vector<TileJob> *> whole, split;
      for (auto *ct : gchunks) (split_max > 0 && dict_bytes_of(*ct) <= split_max ? split : whole).push_back(ct);
      // a job of a whole (large-dictionary) chunk weighs PQG_XCD_WHOLE_W jobs
      // of the split ones (its gathers miss L2 more often)
      static const double ww = knob("PQG_XCD_WHOLE_W") ? atof(knob("PQG_XCD_WHOLE_W")) : 1.0;
      double load[8] = {};
      auto least = [&]() {
        size_t best = 0;
        for (size_t q = 1; q < 8; q++)
          if (load[q] < load[best]) best = q;
        return best;
      };
      double total = 0;
      for (auto *ct : whole) total += ww * (double)ct->size();
      for (auto *ct : split) total += (double)ct->size();
      for (auto *ct : whole) {
        const size_t q = least();
        bins[q].insert(bins[q].end(), ct->begin(), ct->end());
        load[q] += ww * (double)ct->size();
      }
      const double target = total / 8;
      for (auto *ct : split) {
        size_t k = 0;
        while (k < ct->size()) {
          const size_t q = least();
          const double room = load[q] < target ? std::ceil(target - load[q]) : (double)(ct->size() - k);
          const size_t take = std::min((size_t)std::max(room, 1.0), ct->size() - k);
          bins[q].insert(bins[q].end(), ct->begin() + (std::ptrdiff_t)k, ct->begin() + (std::ptrdiff_t)(k + take));
          load[q] += (double)take;
          k += take;
        }
      }
    }
    size_t maxlen = 0, gjobs = 0, ljobs = 0;
    for (auto &v : bins) maxlen = std::max(maxlen, v.size()), gjobs += v.size();
    for (auto &g : ldg) ljobs += (size_t)(g.j1 - g.j0);
    const size_t ngr = (maxlen + LD_WAVES_H - 1) / LD_WAVES_H, nlr = (ldg.size() + 7) / 8;
    size_t gr = 0, lr = 0, gdone = 0, ldone = 0;
    const int32_t nb0 = (int32_t)B->lgroups.size();
    const TileJob none = {nullptr, -1, -1, 0, 0, 0, 0};
    while (gr < ngr || lr < nlr) {
      // the round kind that is behind in its share of the jobs goes next
      // (PQG_MIX_ORDER, analysis: 1 L1/L2 rounds first, 2 LDS rounds first)
      static const int mix_order = knob("PQG_MIX_ORDER") ? atoi(knob("PQG_MIX_ORDER")) : 0;
      bool take_g = lr >= nlr || (gr < ngr && (double)gdone * (double)std::max<size_t>(ljobs, 1) <=
                                                  (double)ldone * (double)std::max<size_t>(gjobs, 1));
      if (mix_order == 1) take_g = gr < ngr;
      if (mix_order == 2) take_g = lr >= nlr;
      for (size_t q = 0; q < 8; q++) {
        // every block owns LD_WAVES_H job slots (wave w: slot 4 b + w), so a
        // global block's waves load their jobs without waiting for the block's
        // descriptor; LDS groups keep their jobs past the slots (ld_tiles)
        LdsGroup g = {};
        g.job0 = (int32_t)slot_tiles.size();
        g.dpage = -1;
        if (take_g) {
          const size_t k0 = gr * LD_WAVES_H, k1 = std::min(k0 + LD_WAVES_H, bins[q].size());
          for (size_t k = k0; k < k1; k++) slot_tiles.push_back(bins[q][k]);
          g.njobs = (int32_t)(k1 > k0 ? k1 - k0 : 0);
          g.kspan = B->ex_lds;
          gdone += (size_t)g.njobs;
          if (g.njobs) B->ldl[ws] = std::max(B->ldl[ws], LD_WAVES_H * B->ex_lds);
        } else if (lr * 8 + q < ldg.size()) {
          const LdG &l = ldg[lr * 8 + q];
          g.job0 = -1 - (int32_t)ld_tiles.size();  // rebased below
          for (int64_t j = l.j0; j < l.j1; j++) ld_tiles.push_back((*l.ct)[(size_t)j]);
          g.njobs = (int32_t)(l.j1 - l.j0);
          g.dpage = (*l.ct)[0].dict;
          g.dict_bytes = l.dict_bytes;
          g.kspan = l.kspan;
          ldone += (size_t)g.njobs;
          B->ldl[ws] = std::max(B->ldl[ws], l.dict_bytes + LD_WAVES_H * l.kspan);
        }
        while (slot_tiles.size() < (size_t)(B->lgroups.size() + 1) * LD_WAVES_H) slot_tiles.push_back(none);
        B->lgroups.push_back(g);
      }
      if (take_g) gr++;
      else lr++;
    }
    B->ldn[ws] = (int32_t)B->lgroups.size() - nb0;
    if (!wg_chunks.empty()) {
      // a chunk's groups go to one XCD residue (its dictionary stays in that
      // L2), chunks dealt to the least-loaded residue by their cost (jobs x
      // slices), largest first; then rounds of 8 blocks (block b on XCD b % 8)
      static const int64_t wg_jobs = knob("PQG_WG_JOBS") ? std::max(1, atoi(knob("PQG_WG_JOBS"))) : WG_JOBS;
      std::vector<std::vector<LdsGroup>> res(8);
      int64_t load[8] = {};
      auto slices = [&](int64_t db) { return (db + WG_SLICE - 1) / WG_SLICE; };
      std::stable_sort(wg_chunks.begin(), wg_chunks.end(), [&](const auto &x, const auto &y) {
        return (int64_t)x.first->size() * slices(x.second) > (int64_t)y.first->size() * slices(y.second);
      });
      for (auto &wc : wg_chunks) {
        const std::vector<TileJob> &ct = *wc.first;
        size_t q = 0;
        for (size_t r = 1; r < 8; r++)
          if (load[r] < load[q]) q = r;
        const int64_t J = (int64_t)ct.size();
        const int64_t G = slices(wc.second) > 1 ? WG_WAVES : wg_jobs;
        const int64_t ng = (J + G - 1) / G;
        for (int64_t k = 0; k < ng; k++) {
          LdsGroup g = {};
          g.job0 = -1 - (int32_t)big_tiles.size();  // rebased below
          for (int64_t jj = k * J / ng; jj < (k + 1) * J / ng; jj++) big_tiles.push_back(ct[(size_t)jj]);
          g.njobs = (int32_t)((k + 1) * J / ng - k * J / ng);
          g.dpage = ct[0].dict;
          g.dict_bytes = (int32_t)wc.second;
          res[q].push_back(g);
        }
        load[q] += J * slices(wc.second);
      }
      size_t rounds = 0;
      for (auto &v : res) rounds = std::max(rounds, v.size());
      for (size_t r = 0; r < rounds; r++)
        for (size_t q = 0; q < 8; q++) {
          LdsGroup g = {};
          g.dpage = -1;
          if (r < res[q].size()) g = res[q][r];
          big_groups[ws].push_back(g);
        }
    }
  }
  // job indices are relative to the launch's first slot (the 8-byte launch
  // starts at block ldn[0])
  for (size_t b = 0; b < B->lgroups.size(); b++) {
    LdsGroup &g = B->lgroups[b];
    if (g.job0 < 0) g.job0 = (int32_t)slot_tiles.size() + (-1 - g.job0);
    if (b >= (size_t)B->ldn[0]) g.job0 -= B->ldn[0] * LD_WAVES_H;
  }
  // k_expand_wg groups after the mixed ones, with absolute job indices (their
  // launches start at the first slot)
  const size_t big_base = slot_tiles.size() + ld_tiles.size();
  for (int ws = 0; ws < 2; ws++) {
    for (LdsGroup g : big_groups[ws]) {
      if (g.njobs > 0) g.job0 = (int32_t)big_base + (-1 - g.job0);
      B->lgroups.push_back(g);
    }
    B->ldn[2 + ws] = (int32_t)big_groups[ws].size();
  }
  B->tiles = std::move(slot_tiles);
  B->tiles.insert(B->tiles.end(), ld_tiles.begin(), ld_tiles.end());
  B->tiles.insert(B->tiles.end(), big_tiles.begin(), big_tiles.end());

  // k_snappy takes pages in list order, one wave each: the longest bodies
  // first (longest-processing-time order), so that the long serial token
  // chains of big pages start with the launch instead of trailing it
  if (!knob("PQG_SNAPPY_LIST_ORDER")) {
    std::stable_sort(B->snappy_list.begin(), B->snappy_list.end(), [&](int32_t x, int32_t y) {
      return B->pages[(size_t)x].body_len > B->pages[(size_t)y].body_len;
    });
    for (size_t q = 0; q < B->snappy_list.size(); q++) B->pages[(size_t)B->snappy_list[q]].sidx = (int32_t)q;
  }
  {  // segments and k_snappy work items (PQG_SNAPPY_SEGMENTS=0: one wave per page)
    const char *se = getenv("PQG_SNAPPY_SEGMENTS");
    const bool use_seg = !(se && se[0] == '0');
    // a page is cut when its serial chain would outlast the launch: its body
    // beyond 1.5x the average body bytes per k_snappy wave slot (20 per CU),
    // and at least 4 segments long
    int64_t staged = 0;
    for (int32_t pi : B->snappy_list) staged += B->pages[(size_t)pi].body_len;
    const int64_t avg_slot = staged / std::max<int64_t>(1, (int64_t)B->ctx->cus * 20);
    const int64_t seg_min = getenv("PQG_SNAPPY_SEG_MIN") ? std::max<int64_t>(atoll(getenv("PQG_SNAPPY_SEG_MIN")), kSnapSeg + 1)
                                                         : std::max<int64_t>(4 * kSnapSeg, avg_slot * 3 / 2);
    struct It {
      int32_t q, k;
      int64_t bytes;
    };
    std::vector<It> items;
    B->seg_base.assign(B->snappy_list.size() + 1, 0);
    for (size_t q = 0; q < B->snappy_list.size(); q++) {
      const int32_t pq = B->snappy_list[q];
      const PageDesc &pd = B->pages[(size_t)pq];
      const int64_t body = pd.body_len;
      // long pages only: their serial token chains set k_snappy's critical
      // path, while the walk that finds segment starts costs a pass over the
      // compressed bytes (PQG_SNAPPY_SEG_MIN: the threshold, bytes).  Not a
      // page of long literals that k_copy takes (it parallelises them
      // already; BYTE_ARRAY dictionaries copy their own)
      bool cut = use_seg && body >= seg_min;
      const bool defers = !(pd.kind == PAGE_DICT && B->cols[(size_t)pd.col].info.physical_type == T_BYTE_ARRAY);
      if (cut && defers) {
        const int64_t lsize = pd.kind == PAGE_V2 ? (int64_t)pd.v2_rep_len + pd.v2_def_len : 0;
        const int64_t fo = B->page_foff[(size_t)pq] + lsize;
        if (fo >= 0 && fo + (int64_t)pd.comp_len <= (int64_t)B->file->len)
          cut = !snappy_long_literals(B->file->data + fo, pd.comp_len);
      }
      const int32_t nseg = cut ? (int32_t)((body + kSnapSeg - 1) / kSnapSeg) : 1;
      B->seg_base[q + 1] = B->seg_base[q] + nseg;
      if (nseg > 1) B->walk_list.push_back((int32_t)q);
      for (int32_t k = 0; k < nseg; k++)
        items.push_back({(int32_t)q, k, nseg > 1 ? std::min<int64_t>(kSnapSeg, body - (int64_t)k * kSnapSeg) : body});
    }
    // three launches: whole data pages (context stream); then, on a side
    // stream, the segments (after k_snappy_walk) and the whole dictionary
    // pages, which k_dict_prepare follows there.  Each part longest first.
    auto part = [&](const It &x) {
      if (B->seg_base[x.q + 1] - B->seg_base[x.q] > 1) return 2;
      return B->pages[(size_t)B->snappy_list[(size_t)x.q]].kind == PAGE_DICT ? 1 : 0;
    };
    std::stable_sort(items.begin(), items.end(), [&](const It &x, const It &y) {
      const int px = part(x), py = part(y);
      return px != py ? px < py : x.bytes > y.bytes;
    });
    for (const It &it : items) {
      B->snap_items.push_back(it.q);
      B->snap_items.push_back(it.k);
      const int pt = part(it);
      if (pt == 0) B->n_whole_items++;
      if (pt == 1) B->n_dict_items++;
    }
  }
  {  // region-parallel length walks: dictionary pages' first (a launch on the
     // dictionary chain), then data pages' (after k_levels); region records
    B->sw_ndict = (int32_t)B->sw_dict.size();
    B->sw_pages = B->sw_dict;
    B->sw_pages.insert(B->sw_pages.end(), B->sw_data.begin(), B->sw_data.end());
    for (auto &pg : B->pages)
      if (pg.swalk >= 0 && pg.kind != PAGE_DICT) pg.swalk += B->sw_ndict;
    for (size_t i = 0; i < B->sw_pages.size(); i++) {
      SwPage &sp = B->sw_pages[i];
      sp.reg0 = (int32_t)B->sw_nreg;
      B->sw_nreg += sp.nreg;
      for (int32_t k = 0; k * 64 < sp.nreg; k++) {
        B->sw_items.push_back((int32_t)i);
        B->sw_items.push_back(k);
      }
      if ((int32_t)i + 1 == B->sw_ndict) B->sw_dict_items = (int32_t)(B->sw_items.size() / 2);
    }
  }
  B->all_srec = !B->data_list.empty();
  for (int32_t pi : B->data_list) B->all_srec &= B->pages[(size_t)pi].srec != 0;
  B->no_levels = !B->data_list.empty();
  for (int32_t pi : B->data_list) {
    const auto &ci = B->cols[(size_t)B->pages[(size_t)pi].col].info;
    B->no_levels &= ci.max_def == 0 && ci.max_rep == 0;
  }
  phase("plan");
  // tables
  std::vector<std::pair<void **, size_t>> tab_fix;
  size_t tab_off = 0;
  // positions of every page's jobs in the launch order; records start stale (epoch 0)
  std::vector<int32_t> pj((size_t)B->page_job_entries + 1, 0);
  for (size_t p = 0; p < B->tiles.size(); p++) {
    const TileJob &tj = B->tiles[p];
    if (tj.page < 0) continue;
    pj[(size_t)B->pages[(size_t)tj.page].job_base + (size_t)(tj.v0 / EX_WAVE_VALUES)] = (int32_t)p;
  }
  // per Snappy page a region of job slots: at most body_len / 16 KB literals are long enough to defer
  std::vector<int32_t> job_base(B->snappy_list.size() + 1), job_owner;
  for (size_t q = 0; q < B->snappy_list.size(); q++) {
    job_base[q] = (int32_t)job_owner.size();
    // BYTE_ARRAY dictionary pages copy their long literals themselves:
    // k_dict_prepare reads them beside the data pages' Snappy decode, before
    // k_copy (fixed-width dictionaries are read after it)
    const PageDesc &sp = B->pages[(size_t)B->snappy_list[q]];
    const bool ba_dict = sp.kind == PAGE_DICT && B->cols[(size_t)sp.col].info.physical_type == T_BYTE_ARRAY;
    int32_t cap = ba_dict ? 0 : std::min(64, sp.body_len / (16 * 1024));
    for (int32_t k = 0; k < cap; k++) job_owner.push_back((int32_t)q);
  }
  B->max_jobs = (uint32_t)job_owner.size();
  B->ngen_flat = (int32_t)B->general_flat.size();
  B->general_list.insert(B->general_list.end(), B->general_flat.begin(), B->general_flat.end());
  B->general_flat.clear();
  {
    // the chain split by length walk (round 6): columns with a
    // region-parallel length walk (C5's l_comment) are scanned and decoded on
    // side stream 0 after the walk, the other columns' scan and decode start
    // when their own k_prepare ends.  Only when every page of a walked column
    // is a k_plain_str or k_decode<4> page and every k_plain_str page belongs
    // to one; their k_decode<4> pages go last in that launch's list
    std::vector<char> &wcol = B->w_col;
    wcol.assign(B->cols.size(), 0);
    std::vector<char> in_p(npages, 0), in_4(npages, 0);
    bool any_w = false, any_o = false;
    for (int32_t pi : B->data_list)
      if (B->pages[(size_t)pi].swalk >= 0) wcol[(size_t)B->pages[(size_t)pi].col] = 1, any_w = true;
    for (size_t i = 0; i < B->pstr_items.size(); i += 2) in_p[(size_t)B->pstr_items[i]] = 1;
    for (int32_t pg : B->general_str4) in_4[(size_t)pg] = 1;
    bool ok = any_w && B->general_nest.empty();
    for (int32_t pi : B->data_list) {
      const PageDesc &pd = B->pages[(size_t)pi];
      if (wcol[(size_t)pd.col]) ok &= in_p[(size_t)pi] || in_4[(size_t)pi];
      else any_o = true, ok &= !in_p[(size_t)pi];
    }
    static const bool no_split = knob_flag("PQG_NO_WALK_SPLIT");  // (analysis: one scan, as before)
    B->sw_split = ok && any_o && !no_split;
    B->ngen_str4_w = 0;
    B->w_cruns.clear();
    B->o_cruns.clear();
    if (B->sw_split) {
      std::stable_partition(B->general_str4.begin(), B->general_str4.end(),
                            [&](int32_t pg) { return !wcol[(size_t)B->pages[(size_t)pg].col]; });
      for (int32_t pg : B->general_str4) B->ngen_str4_w += wcol[(size_t)B->pages[(size_t)pg].col];
      for (int32_t c = 0; c < (int32_t)B->cols.size(); c++) {
        auto &runs = wcol[(size_t)c] ? B->w_cruns : B->o_cruns;
        if (!runs.empty() && runs.back().second == c) runs.back().second = c + 1;
        else runs.push_back({c, c + 1});
      }
    }
  }
  B->ngen_str4 = (int32_t)B->general_str4.size();
  B->ngen_str = (int32_t)(B->general_str4.size() + B->general_str.size());
  {
    // k_decode<2>'s flat dictionary-string pages (nullable: C4's strings;
    // ~20,000 entries a page, one wave each left most of the GPU idle) in
    // parts of ~STR_PART entries, a wave each.  Part boundaries sit on 256-slot
    // steps of the column (the validity words a step writes are its own); a
    // part counts the values before it from k_levels' level scratch and takes
    // their string bytes from k_prepare's per-256-value prefix table
    // (PageDesc::sp_base), then seeks the key stream.  PQG_STR_PART (analysis):
    // entries a part, 0: whole pages.
    B->str_parts.clear();
    B->str_pre_entries = 0;
    B->str_split = false;
    static const int64_t spart = knob("PQG_STR_PART") ? atoll(knob("PQG_STR_PART")) : STR_PART;
    for (int32_t pg : B->general_str) {
      PageDesc &pd = B->pages[(size_t)pg];
      const int64_t n = std::max(pd.num_values, 0);
      pd.sp_base = -1;
      const bool can = spart > 0 && pd.enc == ENC_RLE_DICT && pd.dict >= 0 && (pd.lvl_bits || pd.lvl_base >= 0) &&
                       n >= 2 * spart;
      if (!can) {
        B->str_parts.insert(B->str_parts.end(), {pg, 0, (int32_t)n});
        continue;
      }
      pd.sp_base = B->str_pre_entries;
      B->str_pre_entries += n / 256 + 2;
      B->str_split = true;
      for (int64_t lo = 0; lo < n;) {
        int64_t hi = ((pd.level_base + lo + spart + 255) & ~(int64_t)255) - pd.level_base;
        if (n - hi < spart / 2) hi = n;
        B->str_parts.insert(B->str_parts.end(), {pg, (int32_t)lo, (int32_t)hi});
        lo = hi;
      }
    }
  }
  {
    // the walked columns' k_decode<4> pages (walk split: C5's l_comment
    // dictionary pages, ~20,000 values and a ~1 MiB dictionary each, the
    // step's last 64 waves) in parts as k_decode<2>'s above: a part's values
    // before it are its first entry (required column), their string bytes
    // from k_prepare's prefix table.  PQG_NO_STR4_PARTS (analysis): whole pages
    B->str4w_parts.clear();
    B->str4w_split = false;
    static const bool no_p4 = knob_flag("PQG_NO_STR4_PARTS");
    static const int64_t spart4 = knob("PQG_STR_PART") ? atoll(knob("PQG_STR_PART")) : STR_PART;
    const size_t n4 = B->general_str4.size();
    for (size_t i = n4 - (size_t)B->ngen_str4_w; i < n4; i++) {
      const int32_t pg = B->general_str4[i];
      PageDesc &pd = B->pages[(size_t)pg];
      const int64_t n = std::max(pd.num_values, 0);
      pd.sp_base = -1;
      const bool can = !no_p4 && spart4 > 0 && pd.enc == ENC_RLE_DICT && pd.dict >= 0 &&
                       B->cols[(size_t)pd.col].info.max_def == 0 && n >= 2 * spart4;
      if (!can) {
        B->str4w_parts.insert(B->str4w_parts.end(), {pg, 0, (int32_t)n});
        continue;
      }
      pd.sp_base = B->str_pre_entries;
      B->str_pre_entries += n / 256 + 2;
      B->str4w_split = true;
      for (int64_t lo = 0; lo < n;) {
        int64_t hi = ((pd.level_base + lo + spart4 + 255) & ~(int64_t)255) - pd.level_base;
        if (n - hi < spart4 / 2) hi = n;
        B->str4w_parts.insert(B->str4w_parts.end(), {pg, (int32_t)lo, (int32_t)hi});
        lo = hi;
      }
    }
  }
  B->general_list.insert(B->general_list.end(), B->general_str4.begin(), B->general_str4.end());
  B->general_list.insert(B->general_list.end(), B->general_str.begin(), B->general_str.end());
  B->general_str4.clear();
  B->general_str.clear();
  B->ngen_nest = (int32_t)B->general_nest.size();
  {
    // list pages split into parts of whole 256-entry steps, one k_decode<3>
    // wave each: ~4,096 entries a part (at least 1/16,384 of the batch's
    // entries).  A part starts from the counts k_levels recorded for it
    // (rows, slots, values before it: PageDesc::part0) and seeks the key
    // stream, so only pages with level scratch and PLAIN / RLE_DICTIONARY
    // values are split.  C4 step (ms) by entries a part: whole pages 4.04,
    // 16,384 3.81, 4,096 3.56, 2,048 3.73, 1,024 3.84 — more waves than two a
    // SIMD (k_decode<3>'s occupancy) only queue.  PQG_NEST_PART: entries per
    // part (0: whole pages).
    int64_t tot = 0;
    for (int32_t pg : B->general_nest) tot += std::max(B->pages[(size_t)pg].num_values, 0);
    const int64_t env_part = getenv("PQG_NEST_PART") ? atoll(getenv("PQG_NEST_PART")) : -1;
    int64_t plen = env_part >= 0 ? env_part : std::max<int64_t>(4096, (tot / 16384 + 255) & ~(int64_t)255);
    if (plen > 0) plen = (plen + 255) & ~(int64_t)255;
    B->nest_parts.clear();
    static const bool part_rescan = knob_flag("PQG_PART_RESCAN");  // (analysis: parts count their own prefix)
    for (int32_t pg : B->general_nest) {
      const PageDesc &pd = B->pages[(size_t)pg];
      const int64_t n = std::max(pd.num_values, 0);
      const int64_t np = plen > 0 && pd.lvl_base >= 0 && (pd.enc == ENC_RLE_DICT || pd.enc == ENC_PLAIN) ? n / plen : 1;
      const int64_t step = np > 1 ? ((n + np - 1) / np + 255) & ~(int64_t)255 : std::max<int64_t>(n, 1);
      // (parts after the first start from k_levels' counts: PageDesc::part0)
      if (np > 1 && !part_rescan) B->pages[(size_t)pg].part0 = (int32_t)(B->nest_parts.size() / 3);
      for (int64_t e = 0; e < n || e == 0; e += step) {
        B->nest_parts.push_back(pg);
        B->nest_parts.push_back((int32_t)e);
        B->nest_parts.push_back((int32_t)std::min(e + step, n));
        if (n == 0) break;
      }
    }
  }
  // the chain split by column kind: only when every data page of a repeated
  // column is a k_decode<3> / <5> page (nothing else on the context stream
  // reads their levels, counts or scanned bases) and no data page has a
  // region-parallel length walk (that k_prepare split stays as it is)
  std::vector<int32_t> rep_pages, flat_pages;
  {
    std::vector<char> in_nest(npages, 0);
    for (int32_t pg : B->general_nest) in_nest[(size_t)pg] = 1;
    bool ok = B->lvl_bytes > 0;
    for (int32_t pi : B->data_list) {
      const PageDesc &pd = B->pages[(size_t)pi];
      if (pd.swalk >= 0) ok = false;
      if (B->cols[(size_t)pd.col].info.max_rep > 0) {
        rep_pages.push_back(pi);
        ok &= in_nest[(size_t)pi] != 0;
      } else {
        flat_pages.push_back(pi);
      }
    }
    static const bool no_split = knob_flag("PQG_NO_REP_SPLIT");  // (analysis: one chain, as before)
    B->rep_split = ok && !no_split && !rep_pages.empty() && !flat_pages.empty();
    B->rep_cruns.clear();
    B->flat_cruns.clear();
    for (int32_t c = 0; c < (int32_t)B->cols.size(); c++) {
      auto &runs = B->cols[(size_t)c].info.max_rep > 0 ? B->rep_cruns : B->flat_cruns;
      if (!runs.empty() && runs.back().second == c) runs.back().second = c + 1;
      else runs.push_back({c, c + 1});
    }
  }
  B->general_list.insert(B->general_list.end(), B->general_nest.begin(), B->general_nest.end());
  B->general_nest.clear();
  {
    std::vector<int32_t> lists;
    lists.insert(lists.end(), B->snappy_list.begin(), B->snappy_list.end());
    lists.insert(lists.end(), B->dict_list.begin(), B->dict_list.end());
    lists.insert(lists.end(), B->data_list.begin(), B->data_list.end());
    lists.insert(lists.end(), B->general_list.begin(), B->general_list.end());
    lists.insert(lists.end(), B->dba_list.begin(), B->dba_list.end());
    lists.insert(lists.end(), B->pstr_items.begin(), B->pstr_items.end());
    // k_inflate: longest bodies first (a page is one wave's serial decode,
    // so the launch ends with its longest page; started first, it overlaps
    // the rest — c5gz's ~1 MiB l_comment pages came last in column order)
    std::stable_sort(B->gzip_list.begin(), B->gzip_list.end(), [&](int32_t x, int32_t y) {
      return B->pages[(size_t)x].body_len > B->pages[(size_t)y].body_len;
    });
    B->gz_off = (int32_t)lists.size();
    lists.insert(lists.end(), B->gzip_list.begin(), B->gzip_list.end());
    // (with the walk split, every page of a walked column is prepared after
    // the walk: that chain's k_scan reads all of its columns' pages)
    auto after_walk = [&](int32_t pi) {
      const PageDesc &pd = B->pages[(size_t)pi];
      return pd.swalk >= 0 || (B->sw_split && B->w_col[(size_t)pd.col]);
    };
    B->prep_a_off = (int32_t)lists.size();
    for (int32_t pi : B->data_list)
      if (!after_walk(pi)) lists.push_back(pi);
    B->prep_a_n = (int32_t)lists.size() - B->prep_a_off;
    B->prep_b_off = (int32_t)lists.size();
    // (the walked columns' pages without a walk first: with the walk split
    // they are prepared beside the walk, on side stream 2)
    for (int32_t pi : B->data_list)
      if (after_walk(pi) && B->pages[(size_t)pi].swalk < 0) lists.push_back(pi);
    B->prep_bw = (int32_t)lists.size() - B->prep_b_off;
    for (int32_t pi : B->data_list)
      if (after_walk(pi) && B->pages[(size_t)pi].swalk >= 0) lists.push_back(pi);
    B->prep_b_n = (int32_t)lists.size() - B->prep_b_off;
    B->rep_off = (int32_t)lists.size();
    lists.insert(lists.end(), rep_pages.begin(), rep_pages.end());
    B->rep_n = (int32_t)rep_pages.size();
    B->flat_off = (int32_t)lists.size();
    lists.insert(lists.end(), flat_pages.begin(), flat_pages.end());
    B->flat_n = (int32_t)flat_pages.size();
    // the small tables: one host image (256-byte aligned entries; the
    // zero-initialised ones are zeros in it) and one copy instead of a
    // synchronous copy or memset each (tens of µs apiece)
    struct {
      std::vector<uint8_t> h;
      std::vector<std::pair<void **, size_t>> fix;
      void put(void **dst, const void *src, size_t n) {
        const size_t off = (h.size() + 255) & ~(size_t)255;
        h.resize(off + std::max<size_t>(n, 64), 0);
        if (src && n) memcpy(h.data() + off, src, n);
        fix.push_back({dst, off});
      }
    } tab;
    tab.put((void **)&B->d_pages, B->pages.data(), sizeof(PageDesc) * npages);
    tab.put((void **)&B->d_status0, B->status0.data(), sizeof(uint32_t) * npages);
    tab.put((void **)&B->d_lists, lists.data(), sizeof(int32_t) * lists.size());
    tab.put((void **)&B->d_parts, B->nest_parts.data(), sizeof(int32_t) * B->nest_parts.size());
    tab.put((void **)&B->d_part_pre, nullptr, sizeof(int32_t) * 4 * (B->nest_parts.size() / 3 + 1));
    tab.put((void **)&B->d_str_parts, B->str_parts.data(), sizeof(int32_t) * B->str_parts.size());
    tab.put((void **)&B->d_str_pre, nullptr, sizeof(int64_t) * (size_t)(B->str_pre_entries + 1));
    tab.put((void **)&B->d_str4w_parts, B->str4w_parts.data(), sizeof(int32_t) * B->str4w_parts.size());
    tab.put((void **)&B->d_lgroups, B->lgroups.data(), sizeof(LdsGroup) * (B->lgroups.size() + 1));
    tab.put((void **)&B->d_page_jobs, pj.data(), sizeof(int32_t) * pj.size());
    tab.put((void **)&B->d_sitems, B->snap_items.data(), 4 * B->snap_items.size());
    tab.put((void **)&B->d_seg_base, B->seg_base.data(), 4 * B->seg_base.size());
    tab.put((void **)&B->d_walk, B->walk_list.data(), 4 * B->walk_list.size());
    tab.put((void **)&B->d_seg_flag, nullptr, 4 * (B->snappy_list.size() + 1));
    tab.put((void **)&B->d_copy_cnt, nullptr, 16);
    tab.put((void **)&B->d_job_base, job_base.data(), 4 * job_base.size());
    tab.put((void **)&B->d_job_owner, job_owner.data(), 4 * job_owner.size());
    tab.put((void **)&B->d_hjobs, B->hjobs.data(), 8 * B->hjobs.size());
    tab.put((void **)&B->d_sw_pages, B->sw_pages.data(), sizeof(SwPage) * B->sw_pages.size());
    tab.put((void **)&B->d_sw_items, B->sw_items.data(), 4 * B->sw_items.size());
    // the image travels with the chunk bytes (the end of the input layout):
    // one pinned-ring upload, no separate copy
    B->tab_host = std::move(tab.h);
    tab_off = in.append(B->tab_host.data(), B->tab_host.size(), 256);
    tab_fix = std::move(tab.fix);
  }
  // device buffers
  int rc = 0;
  size_t in_bytes = in.n;
  if (getenv("PQG_DEBUG_INPUT_HIGH_WORD") && in_bytes + kPad < (1u << 30)) {
    // test knob: place the input buffer where every payload address has bit
    // 31 of its low word set (an oversized allocation, d_in shifted inside
    // it), so a 32-bit lane value widened without a uint32_t cast shows up
    // as a wrong address (the round-1 readlane sign-extension fault)
    rc |= alloc_dev((void **)&B->d_in_alloc, in_bytes + (size_t{1} << 32));
    if (!rc) {
      const uint32_t lw = (uint32_t)(uintptr_t)B->d_in_alloc;
      const bool ok = lw >= 0x80000000u && (uint64_t)lw + in_bytes + kPad <= 0xFFFFFFFFull;
      B->d_in = B->d_in_alloc + (ok ? 0 : (size_t)(uint32_t)(0x80000000u - lw));
    }
  } else {
    rc |= alloc_dev((void **)&B->d_in, in_bytes);
    B->d_in_alloc = B->d_in;
  }
  rc |= alloc_dev((void **)&B->d_stage, (size_t)stage_off);
  B->in_alloc = in_bytes + kPad;
  B->stage_alloc = (size_t)stage_off + kPad;
  // two status arrays, by epoch parity: a decode's k_level_check leaves the
  // next decode's array at the planned statuses (no k_reset launch for them)
  rc |= alloc_dev((void **)&B->d_status, 2 * sizeof(uint32_t) * npages);
  // zero-initialised on the upload stream (not shipped as zeros): page infos
  // (failed pages count zero in the scans) and job records (stale: epoch 0)
  rc |= alloc_dev((void **)&B->d_info, sizeof(PageInfo) * npages);
  rc |= alloc_dev(&B->d_recs, sizeof(ExRec) * (B->tiles.size() + 1));
  rc |= alloc_dev((void **)&B->d_cols, sizeof(ColDesc) * B->cols.size());
  rc |= alloc_dev((void **)&B->d_dict, sizeof(uint64_t) * (size_t)B->dict_entries);
  if (getenv("PQG_DEBUG_INPUT_HIGH_WORD") && 8 * (size_t)(B->run_entries + 64) < (1u << 30)) {
    // the same for the run tables (k_expand_wg widens a record's run-table
    // pointer from two lane words)
    const size_t n = 8 * (size_t)(B->run_entries + 64);
    rc |= alloc_dev(&B->d_runs_alloc, n + (size_t{1} << 32));
    if (!rc) {
      const uint32_t lw = (uint32_t)(uintptr_t)B->d_runs_alloc;
      const bool ok = lw >= 0x80000000u && (uint64_t)lw + n <= 0xFFFFFFFFull;
      B->d_runs = (uint8_t *)B->d_runs_alloc + (ok ? 0 : (size_t)(uint32_t)(0x80000000u - lw));
    }
  } else {
    rc |= alloc_dev(&B->d_runs, 8 * (size_t)(B->run_entries + 64));
    B->d_runs_alloc = B->d_runs;
  }
  rc |= alloc_dev(&B->d_tile_info, 8 * (size_t)(B->tile_entries + EX_WAVE_VALUES / RUN_TILE + 1));
  rc |= alloc_dev((void **)&B->d_tiles, sizeof(TileJob) * (B->tiles.size() + 1));
  rc |= alloc_dev(&B->d_jobs, 32 * (size_t)B->max_jobs);
  rc |= alloc_dev((void **)&B->d_njobs, 4 * (B->snappy_list.size() + 1));
  rc |= alloc_dev((void **)&B->d_copy_idx, 4 * (job_owner.size() + 1));
  rc |= alloc_dev((void **)&B->d_lens, 4 * (size_t)(B->lens_entries + 1));
  rc |= alloc_dev((void **)&B->d_sw_regs, sizeof(SwReg) * (size_t)(B->sw_nreg + 1));
  rc |= alloc_dev((void **)&B->d_sw_res, sizeof(SwRes) * (B->sw_pages.size() + 1));
  rc |= alloc_dev((void **)&B->d_lvl, (size_t)B->lvl_bytes + 16);
  rc |= alloc_dev((void **)&B->d_segs, 8 * (size_t)(B->seg_base.back() + 1));
#ifdef PQ_STAMPS
  rc |= alloc_dev((void **)&B->d_dbg, sizeof(uint64_t) * std::max(8 * 4 * (B->tiles.size() + 1), 4 * (npages + 1)));
  rc |= alloc_dev((void **)&B->d_dbg2, sizeof(uint64_t) * (16 * (npages + 1) + 256));  // + k_snappy_walk stamps
#endif
  if (rc) return PQG_ERR_DEVICE;
  phase("alloc");
  hipStream_t s = bstream(B);  // the batch's decode lane (its counting pass)
  // one upload of all chunk bytes through the context's pinned ring, queued on
  // the upload stream (decodes wait on `ready`; the host goes on planning)
  {
    if (in_bytes && ring_upload(ctx, B->d_in, in, ctx->upload, &B->upload_gather_ms, &B->upload_wait_ms)) {
      set_err("input upload failed");
      return PQG_ERR_DEVICE;
    }
    hipMemsetAsync(B->d_in + in_bytes, 0, kPad, ctx->upload);
    B->h2d_bytes += (int64_t)in_bytes;
    for (auto &f : tab_fix) *f.first = B->d_in + tab_off + f.second;
    hipMemsetAsync(B->d_info, 0, sizeof(PageInfo) * npages, ctx->upload);
    // job records: stale (epoch 0), and the host's records of tiled PLAIN
    // pages (EPOCH_STATIC) at their launch positions
    bool any_srec = false;
    for (const TileJob &tj : B->tiles) any_srec |= tj.page >= 0 && B->pages[(size_t)tj.page].srec;
    if (!any_srec) {
      hipMemsetAsync(B->d_recs, 0, sizeof(ExRec) * (B->tiles.size() + 1), ctx->upload);
    } else {
      B->recs_host.assign(B->tiles.size() + 1, ExRec{});
      for (size_t p = 0; p < B->tiles.size(); p++) {
        const TileJob &tj = B->tiles[p];
        if (tj.page < 0 || !B->pages[(size_t)tj.page].srec) continue;
        const PageDesc &d = B->pages[(size_t)tj.page];
        ExRec &rc = B->recs_host[p];
        rc.vals = (d.body_src == BODY_RAW ? B->d_in : B->d_stage) + d.body;
        rc.v0 = tj.v0;
        rc.lim = std::min(tj.v0 + EX_WAVE_VALUES, std::max(d.num_values, 0));
        rc.bw = -1;
        rc.epoch = EPOCH_STATIC;
        rc.val_len = d.body_len;
      }
      hipMemcpyAsync(B->d_recs, B->recs_host.data(), sizeof(ExRec) * B->recs_host.size(), hipMemcpyHostToDevice,
                     ctx->upload);
    }
    if (hipEventCreateWithFlags(&B->ready, hipEventDisableTiming) != hipSuccess) {
      set_err("hipEventCreate failed");
      return PQG_ERR_DEVICE;
    }
  }
  for (auto &hb : host_bodies) {
    HIPCHK(hipMemcpy(B->d_stage + hb.first, hb.second.data(), hb.second.size(), hipMemcpyHostToDevice));
    B->h2d_bytes += (int64_t)hb.second.size();
  }
  phase("upload");

  // column descriptors (outputs allocated after the counting pass)
  B->hcols.resize(B->cols.size());
  for (size_t ci = 0; ci < B->cols.size(); ci++) {
    ColumnPlan &cp = B->cols[ci];
    ColDesc &c = B->hcols[ci];
    memset(&c, 0, sizeof(c));
    c.ptype = cp.info.physical_type;
    c.width = cp.info.value_width;
    c.max_def = cp.info.max_def;
    c.max_rep = cp.info.max_rep;
    // deeper nesting (max_rep >= 2): the column store's own layout — def/rep
    // levels and the dense values (data_store.go:15-31); a slot is a value
    c.rep_def = cp.info.max_rep >= 2 ? cp.info.max_def : cp.info.rep_def;
    c.page_begin = cp.page_begin;
    c.page_end = cp.page_end;
    c.flags = cp.flags;
    c.total_levels = cp.levels;
  }
  const bool any_count = B->any_count;
  // every set-up copy is queued on the upload stream behind the chunk bytes
  // (from host memory the batch keeps): batch creation never waits for the
  // DMA engine, and each decode waits on `ready`
  B->hcols0 = B->hcols;  // hcols changes after the counting pass
  if (!B->cols.empty())
    HIPCHK(hipMemcpyAsync(B->d_cols, B->hcols0.data(), sizeof(ColDesc) * B->cols.size(), hipMemcpyHostToDevice,
                          ctx->upload));
  HIPCHK(hipEventRecord(B->ready, ctx->upload));
  if (any_count) {
    // counting pass: snappy + prepare + scan once to size list/string outputs
    rc = launch_all(B, true, false);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(s));
    std::vector<ColDesc> tmp(B->cols.size());
    HIPCHK(hipMemcpy(tmp.data(), B->d_cols, sizeof(ColDesc) * tmp.size(), hipMemcpyDeviceToHost));
    for (size_t ci = 0; ci < B->cols.size(); ci++) {
      B->hcols[ci].total_rows = tmp[ci].total_rows;
      B->hcols[ci].total_slots = tmp[ci].total_slots;
      B->hcols[ci].total_str = tmp[ci].total_str;
      // list offsets are int32 (Arrow List): a batch whose element count does
      // not fit must be split into fewer row groups
      if (B->hcols[ci].max_rep == 1 && tmp[ci].total_slots > (int64_t)INT32_MAX) {
        set_err("leaf %d: %lld list elements overflow int32 offsets; decode fewer row groups per batch",
                B->cols[ci].leaf, (long long)tmp[ci].total_slots);
        return PQG_ERR_SIZE;
      }
    }
  }
  // outputs
  for (size_t ci = 0; ci < B->cols.size(); ci++) {
    ColumnPlan &cp = B->cols[ci];
    ColDesc &c = B->hcols[ci];
    if (!(cp.flags & COL_NEEDS_COUNT)) {
      c.total_slots = cp.levels;
      c.total_rows = cp.info.max_rep == 0 ? cp.levels : 0;
      c.total_str = 0;
    } else if (cp.info.max_rep == 0) {
      // a flat column's slot of level i is i (k_decode indexes its slot
      // outputs by the page's level base): size them by the levels even when
      // a page failed before its counts were taken (its counts are zero)
      c.total_slots = cp.levels;
      c.total_rows = cp.levels;
    }
    cp.slots = c.total_slots;
    cp.rows = c.total_rows;
    cp.str_bytes = c.total_str;
    bool is_ba = c.ptype == T_BYTE_ARRAY;
    cp.values_bytes = is_ba ? (size_t)c.total_str : (size_t)c.total_slots * (size_t)std::max(c.width, 0);
    rc |= alloc_dev(&cp.values, cp.values_bytes);
    if (c.max_def > 0) {
      cp.validity_bytes = (size_t)((c.total_slots + 63) / 64) * 8;
      rc |= alloc_dev(&cp.validity, cp.validity_bytes);
    }
    if (c.max_rep == 1) {
      cp.list_off_bytes = sizeof(int32_t) * (size_t)(c.total_rows + 1);
      cp.list_val_bytes = (size_t)((c.total_rows + 63) / 64) * 8;
      rc |= alloc_dev(&cp.list_offsets, cp.list_off_bytes);
      rc |= alloc_dev(&cp.list_validity, cp.list_val_bytes);
    }
    if (is_ba) {
      cp.str_off_bytes = sizeof(int64_t) * (size_t)(c.total_slots + 1);
      rc |= alloc_dev(&cp.str_offsets, cp.str_off_bytes);
    }
    if (cp.flags & COL_EMIT_LEVELS) {
      rc |= alloc_dev(&cp.def_out, (size_t)cp.levels);
      rc |= alloc_dev(&cp.rep_out, (size_t)cp.levels);
    }
    c.values = (uint8_t *)cp.values;
    c.validity = (uint32_t *)cp.validity;
    c.list_offsets = (int32_t *)cp.list_offsets;
    c.list_validity = (uint32_t *)cp.list_validity;
    c.str_offsets = (int64_t *)cp.str_offsets;
    c.def_out = (uint8_t *)cp.def_out;
    c.rep_out = (uint8_t *)cp.rep_out;
    if (c.max_rep >= 2 && c.max_rep <= NEST_MAXR && (int)cp.rdefs.size() == c.max_rep) {
      const int R = c.max_rep;
      cp.nest_ostride = cp.levels + 1;
      cp.nest_vstride = (cp.levels + 32) / 32;
      cp.nest_nblocks = (int32_t)((cp.levels + NEST_CH - 1) / NEST_CH);
      rc |= alloc_dev(&cp.nest_off, sizeof(int32_t) * (size_t)(R * cp.nest_ostride));
      rc |= alloc_dev(&cp.nest_val, sizeof(uint32_t) * (size_t)((R + 1) * cp.nest_vstride));
      rc |= alloc_dev(&cp.nest_sums, sizeof(int32_t) * (size_t)(R + 1) * (size_t)(cp.nest_nblocks + 1));
      rc |= alloc_dev(&cp.nest_cnt, sizeof(int64_t) * (size_t)(R + 1));
    }
  }
  if (rc) return PQG_ERR_DEVICE;
  if (!B->cols.empty())
    HIPCHK(hipMemcpyAsync(B->d_cols, B->hcols.data(), sizeof(ColDesc) * B->cols.size(), hipMemcpyHostToDevice,
                          ctx->upload));
  // k_expand jobs: output pointers now that the outputs exist
  for (TileJob &tj : B->tiles) {
    if (tj.page < 0) continue;  // an unused slot
    const PageDesc &d = B->pages[(size_t)tj.page];
    const ColDesc &c = B->hcols[(size_t)d.col];
    tj.width = c.width;
    tj.out = c.values + d.level_base * (int64_t)c.width;
  }
  if (!B->tiles.empty())
    HIPCHK(hipMemcpyAsync(B->d_tiles, B->tiles.data(), sizeof(TileJob) * B->tiles.size(), hipMemcpyHostToDevice,
                          ctx->upload));
  {  // the validity bitmaps k_reset zeroes in every decode
    std::vector<ZeroRange> &zr = B->zr_host;
    for (auto &cp : B->cols) {
      if (cp.validity) zr.push_back({(uint32_t *)cp.validity, cp.validity_bytes / 4});
      if (cp.list_validity) zr.push_back({(uint32_t *)cp.list_validity, cp.list_val_bytes / 4});
    }
    B->nzr = (int32_t)zr.size();
    if (!zr.empty()) {
      if (alloc_dev(&B->d_zr, sizeof(ZeroRange) * zr.size())) {
        set_err("device allocation failed");
        return PQG_ERR_DEVICE;
      }
      HIPCHK(hipMemcpyAsync(B->d_zr, zr.data(), sizeof(ZeroRange) * zr.size(), hipMemcpyHostToDevice, ctx->upload));
    }
  }
  HIPCHK(hipEventRecord(B->ready, ctx->upload));  // decodes wait for every set-up copy
  B->ready_final = true;
  phase("outputs+tables");
  return PQG_OK;
}

static int batch_create_lane(pqg_ctx *ctx, pqg_file *f, int rg_begin, int rg_end, const int *leaves, int nleaves,
                             int flags, int lane, pqg_batch **out);

int pqg_batch_create(pqg_ctx *ctx, pqg_file *f, int rg_begin, int rg_end, const int *leaves, int nleaves, int flags,
                     pqg_batch **out) {
  return batch_create_lane(ctx, f, rg_begin, rg_end, leaves, nleaves, flags, 0, out);
}

static int batch_create_lane(pqg_ctx *ctx, pqg_file *f, int rg_begin, int rg_end, const int *leaves, int nleaves,
                             int flags, int lane, pqg_batch **out) {
  *out = nullptr;
  if (!ctx || !f || rg_begin < 0 || rg_end > (int)f->rgs.size() || rg_begin > rg_end || nleaves < 0) {
    set_err("bad batch arguments");
    return PQG_ERR_ARG;
  }
  HIPCHK(hipSetDevice(ctx->device));
  pqg_batch *B = new pqg_batch();
  B->ctx = ctx;
  B->lane = lane;
  B->file = f;
  B->rg_begin = rg_begin;
  B->rg_end = rg_end;
  B->flags = flags;
  const int rc = batch_init(B, ctx, f, rg_begin, rg_end, leaves, nleaves, flags);
  if (rc != PQG_OK) {
    pqg_batch_destroy(B);
    return rc;
  }
  *out = B;
  return PQG_OK;
}

static int launch_all(pqg_batch *B, bool upto_scan, bool timed) {
  const LaneRef LN = lane_of(B);
  hipStream_t s = LN.stream;
  const size_t npages = B->pages.size();
  // one launch sequence at a time per lane (shared fork/join events)
  std::lock_guard<std::mutex> launch_lock(*LN.mu);
  if (B->ready) hipStreamWaitEvent(s, B->ready, 0);  // the chunk bytes are on the device
  if (timed && !B->ev[B->ring_head][0])  // timing events of this ring slot, made on first use
    for (int i = 0; i < 8; i++) hipEventCreate(&B->ev[B->ring_head][i]);
  pq_launch_args a = {};
  a.snappy_wg = getenv_flag("PQG_SNAPPY_WG") ? 1 : 0;  // (read per decode: tests switch it per batch)
  a.in = B->d_in;
  a.stage = B->d_stage;
  a.in_end = B->d_in + B->in_alloc;
  a.stage_end = B->d_stage + B->stage_alloc;
  a.pages = B->d_pages;
  a.info = B->d_info;
  a.cols = B->d_cols;
  a.dict_ent = B->d_dict;
  a.ncols = (int32_t)B->cols.size();
  a.jobs = B->d_jobs;
  a.njobs = B->d_njobs;
  a.max_jobs = B->max_jobs;
  a.job_base = B->d_job_base;
  a.job_owner = B->d_job_owner;
  a.copy_cnt = B->d_copy_cnt;
  a.hjobs = B->d_hjobs;
  a.sw_pages = B->d_sw_pages;
  a.sw_regs = B->d_sw_regs;
  a.sw_res = B->d_sw_res;
  a.sw_items = B->d_sw_items;
  // (the dictionary pages' part: launches before k_dict_prepare)
  a.n_sw_items = B->sw_dict_items;
  a.sw_page0 = 0;
  a.n_sw_pages = B->sw_ndict;
  a.nhjobs = (int32_t)(B->hjobs.size() / 4);
  a.copy_idx = B->d_copy_idx;
  a.lens = B->d_lens;
  a.lvl = B->d_lvl;
  a.part_tab = B->d_parts;
  a.part_pre = B->d_part_pre;
  a.str_pre = B->d_str_pre;
  a.status0 = B->d_status0;
  a.zr = B->d_zr;
  a.nzr = upto_scan ? 0 : B->nzr;  // the bitmaps are written by the decode kernels only
  a.npages = (int32_t)npages;
  a.dbg = B->d_dbg;
  a.dbg2 = B->d_dbg2;
  a.npages_dbg = (int32_t)B->pages.size() + 1;
  a.runs = B->d_runs;
  a.tile_info = B->d_tile_info;
  a.ex_lds = B->ex_lds;
  a.recs = B->d_recs;
  a.page_jobs = B->d_page_jobs;
  // the first decode after the counting pass resumes from it: the staged
  // pages, level / length scratch, job records and scanned bases it left are
  // this decode's (same epoch), so only the bitmaps are zeroed and the decode
  // phase runs
  // launches are checked with hipGetLastError: drop an error an earlier API
  // call left behind (e.g. a query's hipErrorNotReady), which is not this
  // decode's
  (void)hipGetLastError();
  const bool resume = !upto_scan && B->counted;
  B->counted = upto_scan;
  a.epoch = resume ? B->epoch : ++B->epoch;
  a.status = B->d_status + (a.epoch & 1) * npages;
  a.tiles = B->d_tiles;
  a.lgroups = B->d_lgroups;
  for (int i = 0; i < 6; i++) {
    a.ldn[i] = B->ldn[i];
    a.ldl[i] = B->ldl[i];
  }
  const int32_t ns = (int32_t)B->snappy_list.size(), nd = (int32_t)B->dict_list.size(),
                ndata = (int32_t)B->data_list.size(), ngen = (int32_t)B->general_list.size();
  int e = 0;
  // statuses: already planned when the previous decode's k_level_check set
  // this epoch's array (k_reset then only zeroes the validity bitmaps)
  const bool st_planned = resume || B->st_ready[a.epoch & 1];
  B->st_ready[a.epoch & 1] = false;
  if (st_planned) {
    if (a.nzr) {  // k_reset over the bitmaps only
      pq_launch_args z = a;
      z.npages = 0;
      e |= pq_launch(13, &z, s);
    }
  } else if (npages || a.nzr) {
    e |= pq_launch(13, &a, s);  // k_reset: statuses and validity bitmaps
  }
  if (timed) B->nev = 0;  // an untimed decode keeps the last timed segment count
  hipEvent_t *evs = B->ev[B->ring_head];
  // events cost a gap between dependent kernels: by default only the decode
  // phase is bracketed (the roofline kernel), PQG_SEGMENT_TIMES=1 brackets all
  auto mark = [&](bool decode_edge) {
    if (timed && (B->seg_times || decode_edge)) hipEventRecord(evs[B->nev++], s);
  };
  // k_levels with two waves a page (repetition and definition streams side by
  // side) when a selected column is repeated: C4's lists 2.05 -> 1.61 ms; a
  // flat batch keeps four pages a workgroup (C3's def-only pages: 0.77 vs 0.96 ms)
  bool any_rep = false;
  for (const auto &cp : B->cols) any_rep |= cp.info.max_rep > 0;
  const int lv_id = any_rep ? 24 : 19;
  // V2 level streams are raw bytes of the chunk: with no page waiting on a
  // dictionary, k_levels needs nothing the Snappy phase writes and runs beside
  // it on a side stream (C3: its 0.73 ms left the critical path)
  // PQG_LEVELS_LATE=1 (analysis): k_levels back after the Snappy phase
  static const bool lvl_late_env = knob("PQG_LEVELS_LATE") != nullptr;
  const bool lvl_early = !resume && B->lvl_bytes > 0 && !B->lvl_late && !B->seg_times && !lvl_late_env;
  // repeated columns' level / prepare / scan chain on side stream 2, beside
  // the other columns' (B->rep_split; not with the fused prepare-copy launch
  // or phase timing)
  const bool rsplit = !resume && B->rep_split && B->lvl_bytes > 0 && !lvl_early && !B->seg_times &&
                      !(nd == 0 && (B->max_jobs > 0 || !B->hjobs.empty()));
  // walked columns' scan and decode on side stream 0 after the length walk,
  // the other columns' from the end of their own k_prepare (B->sw_split)
  static const bool prep_serial = knob_flag("PQG_PREP_SERIAL");
  const bool wsplit = !resume && !rsplit && B->sw_split && !B->seg_times && !prep_serial && !B->all_srec &&
                      B->prep_b_n > 0 && B->prep_a_n > 0 && !(nd == 0 && (B->max_jobs > 0 || !B->hjobs.empty()));
  auto scan_runs = [&](const std::vector<std::pair<int32_t, int32_t>> &runs, hipStream_t st) {
    for (const auto &r : runs) {
      pq_launch_args sc = a;
      sc.cols = B->d_cols + r.first;
      sc.ncols = r.second - r.first;
      e |= pq_launch(4, &sc, st);  // k_scan over the run's columns
    }
  };
  if (!resume) {
  mark(false);
  // (k_levels first on the context stream with k_snappy on the side stream
  // was measured slower on C3: 6.4 vs 5.3 ms, the two launches' waves
  // sharing every CU for the whole phase)
  if (lvl_early) {
    pq_launch_args al = a;
    al.list = B->d_lists + ns + nd;
    al.nlist = ndata;
    hipEventRecord(LN.fork, s);
    hipStreamWaitEvent(LN.side[2], LN.fork, 0);
    // PQG_LEVELS_CAP=k: k workgroups per CU looping over the pages, resident
    // from the start beside k_snappy's.  Measured on C3 (ms a step): full
    // grid 5.38, k = 1 6.52, 2 5.91, 4 5.43, 8 5.37 — resident waves beside
    // k_snappy's get too little issue; the full grid stays
    static const int lv_cap = knob("PQG_LEVELS_CAP") ? atoi(knob("PQG_LEVELS_CAP")) : 0;
    al.grid_cap = lv_cap > 0 ? lv_cap * B->ctx->cus : 0;
    e |= pq_launch(lv_id, &al, LN.side[2]);  // k_levels<-1>: every level page
    hipEventRecord(LN.join[2], LN.side[2]);
  }
  if (!B->gzip_list.empty()) {
    // gzip pages (k_inflate, a wave each) before everything that reads a
    // body: the Snappy phase's dictionary preparation forks after this
    InflateArgs ia{B->d_in, B->d_stage, B->d_pages, a.status, B->d_lists + B->gz_off, (int32_t)B->gzip_list.size()};
    if (pq_launch_inflate(&ia, s)) e |= 1;
  }
  a.list = B->d_lists;
  a.nlist = ns;
  a.sitems = B->d_sitems;
  a.nitems = (int32_t)(B->snap_items.size() / 2);
  a.walk = B->d_walk;
  a.nwalk = (int32_t)B->walk_list.size();
  a.seg_base = B->d_seg_base;
  a.segs = B->d_segs;
  a.seg_flag = B->d_seg_flag;
  {
    // Two streams: k_snappy_walk (segment starts of the long pages), their
    // segments, the serial fallback, the whole dictionary pages and
    // k_dict_prepare — a few waves of serial work each, which would idle the
    // GPU on their own — beside the whole data pages.  Only the whole data
    // pages defer literals to k_copy (after the join).
    const int32_t nall = (int32_t)(B->snap_items.size() / 2), nwhole = B->n_whole_items, ndict = B->n_dict_items;
    // without segmented pages or string dictionaries to prepare, the whole
    // data pages and the dictionary pages are one launch on the context
    // stream (items [0, nwhole + ndict) are contiguous): the fork / join
    // around a side stream cost ~10 us of gaps per decode (C2)
    const bool one = B->walk_list.empty() && nd == 0 && nall == nwhole + ndict;
    const bool side = !one && (nall > nwhole || nd > 0) && !B->seg_times;
    // the serial chain (walk -> segments -> ...) goes on the context stream,
    // dispatched first, and the whole data pages on the side stream: a chain
    // on the side stream was dispatched after the whole pages had taken the
    // CUs (PQG_WALK_SIDE=1 restores that order for comparison)
    static const bool walk_side = [] {
      const char *v = knob("PQG_WALK_SIDE");
      return v && v[0] == '1';
    }();
    hipStream_t ss = side && walk_side ? LN.side[0] : s;   // the serial chain
    hipStream_t sw = side && !walk_side ? LN.side[0] : s;  // whole data pages
    // (the whole dictionary pages and k_dict_prepare stay on the chain: a
    // BYTE_ARRAY dictionary page may itself be segmented — C5's l_comment
    // dictionaries — and k_dict_prepare reads what its segments write)
    if (side) {
      hipEventRecord(LN.fork, s);
      hipStreamWaitEvent(LN.side[0], LN.fork, 0);
    }
    if (one) {
      a.nitems = nwhole + ndict;
      e |= pq_launch(0, &a, s);  // k_snappy: every page (whole data pages, then dictionary pages)
    }
    if (!one) e |= pq_launch(17, &a, ss);  // k_snappy_walk
    if (!walk_side && !one) {
      a.nitems = nwhole;
      e |= pq_launch(0, &a, sw);  // k_snappy: whole data pages (side stream)
    }
    pq_launch_args aw = a;
    if (!one) {
      aw.sitems = B->d_sitems + 2 * (size_t)(nwhole + ndict);
      aw.nitems = nall - nwhole - ndict;
      e |= pq_launch(0, &aw, ss);  // k_snappy: segments
      e |= pq_launch(18, &a, ss);  // serial fallback for pages whose segments did not decode alone
      aw.sitems = B->d_sitems + 2 * (size_t)nwhole;
      aw.nitems = ndict;
      e |= pq_launch(0, &aw, ss);  // k_snappy: whole dictionary pages
    }
    if (side) {
      aw = a;
      aw.list = B->d_lists + ns;
      aw.nlist = nd;
      e |= pq_launch(28, &aw, ss);  // long dictionary pages: region-parallel length walk
      e |= pq_launch(29, &aw, ss);
      e |= pq_launch(30, &aw, ss);
      e |= pq_launch(1, &aw, ss);  // k_dict_prepare (its pages are all decoded on this stream)
    }
    if (walk_side && !one) {
      a.nitems = nwhole;
      e |= pq_launch(0, &a, sw);  // k_snappy: whole data pages
    }
    if (side) {
      hipEventRecord(LN.join[0], LN.side[0]);
      hipStreamWaitEvent(s, LN.join[0], 0);
    }
  }
  // without BYTE_ARRAY dictionaries nothing k_prepare reads waits on k_copy
  // except data pages with deferred literals: k_prepare runs beside the copies
  // in one launch and those pages after it (with string dictionaries, the
  // string pages would all wait: measured slower)
  const bool fused = nd == 0 && (B->max_jobs > 0 || !B->hjobs.empty()) && !B->seg_times;
  if (lvl_early) hipStreamWaitEvent(s, LN.join[2], 0);  // the levels and counts k_prepare reads
  const bool lvl_now = B->lvl_bytes && !lvl_early;
  // long PLAIN string pages: the length walk region-parallel (after the
  // copies and k_levels' non-null counts; k_prepare reads the result)
  auto sw_walk = [&](hipStream_t ws) {
    if ((int32_t)B->sw_pages.size() == B->sw_ndict) return;
    pq_launch_args w = a;
    w.sw_items = B->d_sw_items + 2 * (size_t)B->sw_dict_items;
    w.n_sw_items = (int32_t)(B->sw_items.size() / 2) - B->sw_dict_items;
    w.sw_page0 = B->sw_ndict;
    w.n_sw_pages = (int32_t)B->sw_pages.size() - B->sw_ndict;
    e |= pq_launch(28, &w, ws);  // k_sw_regions
    e |= pq_launch(29, &w, ws);  // k_sw_link
    e |= pq_launch(30, &w, ws);  // k_sw_emit
  };
  if (fused) {
    a.list = B->d_lists + ns + nd;
    a.nlist = ndata;
    if (lvl_now) e |= pq_launch(lv_id + 1, &a, s);  // k_levels: pages that do not wait on k_copy
    {
      pq_launch_args pc = a;
      if (B->all_srec) pc.nlist = 0;  // the copies only
      e |= pq_launch(12, &pc, s);  // k_prepare_copy (+ the run walk of tiled RLE_DICTIONARY pages)
    }
    if (B->data_may_defer && !B->all_srec) {  // pages that waited on k_copy (or on the length walk)
      if (lvl_now) e |= pq_launch(lv_id + 2, &a, s);
      sw_walk(s);
      e |= pq_launch(11, &a, s);
    }
  } else {
    e |= pq_launch(6, &a, s);  // k_copy: long literals, timed together with k_snappy
    mark(false);
    if (B->seg_times) {  // phase timing: k_dict_prepare here (not on the side stream)
      a.list = B->d_lists + ns;
      a.nlist = nd;
      e |= pq_launch(28, &a, s);
      e |= pq_launch(29, &a, s);
      e |= pq_launch(30, &a, s);
      e |= pq_launch(1, &a, s);
    }
    mark(false);
    a.list = B->d_lists + ns + nd;
    a.nlist = ndata;
    if (rsplit) {
      // repeated columns' pages on side stream 2: k_levels (two waves a
      // page), k_prepare, k_scan of their columns, then their k_decode<5> /
      // <3> below, beside the other columns' chain on the context stream
      hipEventRecord(LN.fork, s);
      hipStreamWaitEvent(LN.side[2], LN.fork, 0);
      pq_launch_args ar = a;
      ar.list = B->d_lists + B->rep_off;
      ar.nlist = B->rep_n;
      e |= pq_launch(24, &ar, LN.side[2]);  // k_levels<-1, true>
      e |= pq_launch(2, &ar, LN.side[2]);   // k_prepare
      if (B->any_count) scan_runs(B->rep_cruns, LN.side[2]);
      a.list = B->d_lists + B->flat_off;
      a.nlist = B->flat_n;
      e |= pq_launch(19, &a, s);  // k_levels<-1, false>: the other columns' pages
      e |= pq_launch(2, &a, s);   // k_prepare
    } else if (lvl_now) e |= pq_launch(lv_id, &a, s);  // k_levels
    // the region-parallel length walk and k_prepare of the pages that read it
    // on side stream 0, k_prepare of every other page beside them (round 6,
    // C5: 15.46 / 15.48 -> 15.22 / 15.26 ms).  PQG_PREP_SERIAL=1 (analysis):
    // one k_prepare launch after the walk, as before
    if (rsplit) {
      // (k_prepare launched above, per chain)
    } else if (!prep_serial && !B->all_srec && B->prep_b_n > 0 && B->prep_a_n > 0 && !B->seg_times) {
      hipEventRecord(LN.fork, s);
      hipStreamWaitEvent(LN.side[0], LN.fork, 0);
      pq_launch_args pb = a;
      pb.list = B->d_lists + B->prep_b_off;
      pb.nlist = B->prep_b_n;
      if (wsplit && B->prep_bw > 0) {
        // the walked columns' other pages (C5: l_comment's dictionary pages,
        // 0.7 ms) prepared beside the walk on side stream 2
        hipStreamWaitEvent(LN.side[2], LN.fork, 0);
        pq_launch_args pw = pb;
        pw.nlist = B->prep_bw;
        e |= pq_launch(2, &pw, LN.side[2]);
        hipEventRecord(LN.join[2], LN.side[2]);
        pb.list += B->prep_bw;
        pb.nlist -= B->prep_bw;
      }
      sw_walk(LN.side[0]);
      e |= pq_launch(2, &pb, LN.side[0]);  // k_prepare: pages with a length walk
      if (wsplit && B->prep_bw > 0) hipStreamWaitEvent(LN.side[0], LN.join[2], 0);
      if (wsplit && B->any_count) scan_runs(B->w_cruns, LN.side[0]);  // k_scan: the walked columns
      hipEventRecord(LN.join[0], LN.side[0]);
      pq_launch_args pa = a;
      pa.list = B->d_lists + B->prep_a_off;
      pa.nlist = B->prep_a_n;
      e |= pq_launch(2, &pa, s);  // k_prepare: the other pages (+ the run walk of tiled pages)
      if (!wsplit) hipStreamWaitEvent(s, LN.join[0], 0);
    } else {
      sw_walk(s);
      if (!B->all_srec) e |= pq_launch(2, &a, s);  // (+ the run walk of tiled RLE_DICTIONARY pages)
    }
  }
  mark(false);
  }  // !resume
  // scans only feed lists / strings (rerun on resume: with the outputs now
  // allocated they also write the closing list / string offsets)
  if (rsplit) {
    if (B->any_count) scan_runs(B->flat_cruns, s);
    if (upto_scan) {  // the counting pass ends with both chains
      hipEventRecord(LN.join[2], LN.side[2]);
      hipStreamWaitEvent(s, LN.join[2], 0);
    }
  } else if (wsplit) {
    if (B->any_count) scan_runs(B->o_cruns, s);  // (the walked columns': side stream 0, above)
    if (upto_scan) hipStreamWaitEvent(s, LN.join[0], 0);
  } else if (B->any_count) {
    e |= pq_launch(4, &a, s);
  }
  mark(true);
  if (!upto_scan) {
    // the three k_decode instances run side by side: <1> and <2> on side
    // streams forked here, joined before anything reads their output
    const int32_t ng0 = ngen - B->ngen_flat - B->ngen_str - B->ngen_nest;
    const int32_t npstr = (int32_t)(B->pstr_items.size() / 2);
    const bool str_side = B->ngen_str > 0 || npstr > 0;
    const bool fork = B->ngen_flat > 0 || str_side || B->ngen_nest > 0;
    if (fork) hipEventRecord(LN.fork, s);
    // the walked columns' k_decode<4> pages on side stream 2 once their scan
    // (side stream 0) is done, not behind the other columns' <4> pages
    const int32_t n4w = wsplit ? B->ngen_str4_w : 0;
    if (n4w > 0) {
      hipEventRecord(LN.join[2], LN.side[0]);
      hipStreamWaitEvent(LN.side[2], LN.join[2], 0);
      hipStreamWaitEvent(LN.side[2], LN.fork, 0);
      pq_launch_args aw4 = a;
      aw4.list = B->d_lists + ns + nd + ndata + ng0 + B->ngen_flat + (B->ngen_str4 - n4w);
      aw4.nlist = n4w;
      if (B->str4w_split) {
        pq_launch_args ap = aw4;
        ap.parts = B->d_str4w_parts;
        ap.nlist = (int32_t)(B->str4w_parts.size() / 3);
        e |= pq_launch(31, &ap, LN.side[2]);  // k_decode<4>: the walked columns' dictionary pages, in parts
        ap = aw4;
        ap.redo = 1;
        e |= pq_launch(31, &ap, LN.side[2]);  // k_decode<4>: pages whose later parts failed, whole
      } else {
        e |= pq_launch(31, &aw4, LN.side[2]);  // k_decode<4>: the walked columns' dictionary pages
      }
      hipEventRecord(LN.join[2], LN.side[2]);
    }
    if (B->ngen_flat > 0) {
      hipStreamWaitEvent(LN.side[0], LN.fork, 0);
      a.list = B->d_lists + ns + nd + ndata + ng0;
      a.nlist = B->ngen_flat;
      e |= pq_launch(14, &a, LN.side[0]);  // k_decode<1>: flat fixed-width pages
      hipEventRecord(LN.join[0], LN.side[0]);
    }
    // k_plain_str on side stream 0 (after k_decode<1>), beside the
    // dictionary strings on side stream 1 instead of before them (round 6,
    // C5: 15.98 / 15.92 -> 15.70 / 15.72 ms; round 4's k_decode<2> had
    // needed the wave slots).  PQG_PSTR_SERIAL=1 (analysis): the old order
    static const bool pstr_serial = knob_flag("PQG_PSTR_SERIAL");
    const bool pstr0 = !pstr_serial && npstr > 0;
    if (pstr0) {
      if (B->ngen_flat == 0) hipStreamWaitEvent(LN.side[0], LN.fork, 0);
      pq_launch_args ap = a;
      ap.list = B->d_lists + ns + nd + ndata + ngen + (int32_t)B->dba_list.size();
      ap.nlist = npstr;
      e |= pq_launch(23, &ap, LN.side[0]);
      hipEventRecord(LN.join[0], LN.side[0]);
    }
    if (str_side) {
      hipStreamWaitEvent(LN.side[1], LN.fork, 0);
      if (npstr > 0 && !pstr0) {  // k_plain_str: flat required PLAIN string pages, items of PLAIN_STR_ITEM values
        a.list = B->d_lists + ns + nd + ndata + ngen + (int32_t)B->dba_list.size();
        a.nlist = npstr;
        e |= pq_launch(23, &a, LN.side[1]);
      }
      a.list = B->d_lists + ns + nd + ndata + ng0 + B->ngen_flat;
      a.nlist = B->ngen_str4 - n4w;
      e |= pq_launch(31, &a, LN.side[1]);  // k_decode<4>: flat required dictionary strings
      a.list = B->d_lists + ns + nd + ndata + ng0 + B->ngen_flat + B->ngen_str4;
      a.nlist = B->ngen_str - B->ngen_str4;
      if (B->str_split) {
        pq_launch_args ap = a;
        ap.parts = B->d_str_parts;
        ap.nlist = (int32_t)(B->str_parts.size() / 3);
        e |= pq_launch(15, &ap, LN.side[1]);  // k_decode<2>: the other flat BYTE_ARRAY pages, in parts
        ap = a;
        ap.redo = 1;
        e |= pq_launch(15, &ap, LN.side[1]);  // k_decode<2>: pages whose later parts failed, whole
      } else {
        e |= pq_launch(15, &a, LN.side[1]);  // k_decode<2>: the other flat BYTE_ARRAY pages
      }
      hipEventRecord(LN.join[1], LN.side[1]);
    }
    if (B->ngen_nest > 0) {
      if (!rsplit) hipStreamWaitEvent(LN.side[2], LN.fork, 0);  // (split: side stream 2 carries its own chain)
      a.list = B->d_lists + ns + nd + ndata + ng0 + B->ngen_flat + B->ngen_str;
      a.nlist = B->ngen_nest;
      const int32_t nparts = (int32_t)(B->nest_parts.size() / 3);
      if (nparts > B->ngen_nest) {
        pq_launch_args ap = a;
        ap.parts = B->d_parts;
        ap.nlist = nparts;
        static const bool k5_off = knob_flag("PQG_NO_DEC5");  // (analysis: the parts on <3>)
        e |= pq_launch(k5_off ? 16 : 32, &ap, LN.side[2]);  // k_decode<5>: parts of list pages of fixed-width values
        ap = a;
        ap.redo = 1;
        e |= pq_launch(16, &ap, LN.side[2]);  // k_decode<3>: pages whose later parts failed, whole
      } else {
        e |= pq_launch(16, &a, LN.side[2]);  // k_decode<3>: lists of fixed-width values
      }
      hipEventRecord(LN.join[2], LN.side[2]);
    }
    a.list = B->d_lists + ns + nd + ndata;
    a.nlist = ng0;
    e |= pq_launch(3, &a, s);  // k_decode<0>: lists of strings, booleans, level output
    // (round 4: k_plain_str beside k_decode<2> on another side stream, and
    // the tiled expand beside both, measured on C5 24.50 vs 24.28 ms — slower
    // then; with k_decode<4> for the dictionary strings both pay, see above
    // and below)
    // the tiled expand beside the string side stream, joined after it (round
    // 6, C5: 16.12 / 16.11 -> 15.97 / 15.92 ms, C4 unchanged; with round 4's
    // k_decode<2> for the dictionary strings it had been slower).
    // PQG_EXPAND_AFTER_STR=1 (analysis): after the strings, as before
    static const bool expand_after = knob_flag("PQG_EXPAND_AFTER_STR");
    const bool late_str_join = str_side && !expand_after && B->dba_list.empty();
    if (str_side && !late_str_join) hipStreamWaitEvent(s, LN.join[1], 0);
    if (!B->dba_list.empty()) {  // DELTA_BYTE_ARRAY value bytes (after k_decode's offsets)
      a.list = B->d_lists + ns + nd + ndata + ngen;
      a.nlist = (int32_t)B->dba_list.size();
      e |= pq_launch(10, &a, s);
    }
    a.nlist = (int32_t)B->tiles.size();
    // k_expand_wg (dictionaries that need a CU's LDS): after the mixed
    // launch, before it (PQG_BIG_ORDER=1) or beside it on a side stream (=2)
    static const int big_order = knob("PQG_BIG_ORDER") ? atoi(knob("PQG_BIG_ORDER")) : 0;
    const bool big = B->ldn[2] + B->ldn[3] > 0;
    if (big && big_order == 2) {
      hipEventRecord(LN.fork, s);
      hipStreamWaitEvent(LN.side[1], LN.fork, 0);
      e |= pq_launch(22, &a, LN.side[1]);
      hipEventRecord(LN.join[1], LN.side[1]);
    }
    if (big && big_order == 1) e |= pq_launch(22, &a, s);
    // a batch whose data pages all have host-written records (flat required
    // PLAIN: no level streams, no key-stream walk) gives k_level_check nothing
    // to find: k_expand_mix plans the next decode's statuses and the launch is
    // skipped (C1; PQG_LEVEL_CHECK=1 keeps it)
    const bool plan_next = ndata > 0 && !knob_flag("PQG_NO_STATUS_PLAN");
    // (likewise a batch without level streams: the run walk sets its own
    // errors, k_level_check would only re-walk levels — C2)
    const bool skip_check = ((B->all_srec && ngen == 0 && B->dba_list.empty()) || B->no_levels) &&
                            B->ldn[0] + B->ldn[1] > 0 && !knob_flag("PQG_LEVEL_CHECK");
    if (skip_check && plan_next) {
      pq_launch_args ax = a;
      ax.status_next = B->d_status + ((a.epoch + 1) & 1) * npages;
      e |= pq_launch(9, &ax, s);  // k_expand_mix (tiled pages) + the next statuses
    } else {
      e |= pq_launch(9, &a, s);  // k_expand_mix (tiled pages)
    }
    if (big && big_order == 0) e |= pq_launch(22, &a, s);
    if (big && big_order == 2) hipStreamWaitEvent(s, LN.join[1], 0);
    if (late_str_join) hipStreamWaitEvent(s, LN.join[1], 0);
    if (B->ngen_flat > 0 || pstr0 || wsplit) hipStreamWaitEvent(s, LN.join[0], 0);
    if (B->ngen_nest > 0 || n4w > 0) hipStreamWaitEvent(s, LN.join[2], 0);
    // nested (max_rep >= 2) columns: offsets and validity of every level
    // from the levels k_decode emitted
    if (!upto_scan) {
      for (const ColumnPlan &cp : B->cols) {
        if (!cp.nest_off) continue;
        const int R = cp.info.max_rep;
        hipMemsetAsync(cp.nest_val, 0, sizeof(uint32_t) * (size_t)((R + 1) * cp.nest_vstride), s);
        if (cp.levels == 0) {
          hipMemsetAsync(cp.nest_off, 0, sizeof(int32_t) * (size_t)(R * cp.nest_ostride), s);
          hipMemsetAsync(cp.nest_cnt, 0, sizeof(int64_t) * (size_t)(R + 1), s);
          continue;
        }
        NestArgs na;
        memset(&na, 0, sizeof(na));
        na.def = (const uint8_t *)cp.def_out;
        na.rep = (const uint8_t *)cp.rep_out;
        na.n = cp.levels;
        na.max_rep = R;
        na.max_def = cp.info.max_def;
        for (int k = 1; k <= R; k++) na.rdef[k] = cp.rdefs[(size_t)k - 1];
        na.sums = (int32_t *)cp.nest_sums;
        na.off = (int32_t *)cp.nest_off;
        na.val = (uint32_t *)cp.nest_val;
        na.ostride = cp.nest_ostride;
        na.vstride = cp.nest_vstride;
        na.cnt = (int64_t *)cp.nest_cnt;
        na.nblocks = cp.nest_nblocks;
        if (pq_launch_nest(&na, s)) e |= 1;
      }
    }
    mark(true);
    a.list = B->d_lists + ns + nd;
    a.nlist = ndata;
    // k_level_check also plans the next epoch's statuses (grid-strided copy of
    // the initial statuses into the other array)
    a.status_next = plan_next ? B->d_status + ((a.epoch + 1) & 1) * npages : nullptr;
    if (!skip_check) e |= pq_launch(5, &a, s);
    if (plan_next && !e) B->st_ready[(a.epoch + 1) & 1] = true;
    mark(false);
  }
  if (e) {
    set_err("kernel launch failed: kernel id %d: %s", pq_launch_fail_which, hipGetErrorString((hipError_t)pq_launch_fail_err));
    return PQG_ERR_DEVICE;
  }
  if (timed) {
    B->ring_head = (B->ring_head + 1) % pqg_batch::kRing;
    B->ring_count = std::min(B->ring_count + 1, pqg_batch::kRing);
  }
  return PQG_OK;
}

static LaneRef lane_of(pqg_batch *B) {
  pqg_ctx *c = B->ctx;
  if (B->lane == 1) return {c->lane1.stream, c->lane1.side, c->lane1.fork, c->lane1.join, &c->lane1.mu};
  return {c->stream, c->side, c->fork, c->join, &c->launch_mu};
}
static hipStream_t bstream(pqg_batch *B) { return B->lane == 1 ? B->ctx->lane1.stream : B->ctx->stream; }
void *pqg_batch_stream(const pqg_batch *b) {
  return b ? (void *)bstream(const_cast<pqg_batch *>(b)) : nullptr;
}

int pqg_batch_decode(pqg_batch *B) {
  if (!B) return PQG_ERR_ARG;
  HIPCHK(hipSetDevice(B->ctx->device));
  const bool timed = B->time_every > 0 && B->decodes % B->time_every == 0;
  B->decodes++;
  int rc = launch_all(B, false, timed);
  B->decoded = rc == 0;
  return rc;
}

int pqg_batch_set_timing(pqg_batch *B, int every) {
  if (!B || every < 0) return PQG_ERR_ARG;
  B->time_every = every;
  B->decodes = 0;
  return PQG_OK;
}

int pqg_batch_sync(pqg_batch *B) {
  if (!B) return PQG_ERR_ARG;
  HIPCHK(hipSetDevice(B->ctx->device));
  HIPCHK(hipStreamSynchronize(bstream(B)));
  const size_t npages = B->pages.size();
  std::vector<uint32_t> st(npages);
  if (npages)
    HIPCHK(hipMemcpy(st.data(), B->d_status + (B->epoch & 1) * npages, sizeof(uint32_t) * npages,
                     hipMemcpyDeviceToHost));
  // first error in the reference's order: row group, leaf, phase, page ordinal, stage
  struct Key {
    int rg, leaf, phase, ord;
    uint32_t stage, code;
  };
  bool have = false;
  Key best{};
  auto consider = [&](Key k) {
    auto t = [](const Key &x) { return std::make_tuple(x.rg, x.leaf, x.phase, x.ord, x.stage); };
    if (!have || t(k) < t(best)) {
      best = k;
      have = true;
    }
  };
  for (size_t i = 0; i < npages; i++) {
    if (st[i] == STATUS_OK) continue;
    const PageDesc &d = B->pages[i];
    uint32_t stage = st[i] >> 16, code = st[i] & STATUS_CODE;
    consider({d.rg, B->cols[(size_t)d.col].leaf, stage >= ST_PHASE2 ? 1 : 0, d.ord, stage, code});
  }
  for (auto &ce : B->chunk_errors) consider({ce.rg, ce.leaf, 0, ce.ord, ce.stage, ce.code});
  if (!have) {
    B->err_rg = B->err_leaf = B->err_page = -1;
    return PQG_OK;
  }
  B->err_rg = best.rg;
  B->err_leaf = best.leaf;
  B->err_page = best.ord;
  set_err("decode error %u at row group %d, column %d, page %d (stage %u)", best.code, best.rg, best.leaf, best.ord,
          best.stage);
  return (int)best.code;
}

int pqg_batch_row_groups(const pqg_batch *B, int *rg_begin, int *rg_end) {
  if (!B) return PQG_ERR_ARG;
  if (rg_begin) *rg_begin = B->rg_begin;
  if (rg_end) *rg_end = B->rg_end;
  return PQG_OK;
}

int pqg_batch_error_location(const pqg_batch *B, int *rg, int *leaf, int *page) {
  if (rg) *rg = B->err_rg;
  if (leaf) *leaf = B->err_leaf;
  if (page) *page = B->err_page;
  return PQG_OK;
}

int pqg_batch_column(const pqg_batch *B, int i, pqg_column_view *v) {
  if (!B || i < 0 || i >= (int)B->cols.size()) return PQG_ERR_ARG;
  const ColumnPlan &cp = B->cols[(size_t)i];
  memset(v, 0, sizeof(*v));
  v->values = cp.values;
  v->validity = cp.validity;
  v->list_offsets = cp.list_offsets;
  v->list_validity = cp.list_validity;
  v->str_offsets = cp.str_offsets;
  v->def_levels = cp.def_out;
  v->rep_levels = cp.rep_out;
  v->levels = cp.levels;
  v->slots = cp.slots;
  v->rows = cp.rows;
  v->str_bytes = cp.str_bytes;
  v->value_width = cp.info.value_width;
  v->leaf = cp.leaf;
  v->non_null = -1;
  return PQG_OK;
}

int pqg_batch_column_nest(const pqg_batch *B, int i, int level, void **offsets, void **validity, int64_t *count) {
  if (!B || i < 0 || i >= (int)B->cols.size()) return PQG_ERR_ARG;
  const ColumnPlan &cp = B->cols[(size_t)i];
  const int R = cp.info.max_rep;
  if (R < 2 || level < 1 || level > R + 1) return PQG_ERR_ARG;
  if (!cp.nest_off) {
    set_err("leaf %d: nested offsets need max_rep <= %d", cp.leaf, NEST_MAXR);
    return PQG_ERR_UNSUPPORTED;
  }
  HIPCHK(hipSetDevice(B->ctx->device));
  int64_t cnt[NEST_MAXR + 1];
  HIPCHK(hipMemcpy(cnt, cp.nest_cnt, sizeof(int64_t) * (size_t)(R + 1), hipMemcpyDeviceToHost));
  if (offsets) *offsets = level <= R ? (void *)((int32_t *)cp.nest_off + cp.nest_ostride * (level - 1)) : nullptr;
  if (validity) *validity = (void *)((uint32_t *)cp.nest_val + cp.nest_vstride * (level - 1));
  if (count) *count = cnt[level - 1];
  return PQG_OK;
}

int pqg_batch_copy_nest(pqg_batch *B, int i, int level, int what, void *dst, size_t cap, size_t *nbytes) {
  void *off = nullptr, *val = nullptr;
  int64_t n = 0;
  const int rc = pqg_batch_column_nest(B, i, level, &off, &val, &n);
  if (rc) return rc;
  const void *src = what == 0 ? off : val;
  const size_t bytes = what == 0 ? (off ? sizeof(int32_t) * (size_t)(n + 1) : 0) : (size_t)((n + 7) / 8);
  if (what != 0 && what != 1) return PQG_ERR_ARG;
  if (nbytes) *nbytes = bytes;
  if (!dst || !bytes) return PQG_OK;
  if (cap < bytes) {
    set_err("destination too small");
    return PQG_ERR_ARG;
  }
  HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
  return PQG_OK;
}

int pqg_batch_copy(pqg_batch *B, int i, int buf, void *dst, size_t cap, size_t *nbytes) {
  if (!B || i < 0 || i >= (int)B->cols.size()) return PQG_ERR_ARG;
  HIPCHK(hipSetDevice(B->ctx->device));
  const ColumnPlan &cp = B->cols[(size_t)i];
  const void *src = nullptr;
  size_t n = 0;
  switch (buf) {
    case PQG_BUF_VALUES: src = cp.values; n = cp.values_bytes; break;
    case PQG_BUF_VALIDITY: src = cp.validity; n = (size_t)((cp.slots + 7) / 8); break;
    case PQG_BUF_LIST_OFFSETS: src = cp.list_offsets; n = cp.list_off_bytes; break;
    case PQG_BUF_LIST_VALIDITY: src = cp.list_validity; n = (size_t)((cp.rows + 7) / 8); break;
    case PQG_BUF_STR_OFFSETS: src = cp.str_offsets; n = cp.str_off_bytes; break;
    case PQG_BUF_DEF: src = cp.def_out; n = cp.def_out ? (size_t)cp.levels : 0; break;
    case PQG_BUF_REP: src = cp.rep_out; n = cp.rep_out ? (size_t)cp.levels : 0; break;
    default: return PQG_ERR_ARG;
  }
  if (!src) n = 0;
  if (nbytes) *nbytes = n;
  if (!dst) return PQG_OK;
  if (cap < n) {
    set_err("buffer too small (%zu < %zu)", cap, n);
    return PQG_ERR_ARG;
  }
  if (n) {
    HIPCHK(hipStreamSynchronize(bstream(B)));
    HIPCHK(hipMemcpy(dst, src, n, hipMemcpyDeviceToHost));
  }
  return PQG_OK;
}

// ABI 2: the caller passes sizeof its struct; only that many bytes are
// written, so a caller built against an older (shorter) header is never
// overrun, and a newer one sees zeros in fields this library lacks.
int pqg_batch_stats_get(const pqg_batch *B, pqg_batch_stats *out, size_t size) {
  if (!B || !out || size < offsetof(pqg_batch_stats, create_plan_ms)) return PQG_ERR_ARG;
  pqg_batch_stats full;
  pqg_batch_stats *o = &full;
  memset(o, 0, sizeof(*o));
  o->pages = (int64_t)B->pages.size();
  o->data_pages = (int64_t)B->data_list.size();
  o->dict_pages = 0;
  for (const PageDesc &pd : B->pages) o->dict_pages += pd.kind == PAGE_DICT;
  o->snappy_pages = (int64_t)B->snappy_list.size();
  o->host_inflated_pages = B->host_inflated;
  o->gzip_device_pages = (int64_t)B->gzip_list.size();
  o->gzip_in_bytes = B->gzip_in_bytes;
  o->staged_bytes = B->staged_bytes;
  o->h2d_bytes = B->h2d_bytes;
  o->create_plan_ms = B->create_ms[0];
  o->create_alloc_ms = B->create_ms[1];
  o->create_upload_ms = B->create_ms[2];
  o->create_tables_ms = B->create_ms[3];
  o->upload_gather_ms = B->upload_gather_ms;
  o->upload_wait_ms = B->upload_wait_ms;
  // B_in: stored payload bytes of the planned pages
  int64_t bin = 0;
  for (auto &d : B->pages) {
    int64_t lsize = d.kind == PAGE_V2 ? (int64_t)d.v2_rep_len + d.v2_def_len : 0;
    bin += (int64_t)d.comp_len + lsize;
  }
  o->input_bytes = bin;
  for (int32_t pi : B->snappy_list) o->snappy_in_bytes += B->pages[(size_t)pi].comp_len;
  for (auto &d : B->pages)
    if (d.kind == PAGE_DICT) o->dict_bytes += d.body_len;
  int64_t bout = 0;
  for (auto &cp : B->cols) {
    bout += (int64_t)cp.values_bytes;
    if (cp.validity) bout += (cp.slots + 7) / 8;
    if (cp.list_offsets) bout += (int64_t)cp.list_off_bytes + (cp.rows + 7) / 8;
    if (cp.str_offsets) bout += (int64_t)cp.str_off_bytes;
  }
  o->output_bytes = bout;
  memset(out, 0, size);
  memcpy(out, o, std::min(size, sizeof(full)));
  return PQG_OK;
}

// Average per-kernel device time over the decodes issued since the previous
// call (up to the last 64), from HIP events recorded on the context stream
// between consecutive launches: [snappy, dict, prepare, scan, decode, level_check].
int pqg_batch_kernel_times(pqg_batch *B, const char **names, float *ms, int cap) {
  int n = B->nev > 0 ? B->nev - 1 : 0;
  if (hipSetDevice(B->ctx->device) != hipSuccess) return 0;
  if (B->ring_count > 0) {
    hipStreamSynchronize(bstream(B));
    for (int i = 0; i < 8; i++) B->kms_sum[i] = 0;
    B->kms_n = 0;
    for (int k = 0; k < B->ring_count; k++) {
      int slot = (B->ring_head - 1 - k + 2 * pqg_batch::kRing) % pqg_batch::kRing;
      for (int i = 0; i < n; i++) {
        float t = 0;
        hipEventElapsedTime(&t, B->ev[slot][i], B->ev[slot][i + 1]);
        B->kms_sum[i] += t;
      }
      B->kms_n++;
    }
    B->ring_count = 0;
  }
  for (int i = 0; i < n && i < cap; i++) {
    if (names) names[i] = B->seg_times ? kSegNames[i] : kDecodeName[i];
    if (ms) ms[i] = B->kms_n ? (float)(B->kms_sum[i] / B->kms_n) : 0.f;
  }
  return n;
}

void pqg_batch_destroy(pqg_batch *B) {
  if (!B) return;
  hipSetDevice(B->ctx->device);
  // an upload never decoded may still be in flight; a batch whose set-up
  // failed part-way may have copies queued after its last `ready` record
  if (B->ready_final) hipEventSynchronize(B->ready);
  else hipStreamSynchronize(B->ctx->upload);
  hipStreamSynchronize(bstream(B));
  for (auto &cp : B->cols) {
    free_dev(cp.values);
    free_dev(cp.validity);
    free_dev(cp.list_offsets);
    free_dev(cp.list_validity);
    free_dev(cp.str_offsets);
    free_dev(cp.def_out);
    free_dev(cp.rep_out);
    free_dev(cp.nest_off);
    free_dev(cp.nest_val);
    free_dev(cp.nest_sums);
    free_dev(cp.nest_cnt);
  }
  free_dev(B->d_in_alloc);
  free_dev(B->d_info);
  free_dev(B->d_recs);
  free_dev(B->d_stage);
  free_dev(B->d_status);
  free_dev(B->d_cols);
  free_dev(B->d_dict);
  free_dev(B->d_jobs);
  free_dev(B->d_njobs);
  free_dev(B->d_zr);
  free_dev(B->d_copy_idx);
  free_dev(B->d_lens);
  free_dev(B->d_sw_regs);
  free_dev(B->d_sw_res);
  free_dev(B->d_lvl);
  free_dev(B->d_dbg);
  free_dev(B->d_dbg2);
  free_dev(B->d_runs_alloc);
  free_dev(B->d_tile_info);
  free_dev(B->d_tiles);
  free_dev(B->d_segs);
  if (B->ready) hipEventDestroy(B->ready);
  for (int k = 0; k < pqg_batch::kRing; k++)
    for (int i = 0; i < 8; i++)
      if (B->ev[k][i]) hipEventDestroy(B->ev[k][i]);
  delete B;
}

// ---------------------------------------------------------------------------
// pipelined row-group slices (pqg_stream)
// ---------------------------------------------------------------------------
struct pqg_stream {
  pqg_ctx *ctx = nullptr;
  pqg_file *f = nullptr;
  std::vector<int> leaves;
  int flags = 0, depth = 2;
  std::vector<std::pair<int, int>> slices;
  std::vector<pqg_batch *> built;  // per slice, set by the worker
  std::vector<int> rcs;
  std::vector<std::string> errs;
  std::vector<char> done;     // per slice: built (or failed)
  std::vector<char> launched;  // per slice: its decode already launched (ahead of its turn)
  std::vector<int> lrc;        // that launch's status
  int lanes = 2;              // decode lanes: slice k on lane k % 2 (PQG_STREAM_LANES=1: one)
  size_t next_build = 0;      // next slice a worker takes
  size_t ntaken = 0;
  bool stop = false, failed = false;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::thread> workers;
  pqg_batch *cur = nullptr;  // the slice last handed out
};

// Several workers build slices concurrently (host planning, allocation and
// table set-up of different slices overlap; the pinned-ring uploads take
// turns on the context's upload stream), each taking the next slice index
// while at most `depth` slices are built ahead of the one the caller holds.
static void stream_worker(pqg_stream *S) {
  hipSetDevice(S->ctx->device);
  for (;;) {
    size_t k;
    {
      std::unique_lock<std::mutex> lk(S->mu);
      S->cv.wait(lk, [&] {
        return S->stop || S->failed || S->next_build >= S->slices.size() || S->next_build < S->ntaken + (size_t)S->depth;
      });
      if (S->stop || S->failed || S->next_build >= S->slices.size()) return;
      k = S->next_build++;
    }
    pqg_batch *B = nullptr;
    const int rc = batch_create_lane(S->ctx, S->f, S->slices[k].first, S->slices[k].second,
                                     S->leaves.empty() ? nullptr : S->leaves.data(), (int)S->leaves.size(), S->flags,
                                     S->lanes > 1 ? (int)(k & 1) : 0, &B);
    std::lock_guard<std::mutex> lk(S->mu);
    S->built[k] = B;
    S->rcs[k] = rc;
    if (rc) {
      S->errs[k] = g_err;  // the worker's thread-local message
      S->failed = true;    // no slice after a failed one is started
    }
    S->done[k] = 1;
    S->cv.notify_all();
  }
}

int pqg_stream_open(pqg_ctx *ctx, pqg_file *f, int rg_begin, int rg_end, const int *leaves, int nleaves, int flags,
                    int rgs_per_slice, int depth, pqg_stream **out) {
  *out = nullptr;
  if (!ctx || !f || rg_begin < 0 || rg_end > (int)f->rgs.size() || rg_begin > rg_end || nleaves < 0 ||
      rgs_per_slice < 1 || depth < 1) {
    set_err("bad stream arguments");
    return PQG_ERR_ARG;
  }
  for (int i = 0; i < nleaves; i++)
    if (!leaves || leaves[i] < 0 || leaves[i] >= (int)f->leaves.size()) {
      set_err("leaf out of range");
      return PQG_ERR_ARG;
    }
  pqg_stream *S = new pqg_stream();
  S->ctx = ctx;
  S->f = f;
  if (nleaves > 0) S->leaves.assign(leaves, leaves + nleaves);
  S->depth = depth;
  // (PQG_STREAM_RAMP: slices of a quarter and a half first, so the pipeline
  // fills after a short upload; the flag is the stream's, not the batches')
  const bool ramp = (flags & PQG_STREAM_RAMP) != 0;
  S->flags = flags & ~PQG_STREAM_RAMP;
  for (int r = rg_begin, k = 0; r < rg_end; k++) {
    const int per = !ramp || k >= 2 ? rgs_per_slice : std::max(1, rgs_per_slice / (k == 0 ? 4 : 2));
    S->slices.push_back({r, std::min(rg_end, r + per)});
    r += per;
  }
  S->built.assign(S->slices.size(), nullptr);
  S->rcs.assign(S->slices.size(), 0);
  S->errs.assign(S->slices.size(), std::string());
  S->done.assign(S->slices.size(), 0);
  S->launched.assign(S->slices.size(), 0);
  S->lrc.assign(S->slices.size(), 0);
  if (knob("PQG_STREAM_LANES") && atoi(knob("PQG_STREAM_LANES")) == 1) S->lanes = 1;
  const char *w = getenv("PQG_STREAM_WORKERS");
  const int nw = std::max(1, std::min({w ? atoi(w) : 3, depth, (int)std::max<size_t>(1, S->slices.size())}));
  for (int i = 0; i < nw; i++) S->workers.emplace_back(stream_worker, S);
  *out = S;
  return PQG_OK;
}

int pqg_stream_next(pqg_stream *S, pqg_batch **out, int *rg_first) {
  *out = nullptr;
  if (!S) return PQG_ERR_ARG;
  if (S->cur) {  // the caller is done with the previous slice
    pqg_batch_destroy(S->cur);
    S->cur = nullptr;
  }
  size_t k;
  {
    std::unique_lock<std::mutex> lk(S->mu);
    k = S->ntaken;
    if (k >= S->slices.size()) return PQG_OK;
    // a slice never started after an earlier one failed: the stream ends
    S->cv.wait(lk, [&] { return S->done[k] || (S->failed && k >= S->next_build); });
    if (!S->done[k]) {
      S->ntaken = S->slices.size();
      return PQG_OK;
    }
    S->ntaken = k + 1;
    S->cv.notify_all();
    if (S->rcs[k]) {
      set_err("%s", S->errs[k].c_str());
      S->ntaken = S->slices.size();  // nothing after a failed slice
      return S->rcs[k];
    }
  }
  pqg_batch *B = S->built[k];
  S->built[k] = nullptr;
  const int rc = S->launched[k] ? S->lrc[k] : pqg_batch_decode(B);
  S->cur = B;
  if (rc) return rc;
  // decode-ahead: the next slice, if built, starts on the other lane now — it
  // runs beside this one's tail (a slice's decode lasts at least its longest
  // page chain) and while the caller consumes this one
  if (S->lanes > 1 && k + 1 < S->slices.size()) {
    pqg_batch *N = nullptr;
    {
      std::lock_guard<std::mutex> lk(S->mu);
      if (S->done[k + 1] && !S->rcs[k + 1] && S->built[k + 1]) N = S->built[k + 1];
    }
    if (N) {
      S->lrc[k + 1] = pqg_batch_decode(N);
      S->launched[k + 1] = 1;
    }
  }
  *out = B;
  if (rg_first) *rg_first = S->slices[k].first;
  return PQG_OK;
}

void pqg_stream_close(pqg_stream *S) {
  if (!S) return;
  {
    std::lock_guard<std::mutex> lk(S->mu);
    S->stop = true;
    S->cv.notify_all();
  }
  for (auto &t : S->workers)
    if (t.joinable()) t.join();
  if (S->cur) pqg_batch_destroy(S->cur);
  for (pqg_batch *B : S->built)
    if (B) pqg_batch_destroy(B);
  delete S;
}

}  // extern "C"

// single-block device snappy for pqg_decompress_block
static int device_snappy_block(pqg_ctx *ctx, const uint8_t *src, size_t n, uint8_t *dst, size_t expect, int *code) {
  HIPCHK(hipSetDevice(ctx->device));
  hipStream_t s = ctx->stream;
  uint8_t *d_in = nullptr, *d_out = nullptr;
  PageDesc *d_page = nullptr;
  uint32_t *d_st = nullptr;
  int32_t *d_list = nullptr;
  int rc = 0;
  rc |= alloc_dev((void **)&d_in, n);
  rc |= alloc_dev((void **)&d_out, expect);
  rc |= alloc_dev((void **)&d_page, sizeof(PageDesc));
  rc |= alloc_dev((void **)&d_st, sizeof(uint32_t));
  rc |= alloc_dev((void **)&d_list, sizeof(int32_t));
  void *d_jobs = nullptr;
  uint32_t *d_njobs = nullptr;
  int32_t *d_jb = nullptr, *d_jo = nullptr;
  const uint32_t max_jobs = (uint32_t)std::min<size_t>(64, expect / (16 * 1024));
  rc |= alloc_dev(&d_jobs, 32 * (size_t)max_jobs);
  rc |= alloc_dev((void **)&d_njobs, 16);
  rc |= alloc_dev((void **)&d_jb, 16);
  rc |= alloc_dev((void **)&d_jo, 4 * (size_t)(max_jobs + 1));
  uint32_t *d_cc = nullptr;
  int32_t *d_ci = nullptr;
  int32_t *d_sitems = nullptr, *d_sbase = nullptr, *d_walk = nullptr;
  int64_t *d_segs = nullptr;
  uint32_t *d_sflag = nullptr;
  rc |= alloc_dev((void **)&d_cc, 16);
  rc |= alloc_dev((void **)&d_ci, 4 * (size_t)(max_jobs + 1));
  if (!rc) hipMemsetAsync(d_cc, 0, 16, s);
  if (!rc) {
    int32_t zero4[4] = {0, 0, 0, 0};
    hipMemcpyAsync(d_jb, zero4, 16, hipMemcpyHostToDevice, s);
    std::vector<int32_t> owners(max_jobs + 1, 0);
    hipMemcpyAsync(d_jo, owners.data(), 4 * owners.size(), hipMemcpyHostToDevice, s);
    hipStreamSynchronize(s);  // host sources go out of scope
  }
  if (!rc) {
    PageDesc d;
    memset(&d, 0, sizeof(d));
    d.part0 = -1;
    d.sp_base = -1;
    d.kind = PAGE_DICT;
    d.comp_len = (int32_t)n;
    d.body_len = (int32_t)expect;
    d.body_src = BODY_SNAPPY;
    uint32_t st = STATUS_OK;
    int32_t zero = 0;
    hipMemcpyAsync(d_in, src, n, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_page, &d, sizeof(d), hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_st, &st, 4, hipMemcpyHostToDevice, s);
    hipMemcpyAsync(d_list, &zero, 4, hipMemcpyHostToDevice, s);
    pq_launch_args a = {};
    memset(&a, 0, sizeof(a));
    a.snappy_wg = getenv_flag("PQG_SNAPPY_WG") ? 1 : 0;
    a.in = d_in;
    a.stage = d_out;
    a.in_end = d_in + n + kPad;
    a.stage_end = d_out + expect + kPad;
    a.pages = d_page;
    a.status = d_st;
    a.list = d_list;
    a.nlist = 1;
    a.jobs = d_jobs;
    a.njobs = d_njobs;
    a.max_jobs = max_jobs;
    a.job_base = d_jb;
    a.job_owner = d_jo;
    a.copy_cnt = d_cc;
    a.copy_idx = d_ci;
    a.dbg = nullptr;
    // one page, cut into segments like a batch's long pages
    const int32_t nseg = expect > (size_t)kSnapSeg ? (int32_t)((expect + kSnapSeg - 1) / kSnapSeg) : 1;
    std::vector<int32_t> items;
    for (int32_t k = 0; k < nseg; k++) items.push_back(0), items.push_back(k);
    const int32_t seg_base[2] = {0, nseg}, walk0 = 0;
    rc |= alloc_dev((void **)&d_sitems, 4 * items.size());
    rc |= alloc_dev((void **)&d_sbase, 8);
    rc |= alloc_dev((void **)&d_walk, 4);
    rc |= alloc_dev((void **)&d_segs, 8 * (size_t)nseg);
    rc |= alloc_dev((void **)&d_sflag, 4);
    if (!rc) {
      hipMemcpy(d_sitems, items.data(), 4 * items.size(), hipMemcpyHostToDevice);
      hipMemcpy(d_sbase, seg_base, 8, hipMemcpyHostToDevice);
      hipMemcpy(d_walk, &walk0, 4, hipMemcpyHostToDevice);
      hipMemset(d_sflag, 0, 4);
    }
    a.sitems = d_sitems;
    a.nitems = nseg;
    a.walk = d_walk;
    a.nwalk = nseg > 1 ? 1 : 0;
    a.seg_base = d_sbase;
    a.segs = d_segs;
    a.seg_flag = d_sflag;
    PageInfo *d_info = nullptr;
    rc |= alloc_dev((void **)&d_info, sizeof(PageInfo));
    hipMemsetAsync(d_info, 0, sizeof(PageInfo), s);
    a.info = d_info;
    hipDeviceSynchronize();  // null-stream set-up before the launches on the non-blocking stream
    rc |= pq_launch(17, &a, s);
    rc |= pq_launch(0, &a, s);
    rc |= pq_launch(18, &a, s);
    rc |= pq_launch(6, &a, s);
    const hipError_t e1 = hipStreamSynchronize(s);
    if (e1 != hipSuccess) {
      set_err("HIP error %s in the snappy kernels", hipGetErrorString(e1));
      rc |= PQG_ERR_DEVICE;
    }
    PageInfo hi;
    hipMemcpyAsync(&hi, d_info, sizeof(hi), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    if (hi.alias1 && expect) hipMemcpyAsync(d_out, d_in + (hi.alias1 - 1), expect, hipMemcpyDeviceToDevice, s);
    free_dev(d_info);
    hipStreamSynchronize(s);
    hipMemcpyAsync(&st, d_st, 4, hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    *code = st == STATUS_OK ? 0 : (int)(st & 0xffff);
    if (!*code && expect) {
      hipMemcpyAsync(dst, d_out, expect, hipMemcpyDeviceToHost, s);
      hipStreamSynchronize(s);
    }
  }
  free_dev(d_in);
  free_dev(d_out);
  free_dev(d_page);
  free_dev(d_st);
  free_dev(d_list);
  free_dev(d_jobs);
  free_dev(d_njobs);
  free_dev(d_cc);
  free_dev(d_ci);
  free_dev(d_jb);
  free_dev(d_jo);
  free_dev(d_sitems);
  free_dev(d_sbase);
  free_dev(d_walk);
  free_dev(d_segs);
  free_dev(d_sflag);
  if (rc) {
    if (g_err.empty()) set_err("device snappy failed");
    return PQG_ERR_DEVICE;
  }
  return PQG_OK;
}

#ifdef PQ_STAMPS
// diagnostic build only (not part of include/pqgpu.h): copy the stamp buffer
// diagnostic: zero the stamp buffers (before the decode a tool reads back)
extern "C" int pqg_diag_reset(pqg_batch *B) {
  hipStreamSynchronize(bstream(B));
  const size_t n1 = std::max(8 * 4 * (B->tiles.size() + 1), 4 * (B->pages.size() + 1));
  const size_t n2 = 16 * (B->pages.size() + 1) + 256;
  if (B->d_dbg) hipMemset(B->d_dbg, 0, 8 * n1);
  if (B->d_dbg2) hipMemset(B->d_dbg2, 0, 8 * n2);
  return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
// diagnostic: per page (column << 8 | kind), for the stamp tools
extern "C" int pqg_diag_page_cols(pqg_batch *B, int32_t *out, size_t n) {
  size_t k = 0;
  for (; k < n && k < B->pages.size(); k++) out[k] = (B->pages[k].col << 8) | B->pages[k].kind;
  return (int)k;
}
extern "C" int pqg_diag_stamps(pqg_batch *B, uint64_t *out, size_t n) {
  hipStreamSynchronize(bstream(B));
  size_t cap = std::max(8 * 4 * (B->tiles.size() + 1), 4 * (B->pages.size() + 1));
  if (n > cap) n = cap;
  return hipMemcpy(out, B->d_dbg, n * 8, hipMemcpyDeviceToHost) == hipSuccess ? (int)n : -1;
}
extern "C" int pqg_diag_stamps2(pqg_batch *B, uint64_t *out, size_t n) {
  hipStreamSynchronize(bstream(B));
  size_t cap = 16 * (B->pages.size() + 1) + 256;
  if (n > cap) n = cap;
  return hipMemcpy(out, B->d_dbg2, n * 8, hipMemcpyDeviceToHost) == hipSuccess ? (int)n : -1;
}
#endif
