"""GZIP pages: k_inflate on the GPU against zlib on the host, on one file.

usage: python tools/gzip_ab.py [--config c5gz] [--rows N] [--rg-rows N]
                               [--threads T] [--decodes K] [--file PATH]

Writes the config's file (tools/synth.py; c5gz = C5's lineitem columns under
GZIP) unless --file is given, then prints one JSON line:

* members: the file's gzip pages, their compressed and uncompressed bytes
  (from the page headers, walked with tools/page_runs.py's thrift reader);
* zlib on the host: every member inflated by zlib.decompress (the C zlib the
  library's host path calls; it releases the GIL) on 1 thread and on T
  threads — GB/s of uncompressed output;
* k_inflate: the whole file as one batch; the codec phase (PQG_SEGMENT_TIMES=1
  segment 0, which holds k_inflate alone when no page is Snappy) per decode,
  and GB/s of uncompressed output;
* the batch both ways: create (plan) ms — zlib runs inside the plan with
  PQG_BATCH_HOST_INFLATE, single-threaded — and decode ms.
"""
import argparse
import json
import os
import sys
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd"), os.path.join(ROOT, "tools")]

import page_runs  # noqa: E402
import synth  # noqa: E402


def members(path):
    import pyarrow.parquet as pq
    md = pq.ParquetFile(path).metadata
    data = open(path, "rb").read()
    out = []
    for rg in range(md.num_row_groups):
        for c in range(md.num_columns):
            cc = md.row_group(rg).column(c)
            assert cc.compression == "GZIP", cc.compression
            off = cc.dictionary_page_offset if cc.has_dictionary_page and cc.dictionary_page_offset else \
                cc.data_page_offset
            end = off + cc.total_compressed_size
            while off < end:
                h, i = page_runs.skip_struct(data, off)
                usize, csize = h[2], h[3]
                lsize = 0
                if 8 in h:  # DataPageHeaderV2: level bytes stored before the member
                    lsize = h[8].get(5, 0) + h[8].get(6, 0)
                out.append((data[i + lsize:i + csize], usize - lsize))
                off = i + csize
    return out


def zlib_rate(ms, threads):
    def one(m):
        return len(zlib.decompress(m[0], 31))
    t0 = time.perf_counter()
    if threads == 1:
        n = sum(one(m) for m in ms)
    else:
        with ThreadPoolExecutor(threads) as ex:
            n = sum(ex.map(one, ms, chunksize=4))
    dt = time.perf_counter() - t0
    return n, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5gz")
    ap.add_argument("--rows", type=int, default=0)
    ap.add_argument("--rg-rows", type=int, default=0)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--decodes", type=int, default=5)
    ap.add_argument("--file", default=None)
    args = ap.parse_args()
    rows = args.rows or synth.DEFAULTS[args.config][0]
    rg_rows = args.rg_rows or synth.DEFAULTS[args.config][1]
    path = args.file
    if not path:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        path = os.path.join(ROOT, "gpurun_out", "%s_%d_%d.parquet" % (args.config, rows, rg_rows))
        if not os.path.exists(path):
            synth.make(args.config, path, rows, rg_rows)
    ms = members(path)
    comp = sum(len(m) for m, _ in ms)
    unc = sum(u for _, u in ms)
    line = {"file": os.path.basename(path), "members": len(ms), "compressed_bytes": comp,
            "uncompressed_bytes": unc}
    n1, t1 = zlib_rate(ms, 1)
    assert n1 == unc, (n1, unc)
    nt, tt = zlib_rate(ms, args.threads)
    line["zlib_1thread"] = {"ms": round(t1 * 1e3, 2), "GBps": round(unc / t1 / 1e9, 3)}
    line["zlib_threads"] = {"threads": args.threads, "cores": len(os.sched_getaffinity(0)),
                            "ms": round(tt * 1e3, 2), "GBps": round(unc / tt / 1e9, 3)}

    import pqgpu
    ctx = pqgpu.Context(0)
    reader = pqgpu.FileReader(path, ctx=ctx)
    nrg = reader.RowGroupCount()
    leaves = list(range(len(reader.Columns())))
    for name, flags in (("device", 0), ("host", pqgpu.BATCH_HOST_INFLATE)):
        os.environ["PQG_SEGMENT_TIMES"] = "1"
        try:
            t0 = time.perf_counter()
            b = reader.batch(0, nrg, leaves, flags)
            create_ms = (time.perf_counter() - t0) * 1e3
        finally:
            del os.environ["PQG_SEGMENT_TIMES"]
        st = b.stats()
        b.decode()
        b.sync()
        seg = {}
        t0 = time.perf_counter()
        for _ in range(args.decodes):
            b.decode()
            b.sync()
            kt = b.kernel_times()
            for k, v in kt.items():
                seg[k] = seg.get(k, 0.0) + v / args.decodes
        dec_ms = (time.perf_counter() - t0) * 1e3 / args.decodes
        ent = {"create_ms": round(create_ms, 2), "create_plan_ms": round(st["create_plan_ms"], 2),
               "decode_ms_wall": round(dec_ms, 3), "segments_ms": {k: round(v, 4) for k, v in seg.items()},
               "gzip_device_pages": st["gzip_device_pages"], "host_inflated_pages": st["host_inflated_pages"],
               "h2d_bytes": st["h2d_bytes"]}
        if name == "device":
            codec_ms = seg.get("k_snappy+k_copy", 0.0)
            ent["k_inflate_phase_ms"] = round(codec_ms, 4)
            if codec_ms > 0:
                ent["k_inflate_GBps"] = round(unc / (codec_ms * 1e-3) / 1e9, 3)
        line[name] = ent
        b.close()
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
