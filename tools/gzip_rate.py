"""k_inflate's per-wave rate: files of P GZIP pages of one shape, each page
one wave, the codec phase timed (PQG_SEGMENT_TIMES=1 segment 0).  With P at
most the wave slots (4 a CU) the phase time is one page's decode, so
page bytes / time is a single wave's rate; larger P shows the aggregate.

usage: python tools/gzip_rate.py [--pages 1,64,1024] [--kb 1024] [--shape text|ints|random]
Prints one JSON line per (shape, pages)."""
import argparse
import io
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parquet-go_amd")]


def make(shape, pages, kb):
    import pyarrow as pa
    import pyarrow.parquet as pq
    rng = np.random.default_rng(7)
    if shape == "text":  # l_comment-like: random letters and spaces, 10..43 bytes
        letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz     ", np.uint8)
        n = kb * 1024 // 31
        clen = rng.integers(10, 44, n * pages)
        off = np.zeros(n * pages + 1, np.int32)
        off[1:] = np.cumsum(clen)
        dat = letters[rng.integers(0, len(letters), int(off[-1]))]
        arr = pa.StringArray.from_buffers(n * pages, pa.py_buffer(off.tobytes()), pa.py_buffer(dat.tobytes()))
        use_dict = False
    elif shape == "ints":  # small integers: compressible
        n = kb * 1024 // 8
        arr = pa.array(rng.integers(0, 1000, n * pages))
        use_dict = False
    else:  # random 64-bit: stored blocks
        n = kb * 1024 // 8
        arr = pa.array(rng.integers(-(1 << 62), 1 << 62, n * pages))
        use_dict = False
    t = pa.table({"v": arr})
    buf = io.BytesIO()
    pq.write_table(t, buf, compression="gzip", use_dictionary=use_dict, data_page_size=kb * 1024 * 2,
                   row_group_size=n, write_statistics=False)
    return buf.getvalue()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pages", default="1,256,1024,4096")
    ap.add_argument("--kb", type=int, default=1024)
    ap.add_argument("--shape", default="text,ints,random")
    ap.add_argument("--decodes", type=int, default=3)
    args = ap.parse_args()
    import pqgpu
    for shape in args.shape.split(","):
        for pages in [int(x) for x in args.pages.split(",")]:
            data = make(shape, pages, args.kb)
            r = pqgpu.FileReader(data)
            os.environ["PQG_SEGMENT_TIMES"] = "1"
            try:
                b = r.batch(0, r.RowGroupCount(), [0], 0)
            finally:
                del os.environ["PQG_SEGMENT_TIMES"]
            st = b.stats()
            b.decode()
            b.sync()
            ms = 0.0
            for _ in range(args.decodes):
                b.decode()
                b.sync()
                ms += b.kernel_times().get("k_snappy+k_copy", 0.0) / args.decodes
            b.close()
            unc = st["staged_bytes"]
            print(json.dumps({"shape": shape, "pages": st["gzip_device_pages"], "uncompressed_bytes": unc,
                              "compressed_bytes": st["gzip_in_bytes"], "k_inflate_ms": round(ms, 3),
                              "GBps": round(unc / (ms * 1e-3) / 1e9, 3) if ms else None,
                              "per_page_MBps": round(unc / st["gzip_device_pages"] / (ms * 1e-3) / 1e6, 2)
                              if ms else None}), flush=True)


if __name__ == "__main__":
    main()
