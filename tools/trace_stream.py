"""Diagnostic: pqg_stream over a bench file — host time per slice (next() +
sync) and, with PQG_TRACE_CREATE=1, each batch creation's phases on stderr.
usage: python tools/trace_stream.py FILE [rgs_per_slice] [depth]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parquet-go_amd"))
import pqgpu  # noqa: E402

path = sys.argv[1]
per = int(sys.argv[2]) if len(sys.argv) > 2 else 8
depth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
r = pqgpu.FileReader(path)
r.batch(0, 1).close()  # runtime set-up
for rep in range(3):
    t0 = time.perf_counter()
    last = t0
    marks = []
    with r.stream(0, None, per, None, depth) as st:
        for b in st:
            b.sync()
            t = time.perf_counter()
            marks.append(round((t - last) * 1e3, 2))
            last = t
    print("pass %d: %.2f ms total, per slice ms %s" % (rep, (time.perf_counter() - t0) * 1e3, marks), flush=True)
