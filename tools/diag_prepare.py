"""Diagnostic: per-page k_prepare / run-walk times (libpqgpu_diag.so).
usage: python tools/diag_prepare.py BW [ROWS]   (BW 0 = the bench's 1..20 sweep)"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parquet-go_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ["PQGPU_LIB"] = "libpqgpu_diag.so"
import pqgpu  # noqa: E402
import synth  # noqa: E402

bw = int(sys.argv[1])
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 20_000_000
path = "/tmp/diag_bw%d_%d.parquet" % (bw, rows)
if not os.path.exists(path):
    synth.make("c2", path, rows, 1 << 20, fixed_bw=bw)
b = pqgpu.FileReader(path).batch()
for _ in range(3):
    b.decode()
b.sync()
L = pqgpu.lib()
L.pqg_diag_stamps2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
n = 8 * 200000 + 256
out = np.zeros(n, np.uint64)
got = L.pqg_diag_stamps2(b._h, out.ctypes.data, n)
s = out[:got - 256].reshape(-1, 8).astype(np.int64)
s = s[(s[:, 0] > 0) & (s[:, 2] > 0)]
t0 = s[:, 0].min()
pre = (s[:, 1] - s[:, 0]) / 100.0
walk = (s[:, 2] - s[:, 1]) / 100.0
end = (s[:, 2] - t0) / 100.0
print("pages", len(s), "span us %.1f" % end.max())
print("prologue median %.2f p90 %.2f max %.2f" % (np.median(pre), np.percentile(pre, 90), pre.max()))
print("walk     median %.2f p90 %.2f max %.2f" % (np.median(walk), np.percentile(walk, 90), walk.max()))
for w in sorted(set(s[:, 4].tolist())):
    m = s[:, 4] == w
    print("bw %2d pages %5d walk median %6.2f max %6.2f us  runs median %5d  iters median %5d" % (
        w, m.sum(), np.median(walk[m]), walk[m].max(), np.median(s[m, 3]), np.median(s[m, 5])))
st = (s[:, 0] - t0) / 100.0
h, e = np.histogram(st, bins=10)
print("starts:", h, "edges %.1f..%.1f" % (e[0], e[-1]))
# run-walk iterations of page 1 (dbg3, after the per-page block)
npg = (got - 256) // 8
it = out[8 * npg: 8 * npg + 240].reshape(-1, 4).astype(np.int64)
it = it[it[:, 0] > 0]
if len(it):
    print("page 1 walk iterations (us since first, hpos, v, runs):")
    for k in range(len(it)):
        print("  %6.2f  %6d %6d %4d" % ((it[k, 0] - it[0, 0]) / 100.0, it[k, 1], it[k, 2], it[k, 3]))
